#!/bin/bash
# Round evidence on the GPU box: rocprofv3 kernel stats of the bench command,
# then the PMC passes (one counter group per run, --kernel-trace-free) over a
# one-step bench of the same workload (same vocabulary counts, so the same
# default grid and stripes) whose per-example bytes feed roofline.traffic.
#   usage: scripts/profile_round.sh r02 [extra bench args, e.g. the C4 shape, for every run]
set -e
R=${1:?round tag}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$R
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o bench --output-format csv \
  -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench_stats.log" 2>&1
echo "stats pass rc=$?"
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-eval --no-gather-roof $*"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES" "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_ATOMIC_DRAM_sum" "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv \
    -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  echo "pass $i ($grp) rc=$?"
done
python3 scripts/pmc_traffic.py "$OUT" > "$OUT/traffic.json"
cat "$OUT/traffic.json"
