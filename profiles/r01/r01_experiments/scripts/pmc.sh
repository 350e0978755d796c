#!/bin/bash
# PMC passes over a 10M-pair bench run (2 SGNS launches); one counter group per pass
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
ARGS="--pairs 10000000 --steps 1 --warmup 0 --no-cpu-baseline --no-eval"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  echo "pass $i ($grp) rc=$?"
done
