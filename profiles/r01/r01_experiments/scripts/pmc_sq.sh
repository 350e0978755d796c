#!/bin/bash
# SQ instruction-mix passes over a 10M-pair bench run, pipe (0) and atomic (1) kernels
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcsq
rocprofv3 --list-avail > gpurun_out/pmcsq/avail.txt 2>&1 || true
for k in 1; do
ARGS="--pairs 10000000 --steps 1 --warmup 0 --no-cpu-baseline --no-eval"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES" "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmcsq/k${k}p$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmcsq/k${k}p$i.log 2>&1
  echo "kernel $k pass $i rc=$?"
done
done
