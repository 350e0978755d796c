#!/bin/bash
# stall / cache / atomic-path counters over a 10M-pair bench run; kernels in $PMC_KERNELS
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcd
for k in 1; do
ARGS="--pairs 10000000 --steps 1 --warmup 0 --no-cpu-baseline --no-eval"
i=0
for grp in "SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_IFETCH SQ_INSTS_BRANCH" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_ATOMIC_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_UC_ATOMIC_REQ_sum TCP_TCC_RW_ATOMIC_REQ_sum" \
           "TCC_EA0_ATOMIC_sum TCC_EA0_ATOMIC_LEVEL_sum TCC_ATOMIC_sum TCC_BUSY_sum" \
           "TCP_TCC_NC_ATOMIC_REQ_sum TCP_TCC_CC_ATOMIC_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/pmcd/k${k}p$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmcd/k${k}p$i.log 2>&1
  echo "kernel $k pass $i rc=$?"
done
done
