#!/bin/bash
# syn0 rows unstriped (G2V_OPT_DEBUG_WRITE 8) vs production, C2 and sample 0
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python scripts/exp_sweep.py --configs "ld=224" "dbg=8" "ld=224" "dbg=8" \
  "dbg=8,stripe=8x32" "dbg=8,stripe2=32x4" > gpurun_out/syn0_c2.log 2>&1 || exit 1
grep config gpurun_out/syn0_c2.log
timeout -k 10 400 python scripts/exp_sweep.py --sample 0 --configs "ld=224" "dbg=8" "ld=224" "dbg=8" \
  > gpurun_out/syn0_s0.log 2>&1 || exit 1
grep config gpurun_out/syn0_s0.log
