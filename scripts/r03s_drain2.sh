#!/bin/bash
# drained stripe copies, conserving drain + per-chunk L2 acquire, vs production
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python scripts/exp_sweep.py --sample 0 --configs \
  "stripe=8x8,stripe2=0x4" "drain=1,stripe=8x8,stripe2=0x4" "drain=2,stripe=8x8,stripe2=0x4" \
  "drain=4,stripe=8x8,stripe2=0x4" "drain=1001,stripe=8x8,stripe2=0x4" \
  "drain=2,stripe=8x16,stripe2=0x4" "drain=2,stripe=32x8,stripe2=0x4" > gpurun_out/drain2_s0.log 2>&1 || exit 1
grep config gpurun_out/drain2_s0.log
timeout -k 10 400 python scripts/exp_sweep.py --configs \
  "ld=224" "drain=1" "drain=4" "drain=2,stripe=32x16" "ld=224" \
  > gpurun_out/drain2_c2.log 2>&1 || exit 1
grep config gpurun_out/drain2_c2.log
