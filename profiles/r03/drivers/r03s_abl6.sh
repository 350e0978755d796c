#!/bin/bash
# ablation 6 (production atomics into the real tables, readers skip the
# stripe copies: the drained-copy design's ceiling) at sample 0 and C2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python scripts/exp_sweep.py --sample 0 --configs \
  "stripe=8x8,stripe2=0x4" "dbg=6,stripe=8x8,stripe2=0x4" "dbg=6,stripe=8x16,stripe2=0x4" \
  "dbg=6,stripe=8x32,stripe2=0x4" "dbg=6,stripe=32x16,stripe2=0x4" "dbg=6,stripe=128x8,stripe2=0x4" \
  "dbg=4,stripe=8x8,stripe2=0x4" > gpurun_out/abl6_s0.log 2>&1 || exit 1
grep config gpurun_out/abl6_s0.log
timeout -k 10 300 python scripts/exp_sweep.py --configs \
  "ld=224" "dbg=6" "dbg=6,stripe=32x16,stripe2=0x4" "dbg=6,stripe=128x16,stripe2=0x4" \
  > gpurun_out/abl6_c2.log 2>&1 || exit 1
grep config gpurun_out/abl6_c2.log
