#!/bin/bash
# round-3 session 4: one-round stripe-copy loads (tree) vs the previous kernel
# (var_base), interleaved, sample 0 and C2; then waves spread over more CUs.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for who in base tree; do
    R=$GRAFT_REPO_ROOT; [ $who = base ] && R=$GRAFT_REPO_ROOT/var_base
    G2V_ROOT=$R timeout -k 10 200 python scripts/exp_sweep.py --sample 0 --configs "ld=224" \
      > gpurun_out/ab_s0_${who}_$i.log 2>&1 || exit 1
    echo "s0 $who $i $(grep config gpurun_out/ab_s0_${who}_$i.log)"
    G2V_ROOT=$R timeout -k 10 200 python scripts/exp_sweep.py --configs "ld=224" \
      > gpurun_out/ab_c2_${who}_$i.log 2>&1 || exit 1
    echo "c2 $who $i $(grep config gpurun_out/ab_c2_${who}_$i.log)"
  done
done
timeout -k 10 300 python scripts/exp_sweep.py --sample 0 --configs \
  "grid=324,aw=2,stripe=8x8,stripe2=0x4" "grid=648,aw=1,stripe=8x8,stripe2=0x4" \
  "grid=162,stripe=8x8,stripe2=0x4" > gpurun_out/ab_s0_aw.log 2>&1 || exit 1
grep config gpurun_out/ab_s0_aw.log
