#!/bin/bash
# interleaved C2 A/B (tree vs exp_r1/old), 4 rounds
set -e
O=gpurun_out/ab_${1:?tag}; mkdir -p $O
for i in 1 2 3 4; do
  for who in new old; do
    R=$GRAFT_REPO_ROOT; [ $who = old ] && R=$GRAFT_REPO_ROOT/exp_r1/old
    G2V_ROOT=$R timeout -k 10 200 python scripts/exp_sweep.py --reps 3 --configs "ld=224" ${@:2} > $O/c2_${who}_$i.log 2>&1
    echo "$who $i $(grep config $O/c2_${who}_$i.log)"
  done
done
