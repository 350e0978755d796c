#!/bin/bash
# interleaved exp_sweep A/B: the tree's libg2v vs a variant package under $1 (G2V_ROOT)
set -e
V=${1:?variant dir}; shift
for i in 1 2 3; do
  for who in tree variant; do
    R=$GRAFT_REPO_ROOT; [ $who = variant ] && R=$GRAFT_REPO_ROOT/$V
    G2V_ROOT=$R timeout -k 10 200 python scripts/exp_sweep.py "$@" --configs "ld=224" > gpurun_out/abv_${who}_$i.log 2>&1
    echo "$who $i $(grep config gpurun_out/abv_${who}_$i.log)"
  done
done
