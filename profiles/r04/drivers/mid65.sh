#!/bin/bash
# round 4: the DP plan's 50-80 M band at 8 x 65 M pairs per rank (corpus A):
# align vs touch, both at 7 merges per epoch (13,000 jobs -> every 1,858),
# 2 job-seed streams each, against two one-model seeds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 65000000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 --merge-every 1858 \
  --rules align,touch --replica-seeds 1,2 --single-seeds 1,2 --auc-seeds 0 \
  --out gpurun_out/rq_65m_mid > gpurun_out/r04_rq_65m_mid.log 2>&1
