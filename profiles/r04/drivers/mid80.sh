#!/bin/bash
# round 4: the DP plan between its two measured points (8 x 80 M pairs per rank,
# corpus A): align at 7 merges per epoch (the CLI's plan below 125 M) vs touch
# every 4,096 jobs (its plan from 125 M), each at both cadences, 2 job-seed
# streams each, against two one-model seeds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 80000000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 --merge-every 2288,4096 \
  --rules align,touch --replica-seeds 1,2 --single-seeds 1,2 --auc-seeds 0 \
  --out gpurun_out/rq_80m_mid > gpurun_out/r04_rq_80m_mid.log 2>&1
