#!/bin/bash
# round 4: the touch-rule cadence between the two corpora's zero crossings
# (corpus A crosses near 4,096 jobs, corpus B near 2,048): 3,072
# and 3,584 on both corpora, 2 job-seed streams each, against two one-model seeds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 125000000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 --zipf 1.0 \
  --merge-every 3072,3584 --replica-seeds 1,2 --single-seeds 1,2 --auc-seeds 0 --rules touch \
  --out gpurun_out/rq_pick_a > gpurun_out/r04_rq_pick_a.log 2>&1 &&
timeout -k 10 560 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 125000000 \
  --iters 10 --ggipnn-repeat 3 --modules 600 --p-module 0.3 --zipf 1.2 \
  --merge-every 3072,3584 --replica-seeds 1,2 --single-seeds 1,2 --auc-seeds 0 --rules touch \
  --out gpurun_out/rq_pick_b > gpurun_out/r04_rq_pick_b.log 2>&1
