#!/bin/bash
# C3-scale quality study: touch rule at 2,048 / 4,096 / 8,192 jobs (GGIPNN x3 corpus)

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1700 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 125000000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 --merge-every 2048,4096,8192 \
  --auc-seeds 0,1,2 --rules touch --no-single \
  --out gpurun_out/rq_c3e > gpurun_out/r03d_rq_c3e.log 2>&1
