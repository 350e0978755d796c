#!/bin/bash
# C3-scale quality study: the one model's own run-to-run spread (3 job-seed
# streams), the yardstick for the replica gaps of profiles/r03/replica_quality_c3_rep3.json
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1700 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 125000000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 --merge-every 1024 \
  --auc-seeds 0,1,2 --rules touch --single-seeds 1,2,3 \
  --out gpurun_out/rq_c3d > gpurun_out/r03d_rq_c3d.log 2>&1
