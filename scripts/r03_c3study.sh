#!/bin/bash
# C3-scale data-parallel quality study (verdict r2 item 1) with the GGIPNN
# positives repeated 3x (not 30x: less over-training of those genes' rows in
# the one model), touch rule at 1,024 / 16,384 jobs and once per epoch
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1700 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 125000000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 --merge-every 1024,16384,1048576 \
  --auc-seeds 0,1,2 --rules touch \
  --out gpurun_out/rq_c3c > gpurun_out/r03d_rq_c3c.log 2>&1
