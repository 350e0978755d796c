#!/bin/bash
# C3-scale data-parallel quality study (verdict r2 item 1): 8 replicas x 125 M
# pairs (planted co-expression modules + GGIPNN positives x30) vs one model,
# 10-iteration sawtooth, merge every 1,024 jobs: touch / align / align gamma 1.5
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1700 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 125000000 \
  --iters 10 --ggipnn-repeat 30 --modules 1000 --p-module 0.5 --merge-every 1024 --auc-seeds 0,1,2 \
  --rules touch,align,align:1000:1500 \
  --out gpurun_out/rq_c3 > gpurun_out/r03d_rq_c3.log 2>&1
