#!/bin/bash
# reduced replica-quality sweep (8 x 2 M pairs, 3 iterations): merge cadence x touch exponent
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 2000000 \
  --iters 3 --ggipnn-repeat 0 --merge-every 16,8,4 --betas 1000,750,500,0 --no-eval \
  --out gpurun_out/rq_small > gpurun_out/r03b_rq_small.log 2>&1
