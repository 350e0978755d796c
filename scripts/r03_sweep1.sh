#!/bin/bash
# reduced replica-quality sweep on a planted-module corpus (8 x 2 M pairs, 1,000
# modules, half the pairs inside a module, + GGIPNN positives x3, 10 iterations)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 2000000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 --merge-every 16,4 --auc-seeds 0,1 \
  --rules touch,align,align:1000:1500,align:1000:1800 \
  --out gpurun_out/rq_small5 > gpurun_out/r03c_rq_small5.log 2>&1
