#!/bin/bash
# round 4 (verdict r3 item 6): can data parallelism below 125 M pairs per rank
# hold one-model quality?  8 replicas x {12.5 M, 50 M} pairs, {touch, align} x
# {7, 25, 50} merges per epoch, C3's corpus shape (1,000 planted modules, GGIPNN x3)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 12500000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 \
  --merge-every 359,101,51 --rules touch,align --auc-seeds 0 \
  --out gpurun_out/rq_small12 > gpurun_out/r04_rq_small12.log 2>&1 &&
timeout -k 10 700 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 50000000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 \
  --merge-every 1431,401,201 --rules touch,align --auc-seeds 0 \
  --out gpurun_out/rq_small50 > gpurun_out/r04_rq_small50.log 2>&1
