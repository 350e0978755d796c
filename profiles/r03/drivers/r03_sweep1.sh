#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/r03_spread.py > gpurun_out/r03f_spread.log 2>&1
timeout -k 10 900 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 12500000 \
  --iters 2 --ggipnn-repeat 0 --merge-every 410,102 --no-eval --out gpurun_out/rq_mid \
  > gpurun_out/r03f_rq_mid.log 2>&1
timeout -k 10 900 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 5000000 \
  --iters 2 --ggipnn-repeat 0 --merge-every 164 --no-eval --out gpurun_out/rq_mid2 \
  > gpurun_out/r03f_rq_mid2.log 2>&1
