#!/bin/bash
# round 4: merge-cadence sweep on a second structured corpus (verdict r3 item 1):
# Zipf 1.2, 600 planted modules (~41 genes each, under the target function's
# 50-gene pathway cap), p_module 0.3, GGIPNN positives x3; 2 job-seed streams per arm
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1170 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 125000000 \
  --iters 10 --ggipnn-repeat 3 --modules 600 --p-module 0.3 --zipf 1.2 \
  --merge-every "$1" --replica-seeds 1,2 --single-seeds "$2" $3 \
  --auc-seeds 0 --rules touch --out gpurun_out/rq_c3z12_$4 > gpurun_out/r04_rq_c3z12_$4.log 2>&1
