#!/bin/bash
# round 4: the merge-cadence sweep on corpus B (verdict r3 item 1) in two steps
# so each has its own limit: the two one-model seeds + cadences 1,024 / 2,048 /
# 4,096, then 8,192 / 16,384 / once per epoch (30,000 > the epoch's jobs);
# 2 job-seed streams per cadence.  The second step's gaps are taken offline
# against the first step's one-model seeds (profiles/r04/replica_quality_c3_corpusB.json).
set -o pipefail
mkdir -p gpurun_out
C="--replicas 8 --pairs-per-replica 125000000 --iters 10 --ggipnn-repeat 3 --modules 600
   --p-module 0.3 --zipf 1.2 --replica-seeds 1,2 --auc-seeds 0 --rules touch"
timeout -k 10 620 python -u scripts/replica_quality.py $C --merge-every 1024,2048,4096 \
  --single-seeds 1,2 --out gpurun_out/rq_c3z12_b1 > gpurun_out/r04_rq_c3z12_b1.log 2>&1 &&
timeout -k 10 480 python -u scripts/replica_quality.py $C --merge-every 8192,16384,30000 \
  --no-single --out gpurun_out/rq_c3z12_b2 > gpurun_out/r04_rq_c3z12_b2.log 2>&1
