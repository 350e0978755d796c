#!/bin/bash
# round 5: data-parallel plan at the metric's N = 2 and N = 4 points (verdict r4 item 2):
# R replicas x 125 M pairs (the plan dp_merge_plan picks there: touch every 3,584 jobs)
# vs one model, corpora A and B, two job-seed streams against two one-model seeds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
for R in 4 2; do
  for C in A B; do
    eval OPTS=\$$C
    timeout -k 10 500 python -u scripts/replica_quality.py --replicas $R --pairs-per-replica 125000000 \
      --iters 10 --ggipnn-repeat 3 $OPTS --merge-every 3584 --replica-seeds 1,2 --single-seeds 1,2 \
      --auc-seeds 0 --rules touch --out gpurun_out/rq_r05_n${R}_$C > gpurun_out/r05_rq_n${R}_$C.log 2>&1 \
      || { echo "study R=$R corpus $C failed"; tail -20 gpurun_out/r05_rq_n${R}_$C.log; exit 1; }
    grep "^replicas\|^single" gpurun_out/r05_rq_n${R}_$C.log | tail -4
  done
done
