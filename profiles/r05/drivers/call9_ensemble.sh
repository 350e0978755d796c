#!/bin/bash
# round 5: is the replicas' target-function lead at N = 2 / 4 the ensemble effect of averaging?
# Score the plain average of two independently trained one-models (no merges).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
for C in A B; do
  eval OPTS=\$$C
  timeout -k 10 300 python -u scripts/replica_quality.py --replicas 2 --pairs-per-replica 125000000 \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every 25100 --replica-seeds 2 --single-seeds 1,2 \
    --ensemble-singles --auc-seeds 0 --rules touch --out gpurun_out/rq_r05_ens_n2_$C > gpurun_out/r05_rq_ens_n2_$C.log 2>&1 \
    || { echo "study corpus $C failed"; tail -20 gpurun_out/r05_rq_ens_n2_$C.log; exit 1; }
  grep "^replicas\|^single" gpurun_out/r05_rq_ens_n2_$C.log | tail -4 | cut -c1-260
done
