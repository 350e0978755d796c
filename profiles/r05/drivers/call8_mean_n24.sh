#!/bin/bash
# round 5: the mean rule at N = 4 and N = 2 (gaps against call 7's one-model runs, same corpora)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
for R in 4 2; do
  for C in A B; do
    eval OPTS=\$$C
    timeout -k 10 300 python -u scripts/replica_quality.py --replicas $R --pairs-per-replica 125000000 \
      --iters 10 --ggipnn-repeat 3 $OPTS --merge-every 3584,12544 --replica-seeds 1 --no-single \
      --auc-seeds 0 --rules mean --out gpurun_out/rq_r05_mean_n${R}_$C > gpurun_out/r05_rq_mean_n${R}_$C.log 2>&1 \
      || { echo "study R=$R corpus $C failed"; tail -20 gpurun_out/r05_rq_mean_n${R}_$C.log; exit 1; }
    grep "^replicas" gpurun_out/r05_rq_mean_n${R}_$C.log | tail -2 | cut -c1-200
  done
done
