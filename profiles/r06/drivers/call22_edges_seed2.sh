#!/bin/bash
# round 6: second job-seed streams at the windows' most marginal points:
# 8 x 200 M corpus A (wide-shard plan, 4 merges per epoch: +0.85 %) and
# 2 x 200 M corpus B (k^1.85: +0.57 %)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
run() {  # replicas pairs every corpus rules tag
  local R=$1 P=$2 EV=$3 C=$4 RULES=$5 TAG=$6
  eval OPTS=\$$C
  timeout -k 10 500 python -u scripts/replica_quality.py --replicas $R --pairs-per-replica $P \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every $EV --replica-seeds 2,3 --single-seeds 1 \
    --auc-seeds 0 --rules $RULES --out gpurun_out/rq_r06_${TAG}_n${R}_$C > gpurun_out/r06_rq_${TAG}_n${R}_$C.log 2>&1 \
    || { echo "study $TAG $C failed"; tail -20 gpurun_out/r06_rq_${TAG}_n${R}_$C.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/rq_r06_${TAG}_n${R}_$C/replica_quality.json'))
for t, r in d['runs'].items(): print('${R}x$TAG $C', t, {k: r[k] for k in r if k.endswith('gap')})"
}
run 8 200000000 10003 A touch m4s200seeds && run 2 200000000 40100 B touch:1850:1000 b200seeds
