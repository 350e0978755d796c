#!/bin/bash
# round 6 (verdict r5 item 1): 2 ranks past 200 M pairs per rank (C3's 1 B
# pairs over 2 = 500 M) with the damped divisor k^beta, once per epoch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
run() {  # replicas pairs every corpus rules tag
  local R=$1 P=$2 EV=$3 C=$4 RULES=$5 TAG=$6
  eval OPTS=\$$C
  timeout -k 10 500 python -u scripts/replica_quality.py --replicas $R --pairs-per-replica $P \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every $EV --replica-seeds 1 --single-seeds 1 \
    --auc-seeds 0 --rules $RULES --out gpurun_out/rq_r06_${TAG}_n${R}_$C > gpurun_out/r06_rq_${TAG}_n${R}_$C.log 2>&1 \
    || { echo "study $TAG $C failed"; tail -20 gpurun_out/r06_rq_${TAG}_n${R}_$C.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/rq_r06_${TAG}_n${R}_$C/replica_quality.json'))
for t, r in d['runs'].items(): print('${R}x$TAG $C', t, {k: r[k] for k in r if k.endswith('gap')})"
}
for C in B A; do
  run 2 500000000 100100 $C touch:2000:1000,touch:2150:1000 b500 || exit 1
  run 2 300000000 60100 $C touch:1900:1000,touch:2000:1000 b300 || exit 1
done
