#!/bin/bash
# round 6 (verdict r5 item 1): at 8 ranks corpus B reads -0.71 .. -1.12 % at
# C3's shard with the touch rule every 3,584 jobs and corpus A +0.70 %; every
# 3,072 jobs A +1.14 %, B -0.41 .. -0.56 % (round 4): the midpoint 3,328 on
# both corpora, two job-seed streams each, and A's upper edge at 130 M
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
run() {  # pairs every corpus seeds tag
  local P=$1 EV=$2 C=$3 SEEDS=$4 TAG=$5
  eval OPTS=\$$C
  timeout -k 10 450 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica $P \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every $EV --replica-seeds $SEEDS --single-seeds 1 \
    --auc-seeds 0 --rules touch --out gpurun_out/rq_r06_${TAG}_n8_$C > gpurun_out/r06_rq_${TAG}_n8_$C.log 2>&1 \
    || { echo "study $TAG $C failed"; tail -20 gpurun_out/r06_rq_${TAG}_n8_$C.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/rq_r06_${TAG}_n8_$C/replica_quality.json'))
for t, r in d['runs'].items(): print('8x$TAG $C', t, {k: r[k] for k in r if k.endswith('gap')})"
}
run 125000000 3328 B 1,2 c3328s125 && run 125000000 3328 A 1,2 c3328s125 && run 130000000 3328 A 1 c3328s130
