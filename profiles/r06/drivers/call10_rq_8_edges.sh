#!/bin/bash
# round 6 (verdict r5 item 1): the 8-rank default window's edges on the
# corpus that binds each (120 M: corpus B, 135 M: corpus A) and corpus B at
# C3's 125 M on the current kernel (the plan: touch at 7 merges per epoch,
# every 3,584 jobs at 125 M)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
run() {  # pairs every corpus tag
  local P=$1 EV=$2 C=$3 TAG=$4
  eval OPTS=\$$C
  timeout -k 10 400 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica $P \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every $EV --replica-seeds 1 --single-seeds 1 \
    --auc-seeds 0 --rules touch --out gpurun_out/rq_r06_${TAG}_n8_$C > gpurun_out/r06_rq_${TAG}_n8_$C.log 2>&1 \
    || { echo "study $TAG $C failed"; tail -20 gpurun_out/r06_rq_${TAG}_n8_$C.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/rq_r06_${TAG}_n8_$C/replica_quality.json'))
for t, r in d['runs'].items(): print('8x$TAG $C', t, {k: r[k] for k in r if k.endswith('gap')})"
}
run 120000000 3429 B s120 && run 135000000 3584 A s135 && run 125000000 3584 B s125
