#!/bin/bash
# round 6 (verdict r5 item 1): at 8 ranks the corpora agree better at larger
# shards (7 merges per epoch: A - B = 1.9 % at 125 M, 1.2 % at 150 M, 0.4 % at
# 250 M) and fewer merges lower both: 8 x 150 M at 5 merges per epoch and
# 8 x 200 M at 4, corpora A and B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
run() {  # pairs every corpus tag
  local P=$1 EV=$2 C=$3 TAG=$4
  eval OPTS=\$$C
  timeout -k 10 500 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica $P \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every $EV --replica-seeds 1 --single-seeds 1 \
    --auc-seeds 0 --rules touch --out gpurun_out/rq_r06_${TAG}_n8_$C > gpurun_out/r06_rq_${TAG}_n8_$C.log 2>&1 \
    || { echo "study $TAG $C failed"; tail -20 gpurun_out/r06_rq_${TAG}_n8_$C.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/rq_r06_${TAG}_n8_$C/replica_quality.json'))
for t, r in d['runs'].items(): print('8x$TAG $C', t, {k: r[k] for k in r if k.endswith('gap')})"
}
run 150000000 6000 B m5s150 && run 150000000 6000 A m5s150 \
 && run 200000000 10000 B m4s200 && run 200000000 10000 A m4s200
