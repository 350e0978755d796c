#!/bin/bash
# round 6 (verdict r5 item 1): 2 ranks with a damped touch divisor k^beta
# (once per epoch).  beta 1.5 held 2 x 80 M (+0.80 / -0.84 %) and left 2 x
# 125 M B at +1.16 % (A +0.52 %): does a beta rising with the shard hold both
# corpora from 80 to 200 M pairs per rank?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
run() {  # pairs every corpus rules tag
  local P=$1 EV=$2 C=$3 RULES=$4 TAG=$5
  eval OPTS=\$$C
  timeout -k 10 400 python -u scripts/replica_quality.py --replicas 2 --pairs-per-replica $P \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every $EV --replica-seeds 1 --single-seeds 1 \
    --auc-seeds 0 --rules $RULES --out gpurun_out/rq_r06_${TAG}_n2_$C > gpurun_out/r06_rq_${TAG}_n2_$C.log 2>&1 \
    || { echo "study $TAG $C failed"; tail -20 gpurun_out/r06_rq_${TAG}_n2_$C.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/rq_r06_${TAG}_n2_$C/replica_quality.json'))
for t, r in d['runs'].items(): print('2x$TAG $C', t, {k: r[k] for k in r if k.endswith('gap')})"
}
for C in B A; do
  run 100000000 20100 $C touch:1550:1000,touch:1600:1000 b100 || exit 1
  run 125000000 25100 $C touch:1600:1000,touch:1700:1000 b125 || exit 1
  run 150000000 30100 $C touch:1650:1000,touch:1750:1000 b150 || exit 1
  run 200000000 40100 $C touch:1700:1000,touch:1850:1000 b200 || exit 1
done
