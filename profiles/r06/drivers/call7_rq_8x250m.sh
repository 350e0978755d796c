#!/bin/bash
# round 6 (verdict r5 item 1): the 8-rank window above 125 M pairs per rank:
# 8 x 250 M, corpora A and B, touch every 3,584 jobs (the plan so far: 14 per
# epoch at this shard) and at 7 merges per epoch (7,143 jobs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
for C in A B; do
  eval OPTS=\$$C
  timeout -k 10 560 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 250000000 \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every 3584,7143 --replica-seeds 1 --single-seeds 1 \
    --auc-seeds 0 --rules touch --out gpurun_out/rq_r06_s250_n8_$C > gpurun_out/r06_rq_s250_n8_$C.log 2>&1 \
    || { echo "study 8x250M $C failed"; tail -20 gpurun_out/r06_rq_s250_n8_$C.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/rq_r06_s250_n8_$C/replica_quality.json'))
for t, r in d['runs'].items(): print('8x250M $C', t, r.get('train_s'), {k: r[k] for k in r if k.endswith('gap')})"
done
