#!/bin/bash
# round 6 (verdict r5 item 1): the 8-rank window's upper edge (8 x 150 M, touch
# at 7 merges per epoch, corpora A and B), the small-world window gates, and
# the lost-update probe on the production launch layout
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
for C in A B; do
  eval OPTS=\$$C
  timeout -k 10 400 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 150000000 \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every 4286 --replica-seeds 1 --single-seeds 1 \
    --auc-seeds 0 --rules touch --out gpurun_out/rq_r06_s150_n8_$C > gpurun_out/r06_rq_s150_n8_$C.log 2>&1 \
    || { echo "study 8x150M $C failed"; tail -20 gpurun_out/r06_rq_s150_n8_$C.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/rq_r06_s150_n8_$C/replica_quality.json'))
for t, r in d['runs'].items(): print('8x150M $C', t, r.get('train_s'), {k: r[k] for k in r if k.endswith('gap')})"
done
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread \
  tests/test_gpu_c3_quality.py -k small_world > gpurun_out/r06_c3_window_tests.log 2>&1 \
  || echo "window gates failed"
grep -E "PASS|FAIL|replicas x|passed|failed" gpurun_out/r06_c3_window_tests.log | tail -8
timeout -k 10 300 python -u scripts/lost_updates.py --tails auto --out gpurun_out/r06_lost_auto.json \
  > gpurun_out/r06_lost.log 2>&1 || { echo "lost-update probe failed"; tail -20 gpurun_out/r06_lost.log; exit 1; }
tail -5 gpurun_out/r06_lost.log
