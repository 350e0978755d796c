#!/bin/bash
# round 5: the small-N plan (touch once per epoch) at the CLI's smallest default shard, 80 M pairs per rank
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
for R in 4 2; do
  for C in A B; do
    eval OPTS=\$$C
    timeout -k 10 400 python -u scripts/replica_quality.py --replicas $R --pairs-per-replica 80000000 \
      --iters 10 --ggipnn-repeat 3 $OPTS --merge-every 16100 --replica-seeds 1 --single-seeds 1 \
      --auc-seeds 0 --rules touch --out gpurun_out/rq_r05_80m_n${R}_$C > gpurun_out/r05_rq_80m_n${R}_$C.log 2>&1 \
      || { echo "study R=$R corpus $C failed"; tail -20 gpurun_out/r05_rq_80m_n${R}_$C.log; exit 1; }
    grep "^replicas" gpurun_out/r05_rq_80m_n${R}_$C.log | tail -1 | python3 -c "
import sys,ast
for l in sys.stdin:
    tag,d=l.split(' ',1); d=ast.literal_eval(d.strip())
    print('R=$R $C',tag,{k:d[k] for k in d if k.endswith('gap')})"
  done
done
