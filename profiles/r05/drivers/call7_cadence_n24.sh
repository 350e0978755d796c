#!/bin/bash
# round 5: merge cadence at N = 4 and N = 2 (touch rule, 125 M pairs per rank), corpora A and B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
for R in 4 2; do
  if [ $R = 4 ]; then EV="6272,12544,25100"; else EV="8342,12544,25100"; fi
  for C in A B; do
    eval OPTS=\$$C
    timeout -k 10 420 python -u scripts/replica_quality.py --replicas $R --pairs-per-replica 125000000 \
      --iters 10 --ggipnn-repeat 3 $OPTS --merge-every $EV --replica-seeds 1 --single-seeds 1 \
      --auc-seeds 0 --rules touch --out gpurun_out/rq_r05_cad_n${R}_$C > gpurun_out/r05_rq_cad_n${R}_$C.log 2>&1 \
      || { echo "study R=$R corpus $C failed"; tail -20 gpurun_out/r05_rq_cad_n${R}_$C.log; exit 1; }
    grep "^replicas\|^single" gpurun_out/r05_rq_cad_n${R}_$C.log | tail -4 | python3 -c "
import sys,ast
for l in sys.stdin:
    tag,d=l.split(' ',1); d=ast.literal_eval(d.strip())
    print('R=$R $C',tag,{k:d[k] for k in d if k.endswith('gap') or k in ('target_ratio',)})"
  done
done
