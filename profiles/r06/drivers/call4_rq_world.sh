#!/bin/bash
# round 6 (verdict r5 item 1): where the small-N plan holds 1 %, and one point
# each at N = 3 and N = 6 (touch rule; N <= 4 once per epoch, N = 6 the 8-rank
# plan: 7 merges per epoch), corpora A and B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
run() {  # R pairs every corpus seeds tag
  local R=$1 P=$2 EV=$3 C=$4 SEEDS=$5 TAG=$6
  eval OPTS=\$$C
  timeout -k 10 500 python -u scripts/replica_quality.py --replicas $R --pairs-per-replica $P \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every $EV --replica-seeds $SEEDS --single-seeds 1 \
    --auc-seeds 0 --rules touch --out gpurun_out/rq_r06_${TAG}_n${R}_$C > gpurun_out/r06_rq_${TAG}_n${R}_$C.log 2>&1 \
    || { echo "study $TAG R=$R corpus $C failed"; tail -20 gpurun_out/r06_rq_${TAG}_n${R}_$C.log; exit 1; }
  python3 - gpurun_out/rq_r06_${TAG}_n${R}_$C/replica_quality.json "$TAG R=$R $C" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for t, r in d["runs"].items():
    print(sys.argv[2], t, {k: r[k] for k in r if k.endswith("gap")})
PY
}
run 4 100000000 20100 A 1,2 s100 && run 4 100000000 20100 B 1,2 s100 \
 && run 3 80000000 16100 A 1 s80 && run 3 80000000 16100 B 1 s80 \
 && run 3 100000000 20100 A 1 s100 && run 3 100000000 20100 B 1 s100 \
 && run 6 125000000 3584 A 1 s125 && run 6 125000000 3584 B 1 s125 \
 && run 6 80000000 2286 A 1 s80 && run 6 80000000 2286 B 1 s80
