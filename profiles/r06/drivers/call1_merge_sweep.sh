#!/bin/bash
# round 6 (verdict r5 item 1): merge-divisor shape at N = 2 and 4, corpora A and B,
# 125 M and 80 M pairs per rank, touch rule once per epoch (the small-N plan);
# beta > 1 / gamma < 1 damp the summed change of rows several replicas touched
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_gpu_parity.py -k "auto_tail_rows or full_vocab_tracks" > gpurun_out/r06_c1_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/r06_c1_tests.log; exit 1; }
tail -2 gpurun_out/r06_c1_tests.log
A="--modules 1000 --p-module 0.5 --zipf 1.0"
B="--modules 600 --p-module 0.3 --zipf 1.2"
run() {  # R pairs every corpus rules tag
  local R=$1 P=$2 EV=$3 C=$4 RULES=$5 TAG=$6
  eval OPTS=\$$C
  timeout -k 10 600 python -u scripts/replica_quality.py --replicas $R --pairs-per-replica $P \
    --iters 10 --ggipnn-repeat 3 $OPTS --merge-every $EV --replica-seeds 1 --single-seeds 1 \
    --auc-seeds 0 --rules $RULES --out gpurun_out/rq_r06_${TAG}_n${R}_$C > gpurun_out/r06_rq_${TAG}_n${R}_$C.log 2>&1 \
    || { echo "study $TAG R=$R corpus $C failed"; tail -20 gpurun_out/r06_rq_${TAG}_n${R}_$C.log; exit 1; }
  python3 - gpurun_out/rq_r06_${TAG}_n${R}_$C/replica_quality.json "$TAG R=$R $C" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for t, r in d["runs"].items():
    print(sys.argv[2], t, {k: r[k] for k in r if k.endswith("gap")})
PY
}
RULES="touch:1000:1000,touch:1500:1000,touch:2000:1000,touch:1000:750,touch:1000:500"
run 2 125000000 25100 A $RULES s125 && run 2 125000000 25100 B $RULES s125 \
 && run 2 80000000 16100 A $RULES s80 && run 2 80000000 16100 B $RULES s80 \
 && run 4 125000000 25100 B "touch:1500:1000,touch:2000:1000,touch:1000:750" s125
