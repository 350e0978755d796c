#!/bin/bash
# round 6 (verdict r5 item 2): the north-star metrics at C4's shape (60 k genes,
# D 512, K 15, planted modules, the reference's 10-iteration flow): the default
# cold-row stores vs every row atomic vs the C restatement's 16-thread Hogwild
# (gensim workers=16); plus the strong-scaling bench launch test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_bench_launch.py > gpurun_out/r06_c2_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/r06_c2_tests.log; exit 1; }
tail -2 gpurun_out/r06_c2_tests.log
timeout -k 10 1000 python -u scripts/e2e_parity.py --vocab 60000 --dim 512 --negative 15 \
  --modules 2000 --pairs 10000000 --seeds 1,2 --auc-seeds 0,1,2 \
  --engines gpu,gpu_tail0,oracle_hog16 --reference-engine oracle_hog16 \
  --out gpurun_out/e2e_c4 > gpurun_out/r06_e2e_c4.log 2>&1 \
  || { echo "e2e failed"; tail -30 gpurun_out/r06_e2e_c4.log; exit 1; }
tail -60 gpurun_out/r06_e2e_c4.log
