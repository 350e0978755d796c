#!/bin/bash
# round 5: the quality gates with cold-row plain stores (G2V_OPT_TAIL_STORE; verdict r4 item 4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c3
mkdir -p $O
for T in 512 2048; do
  G2V_TEST_TAIL_STORE=$T timeout -k 10 400 python -u -m pytest -x -v -s --timeout 360 --timeout-method thread \
    tests/test_gpu_e2e_parity.py -k "not sample0" > $O/e2e_tail$T.log 2>&1
  echo "e2e tail $T rc=$?"; grep -E "gaps vs|PASS|FAIL|Error" $O/e2e_tail$T.log | cut -c1-400
done
G2V_TEST_TAIL_STORE=2048 timeout -k 10 600 python -u -m pytest -x -v -s --timeout 560 --timeout-method thread \
  "tests/test_gpu_c3_quality.py::test_c3_eight_replicas_within_one_percent_of_one_model" > $O/c3_tail2048.log 2>&1
echo "c3 tail 2048 rc=$?"; grep -E "C3:|PASS|FAIL|Error" $O/c3_tail2048.log | cut -c1-400
