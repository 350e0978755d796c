#!/bin/bash
# round 6 (verdict r5 item 3): rocprofv3 --kernel-trace --stats + the PMC passes
# (now with L2 hit rate and VALU busy) at C2, C4 and sample 0 on the final
# kernel; the lost-update probe on the production launch layout
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_c3_quality.py -k small_world > gpurun_out/r06_c3_window_tests.log 2>&1 \
  || { echo "window gates failed"; tail -30 gpurun_out/r06_c3_window_tests.log; exit 1; }
grep -E "PASS|FAIL|replicas x|passed|failed" gpurun_out/r06_c3_window_tests.log | tail -8
bash scripts/profile_round.sh r06_c2 > gpurun_out/r06_prof_c2.log 2>&1 || { echo "c2 profile failed"; tail -20 gpurun_out/r06_prof_c2.log; exit 1; }
tail -3 gpurun_out/r06_prof_c2.log
timeout -k 10 300 python -u scripts/lost_updates.py --tails auto --out gpurun_out/r06_lost_auto.json \
  > gpurun_out/r06_lost.log 2>&1 || { echo "lost-update probe failed"; tail -20 gpurun_out/r06_lost.log; exit 1; }
tail -5 gpurun_out/r06_lost.log
