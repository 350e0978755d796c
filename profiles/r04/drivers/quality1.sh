#!/bin/bash
# round 4: the C3 quality gate (pytest, full size), then the small-corpus DP sweep
set -o pipefail
mkdir -p gpurun_out/r04q1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 560 --timeout-method thread \
  tests/test_gpu_c3_quality.py > gpurun_out/r04q1/c3_test.log 2>&1
rc=$?
echo "c3 test rc $rc" >> gpurun_out/r04q1/c3_test.log
[ $rc -le 1 ] || exit $rc
bash profiles/r04/drivers/small_dp.sh
