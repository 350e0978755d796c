#!/bin/bash
# round 4: GPU pass over the new code: the whole -m gpu suite but the C3 gate,
# then the stamped-kernel diagnostics (sample 0 and C2)
set -o pipefail
mkdir -p gpurun_out/r04v1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  --deselect tests/test_gpu_c3_quality.py::test_c3_eight_replicas_within_one_percent_of_one_model \
  > gpurun_out/r04v1/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/r04v1/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/stamp_segments.py --sample 0 --pairs 20000000 \
  --out gpurun_out/r04v1/stamps_s0.json > gpurun_out/r04v1/stamps_s0.log 2>&1 &&
timeout -k 10 200 python -u scripts/stamp_segments.py --sample 1e-3 --pairs 20000000 \
  --out gpurun_out/r04v1/stamps_c2.json > gpurun_out/r04v1/stamps_c2.log 2>&1
