#!/bin/bash
# round 4: first GPU pass over the new code (RCCL stand-in tests, dense e2e gate, stamps)
set -o pipefail
mkdir -p gpurun_out/r04v1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_rccl_standin.py "tests/test_gpu_e2e_parity.py::test_gpu_end_to_end_dense_5k_genes" \
  > gpurun_out/r04v1/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/r04v1/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/stamp_segments.py --sample 0 --pairs 20000000 \
  --out gpurun_out/r04v1/stamps_s0.json > gpurun_out/r04v1/stamps_s0.log 2>&1 &&
timeout -k 10 200 python -u scripts/stamp_segments.py --sample 1e-3 --pairs 20000000 \
  --out gpurun_out/r04v1/stamps_c2.json > gpurun_out/r04v1/stamps_c2.log 2>&1
