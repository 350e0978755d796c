#!/bin/bash
# round 4 call 7: deferred copies in 3 slots (199 VGPRs, 2 waves per SIMD, so
# k_job_sample can share the CUs again): kernel parity tests, A/B against the
# eager copy sum, then rocprofv3 stats + PMC traffic at C2 and sample 0, and
# the plain C2 bench line
set -o pipefail
mkdir -p gpurun_out/r04c7
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_atomic_order.py tests/test_gpu_parity.py tests/test_gpu_loss.py \
  > gpurun_out/r04c7/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/r04c7/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/stamp_segments.py --sample 0 --grid 162 --pairs 20000000 \
  --arms production,defer0,production_again,defer0_again \
  --out gpurun_out/r04c7/stamps_s0.json > gpurun_out/r04c7/stamps_s0.log 2>&1 &&
timeout -k 10 300 python -u scripts/stamp_segments.py --sample 1e-3 --pairs 20000000 \
  --arms production,defer0,production_again,defer0_again \
  --out gpurun_out/r04c7/stamps_c2.json > gpurun_out/r04c7/stamps_c2.log 2>&1 &&
timeout -k 10 420 bash scripts/profile_round.sh r04 > gpurun_out/r04c7/profile_c2.log 2>&1 &&
timeout -k 10 420 bash scripts/profile_round.sh r04_s0 --sample 0 > gpurun_out/r04c7/profile_s0.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r04c7/bench.json 2> gpurun_out/r04c7/bench.err
