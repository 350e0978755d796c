#!/bin/bash
# round 4 call 5: final kernel defaults (separate row tails, deferred copies):
# the kernel's parity tests, then rocprofv3 stats + PMC traffic at C2 and at
# sample 0, then the plain C2 bench line
set -o pipefail
mkdir -p gpurun_out/r04c5
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_atomic_order.py tests/test_gpu_parity.py tests/test_gpu_loss.py \
  > gpurun_out/r04c5/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/r04c5/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 420 bash scripts/profile_round.sh r04 > gpurun_out/r04c5/profile_c2.log 2>&1 &&
timeout -k 10 420 bash scripts/profile_round.sh r04_s0 --sample 0 > gpurun_out/r04c5/profile_s0.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r04c5/bench.json 2> gpurun_out/r04c5/bench.err
