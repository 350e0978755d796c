#!/bin/bash
# round 4 call 18: the final kernel sources (comments updated): kernel parity
# tests, rocprofv3 stats + PMC traffic at C2 / sample 0 / C4, the bench line
set -o pipefail
mkdir -p gpurun_out/r04c18
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_atomic_order.py tests/test_gpu_parity.py tests/test_gpu_loss.py \
  > gpurun_out/r04c18/tests.log 2>&1 &&
bash profiles/r04/drivers/call9.sh
