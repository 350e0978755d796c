#!/bin/bash
# round 3, first box: the multi-replica merge tests (new transports), the C2
# bench line, and the sample-0 copy-read ablation (verdict r2 item 4):
# production vs scratch atomics with copy reads (dbg 4) vs scratch atomics
# reading main rows only (dbg 7), at the staleness-bounded default grid
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 180 --timeout-method thread \
  tests/test_gpu_merge_group.py tests/test_gpu_atomic_order.py tests/test_gpu_replica_quality.py tests/test_gpu_merge.py tests/test_gpu_dp_cli.py \
  > gpurun_out/r03a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || exit $?
timeout -k 10 400 python scripts/exp_sweep.py --sample 0 --reps 2 --configs \
  "ld=224" "dbg=4" "dbg=4,stripe=8x16" "dbg=7" "dbg=7,stripe=8x16" "dbg=7,stripe=8x32" \
  "dbg=7,stripe=32x16" "dbg=7,stripe=128x16" "dbg=7,stripe=512x16" "dbg=7,stripe=512x32" \
  > gpurun_out/r03a_s0_copyread.log 2>&1 || exit $?
