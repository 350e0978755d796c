#!/bin/bash
# merge tests (align rule) + reduced replica-quality sweep (8 x 2 M pairs + GGIPNN
# positives x3, 10 iterations): touch vs align, cadence 16 / 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_gpu_merge_group.py tests/test_gpu_merge.py > gpurun_out/r03c_merge_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 1000 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 2000000 \
  --iters 10 --ggipnn-repeat 3 --merge-every 16,4 --auc-seeds 0,1 \
  --rules 1000:1000,align \
  --out gpurun_out/rq_small4 > gpurun_out/r03c_rq_small4.log 2>&1
