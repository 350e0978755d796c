#!/bin/bash
# the two re-gated tests, then rocprofv3 stats + PMC passes of the current
# kernel build at C2, C2 sample 0 and C4 (traffic profiles stamped with the
# kernel hash and launch layout)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 240 --timeout-method thread \
  tests/test_gpu_replica_quality.py tests/test_gpu_shuffle_cli.py > gpurun_out/r03g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
bash scripts/profile_round.sh r03 || exit $?
bash scripts/profile_round.sh r03_s0 --sample 0 || exit $?
bash scripts/profile_round.sh r03_c4 --vocab 60000 --dim 512 --negative 15 || exit $?
