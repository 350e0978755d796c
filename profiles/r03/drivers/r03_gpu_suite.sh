#!/bin/bash
# the whole GPU test suite + smoke on the current library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread \
  > gpurun_out/r03e_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03e_smoke.log 2>&1
