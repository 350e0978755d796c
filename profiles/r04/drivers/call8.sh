#!/bin/bash
# round 4 call 8: the final tree's whole GPU suite (printing the e2e and C3
# gates' measured gaps) and smoke()
set -o pipefail
mkdir -p gpurun_out/r04c8
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rP --timeout 400 --timeout-method thread \
  > gpurun_out/r04c8/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/r04c8/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/r04c8/smoke.log 2>&1
