#!/bin/bash
# round 4 call 21: the final tree -- the whole GPU suite (with durations),
# smoke() and the default bench line
set -o pipefail
mkdir -p gpurun_out/r04c21
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rP --durations=15 --timeout 400 \
  --timeout-method thread > gpurun_out/r04c21/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/r04c21/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/r04c21/smoke.log 2>&1 &&
timeout -k 10 240 python -u bench.py > gpurun_out/r04c21/bench.json 2> gpurun_out/r04c21/bench.err
