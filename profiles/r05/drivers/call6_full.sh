#!/bin/bash
# round 5: the whole GPU suite on the current tree, then the default bench and smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c10
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gpu_tests.log | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH FAILED; tail -5 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2',d['value'],d['roofline']['avg_launch_ms'],d['roofline']['tail_store'],d['quality'],d['cpu_baseline']['value'])"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
