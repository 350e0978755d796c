#!/bin/bash
# round 5, last tree: the whole GPU suite, smoke, the plain C2 bench, the CLI end to end
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c41
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gpu_tests.log | tail -4
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH FAILED; tail -5 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));r=d['roofline'];print('c2',d['value'],r['avg_launch_ms'],r['frac'],r['traffic'] is not None,d['cpu_baseline']['value'])"
timeout -k 10 400 python -u scripts/e2e_cli_timing.py --pairs 100000000 --files 8 --shuffle device \
  > $O/cli_timing.json 2> $O/cli_timing.err || { echo CLI FAILED; tail -5 $O/cli_timing.err; exit 1; }
tail -c 600 $O/cli_timing.json
