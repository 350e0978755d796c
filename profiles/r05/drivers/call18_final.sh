#!/bin/bash
# round 5 final kernel: the whole GPU suite, smoke, the C2 PMC/kernel-stats profile, the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c18
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gpu_tests.log | tail -4
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
bash scripts/profile_round.sh r05f2 > $O/profile.log 2>&1; echo "profile rc=$?"
mkdir -p profiles/r05 && cp gpurun_out/prof_r05f2/traffic.json profiles/r05/traffic_r05.json
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH FAILED; tail -5 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));r=d['roofline'];print('c2',d['value'],r['avg_launch_ms'],r['frac'],r['traffic'],d['quality'],d['cpu_baseline']['value'])"
