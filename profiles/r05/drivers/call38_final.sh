#!/bin/bash
# round 5 final source with 4 striped rows x 16 copies by default: the whole GPU suite, smoke, the C2
# PMC/kernel-stats profile, the bench, the lost-update probe, sample-0 and C4 lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c38
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gpu_tests.log | tail -4
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 $O/smoke.log; exit 1; }
echo smoke ok; tail -1 $O/smoke.log
bash scripts/profile_round.sh r05f5 > $O/profile.log 2>&1 || { echo PROFILE FAILED; tail -20 $O/profile.log; exit 1; }
echo profile ok
mkdir -p profiles/r05 && cp gpurun_out/prof_r05f5/traffic.json profiles/r05/traffic_r05.json
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH FAILED; tail -5 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));r=d['roofline'];print('c2',d['value'],r['avg_launch_ms'],r['frac'],r['traffic'],d['quality'],d['cpu_baseline']['value'])"
timeout -k 10 300 python -u scripts/lost_updates.py --tails auto --epochs 1 --out $O/lost_auto.json > $O/lost_auto.log 2>&1 || { echo LOST FAILED; tail -5 $O/lost_auto.log; exit 1; }
grep "^auto" $O/lost_auto.log
timeout -k 10 300 python bench.py --no-cpu-baseline --sample 0 > $O/bench_s0.json 2> $O/bench_s0.err || { echo S0 FAILED; tail -5 $O/bench_s0.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_s0.json'));r=d['roofline'];print('s0',d['value'],r['avg_launch_ms'],r['frac'],d['quality'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --vocab 60000 --dim 512 --negative 15 > $O/bench_c4.json 2> $O/bench_c4.err || { echo C4 FAILED; tail -5 $O/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c4.json'));r=d['roofline'];print('c4',d['value'],r['avg_launch_ms'],r['frac'],d['quality'])"
