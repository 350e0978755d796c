#!/bin/bash
# round 6, last tree: the whole GPU suite, smoke, the plain C2 bench (the
# driver's command), and the strong-scaling leg at N = 1 (1 B pairs on one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06final5
mkdir -p $O
# the counters this gfx950 exposes (looking for an Infinity-Cache / HBM split)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 || echo "counter listing failed"
grep -i -E "mall|dram|hbm|infinity|_ea0_|df_" $O/counters_list.txt | head -40
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/gpu_tests.log | tail -4
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH FAILED; tail -5 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));r=d['roofline'];print('c2',d['value'],r['avg_launch_ms'],r['frac'],r['traffic'],r.get('l2_hit_rate'),r.get('valu_busy'),d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --scaling strong --no-cpu-baseline > $O/bench_strong_n1.json 2> $O/bench_strong_n1.err || { echo STRONG BENCH FAILED; tail -5 $O/bench_strong_n1.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_strong_n1.json'));print('strong n1',d['value'],d['ms_per_step'],d['config']['workload'])"
