#!/bin/bash
# round 6 (verdict r5 item 2): C4-shape cold-row store boundary vs quality and
# throughput: the default (collision budget) and fixed boundaries, GPU-only arms
# against every row atomic; the new reduced C4 gate
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/e2e_parity.py --vocab 60000 --dim 512 --negative 15 \
  --modules 2000 --pairs 10000000 --seeds 1,2,3 --auc-seeds 0,1,2 \
  --engines gpu_tail0,gpu,gpu_tail30000,gpu_tail45000 --reference-engine gpu_tail0 \
  --out gpurun_out/e2e_c4_tail > gpurun_out/r06_e2e_c4_tail.log 2>&1 \
  || { echo "e2e failed"; tail -30 gpurun_out/r06_e2e_c4_tail.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/e2e_c4_tail/e2e_parity.json'))['summary']
for k in ('heldin','target_ratio','auc_mean'): print(k, {x: d[k][x] for x in d[k] if x.endswith('gap') or x=='oracle_spread'})"
for T in -1 30000 45000 0; do
  timeout -k 10 300 python bench.py --vocab 60000 --dim 512 --negative 15 --tail-store $T \
    --no-cpu-baseline --no-eval --no-gather-roof --steps 3 > gpurun_out/r06_c4_bench_tail$T.json 2> gpurun_out/r06_c4_bench_tail$T.err \
    || { echo "bench $T failed"; tail -5 gpurun_out/r06_c4_bench_tail$T.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06_c4_bench_tail$T.json'));r=d['roofline'];print('tail $T',d['value'],r['avg_launch_ms'],r['stored_rows_per_example'],r['tail_row_syn1neg'])"
done
# 8 ranks x 80 M pairs on corpus B (the 8-rank window's low end; corpus A was measured in round 4)
timeout -k 10 500 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 80000000 \
  --iters 10 --ggipnn-repeat 3 --modules 600 --p-module 0.3 --zipf 1.2 --merge-every 2286 \
  --replica-seeds 1 --single-seeds 1 --auc-seeds 0 --rules touch --out gpurun_out/rq_r06_s80_n8_B \
  > gpurun_out/r06_rq_s80_n8_B.log 2>&1 || { echo "study 8x80M B failed"; tail -20 gpurun_out/r06_rq_s80_n8_B.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/rq_r06_s80_n8_B/replica_quality.json'))
for t, r in d['runs'].items(): print('8x80M B', t, {k: r[k] for k in r if k.endswith('gap')})"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_c4_e2e.py tests/test_gpu_parity.py -k "c4_cold or auto_tail" > gpurun_out/r06_c5_tests.log 2>&1 \
  || echo "tests failed"
grep -E "PASS|FAIL|passed|failed" gpurun_out/r06_c5_tests.log | tail -6
