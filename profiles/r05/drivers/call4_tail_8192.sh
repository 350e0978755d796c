#!/bin/bash
# round 5: tail stores at 4096 / 8192 -- the C2-vocabulary e2e gate (the only
# e2e corpus with rows past 4096) and interleaved bench repeats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c4
mkdir -p $O
for T in 8192 4096; do
  G2V_TEST_TAIL_STORE=$T timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread \
    "tests/test_gpu_e2e_parity.py::test_gpu_end_to_end_at_the_c2_vocabulary" > $O/e2e_c2_tail$T.log 2>&1
  echo "e2e c2 tail $T rc=$?"; grep -E "gaps vs" $O/e2e_c2_tail$T.log | sed 's/.*gaps vs/gaps vs/' | cut -c1-300
done
for rep in 1 2; do
  for T in 0 8192 4096; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-roof --tail-store $T > $O/bench_t${T}_$rep.json 2> $O/bench_t${T}_$rep.err || { echo BENCH FAILED; tail -5 $O/bench_t${T}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_t${T}_$rep.json'));print('tail',$T,d['value'],d['roofline']['avg_launch_ms'],d['quality'])"
  done
done
