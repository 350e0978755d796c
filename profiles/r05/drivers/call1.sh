#!/bin/bash
# round 5, call 1: stripped kernel + tail-store experiment, first look
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_atomic_order.py tests/test_gpu_bench_launch.py tests/test_gpu_loss.py > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH FAILED; tail -20 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2',d['value'],d['roofline']['avg_launch_ms'],d['quality'])"
for T in 8192 2048 512; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-roof --tail-store $T > $O/bench_tail$T.json 2> $O/bench_tail$T.err || { echo BENCH T FAILED; tail -20 $O/bench_tail$T.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_tail$T.json'));print('tail',$T,d['value'],d['roofline']['avg_launch_ms'],d['quality'])"
done
for T in 0 2048; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-roof --sample 0 --tail-store $T > $O/bench_s0_tail$T.json 2> $O/bench_s0_tail$T.err || { echo BENCH S0 FAILED; tail -20 $O/bench_s0_tail$T.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_s0_tail$T.json'));print('s0 tail',$T,d['value'],d['roofline']['avg_launch_ms'],d['quality'])"
done
