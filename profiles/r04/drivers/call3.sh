#!/bin/bash
# round 4 call 3: the repeat-free fast path of k_sgns_atomic -- parity tests
# that exercise the kernel, stamps, bench -- then the 50 M / 80 M align confirmation
set -o pipefail
mkdir -p gpurun_out/r04c3
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_atomic_order.py tests/test_gpu_parity.py tests/test_gpu_loss.py \
  tests/test_gpu_e2e_parity.py tests/test_gpu_c4.py tests/test_gpu_merge_group.py \
  > gpurun_out/r04c3/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/r04c3/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python -u scripts/stamp_segments.py --sample 0 --grid 162 --pairs 20000000 \
  --arms production,stamped,production_again \
  --out gpurun_out/r04c3/stamps_s0.json > gpurun_out/r04c3/stamps_s0.log 2>&1 &&
timeout -k 10 240 python -u scripts/stamp_segments.py --sample 1e-3 --pairs 20000000 \
  --arms production,stamped,production_again \
  --out gpurun_out/r04c3/stamps_c2.json > gpurun_out/r04c3/stamps_c2.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r04c3/bench.json 2> gpurun_out/r04c3/bench.err &&
timeout -k 10 200 python -u bench.py --sample 0 --no-cpu-baseline > gpurun_out/r04c3/bench_s0.json 2> gpurun_out/r04c3/bench_s0.err &&
timeout -k 10 500 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 50000000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 --merge-every 1431 --rules align \
  --replica-seeds 1,2 --single-seeds 1,2 --auc-seeds 0 \
  --out gpurun_out/rq_50m_align > gpurun_out/r04_rq_50m_align.log 2>&1
