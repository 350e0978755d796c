#!/bin/bash
# round 4 call 4: copies-first loads + combined row tails in k_sgns_atomic --
# the kernel's parity tests, stamps and tails A/B, bench lines
set -o pipefail
mkdir -p gpurun_out/r04c4
timeout -k 10 700 python -u -m pytest -x -v -rP --timeout 400 --timeout-method thread \
  tests/test_gpu_atomic_order.py tests/test_gpu_parity.py tests/test_gpu_loss.py \
  tests/test_gpu_e2e_parity.py tests/test_gpu_c4.py \
  "tests/test_gpu_c3_quality.py::test_dp_50m_per_rank_align_within_one_percent" \
  > gpurun_out/r04c4/tests.log 2>&1
rc=$?
echo "tests rc $rc" >> gpurun_out/r04c4/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/stamp_segments.py --sample 0 --grid 162 --pairs 20000000 \
  --arms production,stamped,stamped_defer0,tails0,defer0,production_again,tails0_again,defer0_again \
  --out gpurun_out/r04c4/stamps_s0.json > gpurun_out/r04c4/stamps_s0.log 2>&1 &&
timeout -k 10 300 python -u scripts/stamp_segments.py --sample 1e-3 --pairs 20000000 \
  --arms production,stamped,stamped_defer0,tails0,defer0,production_again,tails0_again,defer0_again \
  --out gpurun_out/r04c4/stamps_c2.json > gpurun_out/r04c4/stamps_c2.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r04c4/bench.json 2> gpurun_out/r04c4/bench.err &&
timeout -k 10 200 python -u bench.py --sample 0 --no-cpu-baseline > gpurun_out/r04c4/bench_s0.json 2> gpurun_out/r04c4/bench_s0.err &&
timeout -k 10 300 python -u bench.py --vocab 60000 --dim 512 --negative 15 --no-cpu-baseline > gpurun_out/r04c4/bench_c4.json 2> gpurun_out/r04c4/bench_c4.err &&
timeout -k 10 400 python -u scripts/replica_quality.py --replicas 8 --pairs-per-replica 80000000 \
  --iters 10 --ggipnn-repeat 3 --modules 1000 --p-module 0.5 --merge-every 2288 --rules align \
  --auc-seeds 0 --out gpurun_out/rq_80m_align > gpurun_out/r04_rq_80m_align.log 2>&1
