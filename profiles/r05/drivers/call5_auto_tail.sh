#!/bin/bash
# round 5: cold-row stores on by default (auto collision budget 0.15): the gates they touch,
# the bench, and the lost-update probe (ablation build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c5
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread \
  tests/test_gpu_atomic_order.py tests/test_gpu_e2e_parity.py \
  "tests/test_gpu_parity.py::test_train_hogwild_full_vocab_tracks_oracle" \
  "tests/test_gpu_parity.py::test_train_hogwild_small_vocabulary_tracks_oracle" \
  "tests/test_gpu_parity.py::test_train_hogwild_objective_matches_oracle" \
  tests/test_gpu_loss.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "gaps vs|passed|failed|FAILED" $O/tests.log | sed 's/.*gaps vs/gaps vs/' | cut -c1-300
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH FAILED; tail -5 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));print('c2',d['value'],d['roofline']['avg_launch_ms'],d['roofline']['tail_store'],d['quality'])"
timeout -k 10 300 python -u scripts/lost_updates.py --tails auto,8192,4096,2048 --out $O/lost.json > $O/lost.log 2>&1
echo "lost rc=$?"; grep -v "^{" $O/lost.log | tail -10
