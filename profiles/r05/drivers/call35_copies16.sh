#!/bin/bash
# round 5: auto stripe copies 16 at D <= 256 whatever the grid (was 8 below one workgroup per CU):
# the parity / e2e / C4 gates, then sample 0 and a budget-held 3,000-gene corpus, auto vs 8 copies
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c35
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_e2e_parity.py \
  tests/test_gpu_parity.py tests/test_gpu_atomic_order.py tests/test_gpu_loss.py tests/test_gpu_c4.py > $O/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
grep -E "e2e|gap|target" $O/tests.log | head -0
for rep in 1 2 3; do
  for cfg in "0 auto" "0 8x8" "0.001 auto3k" "0.001 8x8_3k"; do
    set -- $cfg
    extra=""; st=""
    case $2 in 8x8) st="--stripe 8x8";; auto3k) extra="--vocab 3000";; 8x8_3k) extra="--vocab 3000"; st="--stripe 8x8";; esac
    tag="s$1_$2_$rep"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --sample $1 $extra $st \
      > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];print('$tag',d['value'],r['avg_launch_ms'],r.get('grid_workgroups'),r.get('stripes'))"
  done
done
