#!/bin/bash
# round 5: 4 striped rows instead of 8 (tier-2 default unchanged), interleaved, on every line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c37
mkdir -p $O
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-roof --no-eval "$@" > $O/$tag.json 2> $O/$tag.err \
    || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];print('$tag',d['value'],r['avg_launch_ms'],r.get('stripes'),r.get('stripes_tier2'))"
}
for rep in 1 2 3; do
  run s0_r8_$rep --sample 0 --stripe 8x16 || exit 1
  run s0_r4_$rep --sample 0 --stripe 4x16 || exit 1
  run c2_r8_$rep --stripe 8x16 || exit 1
  run c2_r4_$rep --stripe 4x16 || exit 1
  run v3k_r8_$rep --vocab 3000 --stripe 8x16 || exit 1
  run v3k_r4_$rep --vocab 3000 --stripe 4x16 || exit 1
done
run s0_r2_1 --sample 0 --stripe 2x16 || exit 1
for rep in 1 2; do
  run c4_r8_$rep --vocab 60000 --dim 512 --negative 15 --stripe 8x8 || exit 1
  run c4_r4_$rep --vocab 60000 --dim 512 --negative 15 --stripe 4x8 || exit 1
done
