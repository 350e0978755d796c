#!/bin/bash
# round 5: sample-0 stripe layout re-checked with the cold-row stores (host options only), two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c34
mkdir -p $O
for rep in 1 2; do
  for cfg in "8x8 0x4" "4x8 0x4" "16x8 0x4" "8x16 0x4" "8x8 20x4" "8x8 16x2"; do
    set -- $cfg
    tag="s$1_t$2_$rep"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --sample 0 --stripe $1 --stripe2 $2 \
      > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];print('$tag',d['value'],r['avg_launch_ms'],r.get('stripes'),r.get('stripes_tier2'))"
  done
done
