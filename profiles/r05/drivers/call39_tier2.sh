#!/bin/bash
# round 5: the second stripe tier around the 4 x 16 default, C2 and sample 0, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c39
mkdir -p $O
for rep in 1 2; do
  for cfg in "0.001 20x4" "0.001 20x8" "0.001 12x8" "0.001 12x4" "0.001 32x4" "0 0x4" "0 8x4" "0 8x2" "0 12x4"; do
    set -- $cfg
    tag="s$1_t$2_$rep"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --sample $1 --stripe2 $2 \
      > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];print('$tag',d['value'],r['avg_launch_ms'],r.get('stripes'),r.get('stripes_tier2'))"
  done
done
