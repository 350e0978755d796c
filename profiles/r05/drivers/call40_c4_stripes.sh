#!/bin/bash
# round 5: C4 (D 512, K 15, 121 workgroups) stripe layout around the new 4-row default, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c40
mkdir -p $O
for rep in 1 2; do
  for st in 4x8 4x16 2x8 6x8; do
    tag="c4_$st_$rep"; tag="c4_${st}_$rep"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --vocab 60000 --dim 512 --negative 15 --stripe $st \
      > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];print('$tag',d['value'],r['avg_launch_ms'],r.get('stripes'))"
  done
done
