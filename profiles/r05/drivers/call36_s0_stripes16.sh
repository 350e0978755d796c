#!/bin/bash
# round 5: stripe rows / second tier around the new 16-copy default at sample 0 and on a 3,000-gene corpus
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c36
mkdir -p $O
for rep in 1 2; do
  for cfg in "0 8x16 0x4" "0 4x16 0x4" "0 12x16 0x4" "0 8x16 20x4" "0 8x16 16x2" "0.001 8x16 0x4" "0.001 8x16 20x4" "0.001 12x16 0x4"; do
    set -- $cfg
    extra=""; [ "$1" = "0.001" ] && extra="--vocab 3000"
    tag="s$1_$2_t$3_$rep"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --sample $1 $extra --stripe $2 --stripe2 $3 \
      > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$tag.json'));r=d['roofline'];print('$tag',d['value'],r['avg_launch_ms'])"
  done
done
