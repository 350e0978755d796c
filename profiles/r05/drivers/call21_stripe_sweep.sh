#!/bin/bash
# round 5: re-tune the hot-row stripes now that the cold syn1neg rows are stored (C2 bench lines)
set -o pipefail
O=gpurun_out/r05c21
mkdir -p $O
for rep in 1 2; do
  for ST in "8x16 20x4" "8x8 20x4" "8x16 0x4" "8x16 32x4" "16x8 32x4" "4x16 20x4"; do
    set -- $ST
    tag="${1}_${2}"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --stripe $1 --stripe2 $2 \
      > $O/st_${tag}_$rep.json 2> $O/st_${tag}_$rep.err || { echo "$tag failed"; tail -3 $O/st_${tag}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/st_${tag}_$rep.json'));r=d['roofline'];print('$tag',$rep,d['value'],r['avg_launch_ms'],r['stripes'],r['stripes_tier2'])"
  done
for rep in 1 2; do
  for G in 256 384 512; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --grid $G \
      > $O/grid_${G}_$rep.json 2> $O/grid_${G}_$rep.err || { echo "grid $G failed"; tail -3 $O/grid_${G}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/grid_${G}_$rep.json'));r=d['roofline'];print('grid',$G,$rep,d['value'],r['avg_launch_ms'],r['tail_row_syn1neg'],r['stripes'],d['quality'])"
  done
done
done
