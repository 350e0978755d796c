#!/bin/bash
# round 5: upside of splitting one example over two waves, emulated: dim 100 on twice the waves
# (grid 512 = 2 waves per SIMD) carries the same per-wave and chip-wide write traffic as dim 200
# split in halves; the split's examples/s would be half of that run's, minus the pair's sync
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c30
mkdir -p $O
for cfg in "200 256" "100 512" "100 256" "200 512"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --dim $1 --grid $2 --tail-store 7734 \
    > $O/d$1_g$2.json 2> $O/d$1_g$2.err || { echo "d$1 g$2 failed"; tail -5 $O/d$1_g$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/d$1_g$2.json'));r=d['roofline'];print('D$1 grid$2',d['value'],r['avg_launch_ms'],r.get('waves_last_launch'),r.get('stored_rows_per_example'))"
done
