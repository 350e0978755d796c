#!/bin/bash
# round 5: what a wave's chain costs at fewer bytes per example -- C2 at dim 200 / 128 / 100 / 64
# (examples/s, launch time), sample 1e-3 and 0: does halving the row bytes halve the write-issue time?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c28
mkdir -p $O
for S in 0.001 0; do
  for Dm in 200 128 100 64; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --sample $S --dim $Dm \
      > $O/d${Dm}_s$S.json 2> $O/d${Dm}_s$S.err || { echo "d$Dm failed"; tail -5 $O/d${Dm}_s$S.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/d${Dm}_s$S.json'));r=d['roofline'];print('s$S','D$Dm',d['value'],r['avg_launch_ms'],r.get('waves_last_launch'),r.get('stored_rows_per_example'),r['frac'])"
  done
done
