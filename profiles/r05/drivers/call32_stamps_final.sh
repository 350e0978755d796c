#!/bin/bash
# round 5: per-segment cycles of the final kernel (16-B cold-row stores), C2 and sample 0
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c32
mkdir -p $O
for S in 0.001 0; do
  timeout -k 10 300 python -u scripts/stamp_segments.py --sample $S --out $O/stamps_final_s$S.json > $O/stamps_s$S.log 2>&1 \
    || { echo "s$S failed"; tail -5 $O/stamps_s$S.log; exit 1; }
  python3 -c "import json;d=json.load(open('$O/stamps_final_s$S.json'));a=d['arms'];s=a['stamped'];print('s$S',a['production']['examples_per_s'],a['production_again']['examples_per_s'],s['cycles_per_example_per_wave'],json.dumps(s['segments_cycles']))"
done
