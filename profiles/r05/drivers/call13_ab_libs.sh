#!/bin/bash
# round 5: interleaved A/B of experiment builds (scripts/stamp_segments.py production arm,
# 20 M pairs x 4 epochs, C2 vocabulary; a fresh process per run)
#   prod   = libg2v.so (tail rows: 4 dropped atomics + 4 stores)
#   ie     = if/else store-or-atomics, -structurizecfg-skip-uniform-regions (no dropped atomics)
#   sb15   = all 15 stripe copies of a row in one load batch
#   iesb15 = both
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c13
mkdir -p $O
for S in 0.001 0; do
 for rep in 1 2; do
  for L in prod ie sb15 iesb15; do
    if [ $L = prod ]; then LIB=gene2vec_amd/libg2v.so; else LIB=gene2vec_amd/libg2v_exp_$L.so; fi
    timeout -k 10 200 python -u scripts/stamp_segments.py --sample $S --library $LIB --arms production \
      --out $O/ab_${L}_s${S}_$rep.json > $O/ab_${L}_s${S}_$rep.log 2>&1 || { echo "$L failed"; tail -5 $O/ab_${L}_s${S}_$rep.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_${L}_s${S}_$rep.json'));print('s$S','$L',$rep,d['arms']['production']['examples_per_s'])"
  done
 done
done
