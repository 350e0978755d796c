#!/bin/bash
# round 5: why is sample 0 slower on the final kernel?  Bench A/B (fresh process per run):
#   prod = current (if/else, 15-copy batch, LDS slots), sb7 = current with 7-copy batches,
#   preslot = the kernel before the LDS-slot generalisation (commit 1f8ac6d),
#   adapt = current with the copy batch fitted to each tier (15 / 7 / 3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c19
mkdir -p $O
for S in 0 0.001; do
 for rep in 1 2; do
  for L in prod sb7 preslot adapt; do
    if [ $L = prod ]; then LIB=gene2vec_amd/libg2v.so; else LIB=gene2vec_amd/libg2v_exp_$L.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --sample $S --library $LIB \
      > $O/ab_${L}_s${S}_$rep.json 2> $O/ab_${L}_s${S}_$rep.err || { echo "$L failed"; tail -5 $O/ab_${L}_s${S}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_${L}_s${S}_$rep.json'));r=d['roofline'];print('s$S','$L',$rep,d['value'],r['avg_launch_ms'],r['waves_last_launch'])"
  done
 done
done
