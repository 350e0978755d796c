#!/bin/bash
# round 5: branch-free gradient path (bf) vs the current kernel (prod), bench A/B, fresh process per run
set -o pipefail
O=gpurun_out/r05c23
mkdir -p $O
for S in 0.001 0; do
 for rep in 1 2 3; do
  for L in prod bf; do
    if [ $L = prod ]; then LIB=gene2vec_amd/libg2v.so; else LIB=gene2vec_amd/libg2v_exp_$L.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --sample $S --library $LIB \
      > $O/ab_${L}_s${S}_$rep.json 2> $O/ab_${L}_s${S}_$rep.err || { echo "$L failed"; tail -5 $O/ab_${L}_s${S}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_${L}_s${S}_$rep.json'));r=d['roofline'];print('s$S','$L',$rep,d['value'],r['avg_launch_ms'])"
  done
 done
done
