#!/bin/bash
# round 5: work-queue chunks of 64 examples (ch64) vs 32 (prod), bench A/B; the D 37 tail-store order case
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c26
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_atomic_order.py > $O/atomic_order.log 2>&1 || { echo ORDER FAILED; tail -20 $O/atomic_order.log; exit 1; }
tail -1 $O/atomic_order.log
for S in 0.001 0; do
 for rep in 1 2 3; do
  for L in prod ch64; do
    if [ $L = prod ]; then LIB=gene2vec_amd/libg2v.so; else LIB=gene2vec_amd/libg2v_exp_$L.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --sample $S --library $LIB \
      > $O/ab_${L}_s${S}_$rep.json 2> $O/ab_${L}_s${S}_$rep.err || { echo "$L failed"; tail -5 $O/ab_${L}_s${S}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_${L}_s${S}_$rep.json'));r=d['roofline'];print('s$S','$L',$rep,d['value'],r['avg_launch_ms'],d.get('quality'))"
  done
 done
done
for L in prod ch64; do
  if [ $L = prod ]; then LIB=gene2vec_amd/libg2v.so; else LIB=gene2vec_amd/libg2v_exp_$L.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --vocab 60000 --dim 512 --negative 15 --library $LIB \
    > $O/c4_${L}.json 2> $O/c4_${L}.err || { echo "c4 $L failed"; tail -5 $O/c4_${L}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c4_${L}.json'));r=d['roofline'];print('c4','$L',d['value'],r['avg_launch_ms'])"
done
