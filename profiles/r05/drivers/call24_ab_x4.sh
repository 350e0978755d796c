#!/bin/bash
# round 5: cold-row stores as 16-B lanes (1 b128 + 3 dropped pads per 1 KB) vs
# 4 b32 stores per row (b32): parity of the tail-store order, then bench A/B
# (historical: the b32 arm was an experiment build with -DG2V_STORE_X4=0; that form was removed after this A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c24
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_atomic_order.py > $O/atomic_order.log 2>&1 || { echo ORDER FAILED; tail -20 $O/atomic_order.log; exit 1; }
tail -1 $O/atomic_order.log
for rep in 1 2 3; do
  for L in prod b32; do
    if [ $L = prod ]; then LIB=gene2vec_amd/libg2v.so; else LIB=gene2vec_amd/libg2v_exp_$L.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --library $LIB \
      > $O/c2_${L}_$rep.json 2> $O/c2_${L}_$rep.err || { echo "$L failed"; tail -5 $O/c2_${L}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c2_${L}_$rep.json'));r=d['roofline'];print('c2','$L',$rep,d['value'],r['avg_launch_ms'])"
  done
done
for rep in 1 2; do
  for L in prod b32; do
    if [ $L = prod ]; then LIB=gene2vec_amd/libg2v.so; else LIB=gene2vec_amd/libg2v_exp_$L.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-roof --no-eval --vocab 60000 --dim 512 --negative 15 --library $LIB \
      > $O/c4_${L}_$rep.json 2> $O/c4_${L}_$rep.err || { echo "c4 $L failed"; tail -5 $O/c4_${L}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c4_${L}_$rep.json'));r=d['roofline'];print('c4','$L',$rep,d['value'],r['avg_launch_ms'])"
  done
done
