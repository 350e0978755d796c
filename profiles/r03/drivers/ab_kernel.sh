#!/bin/bash
# A/B of the SGNS kernel on one box: the tree's libg2v vs a previous build
# placed under exp_r1/old (G2V_ROOT), at C2, C2 sample 0 and C4, then the SQ
# instruction mix of the tree's kernel.   usage: scripts/ab_kernel.sh TAG
set -e
T=${1:?tag}
O=gpurun_out/ab_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for who in new old; do
  R=$GRAFT_REPO_ROOT; [ $who = old ] && R=$GRAFT_REPO_ROOT/exp_r1/old
  G2V_ROOT=$R timeout -k 10 200 python scripts/exp_sweep.py --configs "ld=224" > $O/c2_$who.log 2>&1
  G2V_ROOT=$R timeout -k 10 200 python scripts/exp_sweep.py --sample 0 --configs "ld=224" > $O/s0_$who.log 2>&1
  G2V_ROOT=$R timeout -k 10 300 python scripts/exp_sweep.py --vocab 60000 --dim 512 --negative 15 --pairs 10000000 --configs "ld=512" > $O/c4_$who.log 2>&1
  echo "$who done"
done
for f in $O/*.log; do echo "== $f"; grep config $f; done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES -d $O/sq -o run --output-format csv \
  -- python3 bench.py --pairs 10000000 --steps 1 --warmup 0 --no-cpu-baseline --no-eval --no-gather-roof > $O/sq.log 2>&1
echo "sq rc=$?"
