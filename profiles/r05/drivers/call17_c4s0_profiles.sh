#!/bin/bash
# round 5: lost-update probe at C2 and C4, PMC traffic + kernel stats at C4 and sample 0
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c17
mkdir -p $O
timeout -k 10 300 python -u scripts/lost_updates.py --tails auto --epochs 1 --out $O/lost_c2.json > $O/lost_c2.log 2>&1; echo "lost c2 rc=$?"; grep "^auto" $O/lost_c2.log
timeout -k 10 300 python -u scripts/lost_updates.py --vocab 60000 --dim 512 --negative 15 --tails auto,0 --epochs 1 --out $O/lost_c4.json > $O/lost_c4.log 2>&1; echo "lost c4 rc=$?"; grep "^auto\|^0 " $O/lost_c4.log
bash scripts/profile_round.sh r05c4 --vocab 60000 --dim 512 --negative 15 > $O/profile_c4.log 2>&1; echo "profile c4 rc=$?"
bash scripts/profile_round.sh r05s0 --sample 0 > $O/profile_s0.log 2>&1; echo "profile s0 rc=$?"
for f in gpurun_out/prof_r05c4/bench_stats.log gpurun_out/prof_r05s0/bench_stats.log; do
  python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); r=d['roofline']; print('$f'.split('/')[1], d['value'], r['avg_launch_ms'], r['frac'], r['stored_rows_per_example'])"
done
