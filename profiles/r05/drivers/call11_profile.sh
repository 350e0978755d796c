#!/bin/bash
# round 5 evidence: rocprofv3 kernel stats + PMC traffic of the C2 bench on the final kernel,
# the lost-update probe at the default (syn1neg-only auto), sample-0 and C4 lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c11
mkdir -p $O
bash scripts/profile_round.sh r05 > $O/profile.log 2>&1; echo "profile rc=$?"; tail -30 $O/profile.log | grep -E "rc=|fetch_bytes|write_bytes|traffic_over|l2_hit|atomic_req" | head -12
timeout -k 10 300 python -u scripts/lost_updates.py --tails auto --epochs 1 --out $O/lost_auto.json > $O/lost_auto.log 2>&1
echo "lost rc=$?"; grep "^auto" $O/lost_auto.log
timeout -k 10 300 python bench.py --no-cpu-baseline --sample 0 > $O/bench_s0.json 2> $O/bench_s0.err; echo "s0 rc=$?"
python -c "import json;d=json.load(open('$O/bench_s0.json'));r=d['roofline'];print('s0',d['value'],r['avg_launch_ms'],r['frac'],r['tail_row_syn1neg'] if 'tail_row_syn1neg' in r else '',d['quality'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --vocab 60000 --dim 512 --negative 15 > $O/bench_c4.json 2> $O/bench_c4.err; echo "c4 rc=$?"
python -c "import json;d=json.load(open('$O/bench_c4.json'));r=d['roofline'];print('c4',d['value'],r['avg_launch_ms'],r['frac'],d['quality'])"
