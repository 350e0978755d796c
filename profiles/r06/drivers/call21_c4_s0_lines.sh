#!/bin/bash
# round 6 (verdict r5 item 3): the C4 and sample-0 bench lines on the final
# tree, now carrying roofline.traffic / l2_hit_rate / valu_busy from the r06 profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06lines
timeout -k 10 300 python bench.py --vocab 60000 --dim 512 --negative 15 --no-cpu-baseline > gpurun_out/r06lines/final_bench_c4.json 2> gpurun_out/r06lines/c4.err \
  || { echo "C4 bench failed"; tail -5 gpurun_out/r06lines/c4.err; exit 1; }
timeout -k 10 300 python bench.py --sample 0 --no-cpu-baseline > gpurun_out/r06lines/final_bench_s0.json 2> gpurun_out/r06lines/s0.err \
  || { echo "s0 bench failed"; tail -5 gpurun_out/r06lines/s0.err; exit 1; }
for c in c4 s0; do python3 -c "
import json;d=json.load(open('gpurun_out/r06lines/final_bench_$c.json'));r=d['roofline']
print('$c', d['value'], r['avg_launch_ms'], r['frac'], r['traffic'], r.get('l2_hit_rate'), r.get('valu_busy'), r.get('traffic_over_algorithmic'))"; done
