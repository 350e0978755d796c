#!/bin/bash
# round 5: tail stores generalised to D > 256 / negative > 7 (LDS slots): parity + C4 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c16
mkdir -p $O
for rep in 1 2; do
  for T in -1 0; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-roof --vocab 60000 --dim 512 --negative 15 --tail-store $T \
      > $O/c4_t${T}_$rep.json 2> $O/c4_t${T}_$rep.err || { echo C4 FAILED; tail -5 $O/c4_t${T}_$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c4_t${T}_$rep.json'));r=d['roofline'];print('c4 tail',$T,d['value'],r['avg_launch_ms'],r['frac'],r['tail_row_syn1neg'],r['stored_rows_per_example'],d['quality'])"
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gather-roof > $O/c2.json 2> $O/c2.err; python -c "import json;d=json.load(open('$O/c2.json'));r=d['roofline'];print('c2',d['value'],r['avg_launch_ms'],r['frac'])"
