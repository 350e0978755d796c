#!/bin/bash
# bench C2 with the second stripe tier off / auto, interleaved
set -e
for i in 1 2 3 4; do
  for t in off auto; do
    opt=""; [ $t = off ] && opt="--stripe2 0x4"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --steps 6 $opt > gpurun_out/s2_${t}_$i.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/s2_${t}_$i.json'));r=d['roofline'];print('tier2', '$t', $i, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['stripes_tier2'], d['quality'])"
  done
done
