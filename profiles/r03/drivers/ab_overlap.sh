#!/bin/bash
# bench C2 with the sampler overlapped (G2V_OPT_SAMPLE_OVERLAP) or not, interleaved
set -e
for i in 1 2 3 4 5; do
  for ov in 0 1; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-gather-roof --sample-overlap $ov ${@} > gpurun_out/ov_${ov}_$i.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/ov_${ov}_$i.json'));r=d['roofline'];print('overlap', $ov, $i, d['value'], d['ms_per_step'], r['avg_launch_ms'], d['quality'])"
  done
done
