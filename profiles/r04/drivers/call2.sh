#!/bin/bash
# round 4 call 2: finer stamps + instruction-count probes, then the C3 gate and the small-DP sweep
set -o pipefail
mkdir -p gpurun_out/r04c2
timeout -k 10 240 python -u scripts/stamp_segments.py --sample 0 --grid 162 --pairs 20000000 \
  --arms production,stamped,notail,copies4,production_again,notail_again,copies4_again \
  --out gpurun_out/r04c2/stamps_s0.json > gpurun_out/r04c2/stamps_s0.log 2>&1 &&
timeout -k 10 240 python -u scripts/stamp_segments.py --sample 1e-3 --pairs 20000000 \
  --arms production,stamped,notail,production_again,notail_again \
  --out gpurun_out/r04c2/stamps_c2.json > gpurun_out/r04c2/stamps_c2.log 2>&1 &&
bash profiles/r04/drivers/quality1.sh
