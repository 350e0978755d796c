#!/bin/bash
# round 4 call 23: LDS-DMA chunk pipeline, throughput probe only
# (stamps harness, production + stamped arms at sample 0 and C2)
set -o pipefail
mkdir -p gpurun_out/r04c23
timeout -k 10 300 python -u scripts/stamp_segments.py --sample 0 --grid 162 --pairs 20000000 \
  --arms production,stamped,production_again \
  --out gpurun_out/r04c23/stamps_s0.json > gpurun_out/r04c23/stamps_s0.log 2>&1 &&
timeout -k 10 300 python -u scripts/stamp_segments.py --sample 1e-3 --pairs 20000000 \
  --arms production,stamped,production_again \
  --out gpurun_out/r04c23/stamps_c2.json > gpurun_out/r04c23/stamps_c2.log 2>&1
