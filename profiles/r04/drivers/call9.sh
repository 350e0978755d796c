#!/bin/bash
# round 4 call 9: the final kernel build's rocprofv3 stats + PMC traffic at
# C2, sample 0 and C4, then the plain bench lines (C2 with the CPU baseline)
set -o pipefail
mkdir -p gpurun_out/r04c18
timeout -k 10 360 bash scripts/profile_round.sh r04 > gpurun_out/r04c18/profile_c2.log 2>&1 &&
timeout -k 10 360 bash scripts/profile_round.sh r04_s0 --sample 0 > gpurun_out/r04c18/profile_s0.log 2>&1 &&
timeout -k 10 420 bash scripts/profile_round.sh r04_c4 --vocab 60000 --dim 512 --negative 15 \
  > gpurun_out/r04c18/profile_c4.log 2>&1 &&
timeout -k 10 240 python -u bench.py > gpurun_out/r04c18/bench.json 2> gpurun_out/r04c18/bench.err
