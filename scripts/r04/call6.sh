#!/bin/bash
# round 4 call 6: rocprofv3 stats + PMC traffic at C4, then the stability-cap
# re-check at sample 0 on an 8,000-gene corpus (scripts/r04/cap_check.sh)
set -o pipefail
mkdir -p gpurun_out/r04c6
timeout -k 10 500 bash scripts/profile_round.sh r04_c4 --vocab 60000 --dim 512 --negative 15 \
  > gpurun_out/r04c6/profile_c4.log 2>&1 &&
bash scripts/r04/cap_check.sh
