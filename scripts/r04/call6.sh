#!/bin/bash
# round 4 call 6: rocprofv3 kernel stats + PMC traffic of the round-4 kernel
# build (C2), then the stability-cap re-check at sample 0 on an 8,000-gene corpus
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash scripts/profile_round.sh r04 > gpurun_out/r04_profile_round.log 2>&1
rc=$?
echo "profile rc $rc" >> gpurun_out/r04_profile_round.log
[ $rc -eq 0 ] || exit $rc
bash scripts/r04/cap_check.sh
