#!/bin/bash
# round 6 (verdict r5 item 3): rocprofv3 --kernel-trace --stats + the PMC passes
# (with L2 hit rate and VALU busy) at C2, C4 and sample 0 on the final kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/profile_round.sh r06_c2 > gpurun_out/r06_prof_c2.log 2>&1 || { echo "c2 profile failed"; tail -20 gpurun_out/r06_prof_c2.log; exit 1; }
tail -3 gpurun_out/r06_prof_c2.log
bash scripts/profile_round.sh r06_c4 --vocab 60000 --dim 512 --negative 15 > gpurun_out/r06_prof_c4.log 2>&1 || { echo "c4 profile failed"; tail -20 gpurun_out/r06_prof_c4.log; exit 1; }
tail -3 gpurun_out/r06_prof_c4.log
bash scripts/profile_round.sh r06_s0 --sample 0 > gpurun_out/r06_prof_s0.log 2>&1 || { echo "s0 profile failed"; tail -20 gpurun_out/r06_prof_s0.log; exit 1; }
tail -3 gpurun_out/r06_prof_s0.log
