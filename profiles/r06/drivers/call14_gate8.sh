#!/bin/bash
# round 6: the new 8-rank window gate (8 x 150 M, corpus B, the wide-shard plan)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -v --timeout 700 --timeout-method thread \
  tests/test_gpu_c3_quality.py -k wide_shard -s > gpurun_out/r06_gate8.log 2>&1 \
  || { echo "gate failed"; tail -30 gpurun_out/r06_gate8.log; exit 1; }
grep -E "PASS|FAIL|replicas x|passed|failed" gpurun_out/r06_gate8.log | tail -4
