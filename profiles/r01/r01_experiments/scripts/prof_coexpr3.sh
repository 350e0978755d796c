#!/bin/bash
# coexpr: GPU parity tests, live-roofline bench, rocprof kernel stats of the same bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_coexpr.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_coexpr.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_coexpr.py > gpurun_out/bench_coexpr.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_coexpr3 -o run --output-format csv -- python3 scripts/bench_coexpr.py > gpurun_out/prof_coexpr3.log 2>&1 &&
cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 600 python -u scripts/bench_ingest.py > gpurun_out/bench_ingest.log 2>&1 &&
timeout -k 10 300 python -u scripts/e2e_cli_timing.py > gpurun_out/e2e_cli.log 2>&1
