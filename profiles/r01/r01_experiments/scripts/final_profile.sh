#!/bin/bash
# round-end evidence: GPU tests, smoke, bench JSON, rocprofv3 kernel stats of the same bench command
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/final/bench.json.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/final/bench_prof.log 2>&1
timeout -k 10 400 python -u scripts/e2e_cli_timing.py --pairs 100000000 --files 8 > gpurun_out/final/e2e_100m.log 2>&1
