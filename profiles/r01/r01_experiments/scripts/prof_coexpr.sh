set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_coexpr -o run --output-format csv -- python3 scripts/bench_coexpr.py > gpurun_out/prof_coexpr.log 2>&1
