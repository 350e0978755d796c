#!/bin/bash
# the round's bench lines: C2 (default), C4, sample 0
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python bench.py > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err || exit $?
timeout -k 10 500 python bench.py --vocab 60000 --dim 512 --negative 15 --no-cpu-baseline \
  > gpurun_out/r03h_bench_c4.json 2> gpurun_out/r03h_bench_c4.err || exit $?
timeout -k 10 500 python bench.py --sample 0 --no-cpu-baseline \
  > gpurun_out/r03h_bench_s0.json 2> gpurun_out/r03h_bench_s0.err || exit $?
