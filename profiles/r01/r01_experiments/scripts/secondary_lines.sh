#!/bin/bash
# secondary bench lines asked by SURVEY 8(d): sample=0 (workload-stable) and a 1-core CPU baseline
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "hogwild_disjoint" -x -v --timeout 120 --timeout-method thread > gpurun_out/t_hogwild_k.log 2>&1 &&
timeout -k 10 400 python -u bench.py --sample 0 > gpurun_out/bench_sample0.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 2 --cpu-threads 1 --cpu-sample-pairs 4000000 --no-gather-roof > gpurun_out/bench_cpu1.log 2>&1
