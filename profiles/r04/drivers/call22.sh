#!/bin/bash
# round 4 call 22: rehearsals on the final tree -- bench.py with 8 ranks sharing
# the one GPU over gloo (C3 volume: 125 M pairs per rank, libg2v's host
# transport, the default 3,584-job touch cadence), then the CLI end to end
# (100 M pairs, 10 iterations, device shuffles, every checkpoint and export)
set -o pipefail
mkdir -p gpurun_out/r04c22
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 8 --backend gloo --steps 2 \
  --warmup 1 --no-cpu-baseline > gpurun_out/r04c22/bench_gloo_n8.json 2> gpurun_out/r04c22/bench_gloo_n8.err &&
timeout -k 10 400 python -u scripts/e2e_cli_timing.py --pairs 100000000 --files 8 --shuffle device \
  > gpurun_out/r04c22/cli_timing.json 2> gpurun_out/r04c22/cli_timing.err
