#!/bin/bash
# round 5 rehearsals on the final tree: bench.py --gpus 8 with NO outer launcher
# (its own torch.distributed.run child; 8 ranks sharing the one GPU over gloo, C3 volume,
# the 8-rank plan), --gpus 4 the same (the once-per-epoch plan), then the CLI end to end
set -o pipefail
O=gpurun_out/r05c20
mkdir -p $O
timeout -k 10 500 python bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_gloo_n8.json 2> $O/bench_gloo_n8.err; echo "n8 rc=$?"
python3 -c "import json;d=json.load(open('$O/bench_gloo_n8.json'));print('n8',d['n_gpus'],d['value'],d['value_per_gpu'],d['pairs_per_gpu'],d['merge'],d['quality'])"
timeout -k 10 400 python bench.py --gpus 4 --backend gloo --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/bench_gloo_n4.json 2> $O/bench_gloo_n4.err; echo "n4 rc=$?"
python3 -c "import json;d=json.load(open('$O/bench_gloo_n4.json'));print('n4',d['n_gpus'],d['value'],d['value_per_gpu'],d['pairs_per_gpu'],d['merge'],d['quality'])"
timeout -k 10 400 python -u scripts/e2e_cli_timing.py --pairs 100000000 --files 8 --shuffle device \
  > $O/cli_timing.json 2> $O/cli_timing.err; echo "cli rc=$?"; tail -1 $O/cli_timing.json
