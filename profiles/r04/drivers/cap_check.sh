#!/bin/bash
# round 4 (verdict r3 item 4): the stability cap's constant (100) on one more
# corpus at sample 0: 8,000 genes, 250 planted modules, 3 M pairs + GGIPNN x1;
# capped (default) vs uncapped (set_vocab's grid fixed) vs grid 16, and the
# sequential oracle; per-iteration |syn0|^2 / |syn1neg|^2 and the cap product
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/e2e_parity.py --sample 0 --vocab 8000 --modules 250 \
  --pairs 3000000 --ggipnn-repeat 1 --engines gpu,gpu_uncapped,gpu_grid16,oracle --seeds 1,2 \
  --auc-seeds "" --per-iter --out gpurun_out/cap_check_v8k > gpurun_out/r04_cap_check_v8k.log 2>&1
