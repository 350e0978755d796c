#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
SPEC="0:512:8:8,0:512:8:4,0:512:16:4,0:512:4:8,0:512:16:8,0:512:4:16,0:512:2:16,0:512:8:12,0:512:32:4"
SAMPLE=0 timeout -k 10 300 python -u scratch/ablate.py $SPEC > gpurun_out/stripe_sweep_s0.log 2>&1 &&
SAMPLE=1e-3 timeout -k 10 300 python -u scratch/ablate.py $SPEC > gpurun_out/stripe_sweep_s1e-3.log 2>&1
