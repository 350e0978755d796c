#!/bin/bash
# round 5 (final build, 4 x 16 stripes): north-star metrics (loss, held-in objective, target function, GGIPNN AUC) at the C2
# vocabulary with the cold-row stores (gpu = default) vs every row atomic (gpu_tail0), against
# the C restatement's 16-thread Hogwild (gensim workers=16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c42
mkdir -p $O
timeout -k 10 1000 python -u scripts/e2e_parity.py --vocab 24447 --modules 1000 --pairs 10000000 \
  --engines gpu,gpu_tail0,oracle_hog16 --reference-engine oracle_hog16 --seeds 1,2 --out $O > $O/e2e.log 2>&1 \
  || { echo E2E FAILED; tail -20 $O/e2e.log; exit 1; }
grep -E "^(gpu|gpu_tail0|oracle_hog16) " $O/e2e.log | cut -c1-300
python3 -c "import json;d=json.load(open('$O/e2e_parity.json'));print(json.dumps(d['summary'],indent=1))"
