#!/bin/bash
# round 5: where a wave's cycles go with the cold-row stores (stamped build, debug write 8),
# and the e2e gates' numbers at the default tail stores
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c12
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 360 --timeout-method thread \
  tests/test_gpu_e2e_parity.py > $O/e2e.log 2>&1
echo "e2e rc=$?"; grep -E "gaps vs" $O/e2e.log | sed 's/.*gaps vs/gaps vs/' | cut -c1-260
timeout -k 10 400 python -u scripts/stamp_segments.py --arms production,stamped,tail0,stamped_tail0,production_again \
  --out $O/stamps_c2.json > $O/stamps_c2.log 2>&1; echo "stamps c2 rc=$?"
timeout -k 10 400 python -u scripts/stamp_segments.py --sample 0 --arms production,stamped,tail0,stamped_tail0 \
  --out $O/stamps_s0.json > $O/stamps_s0.log 2>&1; echo "stamps s0 rc=$?"
for S in 0.001 0; do
  timeout -k 10 300 python -u scripts/stamp_segments.py --sample $S --library gene2vec_amd/libg2v_exp_sb15.so \
    --arms production,stamped,production_again --out $O/stamps_sb15_s$S.json > $O/stamps_sb15_s$S.log 2>&1; echo "sb15 s$S rc=$?"
done
python3 - <<'PY'
import json
for f in ("gpurun_out/r05c12/stamps_c2.json","gpurun_out/r05c12/stamps_s0.json","gpurun_out/r05c12/stamps_sb15_s0.001.json","gpurun_out/r05c12/stamps_sb15_s0.json"):
    d=json.load(open(f))
    for arm,r in d["arms"].items():
        seg=r.get("segments_cycles") or {}
        print(f.split("_")[-1], arm, r.get("examples_per_s"), r.get("cycles_per_example_per_wave"), {k:round(v) for k,v in seg.items()} if seg else "")
PY
