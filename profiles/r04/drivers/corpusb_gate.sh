#!/bin/bash
# round 4: the corpus-B C3 gate twice (its run-to-run spread before it joins
# the round-end suite)
set -o pipefail
mkdir -p gpurun_out/r04cb
for i in 1 2; do
  timeout -k 10 500 python -u -m pytest -x -v -rP --timeout 450 --timeout-method thread \
    "tests/test_gpu_c3_quality.py::test_c3_second_corpus_within_one_percent" \
    > gpurun_out/r04cb/run$i.log 2>&1
  rc=$?
  echo "rc $rc" >> gpurun_out/r04cb/run$i.log
  [ $rc -le 1 ] || exit $rc
done
