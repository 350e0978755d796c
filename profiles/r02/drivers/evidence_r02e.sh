set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err &&
timeout -k 10 300 python bench.py --vocab 60000 --dim 512 --negative 15 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err &&
timeout -k 10 300 python bench.py --sample 0 --no-cpu-baseline > gpurun_out/bench_s0.json 2> gpurun_out/bench_s0.err &&
timeout -k 10 500 python -u scripts/quality_full_c2.py --vocab 60000 --dim 512 --negative 15 --pairs 20000000 > gpurun_out/quality_c4.log 2>&1
