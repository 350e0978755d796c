set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m cProfile -o gpurun_out/e2e.prof scripts/e2e_cli_timing.py --pairs 100000000 --files 8 --iters 10 > gpurun_out/e2e_prof.log 2>&1
python -c "
import pstats; p=pstats.Stats('gpurun_out/e2e.prof'); p.sort_stats('cumulative').print_stats(45)" > gpurun_out/e2e_pstats.txt 2>&1
