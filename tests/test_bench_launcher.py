"""bench.py --gpus N: the benchmark's own process shape (verdict r4 item 1).

The driver runs `python bench.py --gpus N ...` for its BENCH line and wraps
N > 1 in torch.distributed.run for SCALE; both shapes must train N ranks.
Without a launcher, --gpus N > 1 starts one `torch.distributed.run` child
before anything touches the GPU; under a launcher --gpus must equal
WORLD_SIZE.  CPU-only here: --launch-probe makes the ranks meet over gloo and
rank 0 report the world instead of training (the training run of the same
shape is tests/test_gpu_bench_launch.py).  The reference is one process
(src/gene2vec.py:59,70)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra)
    return env


def test_gpus_n_without_launcher_starts_n_ranks():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--launch-probe"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # exactly one JSON line on stdout
    out = json.loads(lines[0])
    assert out["probe"] and out["n_gpus"] == 3
    assert out["rank_sum"] == out["ranks_expected_sum"] == 6  # ranks 0, 1, 2 all joined


def test_gpus_must_match_launcher_world():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--launch-probe"], cwd=ROOT,
                       env=_env(WORLD_SIZE="2", RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "--gpus 3" in r.stderr and "WORLD_SIZE=2" in r.stderr


def test_gpus_one_stays_one_process():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--launch-probe"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip())
    assert out["n_gpus"] == 1 and out["rank_sum"] == 1
    assert "torch.distributed.run" not in r.stderr


def test_strong_scaling_splits_the_total():
    """--scaling strong (verdict r5 item 4): each of N ranks trains
    --total-pairs / N (1 B / N by default); weak keeps 125 M per rank"""
    for argv, n, per in ((["--gpus", "4", "--scaling", "strong"], 4, 250_000_000),
                         (["--gpus", "2", "--scaling", "strong", "--total-pairs", "1000"], 2, 500),
                         (["--gpus", "1", "--scaling", "strong"], 1, 1_000_000_000),
                         (["--gpus", "2"], 2, 125_000_000),
                         (["--gpus", "1"], 1, 100_000_000)):
        r = subprocess.run([sys.executable, "bench.py", *argv, "--launch-probe"], cwd=ROOT,
                           env=_env(), capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-3000:]
        out = json.loads(r.stdout.strip())
        assert out["n_gpus"] == n and out["rank_sum"] == out["ranks_expected_sum"]
        assert out["pairs_per_rank"] == per, (argv, out)
        assert out["scaling"] == ("strong" if "strong" in argv else "weak")


def test_strong_scaling_refuses_pairs():
    r = subprocess.run([sys.executable, "bench.py", "--scaling", "strong", "--pairs", "10",
                        "--launch-probe"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0 and "--total-pairs" in r.stderr
