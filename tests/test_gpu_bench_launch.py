"""GPU: `python bench.py --gpus 2` with NO outer launcher trains two ranks
(verdict r4 item 1): bench.py starts its own torch.distributed.run child, the
ranks (sharing the one GPU, gloo rehearsal) train their shards with libg2v's
in-call merges, and the one JSON line reports n_gpus 2 and the merges.  The
launcher logic alone is tests/test_bench_launcher.py (CPU)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_two_without_launcher():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo", "--pairs", "2000000",
           "--steps", "1", "--warmup", "0", "--avg-every-jobs", "100", "--no-cpu-baseline",
           "--no-eval", "--no-gather-roof"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["merge"]["merges"] > 0, line
    assert line["merge"]["backend"] == "libg2v-host"
    assert line["value_per_gpu"] * 2 == pytest.approx(line["value"], rel=1e-6)
    assert line["pairs_per_gpu"] == 2_000_000
    assert line["effective_examples"] > 2 * 2_000_000  # both ranks' examples counted


def test_bench_strong_scaling_two_ranks():
    """--scaling strong (verdict r5 item 4): 2 ranks split --total-pairs, the
    line says strong and names the whole corpus"""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo", "--scaling", "strong",
           "--total-pairs", "4000000", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
           "--no-eval", "--no-gather-roof"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["scaling"] == "strong" and line["n_gpus"] == 2
    assert line["pairs_per_gpu"] == 2_000_000
    assert line["config"]["total_pairs"] == 4_000_000
    assert "4000000 pairs in all" in line["config"]["workload"]
    assert line["value"] == pytest.approx(4_000_000 / (line["ms_per_step"] / 1e3), rel=1e-3)
