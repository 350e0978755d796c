"""GPU: libg2v's RCCL transport with TWO ranks on the one-GPU box (verdict r3
item 3).

The kCommRccl lines of g2v_api.hip -- ncclCommInitRank, the grouped
ncclBroadcast of the tables (comm_broadcast_tables), the grouped ncclAllReduce
of every merge (comm_allreduce), ncclCommAbort on failure -- are the default
under torchrun, but real RCCL refuses two ranks on one GPU ("Duplicate GPU
detected").  G2V_RCCL_LIB points libg2v's dlopen at the test-only stand-in
tests/rccl_standin/libg2v_rccl_standin.so, which carries the same calls
through shared memory with the host transport's rank-order sum, so:
  * the merged tables of a two-rank run are bit-identical to the host
    transport's (distributed.HostCollective over gloo), sequential kernel
    (deterministic), touch / mean / align rules;
  * a rank failing between in-call merges (G2V_OPT_DEBUG_FAIL_MERGE) aborts
    the communicator and its peer fails out of its merge at once (no hang),
    on both transports (the host one is ADVICE r3's medium finding);
  * the DP CLI and bench.py run their RCCL merge path through it.
The reference has no counterpart (one process, src/gene2vec.py:59)."""
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def standin():
    from tests.rccl_standin import build as B
    return B.build()


def _env(standin, **extra):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", G2V_RCCL_LIB=standin,
               G2V_ALLOW_RCCL_STANDIN="1",
               G2V_RCCL_STANDIN_MB="64", G2V_RCCL_STANDIN_TIMEOUT_S="90",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.update(extra)
    return env


def _run_pair(tmp_path, standin, transport, tag, *extra):
    port = _free_port()
    out = str(tmp_path / tag)
    procs = [subprocess.Popen([sys.executable, "-u", "-m", "tests.rccl_standin.worker",
                               "--rank", str(r), "--port", str(port), "--transport", transport,
                               "--out", out, *extra],
                              cwd=ROOT, env=_env(standin), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True)
             for r in range(2)]
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, lg in zip(procs, logs):
        assert p.returncode == 0, lg[-3000:]
    return [json.load(open(f"{out}_rank{r}.json")) for r in range(2)], out


@pytest.mark.parametrize("rule", ["touch", "mean", "align"])
def test_rccl_two_ranks_bit_identical_to_host_transport(tmp_path, standin, rule):
    st_r, out_r = _run_pair(tmp_path, standin, "rccl", f"rccl_{rule}", "--rule", rule)
    st_h, out_h = _run_pair(tmp_path, standin, "host", f"host_{rule}", "--rule", rule)
    for s in st_r + st_h:
        assert s["ok"], s
    # 120,000 pairs per rank = 24 jobs, a merge every 8 jobs: 3 per epoch, 2 epochs;
    # the stand-in ran every one of them (+ the 2 table broadcasts of comm_init)
    assert st_r[0]["merges"] == st_r[1]["merges"] == 6
    n_coll = {"touch": 3, "mean": 2, "align": 3}[rule]
    assert st_r[0]["standin_calls"] == st_r[1]["standin_calls"] == 2 + 6 * n_coll
    a = [np.load(f"{out_r}_rank{r}.npz") for r in range(2)]
    b = [np.load(f"{out_h}_rank{r}.npz") for r in range(2)]
    for t in ("syn0", "syn1neg"):
        assert np.array_equal(a[0][t], a[1][t])  # the replicas agree
        assert np.array_equal(a[0][t], b[0][t]), t  # RCCL path == host transport, bit for bit
        assert np.array_equal(b[0][t], b[1][t])
    assert np.abs(a[0]["syn1neg"]).max() > 0


@pytest.mark.parametrize("transport", ["rccl", "host"])
def test_failure_between_merges_reaches_the_peer(tmp_path, standin, transport):
    t = time.time()
    st, _ = _run_pair(tmp_path, standin, transport, f"fail_{transport}", "--fail-merge", "2")
    took = time.time() - t
    assert not st[0]["ok"] and not st[1]["ok"], st
    assert "injected failure before in-call merge 2" in st[1]["error"], st[1]
    if transport == "rccl":
        # the failing rank's g2v_train aborted the communicator (ncclCommAbort):
        # the peer's ncclAllReduce returned at once instead of timing out
        assert "ncclAllReduce failed" in st[0]["error"], st[0]
        assert "communicator aborted" in st[0]["error"], st[0]
    else:
        # the failing rank joined the pending gather with its ok flag cleared
        assert st[0]["error"].startswith("PeerFailed"), st[0]
    assert max(s["seconds"] for s in st) < 80, (took, st)  # far below the 90 s barrier timeout


def test_dp_cli_rccl_path_equals_host_path(tmp_path, standin):
    """torchrun -m gene2vec_amd.gene2vec with --merge-transport rccl (the
    torchrun default's libg2v path, bootstrapped over gloo here) and with the
    host transport: same shuffles, sequential kernel -> identical checkpoints"""
    from gene2vec_amd import Word2Vec
    from gene2vec_amd import synthetic as S
    V, n_pairs = 800, 120_000
    names = S.gene_names(V)
    pairs = S.zipf_gene_pairs(n_pairs, V, 1.0, seed=12)
    data = tmp_path / "data"
    data.mkdir()
    for k, part in enumerate(np.array_split(pairs, 3)):
        (data / f"pairs_{k}.txt").write_text(
            "\n".join(f"{names[a]} {names[b]}" for a, b in part) + "\n", encoding="windows-1252")
    log = tmp_path / "standin.log"
    outs = {}
    for transport in ("rccl", "host"):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               "-m", "gene2vec_amd.gene2vec", str(data), str(tmp_path / transport), "txt",
               "--backend", "gloo", "--merge-transport", transport, "--dp-min-pairs-per-rank", "0",
               "--mode", "sequential", "--iters", "2", "--dim", "32", "--hash", "crc32",
               "--shuffle-seed", "3", "--native-ingest", "--no-txt", "--no-w2v",
               "--merge-every-jobs", "4"]
        r = subprocess.run(cmd, env=_env(standin, G2V_RCCL_STANDIN_LOG=str(log)), cwd=ROOT,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        outs[transport] = Word2Vec.load(str(tmp_path / transport / "gene2vec_dim_32_iter_2"))
    lines = log.read_text().split("\n")
    assert sum(1 for ln in lines if "collectives" in ln) == 2, lines  # both rccl ranks, not host
    assert np.array_equal(outs["rccl"].wv.vectors, outs["host"].wv.vectors)
    assert np.array_equal(outs["rccl"].syn1neg, outs["host"].syn1neg)


def test_bench_two_ranks_rccl_merge(tmp_path, standin):
    """bench.py's N > 1 path (C3 shape, reduced to 2 M pairs per rank) with
    libg2v's RCCL merge: the line names the rccl backend and its merges"""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--backend", "gloo", "--merge-transport", "rccl", "--pairs", "2000000",
           "--steps", "2", "--warmup", "1", "--avg-every-jobs", "100", "--no-cpu-baseline",
           "--no-gather-roof"]
    r = subprocess.run(cmd, env=_env(standin, G2V_RCCL_STANDIN_MB="256"), cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["merge"]["backend"] == "rccl", line["merge"]
    assert line["merge"]["merges"] == 3 * 4  # 400 jobs per rank, every 100: 4 per epoch, 3 epochs
    assert line["value"] > 0 and line["quality"]["sgns_loss_heldin"] < line["quality"]["init_loss"]
