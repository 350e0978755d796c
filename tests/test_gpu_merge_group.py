"""GPU: libg2v's replica merge with MORE THAN ONE replica (SURVEY.md 8(e);
verdict r2 "what's missing" #2).

RCCL refuses two ranks on one GPU, so the N > 1 path runs here through the
two other transports of the same merge (include/g2v.h): an in-process group
of contexts driven by one thread each (g2v_comm_init_local: the all-reduce is
a device sum in rank order) and the host collective over gloo between
processes (g2v_comm_init_host).  Only the all-reduce differs from the RCCL
path: k_merge_delta / k_merge_apply, the touched counts, the rank-0
broadcast of g2v_comm_init* and the in-call merges of g2v_train with uneven
window counts are the lines RCCL runs.  Replicas train SEQUENTIAL (one wave,
gensim order) so every result is deterministic and the comparisons are bit
for bit: against g2v_average_local (k_merge_local, one kernel over all
replicas, the same summation order) and the numpy restatement of the touch
rule (distributed.touch_merge_)."""
import os
import socket
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd import distributed as Dd
from gene2vec_amd import engine as E
from tests.helpers import vocab_from_ids, zipf_pairs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _corpus(V0=600, D=48, K=5, n_total=60_000, seed=21):
    pairs = zipf_pairs(n_total, V0, seed=seed)
    flat = pairs.reshape(-1)
    _, remap, counts = vocab_from_ids(flat, V0)
    tok = remap[flat]
    V = len(counts)
    rng = np.random.Generator(np.random.PCG64(5))
    syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
    return tok, counts, syn0, V, D, K


def _engine(counts, syn0, D, K, tok_shard, syn0_override=None):
    e = E.SGNSEngine(len(counts), D, K)
    e.set_vocab(counts, 1e-3)
    s0 = syn0 if syn0_override is None else syn0_override
    e.set_weights(s0, np.zeros_like(s0))
    e.set_corpus(tok_shard, sent_len=2)
    return e


def _shards(tok, sizes):
    out, p = [], 0
    for n in sizes:
        out.append(tok[2 * p:2 * (p + n)])
        p += n
    return out


def _schedule(n_pairs, seed):
    js = E.plan_jobs(n_sent=n_pairs, sent_len=2)
    return js, E.job_alphas(js, n_pairs), E.job_seeds(np.random.RandomState(seed), len(js) - 1)


def _touch_ref(ts, olds):
    d = [t - o for t, o in zip(ts, olds)]
    k = sum((x != 0).any(axis=1).astype(np.float32) for x in d)
    s = np.zeros_like(d[0])
    for x in d:
        s = s + x
    return olds[0] + s / np.maximum(k, np.float32(1))[:, None]


def _align_ref(ts, olds):
    """G2V_MERGE_ALIGN restated: new = old + s / clamp(|s|^2 / sum_r |d_r|^2, 1, k)"""
    d = [t - o for t, o in zip(ts, olds)]
    k = sum((x != 0).any(axis=1).astype(np.float32) for x in d)
    s = np.zeros_like(d[0])
    for x in d:
        s = s + x
    nsq = sum((x.astype(np.float64) ** 2).sum(1) for x in d)
    tsq = (s.astype(np.float64) ** 2).sum(1)
    div = np.where(nsq > 0, np.clip(tsq / np.maximum(nsq, 1e-300), 1, np.maximum(k, 1)), 1)
    return olds[0] + s / div.astype(np.float32)[:, None]


def _run_threads(fns):
    with ThreadPoolExecutor(max_workers=len(fns)) as ex:
        futs = [ex.submit(f) for f in fns]
        return [f.result(timeout=300) for f in futs]


@pytest.mark.parametrize("n", [2, 3, 5, 8])
@pytest.mark.parametrize("rule", [N.MERGE_TOUCH, N.MERGE_MEAN, N.MERGE_ALIGN])
def test_group_merge_equals_average_local_and_restatement(n, rule):
    """one window per replica, then g2v_average over the group: every rank
    holds g2v_average_local's tables bit for bit, which are the restated rule;
    the snapshot is refreshed, so a second window merges against it"""
    tok, counts, syn0, V, D, K = _corpus()
    per = 5000
    shards = _shards(tok, [per] * n)
    sched = [_schedule(per, 100 + r) for r in range(n)]
    grp = E.LocalGroup(n)
    ga = [_engine(counts, syn0, D, K, shards[r]) for r in range(n)]
    gb = [_engine(counts, syn0, D, K, shards[r]) for r in range(n)]
    for e in gb:
        e.merge_snapshot()
    _run_threads([lambda r=r: ga[r].comm_init_local(grp, r) for r in range(n)])

    def window(e, r, w):
        js, al, sd = sched[r]
        h = len(js) // 2
        lo, hi = (0, h) if w == 0 else (h, len(js) - 1)
        e.train(js[lo:hi + 1], al[lo:hi], sd[lo:hi], N.MODE_SEQUENTIAL)

    pre = None
    for w in range(2):
        for r, e in enumerate(gb):
            window(e, r, w)
        if w == 0:
            pre = [e.get_weights() for e in gb]
        E.SGNSEngine.average_local(gb, rule)

        def rank(r, w=w):
            window(ga[r], r, w)
            ga[r].average(rule)
            return ga[r].get_weights()
        got = _run_threads([lambda r=r: rank(r) for r in range(n)])
        ref = gb[0].get_weights()
        for g in got:
            assert np.array_equal(g[0], ref[0]) and np.array_equal(g[1], ref[1])
        if w == 0:
            for tbl, init in ((0, syn0), (1, np.zeros_like(syn0))):
                if rule == N.MERGE_TOUCH:
                    exp = _touch_ref([p[tbl] for p in pre], [init] * n)
                elif rule == N.MERGE_ALIGN:
                    exp = _align_ref([p[tbl] for p in pre], [init] * n)
                else:
                    s = np.zeros_like(init)
                    for p in pre:
                        s = s + p[tbl]
                    exp = s * np.float32(1.0 / n)
                # (align: the divisor's norms are summed in another order here)
                np.testing.assert_allclose(ref[tbl], exp, rtol=1e-6 if rule != N.MERGE_ALIGN
                                           else 1e-5, atol=1e-9)
                # a row trained by one replica only keeps that replica's full update
                if rule != N.MERGE_MEAN and tbl == 1:
                    touched = [(p[1] != 0).any(axis=1) for p in pre]
                    only0 = touched[0] & ~np.any(touched[1:], axis=0)
                    if only0.any():
                        assert np.array_equal(ref[1][only0], pre[0][1][only0])
    for e in ga + gb:
        e.close()
    grp.close()


@pytest.mark.parametrize("overlap", [0, 1])
def test_group_in_call_merges_uneven_windows(overlap):
    """G2V_OPT_MERGE_EVERY_JOBS inside one g2v_train per rank, shards of
    different sizes (3, 2 and 1 windows of 2 jobs, the last ones short): the
    ranks with fewer windows join the remaining merges through g2v_average
    (ReplicaTrainer's rule) -- equal, bit for bit, to per-window training with
    g2v_average_local after every window"""
    tok, counts, syn0, V, D, K = _corpus(n_total=60_000)
    sizes = [27_000, 18_500, 6_000]  # 6, 4 and 2 jobs of <= 5,000 pairs
    n, every = len(sizes), 2
    shards = _shards(tok, sizes)
    sched = [_schedule(sizes[r], 7 + r) for r in range(n)]
    grp = E.LocalGroup(n)
    agree = Dd.ThreadAgreement(n)
    ga = [_engine(counts, syn0, D, K, shards[r]) for r in range(n)]
    for e in ga:
        e.set_option(N.OPT_SEG_JOBS, 1)  # several segments per window: the pipeline spans merges
        e.set_option(N.OPT_SAMPLE_OVERLAP, overlap)
    gb = [_engine(counts, syn0, D, K, shards[r]) for r in range(n)]
    for e in gb:
        e.merge_snapshot()
    _run_threads([lambda r=r: ga[r].comm_init_local(grp, r) for r in range(n)])
    trainers = [Dd.ReplicaTrainer(ga[r], (), every, N.MODE_SEQUENTIAL, backend="libg2v", world=n,
                                  agree=agree.for_rank(r)) for r in range(n)]
    _run_threads([lambda r=r: trainers[r].train_epoch(*sched[r]) for r in range(n)])
    wins = [(len(s[0]) - 1 + every - 1) // every for s in sched]
    assert wins == [3, 2, 1] and all(t.averages == 3 for t in trainers)
    for w in range(max(wins)):
        for r, e in enumerate(gb):
            js, al, sd = sched[r]
            j0, j1 = w * every, min(len(js) - 1, (w + 1) * every)
            if j0 < len(js) - 1:
                e.train(js[j0:j1 + 1], al[j0:j1], sd[j0:j1], N.MODE_SEQUENTIAL)
        E.SGNSEngine.average_local(gb, N.MERGE_TOUCH)
    ref = gb[0].get_weights()
    for e in ga:
        g = e.get_weights()
        assert np.array_equal(g[0], ref[0]) and np.array_equal(g[1], ref[1])
    for e in ga + gb:
        e.close()
    grp.close()


def test_group_hogwild_replicas_agree():
    """production Hogwild kernel, 4 replicas, in-call merges: after the
    epoch-final merge every replica holds the same bits and the model has
    learned (the DP CLI keeps these replicas across iterations)"""
    tok, counts, syn0, V, D, K = _corpus(V0=2000, D=64, n_total=200_000)
    n, per, every = 4, 50_000, 3
    shards = _shards(tok, [per] * n)
    sched = [_schedule(per, 40 + r) for r in range(n)]
    grp = E.LocalGroup(n)
    agree = Dd.ThreadAgreement(n)
    ga = [_engine(counts, syn0, D, K, shards[r]) for r in range(n)]
    _run_threads([lambda r=r: ga[r].comm_init_local(grp, r) for r in range(n)])
    tr = [Dd.ReplicaTrainer(ga[r], (), every, N.MODE_HOGWILD, backend="libg2v", world=n,
                            agree=agree.for_rank(r)) for r in range(n)]
    _run_threads([lambda r=r: tr[r].train_epoch(*sched[r]) for r in range(n)])
    w = [e.get_weights() for e in ga]
    for g in w[1:]:
        assert np.array_equal(g[0], w[0][0]) and np.array_equal(g[1], w[0][1])
    assert np.isfinite(w[0][0]).all() and np.abs(w[0][1]).max() > 0
    st = ga[0].read_stats()
    assert st["sgns_grid"] > 0 and st["stripe_copies"] >= 1
    for e in ga:
        e.close()
    grp.close()


def test_group_broadcast_takes_rank0_tables():
    """g2v_comm_init_local is g2v_comm_init's broadcast: replicas created with
    different tables (Python's hash() seeds each process differently) all
    hold rank 0's after joining"""
    tok, counts, syn0, V, D, K = _corpus()
    n = 3
    inits = [syn0 * np.float32(r + 1) for r in range(n)]
    grp = E.LocalGroup(n)
    es = [_engine(counts, syn0, D, K, tok[:2000], syn0_override=inits[r]) for r in range(n)]
    _run_threads([lambda r=r: es[r].comm_init_local(grp, r) for r in range(n)])
    for e in es:
        assert np.array_equal(e.get_weights()[0], inits[0])
        e.close()
    grp.close()


def test_group_failure_aborts_peers():
    """a rank whose g2v_train fails between in-call merges aborts the group:
    its peers return G2V_ECOMM from their merges instead of waiting forever"""
    tok, counts, syn0, V, D, K = _corpus()
    n = 3
    grp = E.LocalGroup(n, timeout_s=120)
    es = [_engine(counts, syn0, D, K, tok[:20_000]) for _ in range(n)]
    _run_threads([lambda r=r: es[r].comm_init_local(grp, r) for r in range(n)])
    js, al, sd = _schedule(10_000, 3)

    def rank(r):
        e = es[r]
        e.set_option(N.OPT_MERGE_EVERY_JOBS, 1)
        if r == 1:  # a job range past the corpus: rejected before any merge
            bad = js.copy()
            bad[-1] = 10**9
            with pytest.raises(N.G2VError) as x:
                e.train(bad, al, sd, N.MODE_SEQUENTIAL)
            return x.value.code
        with pytest.raises(N.G2VError) as x:
            e.train(js, al, sd, N.MODE_SEQUENTIAL)
        return x.value.code

    codes = _run_threads([lambda r=r: rank(r) for r in range(n)])
    assert codes[1] == N.G2V_EINVAL and codes[0] == codes[2] == N.G2V_ECOMM
    # the contexts stay usable without a communicator
    es[0].set_option(N.OPT_MERGE_EVERY_JOBS, 0)
    es[0].train(js, al, sd, N.MODE_SEQUENTIAL)
    for e in es:
        e.close()
    grp.close()


def test_bind_tables_over_2gib_rejected():
    """a bound table of 2 GiB or more would be addressed past the
    kernels' 32-bit buffer offsets -- rejected with G2V_ERANGE"""
    e = E.SGNSEngine(300_000, 8, 5)
    with pytest.raises(N.G2VError) as x:
        e.bind_tables(1 << 20, 1 << 20, 1792)  # 300,000 x 1,792 x 4 B = 2.15 GB; never read
    assert x.value.code == N.G2V_ERANGE
    e.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


_HOST_CHILD = r"""
import os, sys, numpy as np
sys.path.insert(0, os.environ["G2V_TEST_ROOT"])
import torch, torch.distributed as dist
from gene2vec_amd import _native as N, distributed as Dd, engine as E
from tests.test_gpu_merge_group import _corpus, _engine, _shards, _schedule
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
tok, counts, syn0, V, D, K = _corpus(n_total=60_000)
sizes = [int(x) for x in os.environ["G2V_TEST_SIZES"].split(",")]
e = _engine(counts, syn0 * np.float32(rank + 1), D, K, _shards(tok, sizes)[rank])
e.comm_init_host(Dd.host_collective(), world, rank)
t = Dd.ReplicaTrainer(e, (), 2, N.MODE_SEQUENTIAL, backend="libg2v")
t.train_epoch(*_schedule(sizes[rank], 7 + rank))
s0, s1 = e.get_weights()
np.savez(os.environ["G2V_TEST_OUT"] + f"_{rank}.npz", s0=s0, s1=s1, merges=t.averages)
dist.destroy_process_group()
"""


def test_host_transport_two_processes(tmp_path):
    """g2v_comm_init_host over gloo, 2 processes sharing the GPU, in-call
    merges with uneven windows: both ranks end bit-identical to
    g2v_average_local's per-window merges of the same replicas (rank 1 started
    from other tables: the broadcast took rank 0's)"""
    sizes = [16_000, 7_000]
    script = tmp_path / "child.py"
    script.write_text(_HOST_CHILD)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", G2V_TEST_ROOT=ROOT,
               G2V_TEST_SIZES=",".join(map(str, sizes)), G2V_TEST_OUT=str(tmp_path / "rank"),
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(script)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    got = [np.load(str(tmp_path / f"rank_{k}.npz")) for k in range(2)]
    assert int(got[0]["merges"]) == int(got[1]["merges"]) == 2
    tok, counts, syn0, V, D, K = _corpus(n_total=60_000)
    shards = _shards(tok, sizes)
    gb = [_engine(counts, syn0, D, K, shards[k]) for k in range(2)]
    for e in gb:
        e.merge_snapshot()
    sched = [_schedule(sizes[k], 7 + k) for k in range(2)]
    for w in range(2):
        for k, e in enumerate(gb):
            js, al, sd = sched[k]
            j0, j1 = 2 * w, min(len(js) - 1, 2 * w + 2)
            if j0 < len(js) - 1:
                e.train(js[j0:j1 + 1], al[j0:j1], sd[j0:j1], N.MODE_SEQUENTIAL)
        E.SGNSEngine.average_local(gb, N.MERGE_TOUCH)
    ref = gb[0].get_weights()
    for g in got:
        assert np.array_equal(g["s0"], ref[0]) and np.array_equal(g["s1"], ref[1])
    for e in gb:
        e.close()
