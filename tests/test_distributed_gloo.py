"""World-size-2 gloo tests (CPU) of the multi-GPU path: sharding, global
vocabulary, replica averaging and the averaging cadence of ReplicaTrainer.
The RCCL (nccl backend) run uses the same code with device tensors."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from gene2vec_amd import distributed as Dd
from gene2vec_amd import engine as E
from gene2vec_amd import synthetic as S


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FakeEngine:
    """stands in for SGNSEngine: every job adds (rank+1) * job_index to the tables"""

    def __init__(self, tables, rank):
        self.tables, self.rank, self.calls = tables, rank, []

    def train(self, js, al, sd, mode, timing=False, compute_loss=False):
        self.calls.append((int(js[0]), int(js[-1]), len(al), len(sd)))
        for t in self.tables:
            t += float((self.rank + 1) * len(al))


class FailingEngine:
    """libg2v-backend stand-in: train raises on one rank, average / abort recorded"""

    def __init__(self, fail):
        self.fail, self.aborted, self.opts, self.averages = fail, False, {}, 0

    def set_option(self, k, v):
        self.opts[k] = v

    def train(self, js, al, sd, mode, timing=False, compute_loss=False):
        if self.fail:
            raise RuntimeError("boom")

    def average(self, rule):
        self.averages += 1

    def comm_abort(self):
        self.aborted = True


class HostMergingEngine:
    """libg2v over the host transport, as ReplicaTrainer sees it: train() runs
    one merge collective (Dd.HostCollective, flagged) at the end of every
    window of OPT_MERGE_EVERY_JOBS jobs, as g2v_train's in-call merges do, and
    fails before merge `fail_before` (1-based) like G2V_OPT_DEBUG_FAIL_MERGE"""

    def __init__(self, fail_before=0, V=5, ld=4):
        from gene2vec_amd import _native as N
        self.N, self.V, self.ld, self.fail_before = N, V, ld, fail_before
        self.opts, self.aborted = {}, False
        self.host_collective = Dd.HostCollective()

    def set_option(self, k, v):
        self.opts[k] = v

    def _merge(self):
        buf = np.ones(Dd.merge_floats(self, "touch"), np.float32)
        self.host_collective(self.N.COLL_SUM, buf)

    def train(self, js, al, sd, mode, timing=False, compute_loss=False):
        every = self.opts[self.N.OPT_MERGE_EVERY_JOBS]
        for w in range((len(al) + every - 1) // every):
            if w + 1 == self.fail_before:
                raise RuntimeError("injected failure before in-call merge")
            self._merge()

    def average(self, rule):
        self._merge()

    def comm_abort(self):
        self.aborted = True


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        # sharding of one synthetic corpus
        n = 10001
        s0, s1 = Dd.shard_range(n, rank, world)
        pairs = S.zipf_gene_pairs(n, 500, seed=3)[s0:s1]
        flat = pairs.reshape(-1)
        c, f = E.count_ids(flat, 500)
        gc, gf = Dd.global_vocab(c, f, token_offset=2 * s0)
        out["counts"], out["first"] = gc, gf
        # averaging
        t = torch.full((4, 3), float(rank + 1))
        Dd.average_([t])
        out["avg"] = t.numpy()
        # cadence: 10 jobs, average every 4 -> windows of 4, 4, 2
        tabs = [torch.zeros(2, 2), torch.zeros(3)]
        eng = FakeEngine(tabs, rank)
        tr = Dd.ReplicaTrainer(eng, tabs, avg_every_jobs=4, merge="mean")
        js = np.arange(0, 21, 2, dtype=np.int64)
        tr.train_epoch(js, np.zeros(10), np.zeros(10, np.uint64))
        out["calls"] = eng.calls
        out["tables"] = [x.numpy() for x in tabs]
        out["averages"] = tr.averages
        # row-wise touch merge: rank 0 changes rows {0, 1}, rank 1 rows {1, 2}
        t = torch.zeros(4, 3)
        olds = [t.clone()]
        rows = [0, 1] if rank == 0 else [1, 2]
        t[rows] += float(rank + 1)
        Dd.touch_merge_([t], olds)
        out["touch"] = t.numpy()
        out["touch_old"] = olds[0].numpy()
        # align rule: row 0 both ranks move alike (agree: their mean), row 1
        # orthogonally (independent: their sum), row 2 rank 1 only
        t = torch.zeros(3, 2)
        olds = [t.clone()]
        t[0] = torch.tensor([1.0, 1.0])
        t[1] = torch.tensor([1.0, 0.0]) if rank == 0 else torch.tensor([0.0, 2.0])
        if rank == 1:
            t[2] = torch.tensor([3.0, 0.0])
        Dd.touch_merge_([t], olds, align=True)
        out["align"] = t.numpy()
        # both tables in one [2][V][ld] buffer (bench.py's layout): same result
        # as merging each table on its own
        g = torch.Generator().manual_seed(rank)
        both = torch.zeros(2, 5, 3)
        olds2 = [both.clone()]
        sep = [both[0].clone(), both[1].clone()]
        sep_old = [x.clone() for x in sep]
        upd = (torch.rand(2, 5, 3, generator=g) > 0.6).float() * (rank + 1)
        both += upd
        sep[0] += upd[0]
        sep[1] += upd[1]
        Dd.touch_merge_([both], olds2)
        Dd.touch_merge_(sep, sep_old)
        out["fused"] = both.numpy()
        out["separate"] = np.stack([x.numpy() for x in sep])
        # shards whose job counts differ (rank 0: 10 jobs, rank 1: 6, merges every
        # 4): both ranks must run max(3, 2) = 3 merge windows, or rank 0 would
        # wait forever in its third all-reduce
        tabs2 = [torch.zeros(3)]
        eng2 = FakeEngine(tabs2, rank)
        tr2 = Dd.ReplicaTrainer(eng2, tabs2, avg_every_jobs=4, merge="mean")
        nj = 10 if rank == 0 else 6
        tr2.train_epoch(np.arange(0, 2 * nj + 1, 2, dtype=np.int64), np.zeros(nj),
                        np.zeros(nj, np.uint64))
        out["uneven_calls"] = eng2.calls
        out["uneven_averages"] = tr2.averages
        out["uneven_tables"] = tabs2[0].numpy()
        # g2v_comm_init_host's collective over gloo: rank-order sum, broadcast
        from gene2vec_amd import _native as N
        coll = Dd.host_collective()
        a = np.array([0.1, 1e8, -3.0, 7.0], np.float32) * np.float32(rank + 1)
        coll(N.COLL_SUM, a)
        out["coll_sum"] = a
        b = np.full(3, 10.0 * (rank + 1), np.float32)
        coll(N.COLL_BCAST0, b)
        out["coll_bcast"] = b
        # libg2v backend: a rank whose epoch fails re-raises its error, its peer
        # learns of it from the ok-flag agreement and leaves the communicator
        fe = FailingEngine(fail=(rank == 1))
        tr3 = Dd.ReplicaTrainer(fe, (), avg_every_jobs=4, backend="libg2v")
        try:
            tr3.train_epoch(np.arange(0, 21, 2, dtype=np.int64), np.zeros(10),
                            np.zeros(10, np.uint64))
            out["fail"] = None
        except RuntimeError as e:
            out["fail"] = str(e)
        out["aborted"] = fe.aborted
        out["merge_every_reset"] = fe.opts.get(N.OPT_MERGE_EVERY_JOBS)
        # host transport: rank 1 fails between its in-call merges while rank 0
        # waits inside merge 2's gather; rank 1 joins that gather with its ok
        # flag cleared, rank 0 fails out of it, and both agree (no mismatched
        # gloo collectives, no hang: the agreements below still line up)
        he = HostMergingEngine(fail_before=2 if rank == 1 else 0)
        tr4 = Dd.ReplicaTrainer(he, (), avg_every_jobs=4, backend="libg2v")
        try:
            tr4.train_epoch(np.arange(0, 21, 2, dtype=np.int64), np.zeros(10),
                            np.zeros(10, np.uint64))
            out["host_fail"] = None
        except Exception as e:
            out["host_fail"] = f"{type(e).__name__}: {e}"
        out["host_sums"] = he.host_collective.sums
        out["max_int"] = Dd.allreduce_max_int(5 + rank)
        out["sum_float"] = Dd.allreduce_sum_float(0.5 * (rank + 1))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def results():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_shard_range_partitions():
    for n in (0, 1, 7, 10001):
        for w in (1, 2, 3, 8):
            r = [Dd.shard_range(n, k, w) for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))


def test_global_vocab_equals_single_process(results):
    pairs = S.zipf_gene_pairs(10001, 500, seed=3)
    c, f = E.count_ids(pairs.reshape(-1), 500)
    for r in (0, 1):
        assert np.array_equal(results[r]["counts"], c)
        assert np.array_equal(results[r]["first"], f)


def test_average_is_mean(results):
    for r in (0, 1):
        assert np.allclose(results[r]["avg"], 1.5)


def test_replica_trainer_cadence_and_consistency(results):
    for r in (0, 1):
        assert results[r]["calls"] == [(0, 8, 4, 4), (8, 16, 4, 4), (16, 20, 2, 2)]
        assert results[r]["averages"] == 3
    # window adds (rank+1)*jobs, then the mean over ranks: 1.5*4 + 1.5*4 + 1.5*2
    for t0, t1 in zip(results[0]["tables"], results[1]["tables"]):
        assert np.array_equal(t0, t1)
        assert np.allclose(t0, 15.0)


def test_touch_merge_rowwise(results):
    for r in (0, 1):
        t = results[r]["touch"]
        assert np.allclose(t[0], 1.0)        # only rank 0: full update kept
        assert np.allclose(t[1], 1.5)        # both ranks: mean of (1, 2)
        assert np.allclose(t[2], 2.0)        # only rank 1
        assert np.allclose(t[3], 0.0)        # untouched
        assert np.array_equal(results[r]["touch_old"], t)


def test_align_merge_rowwise(results):
    for r in (0, 1):
        a = results[r]["align"]
        assert np.allclose(a[0], [1.0, 1.0])   # agreeing changes: their mean
        assert np.allclose(a[1], [1.0, 2.0])   # orthogonal changes: their sum
        assert np.allclose(a[2], [3.0, 0.0])   # one replica: its change


def test_touch_merge_fused_buffer_equals_per_table(results):
    for r in (0, 1):
        assert np.array_equal(results[r]["fused"], results[r]["separate"])
    assert np.array_equal(results[0]["fused"], results[1]["fused"])


def test_uneven_shards_same_merge_count(results):
    assert results[0]["uneven_calls"] == [(0, 8, 4, 4), (8, 16, 4, 4), (16, 20, 2, 2)]
    assert results[1]["uneven_calls"] == [(0, 8, 4, 4), (8, 12, 2, 2)]
    assert results[0]["uneven_averages"] == results[1]["uneven_averages"] == 3
    # window adds: rank 0 4, 4, 2; rank 1 8, 4, 0 -> means 6, 4, 1 -> 11
    assert np.array_equal(results[0]["uneven_tables"], results[1]["uneven_tables"])
    assert np.allclose(results[0]["uneven_tables"], 11.0)


def test_host_collective_rank_order_sum_and_broadcast(results):
    a = np.array([0.1, 1e8, -3.0, 7.0], np.float32)
    expect = np.zeros(4, np.float32) + a + a * np.float32(2)
    for r in (0, 1):
        assert np.array_equal(results[r]["coll_sum"], expect)
        assert np.array_equal(results[r]["coll_bcast"], np.full(3, 10.0, np.float32))


def test_libg2v_backend_failure_reaches_every_rank(results):
    assert results[1]["fail"] == "boom" and not results[1]["aborted"]
    assert "another rank" in results[0]["fail"] and results[0]["aborted"]
    for r in (0, 1):
        assert results[r]["merge_every_reset"] == 0


def test_host_transport_failure_between_merges(results):
    """the failing rank joins its peer's pending merge with
    the ok flag cleared; the peer raises PeerFailed, the failing rank its own
    error, and the later scalar agreement (max_int) still matches up"""
    assert results[1]["host_fail"] == "RuntimeError: injected failure before in-call merge"
    assert results[0]["host_fail"].startswith("PeerFailed: rank(s) [1] failed")
    assert results[0]["host_sums"] == 1 and results[1]["host_sums"] == 1
    assert results[0]["max_int"] == results[1]["max_int"] == 6


def test_thread_agreement_min():
    import threading
    ag = Dd.ThreadAgreement(3)
    got = [None] * 3

    def run(r):
        f = ag.for_rank(r)
        got[r] = (f(5 - r), f(10 + r))
    th = [threading.Thread(target=run, args=(r,)) for r in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    assert got == [(3, 10)] * 3


def test_scalar_agreements(results):
    for r in (0, 1):
        assert results[r]["max_int"] == 6
        assert results[r]["sum_float"] == 1.5


def test_single_process_trainer_never_merges():
    """world 1 (no process group): the windows train, no merge runs (the N = 1
    bench carries no merge work)"""
    import torch
    t = [torch.zeros(2)]
    eng = FakeEngine(t, 0)
    tr = Dd.ReplicaTrainer(eng, t, avg_every_jobs=3, merge="touch")
    tr.train_epoch(np.arange(0, 15, 2, dtype=np.int64), np.zeros(7), np.zeros(7, np.uint64))
    assert tr.averages == 0 and len(eng.calls) == 3


def _gather_worker(rank, world, port, paths, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = Dd.gather_corpus(paths)
        q.put((rank, None if c is None else (c.tokens.copy(), list(c.words), c.counts.copy(),
                                             c.n_sent, c.pairs_only)))
    finally:
        dist.destroy_process_group()


def _run_gather(paths, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, paths, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _write_pairs(d, k, pairs, names):
    p = d / f"pairs_{k}.txt"
    p.write_text("\n".join(f"{names[a]} {names[b]}" for a, b in pairs) + "\n",
                 encoding="windows-1252")
    return str(p)


@pytest.mark.parametrize("world,n_files", [(2, 3), (3, 2)])
def test_gather_corpus_equals_single_reader(tmp_path, world, n_files):
    """rank-sharded ingest (each rank tokenises its file range, the ranks share
    words and tokens) builds the single-process reader's corpus on every rank;
    with more ranks than files a rank reads nothing and still takes part"""
    from gene2vec_amd import ingest
    names = S.gene_names(300)
    pairs = S.zipf_gene_pairs(3000, 300, 1.0, seed=5)
    paths = [_write_pairs(tmp_path, k, part, names)
             for k, part in enumerate(np.array_split(pairs, n_files))]
    ref = ingest.read_corpus(paths)
    res = _run_gather(paths, world)
    for r in range(world):
        tok, words, counts, n_sent, pairs_only = res[r]
        assert words == list(ref.words)
        assert np.array_equal(counts, ref.counts)
        assert np.array_equal(tok, ref.tokens)
        assert n_sent == ref.n_sent and pairs_only


def test_gather_corpus_declines_non_pairs(tmp_path):
    names = S.gene_names(50)
    pairs = S.zipf_gene_pairs(200, 50, 1.0, seed=6)
    p0 = _write_pairs(tmp_path, 0, pairs, names)
    p1 = tmp_path / "pairs_1.txt"
    p1.write_text("G00001 G00002 G00003\n", encoding="windows-1252")
    res = _run_gather([p0, str(p1)], 2)
    assert res[0] is None and res[1] is None


class _OptEngine:
    """records set_option / comm_init_host calls (libg2v-backend stand-in)"""

    def __init__(self):
        self.opts, self.host = {}, None

    def set_option(self, k, v):
        self.opts[k] = v

    def comm_init_host(self, hc, world, rank):
        self.host = (world, rank)


def _bind_worker(rank, world, port, betas, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from types import SimpleNamespace

    from gene2vec_amd import _native as N
    from gene2vec_amd import word2vec as W
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        for beta in betas:
            me = SimpleNamespace(mode="hogwild", merge_beta=beta, merge_every_jobs=100,
                                 merge_rule="touch")
            eng = _OptEngine()
            W.Word2Vec._bind_replica(me, eng)
            out.append((eng.opts.get(N.OPT_MERGE_BETA_MILLI), eng.host,
                        me._replica.avg_every_jobs, me._replica.merge))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_bind_replica_sets_the_plans_merge_beta():
    """the CLI's damped divisor (distributed.dp_merge_beta)
    reaches libg2v: Word2Vec._bind_replica sets G2V_OPT_MERGE_BETA_MILLI on
    every rank's engine when the plan damps (beta != 1), and leaves the
    library default otherwise; world size 2 over gloo (the host transport)"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bind_worker, args=(r, 2, port, (1.7, 1.0), q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        damped, plain = res[rank]
        assert damped == (1700, (2, rank), 100, "touch")
        assert plain == (None, (2, rank), 100, "touch")
