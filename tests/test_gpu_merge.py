"""GPU: the replica merge of the multi-GPU path inside libg2v (SURVEY.md 8(b)
g2v_comm_init / g2v_average, 8(e)).

RCCL refuses two ranks on one GPU ("Duplicate GPU detected", measured on
this pool), so a one-GPU box checks (a) the merge arithmetic through
g2v_average_local -- the same rule over replicas trained by separate
contexts -- against a numpy restatement of distributed.touch_merge_, and
(b) the RCCL path end to end with a one-rank communicator (unique id,
broadcast, grouped all-reduce, delta/apply kernels), whose merge must equal
the restated formula bit for bit.  The N > 1 all-reduce itself runs in the
driver's 8-GPU bench.
"""
import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd import engine as E
from tests.helpers import vocab_from_ids, zipf_pairs

pytestmark = pytest.mark.gpu


def _setup(n_rep, V0=800, D=100, K=5, n_pairs=30000):
    pairs = zipf_pairs(n_pairs * n_rep, V0, seed=11)
    flat = pairs.reshape(-1)
    _, remap, counts = vocab_from_ids(flat, V0)
    tok = remap[flat]
    V = len(counts)
    rng = np.random.Generator(np.random.PCG64(3))
    syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
    syn1 = np.zeros((V, D), np.float32)
    engs = []
    for r in range(n_rep):
        e = E.SGNSEngine(V, D, K)
        e.set_vocab(counts, 1e-3)
        e.set_weights(syn0, syn1)
        e.merge_snapshot()
        e.set_corpus(tok[2 * n_pairs * r:2 * n_pairs * (r + 1)], sent_len=2)
        engs.append(e)
    return engs, syn0, syn1, n_pairs


def _train(e, n, seed):
    js = E.plan_jobs(n_sent=n, sent_len=2)
    e.train(js, E.job_alphas(js, n), E.job_seeds(np.random.RandomState(seed), len(js) - 1))


def _touch_ref(ts, olds):
    """distributed.touch_merge_ restated in float32 numpy: new = old +
    sum_r(t_r - old_r) / max(k, 1), k = replicas whose row changed"""
    d = [t - o for t, o in zip(ts, olds)]
    k = sum((x != 0).any(axis=1).astype(np.float32) for x in d)
    s = d[0].copy()
    for x in d[1:]:
        s = s + x
    return olds[0] + s / np.maximum(k, np.float32(1))[:, None]


@pytest.mark.parametrize("n_rep", [2, 3])
def test_average_local_touch_matches_restatement(n_rep):
    engs, syn0, syn1, n = _setup(n_rep)
    for r, e in enumerate(engs):
        _train(e, n, seed=r + 1)
    pre = [e.get_weights() for e in engs]
    E.SGNSEngine.average_local(engs, N.MERGE_TOUCH)
    for tbl, init in ((0, syn0), (1, syn1)):
        ref = _touch_ref([p[tbl] for p in pre], [init] * n_rep)
        for e in engs:
            got = e.get_weights()[tbl]
            np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-9)
    # a second window merges against the refreshed snapshot (the first merge)
    merged1 = engs[0].get_weights()
    for r, e in enumerate(engs):
        _train(e, n, seed=10 + r)
    pre2 = [e.get_weights() for e in engs]
    E.SGNSEngine.average_local(engs, N.MERGE_TOUCH)
    ref = _touch_ref([p[1] for p in pre2], [merged1[1]] * n_rep)
    np.testing.assert_allclose(engs[-1].get_weights()[1], ref, rtol=1e-6, atol=1e-9)
    for e in engs:
        e.close()


def test_average_local_mean():
    engs, syn0, syn1, n = _setup(2)
    for r, e in enumerate(engs):
        _train(e, n, seed=r + 1)
    pre = [e.get_weights() for e in engs]
    E.SGNSEngine.average_local(engs, N.MERGE_MEAN)
    for tbl in (0, 1):
        ref = (pre[0][tbl] + pre[1][tbl]) * np.float32(0.5)
        for e in engs:
            np.testing.assert_allclose(e.get_weights()[tbl], ref, rtol=1e-6, atol=1e-9)
    for e in engs:
        e.close()


def test_average_local_requires_snapshot():
    e = E.SGNSEngine(10, 8, 5)
    e.set_weights(np.zeros((10, 8), np.float32), np.zeros((10, 8), np.float32))
    with pytest.raises(N.G2VError) as x:
        E.SGNSEngine.average_local([e, e], N.MERGE_TOUCH)
    assert x.value.code == N.G2V_ESTATE
    e.close()


@pytest.mark.parametrize("rule", [N.MERGE_TOUCH, N.MERGE_MEAN])
def test_rccl_one_rank_merge(rule):
    """g2v_comm_unique_id -> g2v_comm_init (1 rank) -> train -> g2v_average:
    the whole RCCL path on the context's stream; with one rank the merge is
    old + (t - old) / 1 (touch) or t * 1 (mean)"""
    engs, syn0, syn1, n = _setup(1)
    e = engs[0]
    uid = E.SGNSEngine.comm_unique_id()
    assert len(uid) == N.UNIQUE_ID_BYTES
    e.comm_init(uid, 1, 0)
    _train(e, n, seed=5)
    t0, t1 = e.get_weights()
    e.average(rule)
    g0, g1 = e.get_weights()
    for t, g, init in ((t0, g0, syn0), (t1, g1, syn1)):
        if rule == N.MERGE_TOUCH:
            ref = init + (t - init) / np.float32(1)
        else:
            ref = t * np.float32(1)
        assert np.array_equal(g, ref)
    # the snapshot was refreshed: a second merge without training is a no-op
    e.average(rule)
    h0, h1 = e.get_weights()
    assert np.array_equal(h0, g0) and np.array_equal(h1, g1)
    e.close()


@pytest.mark.parametrize("overlap", [0, 1])
def test_rccl_in_call_merges_equal_external(overlap):
    """G2V_OPT_MERGE_EVERY_JOBS: one g2v_train call that merges at the end of
    every window of 3 jobs (and of the shorter last window) trains and merges
    exactly what separate per-window train calls with g2v_average in between
    do -- SEQUENTIAL mode, one-rank communicator, so the results are bit for
    bit; with and without the overlapped sampler."""
    res = []
    for inner in (False, True):
        engs, syn0, syn1, n = _setup(1, n_pairs=36_000)
        e = engs[0]
        e.set_option(N.OPT_SEG_JOBS, 2)
        e.set_option(N.OPT_SAMPLE_OVERLAP, overlap)
        e.comm_init(E.SGNSEngine.comm_unique_id(), 1, 0)
        js = E.plan_jobs(n_sent=n, sent_len=2)
        al = E.job_alphas(js, n)
        sd = E.job_seeds(np.random.RandomState(3), len(js) - 1)
        nj = len(js) - 1
        assert nj % 3 != 0  # a shorter last window
        if inner:
            e.set_option(N.OPT_MERGE_RULE, N.MERGE_TOUCH)
            e.set_option(N.OPT_MERGE_EVERY_JOBS, 3)
            e.train(js, al, sd, N.MODE_SEQUENTIAL)
            e.set_option(N.OPT_MERGE_EVERY_JOBS, 0)
        else:
            for j0 in range(0, nj, 3):
                j1 = min(nj, j0 + 3)
                e.train(js[j0:j1 + 1], al[j0:j1], sd[j0:j1], N.MODE_SEQUENTIAL)
                e.average(N.MERGE_TOUCH)
        res.append(e.get_weights())
        e.close()
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])
