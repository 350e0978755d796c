"""GPU parity: libg2v.so on the MI355X against the CPU oracle and the golden
fixtures.  All calls go through the C ABI (gene2vec_amd.engine -> ctypes).

Bars (north star): vocabulary/sampling tables and the sampled
(center, input, negatives) stream bit-exact; a synchronous or sequential
SGNS step within 1e-5 relative of the NumPy/C restatement; Hogwild training
judged by its SGNS objective against the oracle's.
"""
import json
import os

import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd import engine as E
from oracle import c_oracle as CO
from oracle import sgns_oracle as O
from tests.conftest import GOLDEN
from tests.helpers import crc_hash, vocab_from_ids, zipf_pairs

pytestmark = pytest.mark.gpu

RTOL = 1e-5  # north star: "within 1e-5 relative"


def _close(a, b, rtol=RTOL, atol=1e-7):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


def _corpus_from_pairs(pairs, V):
    flat = pairs.reshape(-1)
    order, remap, counts = vocab_from_ids(flat, V)
    tok = remap[flat]
    return tok, counts


def _engine(V, D, K, counts, sample, syn0=None, syn1=None):
    eng = E.SGNSEngine(V, D, K)
    eng.set_vocab(counts, sample)
    if syn0 is None:
        rng = np.random.Generator(np.random.PCG64(11))
        syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
        syn1 = np.zeros((V, D), np.float32)
    eng.set_weights(syn0, syn1)
    return eng, syn0, syn1


# ---------------------------------------------------------------------------
# vocabulary tables (bit-exact)
# ---------------------------------------------------------------------------
def test_vocab_tables_bit_exact(golden):
    g = golden["test_pairs"]
    counts = np.array(g["counts"], np.int64)
    eng = E.SGNSEngine(len(counts), 16, 5)
    cum, si = eng.set_vocab(counts, 1e-3, return_tables=True)
    assert cum.tolist() == g["cum_table"]
    assert si.tolist() == [min(x, 2 ** 32 - 1) for x in g["sample_int"]]
    for V in (1000, 24447, 60000):
        z = np.load(os.path.join(GOLDEN, f"zipf{V}_tables.npz"))
        eng = E.SGNSEngine(V, 16, 5)
        cum, si = eng.set_vocab(z["counts"], 1e-3, return_tables=True)
        assert np.array_equal(cum, z["cum"]), f"cum_table mismatch V={V}"
        assert np.array_equal(si, np.minimum(z["sample_int"], 2 ** 32 - 1).astype(np.uint32))
        eng.close()


# ---------------------------------------------------------------------------
# sampled example stream (bit-exact vs the C oracle)
# ---------------------------------------------------------------------------
def _sampler_case(tok, off, counts, sample, K, seed_rs=1):
    V = len(counts)
    eng = E.SGNSEngine(V, 8, K)
    eng.set_vocab(counts, sample)
    eng.set_corpus(tok, sent_off=off)
    js = E.plan_jobs(sent_off=off)
    seeds = E.job_seeds(np.random.RandomState(seed_rs), len(js) - 1)
    got = eng.debug_sample(js, seeds)
    cum = CO.make_cum_table(counts)
    si = CO.sample_int(counts, sample)
    ref = CO.sample_records(tok, off, js, seeds, si, sample != 0, cum, K)
    eng.close()
    return got, ref


@pytest.mark.parametrize("sample", [0.0, 1e-3])
def test_sampler_reference_corpus(test_pairs, sample):
    voc = O.build_vocab(test_pairs, 1, sample)
    ids = O.sentences_to_ids(test_pairs, voc.word2index)
    tok = np.array([w for s in ids for w in s], np.int32)
    off = np.cumsum([0] + [len(s) for s in ids]).astype(np.int64)
    got, ref = _sampler_case(tok, off, voc.counts, sample, 5)
    assert got.shape == ref.shape and np.array_equal(got, ref)
    # and the numpy restatement agrees on the single job
    seeds = E.job_seeds(np.random.RandomState(1), 1)
    ref2 = O.sample_job_records(ids, int(seeds[0]), voc.sample_int, sample != 0,
                                O.make_cum_table(voc.counts), 5)
    assert got.tolist() == [[c, j] + n for c, j, n in ref2]


@pytest.mark.parametrize("K", [5, 15, 7, 20])
@pytest.mark.parametrize("sample", [0.0, 1e-3, 1e-5])
def test_sampler_zipf_pairs(K, sample):
    pairs = zipf_pairs(60000, 3000, seed=5)
    tok, counts = _corpus_from_pairs(pairs, 3000)
    off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)
    got, ref = _sampler_case(tok, off, counts, sample, K)
    assert len(ref) > 1000 and np.array_equal(got, ref)


def test_sampler_ragged_oov_empty():
    """irregular sentences (0..9 tokens, the 4-token boundary lines of
    generate_gene_pairs.py:208-209), OOV tokens (-1) and empty lines"""
    rng = np.random.RandomState(2)
    V = 500
    lengths = rng.choice([0, 1, 2, 2, 2, 3, 4, 9], size=20000)
    lengths[:3] = [0, 0, 9999]      # near-maximal sentence in the first job
    tok = rng.randint(-1, V, size=int(lengths.sum())).astype(np.int32)
    counts = np.bincount(tok[tok >= 0], minlength=V).astype(np.int64)
    counts[counts == 0] = 1
    counts = np.sort(counts)[::-1].copy()
    off = np.cumsum(np.concatenate([[0], lengths])).astype(np.int64)
    for sample in (0.0, 1e-3):
        got, ref = _sampler_case(tok, off, counts, sample, 5, seed_rs=9)
        assert np.array_equal(got, ref)


# ---------------------------------------------------------------------------
# explicit-negative steps (1e-5 relative)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["step_V60_D200_K5", "step_V40_D512_K15"])
def test_step_sequential_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    V, D = z["syn0"].shape
    K = z["negs"].shape[1]
    eng = E.SGNSEngine(V, D, K)
    eng.set_weights(z["syn0"], z["syn1neg"])
    eng.step_explicit(z["center"], z["input"], z["negs"], float(z["alpha"]), N.MODE_SEQUENTIAL)
    s0, s1 = eng.get_weights()
    _close(s0, z["syn0_out"])
    _close(s1, z["syn1neg_out"])


@pytest.mark.parametrize("D,K", [(200, 5), (512, 15), (100, 5), (50, 3), (7, 1), (256, 20),
                                 (300, 10), (64, 2), (200, 4), (128, 7), (333, 12), (512, 19),
                                 (1, 5), (2, 1), (65, 3)])
def test_step_sequential_vs_c_oracle(D, K):
    rng = np.random.Generator(np.random.PCG64(D * 100 + K))
    V, B = 37, 500  # small V: many repeated rows and repeated negatives
    syn0 = ((rng.random((V, D)) - 0.5) / D * 80).astype(np.float32)
    syn1 = ((rng.random((V, D)) - 0.5) / D * 80).astype(np.float32)
    center = rng.integers(0, V, B).astype(np.int32)
    inp = rng.integers(0, V, B).astype(np.int32)
    negs = rng.integers(-1, V, (B, K)).astype(np.int32)
    negs[:5] = center[:5, None]  # negative == center is skipped
    eng = E.SGNSEngine(V, D, K)
    eng.set_weights(syn0, syn1)
    eng.step_explicit(center, inp, negs, 0.05, N.MODE_SEQUENTIAL)
    g0, g1 = eng.get_weights()
    a0, a1 = syn0.copy(), syn1.copy()
    CO.sgns_step_sequential(a0, a1, np.ones(V, np.float32), center, inp, negs, 0.05)
    _close(g0, a0, atol=1e-6)
    _close(g1, a1, atol=1e-6)


@pytest.mark.parametrize("D,K", [(200, 5), (512, 15), (7, 1), (64, 2), (100, 3), (300, 10),
                                 (256, 20), (508, 5), (200, 4), (150, 8), (260, 13), (512, 18),
                                 (1, 2), (65, 6)])
def test_step_hogwild_disjoint_equals_sequential(D, K):
    """examples touching disjoint rows: every update order gives the same
    result -- the production atomic kernel for every compiled negative count,
    ragged and wide dimensions"""
    B = 64
    V = B * (K + 2)
    rng = np.random.Generator(np.random.PCG64(3))
    syn0 = ((rng.random((V, D)) - 0.5) / D * 40).astype(np.float32)
    syn1 = ((rng.random((V, D)) - 0.5) / D * 40).astype(np.float32)
    perm = rng.permutation(V).astype(np.int32).reshape(B, K + 2)
    center, inp, negs = perm[:, 0], perm[:, 1], perm[:, 2:]
    eng = E.SGNSEngine(V, D, K)
    eng.set_weights(syn0, syn1)
    eng.step_explicit(center, inp, negs, 0.025, N.MODE_HOGWILD)
    g0, g1 = eng.get_weights()
    a0, a1 = syn0.copy(), syn1.copy()
    CO.sgns_step_sequential(a0, a1, np.ones(V, np.float32), center, inp, negs, 0.025)
    _close(g0, a0)
    _close(g1, a1)


def test_step_minibatch_vs_numpy():
    D, K, V, B = 200, 5, 50, 300
    rng = np.random.Generator(np.random.PCG64(4))
    syn0 = ((rng.random((V, D)) - 0.5) / D * 40).astype(np.float32)
    syn1 = ((rng.random((V, D)) - 0.5) / D * 40).astype(np.float32)
    center = rng.integers(0, V, B).astype(np.int32)
    inp = rng.integers(0, V, B).astype(np.int32)
    negs = rng.integers(-1, V, (B, K)).astype(np.int32)
    eng = E.SGNSEngine(V, D, K)
    eng.set_weights(syn0, syn1)
    eng.step_explicit(center, inp, negs, 0.025, N.MODE_MINIBATCH)
    g0, g1 = eng.get_weights()
    a0, a1 = syn0.copy(), syn1.copy()
    O.sgns_step_minibatch(a0, a1, np.ones(V, np.float32), center, inp, negs, 0.025)
    _close(g0, a0, atol=1e-6)
    _close(g1, a1, atol=1e-6)


# ---------------------------------------------------------------------------
# full training
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("tag,sample", [("s0", 0.0), ("s1e-3", 1e-3)])
def test_train_sequential_reference_corpus_golden(test_pairs, tag, sample):
    z = np.load(os.path.join(GOLDEN, f"e2e_test_pairs_{tag}.npz"))
    voc = O.build_vocab(test_pairs, 1, sample)
    ids = O.sentences_to_ids(test_pairs, voc.word2index)
    tok = np.array([w for s in ids for w in s], np.int32)
    off = np.cumsum([0] + [len(s) for s in ids]).astype(np.int64)
    V, D = len(voc.index2word), 200
    eng = E.SGNSEngine(V, D, 5)
    eng.set_vocab(voc.counts, sample)
    eng.set_weights(z["syn0_init"], np.zeros((V, D), np.float32))
    eng.set_corpus(tok, sent_off=off)
    js = E.plan_jobs(sent_off=off)
    rs = np.random.RandomState(1)
    stats = []
    for _ in range(3):
        eng.train(js, E.job_alphas(js, len(ids)), E.job_seeds(rs, len(js) - 1),
                  N.MODE_SEQUENTIAL)
        stats.append(eng.read_stats())
    s0, s1 = eng.get_weights()
    _close(s0, z["syn0"])
    _close(s1, z["syn1neg"])
    gst = json.loads(str(z["stats"]))
    for a, b in zip(stats, gst):
        assert (a["effective_words"], a["examples"], a["raw_words"]) == (
            b["effective_words"], b["examples"], b["raw_words"])


def _zipf_setup(n_pairs, V, D, K, sample, seed=20250114):
    pairs = zipf_pairs(n_pairs, V, seed=seed)
    tok, counts = _corpus_from_pairs(pairs, V)
    V = len(counts)
    rng = np.random.Generator(np.random.PCG64(1))
    syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
    return tok, counts, syn0


@pytest.mark.parametrize("seg_jobs", [0, 3, 1])
def test_train_sequential_vs_c_oracle_zipf(seg_jobs):
    """seg_jobs > 0 splits the 8 jobs into several sample -> update segments
    (sampler state, LCG streams and alpha carried across segment boundaries)"""
    D, K, sample = 200, 5, 1e-3
    tok, counts, syn0 = _zipf_setup(40000, 2000, D, K, sample)
    V = len(counts)
    off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)
    js = E.plan_jobs(n_sent=len(tok) // 2, sent_len=2)
    al = E.job_alphas(js, len(tok) // 2)
    sd = E.job_seeds(np.random.RandomState(1), len(js) - 1)
    eng = E.SGNSEngine(V, D, K)
    if seg_jobs:
        eng.set_option(N.OPT_SEG_JOBS, seg_jobs)
    eng.set_vocab(counts, sample)
    eng.set_weights(syn0, np.zeros((V, D), np.float32))
    eng.set_corpus(tok, sent_len=2)
    eng.train(js, al, sd, N.MODE_SEQUENTIAL)
    st = eng.read_stats()
    g0, g1 = eng.get_weights()
    a0, a1 = syn0.copy(), np.zeros((V, D), np.float32)
    ref = CO.train(tok, off, js, al.astype(np.float32), sd, CO.sample_int(counts, sample), True,
                   CO.make_cum_table(counts), a0, a1, np.ones(V, np.float32), K)
    assert (st["effective_words"], st["examples"]) == (ref["effective_words"], ref["examples"])
    _close(g0, a0, atol=1e-6)
    _close(g1, a1, atol=1e-6)


@pytest.mark.parametrize("V", [1, 2, 3])
@pytest.mark.parametrize("mode", ["sequential", "hogwild"])
def test_train_tiny_vocabulary(V, mode):
    """degenerate vocabularies: one gene (every negative equals the center and
    is skipped), two and three genes; sequential vs the C oracle at 1e-5,
    Hogwild: identical counts and the pair objective within 1 % of the
    sequential oracle's"""
    D, K, sample = 16, 5, 1e-3
    rng = np.random.RandomState(V)
    n = 3000
    pairs = rng.randint(0, V, (n, 2)).astype(np.int32)
    tok = pairs.reshape(-1)
    counts = np.bincount(tok, minlength=V).astype(np.int64)
    order = np.argsort(-counts, kind="stable")
    remap = np.empty(V, np.int32)
    remap[order] = np.arange(V, dtype=np.int32)
    tok = remap[tok]
    counts = counts[order]
    syn0 = ((np.random.Generator(np.random.PCG64(2)).random((V, D)) - 0.5) / D).astype(np.float32)
    off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    al = E.job_alphas(js, n)
    sd = E.job_seeds(np.random.RandomState(1), len(js) - 1)
    eng = E.SGNSEngine(V, D, K)
    eng.set_vocab(counts, sample)
    eng.set_weights(syn0, np.zeros((V, D), np.float32))
    eng.set_corpus(tok, sent_len=2)
    eng.train(js, al, sd, N.MODE_SEQUENTIAL if mode == "sequential" else N.MODE_HOGWILD)
    st = eng.read_stats()
    g0, g1 = eng.get_weights()
    a0, a1 = syn0.copy(), np.zeros((V, D), np.float32)
    ref = CO.train(tok, off, js, al.astype(np.float32), sd, CO.sample_int(counts, sample), True,
                   CO.make_cum_table(counts), a0, a1, np.ones(V, np.float32), K)
    assert (st["effective_words"], st["examples"]) == (ref["effective_words"], ref["examples"])
    assert np.isfinite(g0).all() and np.isfinite(g1).all()
    if mode == "sequential":
        _close(g0, a0, atol=1e-6)
        _close(g1, a1, atol=1e-6)
    else:
        # Hogwild on 1-3 rows: every example in flight shares the rows; the
        # staleness-bounded grid keeps the learned objective at the sequential
        # oracle's (the same corpus pairs, gensim's negatives skipped when they
        # equal the centre)
        got = _pair_objective(g0, g1, tok, counts, K)
        exp = _pair_objective(a0, a1, tok, counts, K)
        init = _pair_objective(syn0, np.zeros((V, D), np.float32), tok, counts, K)
        print("tiny vocabulary V=%d: init %.5f hogwild %.5f sequential %.5f" % (V, init, got, exp))
        assert exp < init
        assert abs(got - exp) / exp < 0.01, (got, exp)


def _pair_objective(syn0, syn1, tok, counts, K, seed=3):
    """SGNS objective over every directed pair of the corpus: -log s(u.v_c) -
    sum over K unigram^0.75 negatives (skipped when equal to the centre) of
    log s(-u.v_n), in double"""
    rng = np.random.RandomState(seed)
    c, j = tok[0::2], tok[1::2]
    c, j = np.concatenate([c, j]), np.concatenate([j, c])
    p = counts.astype(np.float64) ** 0.75
    negs = rng.choice(len(counts), size=(len(c), K), p=p / p.sum())
    u = syn0[j].astype(np.float64)
    pos = np.einsum("nd,nd->n", u, syn1[c].astype(np.float64))
    neg = np.einsum("nd,nkd->nk", u, syn1[negs].astype(np.float64))
    keep = negs != c[:, None]
    return float((np.logaddexp(0, -pos) + (np.logaddexp(0, neg) * keep).sum(1)).mean())


def _eval_loss(syn0, syn1, tok, counts, K, n_eval=20000, seed=99):
    rng = np.random.Generator(np.random.PCG64(seed))
    n = len(tok) // 2
    idx = rng.integers(0, n, n_eval)
    c, j = tok[2 * idx], tok[2 * idx + 1]
    p = counts.astype(np.float64) ** 0.75
    negs = rng.choice(len(counts), size=(n_eval, K), p=p / p.sum())
    return O.sgns_loss(syn0, syn1, c, j, negs)


@pytest.mark.parametrize("D,K,seg_jobs,overlap",
                         [(200, 5, 0, 1), (512, 15, 0, 1), (200, 5, 7, 1), (200, 5, 0, 0)])
def test_train_hogwild_objective_matches_oracle(D, K, seg_jobs, overlap):
    """Hogwild GPU vs the sequential oracle on the same jobs/seeds: the SGNS
    objective on held-in pairs must agree within 0.5 % (Hogwild reorders
    updates; it is judged end-to-end).  Measured at the
    default grid over 5 seed streams: -0.06..+0.11 %, mean +0.05 %; the
    sequential oracle's own seed-to-seed spread is 0.5 %
    (profiles/r02/r02_pipeline/hogwild_dev_*.log).  overlap = G2V_OPT_ATOMIC_OVERLAP."""
    sample = 1e-3
    tok, counts, syn0 = _zipf_setup(200000, 3000, D, K, sample)
    V = len(counts)
    off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)
    js = E.plan_jobs(n_sent=len(tok) // 2, sent_len=2)
    eng = E.SGNSEngine(V, D, K)
    if seg_jobs:
        eng.set_option(N.OPT_SEG_JOBS, seg_jobs)  # pipelined sampler/SGNS segments
    eng.set_option(N.OPT_ATOMIC_OVERLAP, overlap)
    eng.set_vocab(counts, sample)
    eng.set_weights(syn0, np.zeros((V, D), np.float32))
    eng.set_corpus(tok, sent_len=2)
    a0, a1 = syn0.copy(), np.zeros((V, D), np.float32)
    rs_g, rs_c = np.random.RandomState(1), np.random.RandomState(1)
    for it in range(3):
        al = E.job_alphas(js, len(tok) // 2)
        eng.train(js, al, E.job_seeds(rs_g, len(js) - 1), N.MODE_HOGWILD)
        CO.train(tok, off, js, al.astype(np.float32), E.job_seeds(rs_c, len(js) - 1),
                 CO.sample_int(counts, sample), True, CO.make_cum_table(counts), a0, a1,
                 np.ones(V, np.float32), K)
    g0, g1 = eng.get_weights()
    assert np.isfinite(g0).all() and np.isfinite(g1).all()
    l_gpu = _eval_loss(g0, g1, tok, counts, K)
    l_ref = _eval_loss(a0, a1, tok, counts, K)
    l_init = _eval_loss(syn0, np.zeros_like(a1), tok, counts, K)
    assert l_ref < l_init * 0.95
    assert abs(l_gpu - l_ref) / l_ref < 0.005, (l_gpu, l_ref, l_init)


def test_train_counts_at_scale_bit_exact():
    """10 M pairs: effective words and example counts of the device sampler
    equal the C oracle's (downsampling is bit-exact at any size)."""
    V, n = 24447, 10_000_000
    pairs = zipf_pairs(n, V, seed=20250114)
    tok, counts = _corpus_from_pairs(pairs, V)
    V = len(counts)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    sd = E.job_seeds(np.random.RandomState(1), len(js) - 1)
    eng = E.SGNSEngine(V, 200, 5)
    eng.set_vocab(counts, 1e-3)
    eng.set_weights(np.zeros((V, 200), np.float32), np.zeros((V, 200), np.float32))
    eng.set_corpus(tok, sent_len=2)
    eng.train(js, E.job_alphas(js, n), sd, N.MODE_HOGWILD)
    st = eng.read_stats()
    off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)
    ref = CO.sample_records(tok[:20000], off[:10001], np.array([0, 5000, 10000]), sd[:2],
                            CO.sample_int(counts, 1e-3), True, CO.make_cum_table(counts), 5)
    got = eng.debug_sample(js[:3], sd[:2])
    assert np.array_equal(got, ref)
    assert st["raw_words"] == 2 * n and st["jobs"] == len(js) - 1
    n_ref = CO.count_records(tok, off, js, sd, CO.sample_int(counts, 1e-3), True,
                             CO.make_cum_table(counts), 5)
    assert st["examples"] == n_ref
    assert 0.5 * n < st["examples"] < 1.5 * n


def test_train_hogwild_full_vocab_tracks_oracle():
    """C2 vocabulary (V=24447, Zipf 1.0), 2M pairs, 2 gensim iterations:
    the production kernel (striped hot rows, bounded grid) stays within 0.3 %
    of the sequential oracle's objective (measured 0.01-0.1 %)."""
    D, K, sample = 200, 5, 1e-3
    tok, counts, syn0 = _zipf_setup(2_000_000, 24447, D, K, sample)
    V = len(counts)
    n = len(tok) // 2
    off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    eng = E.SGNSEngine(V, D, K)
    eng.set_vocab(counts, sample)
    eng.set_weights(syn0, np.zeros((V, D), np.float32))
    eng.set_corpus(tok, sent_len=2)
    a0, a1 = syn0.copy(), np.zeros((V, D), np.float32)
    rs_g, rs_c = np.random.RandomState(1), np.random.RandomState(1)
    for _ in range(2):
        al = E.job_alphas(js, n)
        eng.train(js, al, E.job_seeds(rs_g, len(js) - 1), N.MODE_HOGWILD)
        CO.train(tok, off, js, al.astype(np.float32), E.job_seeds(rs_c, len(js) - 1),
                 CO.sample_int(counts, sample), True, CO.make_cum_table(counts), a0, a1,
                 np.ones(V, np.float32), K)
    g0, g1 = eng.get_weights()
    st = eng.read_stats()
    l_gpu = _eval_loss(g0, g1, tok, counts, K, n_eval=50000)
    l_ref = _eval_loss(a0, a1, tok, counts, K, n_eval=50000)
    assert abs(l_gpu - l_ref) / l_ref < 0.003, (l_gpu, l_ref)
    # the default cold-row stores (G2V_OPT_TAIL_STORE auto): at
    # 1,024 waves the collision budget (waves x updates per example <= 0.15)
    # starts syn1neg at row ~7,700 for this vocabulary; syn0 stays atomic
    assert st["sgns_grid"] == 256
    assert 7000 < st["tail_row_syn1neg"] < 8500, st
    assert st["tail_row_syn0"] == -1, st


@pytest.mark.parametrize("case", ["sorted", "ns_negative", "reversed"])
def test_auto_tail_rows_follow_suffix_max(case):
    """the auto cold-row boundary (G2V_OPT_TAIL_STORE -1) is the
    first row from which every later row is under the collision budget --
    with a negative ns_exponent or unsorted counts the hot rows sit late and
    no row before them may take plain stores (engine.tail_store_row restates
    the rule on the host)"""
    D, K, sample = 200, 5, 1e-3
    tok, counts, syn0 = _zipf_setup(400_000, 24447, D, K, sample)
    V = len(counts)
    ns = -0.75 if case == "ns_negative" else 0.75
    if case == "reversed":
        tok = (V - 1 - tok).astype(np.int32)
        counts = counts[::-1].copy()
        syn0 = syn0[::-1].copy()
    n = len(tok) // 2
    js = E.plan_jobs(n_sent=n, sent_len=2)
    eng = E.SGNSEngine(V, D, K)
    eng.set_vocab(counts, sample, ns_exponent=ns)
    eng.set_weights(syn0, np.zeros((V, D), np.float32))
    eng.set_corpus(tok, sent_len=2)
    eng.train(js, E.job_alphas(js, n), E.job_seeds(np.random.RandomState(1), len(js) - 1),
              N.MODE_HOGWILD)
    st = eng.read_stats()
    t = E.tail_store_row(counts, sample, K, st["sgns_grid"] * 4, ns_exponent=ns)
    got = st["tail_row_syn1neg"]
    if case == "sorted":
        assert 0 < got < V
    if t >= V:
        assert got == -1, (st, t)
    else:
        assert abs(got - max(t, st["stripe2_rows"])) <= 1, (st, t)
    assert st["tail_row_syn0"] == -1
    g0, g1 = eng.get_weights()
    assert np.isfinite(g0).all() and np.isfinite(g1).all()


def test_striping_keeps_values_exact():
    """hot-row striping only changes where atomics land: with disjoint rows,
    striped == unstriped == sequential"""
    D, K, B = 200, 5, 64
    V = B * (K + 2)
    rng = np.random.Generator(np.random.PCG64(8))
    syn0 = ((rng.random((V, D)) - 0.5) / D * 40).astype(np.float32)
    syn1 = ((rng.random((V, D)) - 0.5) / D * 40).astype(np.float32)
    perm = rng.permutation(V).astype(np.int32).reshape(B, K + 2)
    center, inp, negs = perm[:, 0], perm[:, 1], perm[:, 2:]
    outs = []
    # (rows, copies, second-tier end row, second-tier copies)
    for rows, copies, r2, c2 in ((0, 1, 0, 4), (V, 8, 0, 4), (16, 3, 0, 4), (16, 3, 200, 4),
                                 (8, 16, V, 2)):
        eng = E.SGNSEngine(V, D, K)
        eng.set_option(N.OPT_STRIPE_ROWS, rows)
        eng.set_option(N.OPT_STRIPE_COPIES, copies)
        eng.set_option(N.OPT_STRIPE2_ROWS, r2)
        eng.set_option(N.OPT_STRIPE2_COPIES, c2)
        eng.set_weights(syn0, syn1)
        eng.step_explicit(center, inp, negs, 0.025, N.MODE_HOGWILD)
        outs.append(eng.get_weights())
        eng.close()
    a0, a1 = syn0.copy(), syn1.copy()
    CO.sgns_step_sequential(a0, a1, np.ones(V, np.float32), center, inp, negs, 0.025)
    for g0, g1 in outs:
        _close(g0, a0)
        _close(g1, a1)


def test_striped_reads_sum_every_copy():
    """One chunk (32 examples, one wave, deterministic) over 12 rows, so rows
    are re-read after their own earlier updates landed in stripe copies: 16
    copies (two load batches of 7 + one), 3 copies, two-tier layouts and no
    striping agree to float rounding of the copy sums."""
    D, K, B, V = 200, 5, 32, 12
    rng = np.random.Generator(np.random.PCG64(21))
    syn0 = ((rng.random((V, D)) - 0.5) / D * 40).astype(np.float32)
    syn1 = ((rng.random((V, D)) - 0.5) / D * 40).astype(np.float32)
    center = rng.integers(0, V, B).astype(np.int32)
    inp = ((center + 1 + rng.integers(0, V - 1, B)) % V).astype(np.int32)
    negs = rng.integers(0, V, (B, K)).astype(np.int32)
    outs = []
    # the last two: a second tier (rows 4..11 with 4 copies, rows 2..7 with 8)
    for rows, copies, r2, c2 in ((0, 1, 0, 4), (V, 16, 0, 4), (V, 3, 0, 4), (4, 16, V, 4),
                                 (2, 3, 8, 8)):
        eng = E.SGNSEngine(V, D, K)
        eng.set_option(N.OPT_STRIPE_ROWS, rows)
        eng.set_option(N.OPT_STRIPE_COPIES, copies)
        eng.set_option(N.OPT_STRIPE2_ROWS, r2)
        eng.set_option(N.OPT_STRIPE2_COPIES, c2)
        eng.set_weights(syn0, syn1)
        eng.step_explicit(center, inp, negs, 0.025, N.MODE_HOGWILD)
        outs.append(eng.get_weights())
        eng.close()
    for g0, g1 in outs[1:]:
        np.testing.assert_allclose(g0, outs[0][0], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(g1, outs[0][1], rtol=1e-5, atol=1e-6)
    assert not np.array_equal(outs[0][1], syn1)


def test_sampler_at_c2_full_size_bit_exact():
    """BASELINE C2 at full size (V=24447, 100 M pairs, the bench corpus):
    effective words and directed examples of one production train() equal the
    C oracle's count, and the sampled records (downsampling + LCG jump-ahead +
    bisected negatives) of job windows at the start, middle and end of the
    corpus equal the oracle's bit for bit."""
    from gene2vec_amd import synthetic as S
    n, V0 = 100_000_000, 24447
    pairs = S.zipf_gene_pairs(n, V0, 1.0, seed=20250114)
    flat = pairs.reshape(-1)
    del pairs
    counts, first = E.count_ids(flat, V0)
    order, remap = S.vocab_order(counts, first)
    tok = remap[flat]
    del flat
    vc = counts[order].astype(np.int64)
    V = len(order)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    sd = E.job_seeds(np.random.RandomState(1), len(js) - 1)
    eng = E.SGNSEngine(V, 200, 5)
    eng.set_vocab(vc, 1e-3)
    eng.set_corpus(tok, sent_len=2)
    rng = np.random.Generator(np.random.PCG64(5))
    eng.set_weights(((rng.random((V, 200)) - 0.5) / 200).astype(np.float32),
                    np.zeros((V, 200), np.float32))
    eng.train(js, E.job_alphas(js, n), sd, N.MODE_HOGWILD)
    st = eng.read_stats()
    off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)
    si, cum = CO.sample_int(vc, 1e-3), CO.make_cum_table(vc)
    assert st["raw_words"] == 2 * n and st["jobs"] == len(js) - 1
    assert st["examples"] == CO.count_records(tok, off, js, sd, si, True, cum, 5)
    nj = len(js) - 1
    for j0 in (0, nj // 2, nj - 3):
        w = js[j0:j0 + 4] - js[j0]
        s0, s1 = js[j0], js[j0 + 3]
        sub_tok = tok[2 * s0:2 * s1]
        ref = CO.sample_records(sub_tok, off[:s1 - s0 + 1], w, sd[j0:j0 + 3], si, True, cum, 5)
        got = eng.debug_sample(js[j0:j0 + 4], sd[j0:j0 + 3])
        assert np.array_equal(got, ref), j0
    g0, g1 = eng.get_weights()
    assert np.isfinite(g0).all() and np.isfinite(g1).all() and np.abs(g1).max() > 0


@pytest.mark.parametrize("V,zipf_s,sample", [(300, 1.0, 1e-3), (2000, 1.0, 1e-3), (300, 0.0, 1e-3),
                                             (3000, 1.0, 0.0)])
def test_train_hogwild_small_vocabulary_tracks_oracle(V, zipf_s, sample):
    """Small vocabularies, where every row is hot: the default grid is cut by
    the staleness budget (waves x hottest-row updates per example), and the
    Hogwild objective stays within 0.5 % of the sequential oracle after 3
    gensim iterations (Zipf 1.0 and uniform genes; V 3,000 without
    downsampling diverged at 318 workgroups under a negatives-only budget)."""
    D, K = 200, 5
    n = 300000
    tok, counts, syn0 = _zipf_setup(n, V, D, K, sample, seed=31) if zipf_s else (None,) * 3
    if not zipf_s:
        rng = np.random.RandomState(31)
        pairs = rng.randint(0, V, (n, 2)).astype(np.int32)
        pairs[:, 1] = np.where(pairs[:, 1] == pairs[:, 0], (pairs[:, 0] + 1) % V, pairs[:, 1])
        tok, counts = _corpus_from_pairs(pairs, V)
        syn0 = ((np.random.Generator(np.random.PCG64(1)).random((len(counts), D)) - 0.5)
                / D).astype(np.float32)
    V = len(counts)
    off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    eng = E.SGNSEngine(V, D, K)
    eng.set_vocab(counts, sample)
    grid = eng.get_option(N.OPT_GRID)
    if zipf_s and V <= 300:
        assert grid < 512, grid  # hotter than C4: fewer waves in flight
    if zipf_s and not sample:
        assert grid < 250, grid  # the top gene's tokens count too (negatives alone: 313)
    eng.set_weights(syn0, np.zeros((V, D), np.float32))
    eng.set_corpus(tok, sent_len=2)
    a0, a1 = syn0.copy(), np.zeros((V, D), np.float32)
    rs_g, rs_c = np.random.RandomState(1), np.random.RandomState(1)
    for _ in range(3):
        al = E.job_alphas(js, n)
        eng.train(js, al, E.job_seeds(rs_g, len(js) - 1), N.MODE_HOGWILD)
        CO.train(tok, off, js, al.astype(np.float32), E.job_seeds(rs_c, len(js) - 1),
                 CO.sample_int(counts, sample), sample != 0, CO.make_cum_table(counts), a0, a1,
                 np.ones(V, np.float32), K)
    g0, g1 = eng.get_weights()
    eng.close()
    l_gpu = _eval_loss(g0, g1, tok, counts, K)
    l_ref = _eval_loss(a0, a1, tok, counts, K)
    assert abs(l_gpu - l_ref) / l_ref < 0.005, (V, zipf_s, sample, grid, l_gpu, l_ref)
