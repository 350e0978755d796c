"""The CPU oracle against the golden fixtures and the independent anchors.

Anchors independent of the oracle itself: the reference's own corpus
data/test.txt (counts / vocabulary size, SURVEY.md section 4 KATs) and numpy's
RandomState (the generator gensim calls in seeded_vector / model.random).
"""
import json
import os

import numpy as np
import pytest

from oracle import c_oracle as CO
from oracle import sgns_oracle as O
from tests.conftest import GOLDEN
from tests.helpers import crc_hash, long_sentence_corpus


def test_reference_fixture_vocab(golden, test_pairs):
    voc = O.build_vocab(test_pairs, 1, 1e-3)
    # 80 raw words, 79 unique, TLE1 x2 at index 0
    assert voc.total_words == 80 and len(voc.index2word) == 79 and voc.corpus_count == 40
    assert voc.index2word[0] == "TLE1" and voc.counts[0] == 2
    g = golden["test_pairs"]
    assert voc.index2word == g["index2word"]
    assert voc.first_order == g["first_order"]
    assert voc.counts.tolist() == g["counts"]


def test_known_answer_tables(golden):
    g = golden["test_pairs"]
    cum = g["cum_table"]
    assert cum[:4] == [45325569, 72276314, 99227058, 126177803]
    assert cum[-1] == 2 ** 31 - 1
    si = dict(zip(g["counts"], g["sample_int"]))
    assert si[1] == 1558397584 and si[2] == 1030792151
    assert set(g["sample_int_s0"]) == {2 ** 32}  # sample=0: never downsampled


def test_oracle_tables_match_golden(golden, test_pairs):
    voc = O.build_vocab(test_pairs, 1, 1e-3)
    assert O.make_cum_table(voc.counts).tolist() == golden["test_pairs"]["cum_table"]
    assert [int(x) for x in voc.sample_int] == golden["test_pairs"]["sample_int"]
    for V in (1000, 24447, 60000):
        z = np.load(os.path.join(GOLDEN, f"zipf{V}_tables.npz"))
        assert np.array_equal(CO.make_cum_table(z["counts"]), z["cum"])
        assert np.array_equal(CO.sample_int(z["counts"], 1e-3), z["sample_int"])
    z = np.load(os.path.join(GOLDEN, "zipf1000_tables.npz"))
    assert np.array_equal(O.make_cum_table(z["counts"]), z["cum"])


def test_exp_table():
    g = np.load(os.path.join(GOLDEN, "exp_table.npy"))
    assert np.array_equal(O.exp_table(), g)
    assert np.array_equal(CO.exp_table(), g)
    assert O.LUT_SCALE == 83
    # monotone sigmoid over [-6, 6)
    assert np.all(np.diff(g) > 0) and 0 < g[0] < 0.003 and 0.997 < g[-1] < 1


def test_lcg_and_negatives(golden):
    g = golden["lcg"]
    z = np.load(os.path.join(GOLDEN, "zipf1000_tables.npz"))
    x = g["seed"]
    outs, negs = [], []
    for _ in range(1000):
        outs.append(x >> 16)
        t, x = O.draw_negative(z["cum"], x)
        negs.append(t)
    assert outs == g["outputs"] and negs == g["negatives_zipf1000"]
    y = g["seed"]
    for _ in range(1000):
        y = O.lcg_next(y)
    assert y == O.lcg_jump(g["seed"], 1000) == g["jump_1000"]
    assert O.lcg_jump(g["seed"], 123457) == g["jump_123457"]


def test_schedule(golden):
    s = golden["schedule"]
    assert [list(j) for j in O.plan_jobs([2] * 40)] == s["jobs40"]
    assert O.job_alphas(O.plan_jobs([2] * 40), 40) == s["alphas40"] == [0.025]
    j = O.plan_jobs([2] * 1000000)
    assert len(j) == s["jobs1m_n"] == 200
    a = O.job_alphas(j, 1000000)
    assert a[:5] == s["alphas1m_head"] and a[-5:] == s["alphas1m_tail"]
    assert a[1] == pytest.approx(0.025 - 0.0249 * 5000 / 1e6, rel=1e-15)
    assert [list(x) for x in O.plan_jobs(s["mixed_lengths"])] == s["mixed_jobs"]
    assert O.job_seeds(np.random.RandomState(1), 5) == s["seeds_rs1"]


def test_seeded_vector_is_numpy_randomstate(golden):
    g = golden["seeded_vector"]
    v = O.seeded_vector(g["word"] + str(g["seed"]), g["dim"], crc_hash).astype(np.float32)
    assert v.tolist() == g["values"]
    rs = np.random.RandomState(crc_hash("TLE11") & 0xFFFFFFFF)
    assert np.array_equal(((rs.rand(8) - 0.5) / 8).astype(np.float32), v)


@pytest.mark.parametrize("name", ["step_V60_D200_K5", "step_V40_D512_K15"])
def test_step_golden_numpy_and_c(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    for impl in ("numpy", "c"):
        a0, a1 = z["syn0"].copy(), z["syn1neg"].copy()
        lockf = np.ones(len(a0), dtype=np.float32)
        if impl == "numpy":
            O.sgns_step_sequential(a0, a1, lockf, z["center"], z["input"], z["negs"],
                                   float(z["alpha"]))
        else:
            CO.sgns_step_sequential(a0, a1, lockf, z["center"], z["input"], z["negs"],
                                    float(z["alpha"]))
        np.testing.assert_allclose(a0, z["syn0_out"], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(a1, z["syn1neg_out"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("tag,sample", [("s0", 0.0), ("s1e-3", 1e-3)])
def test_e2e_numpy_vs_c_vs_golden(test_pairs, tag, sample):
    z = np.load(os.path.join(GOLDEN, f"e2e_test_pairs_{tag}.npz"))
    voc = O.build_vocab(test_pairs, 1, sample)
    syn0, syn1, lockf = O.reset_weights(voc.index2word, 200, 1, crc_hash)
    assert np.array_equal(syn0, z["syn0_init"])
    ids = O.sentences_to_ids(test_pairs, voc.word2index)
    tok = np.array([w for s in ids for w in s], np.int32)
    off = np.cumsum([0] + [len(s) for s in ids]).astype(np.int64)
    jobs = O.plan_jobs([len(s) for s in ids])
    js = np.array([jobs[0][0]] + [j[1] for j in jobs], np.int64)
    cum = O.make_cum_table(voc.counts)
    rs = np.random.RandomState(1)
    stats = []
    for _ in range(3):
        al = np.array(O.job_alphas(jobs, len(ids)), np.float32)
        sd = np.array(O.job_seeds(rs, len(jobs)), np.uint64)
        stats.append(CO.train(tok, off, js, al, sd, voc.sample_int, bool(sample), cum, syn0,
                              syn1, lockf, 5))
    gst = json.loads(str(z["stats"]))
    for a, b in zip(stats, gst):
        assert (a["effective_words"], a["examples"], a["jobs"]) == (
            b["effective_words"], b["examples"], b["jobs"])
    np.testing.assert_allclose(syn0, z["syn0"], rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(syn1, z["syn1neg"], rtol=1e-6, atol=1e-8)
    assert np.abs(syn1).max() > 0  # it trained


def test_c_records_match_numpy(test_pairs):
    voc = O.build_vocab(test_pairs, 1, 1e-3)
    ids = O.sentences_to_ids(test_pairs, voc.word2index)
    cum = O.make_cum_table(voc.counts)
    tok = np.array([w for s in ids for w in s], np.int32)
    off = np.cumsum([0] + [len(s) for s in ids]).astype(np.int64)
    for seed in (1, 987654321, 2 ** 47 + 5):
        rec = CO.sample_records(tok, off, np.array([0, len(ids)]), np.array([seed], np.uint64),
                                voc.sample_int, True, cum, 5)
        ref = O.sample_job_records(ids, seed, voc.sample_int, True, cum, 5)
        assert rec.tolist() == [[c, j] + n for c, j, n in ref]


# ---------------------------------------------------------------------------
# compute_loss ([ext] fast_sentence_sg_neg's LOG_TABLE tally) and the
# MAX_SENTENCE_LEN truncation of train_batch_sg
# ---------------------------------------------------------------------------
def test_log_table():
    lt = O.log_table()
    assert np.array_equal(lt, CO.log_table())
    e = O.exp_table()
    assert np.array_equal(lt, np.log(e.astype(np.float64)).astype(np.float32))
    assert np.all(np.diff(lt) > 0) and np.all(lt < 0)
    # the index int((0 + 6) * 83) = 498 of an untrained model: log(sigmoid(-0.024))
    assert lt[498] == pytest.approx(np.log(1 / (1 + np.exp(0.024))), rel=1e-5)


@pytest.mark.parametrize("sample", [0.0, 1e-3])
def test_compute_loss_numpy_equals_c(test_pairs, sample):
    """gensim's float32 running loss (workers=1 order) from both restatements,
    over three train() calls continued (no reset between them)."""
    voc = O.build_vocab(test_pairs, 1, sample)
    ids = O.sentences_to_ids(test_pairs, voc.word2index)
    tok = np.array([w for s in ids for w in s], np.int32)
    off = np.cumsum([0] + [len(s) for s in ids]).astype(np.int64)
    jobs = O.plan_jobs([len(s) for s in ids])
    js = np.array([jobs[0][0]] + [j[1] for j in jobs], np.int64)
    cum = O.make_cum_table(voc.counts)
    n0, n1, nl = O.reset_weights(voc.index2word, 50, 1, crc_hash)
    c0, c1 = n0.copy(), n1.copy()
    l_np = np.zeros(1, np.float32)
    l_c = np.zeros(1, np.float32)
    rs_n, rs_c = np.random.RandomState(1), np.random.RandomState(1)
    for _ in range(3):
        O.train_epoch_sequential(ids, voc, n0, n1, nl, cum, 5, rs_n, sample=sample, loss=l_np)
        al = np.array(O.job_alphas(jobs, len(ids)), np.float32)
        sd = np.array(O.job_seeds(rs_c, len(jobs)), np.uint64)
        CO.train(tok, off, js, al, sd, voc.sample_int, bool(sample), cum, c0, c1, nl, 5,
                 loss=l_c)
    assert l_np[0] == l_c[0] and l_c[0] > 0
    np.testing.assert_allclose(c0, n0, rtol=1e-6, atol=1e-8)


def test_compute_loss_first_example_is_log2_per_target():
    """untrained syn1neg (zeros): every dot is 0 -> each applied target adds
    -LOG_TABLE[498] = 0.7052...; a negative equal to the center is skipped"""
    V, D, K = 10, 8, 5
    syn0 = np.full((V, D), 0.01, np.float32)
    syn1 = np.zeros((V, D), np.float32)
    loss = np.zeros(1, np.float32)
    negs = np.array([[1, 2, 0, 3, -1]], np.int32)  # 0 == center: skipped; -1 skipped
    CO.sgns_step_sequential(syn0, syn1, np.ones(V, np.float32), np.array([0], np.int32),
                            np.array([4], np.int32), negs, 0.025, loss=loss)
    assert loss[0] == np.float32(-O.log_table()[498] * 4)


@pytest.mark.parametrize("sample", [0.0, 1e-3])
def test_long_sentence_truncation_numpy_equals_c(sample):
    """sentences over batch_words: a job of their own (an empty job first when
    the corpus starts with one), truncated at 10000 effective words"""
    tok, off, counts = long_sentence_corpus()
    lengths = np.diff(off).tolist()
    jobs = O.plan_jobs(lengths)
    assert jobs[0] == (0, 0)
    js = np.array([jobs[0][0]] + [j[1] for j in jobs], np.int64)
    seeds = np.array(O.job_seeds(np.random.RandomState(4), len(jobs)), np.uint64)
    cum = O.make_cum_table(counts)
    si = O.sample_int_from_counts(counts, sample)
    rec = CO.sample_records(tok, off, js, seeds, si, sample != 0, cum, 5)
    ref = []
    sents = [tok[off[i]:off[i + 1]].tolist() for i in range(len(lengths))]
    effs = []
    for (s0, s1), sd in zip(jobs, seeds):
        ref += O.sample_job_records(sents[s0:s1], int(sd), si, sample != 0, cum, 5)
        effs.append(O.downsample_job(sents[s0:s1], si, int(sd), sample != 0)[2])
    assert rec.tolist() == [[c, j] + n for c, j, n in ref]
    assert max(effs) == 10000 and effs[0] == 0


def test_atomic_one_wave_restatement_degenerates_to_sequential():
    """orc_atomic_one_wave (k_sgns_atomic's order on one wave) with chunks of
    one example and no stripes is gensim's sequential order, up to the
    kernel's float atomics rounding coef*src and the add separately where
    saxpy fuses them (~1e-7); with 32-example chunks the one-example lag
    moves it by ~0.5 %, and stripes only re-associate sums (~1e-6)"""
    from oracle import c_oracle as CO
    rng = np.random.RandomState(0)
    V, D, K, n = 40, 200, 5, 3000
    s0 = ((rng.rand(V, D) - 0.5) / D).astype(np.float32)
    s1 = np.zeros((V, D), np.float32)
    c, i = rng.randint(0, V, n), rng.randint(0, V, n)
    ng = rng.randint(0, V, (n, K))
    ng[ng == c[:, None]] = -1
    lf = np.ones(V, np.float32)

    def rel(a, b):
        return float(np.abs(a - b).max() / np.abs(b).max())
    a0, a1 = s0.copy(), s1.copy()
    CO.sgns_step_sequential(a0, a1, lf, c, i, ng, 0.025)
    b0, b1 = s0.copy(), s1.copy()
    CO.atomic_one_wave(b0, b1, lf, c, i, ng, 0.025, chunk=1)
    assert rel(b0, a0) < 1e-6 and rel(b1, a1) < 1e-6
    d0, d1 = s0.copy(), s1.copy()
    CO.atomic_one_wave(d0, d1, lf, c, i, ng, 0.025, chunk=32)
    assert rel(d1, a1) > 1e-3
    f0, f1 = s0.copy(), s1.copy()
    CO.atomic_one_wave(f0, f1, lf, c, i, ng, 0.025, 8, 16, 20, 4, chunk=32)
    assert rel(f0, d0) < 1e-5 and rel(f1, d1) < 1e-5
