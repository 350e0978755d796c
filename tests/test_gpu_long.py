"""GPU: sentences longer than gensim's batch_words and corpus validation.

[ext] _job_producer gives a sentence over batch_words = 10000 raw words a job
of its own (queuing an EMPTY job first when it is the first sentence, which
still draws its two model.random seeds), and [ext] train_batch_sg stops at
MAX_SENTENCE_LEN = 10000 effective words (the reference reads any line
length, src/gene2vec.py:45).  Records bit-exact and sequential training at
1e-5 against the C oracle (oracle/sgns_oracle.c train_job, which restates
the truncation); ids outside [-1, V) are rejected (host corpus) or latched
as a device fault (device corpus).
"""
import numpy as np
import pytest
import torch

from gene2vec_amd import _native as N
from gene2vec_amd import engine as E
from oracle import c_oracle as CO
from tests.helpers import long_sentence_corpus

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sample", [0.0, 1e-3])
@pytest.mark.parametrize("K", [5, 15])
def test_long_sentence_records_bit_exact(sample, K):
    tok, off, counts = long_sentence_corpus()
    V = len(counts)
    js = E.plan_jobs(sent_off=off)
    assert js[0] == js[1] == 0  # the empty first job
    seeds = E.job_seeds(np.random.RandomState(7), len(js) - 1)
    eng = E.SGNSEngine(V, 8, K)
    eng.set_vocab(counts, sample)
    eng.set_corpus(tok, sent_off=off)
    got = eng.debug_sample(js, seeds)
    ref = CO.sample_records(tok, off, js, seeds, CO.sample_int(counts, sample), sample != 0,
                            CO.make_cum_table(counts), K)
    assert len(ref) > 20000 and np.array_equal(got, ref)
    eng.close()


def test_long_sentence_train_sequential_vs_oracle():
    tok, off, counts = long_sentence_corpus(seed=3)
    V, D, K = len(counts), 64, 5
    js = E.plan_jobs(sent_off=off)
    n = len(off) - 1
    al = E.job_alphas(js, n)
    sd = E.job_seeds(np.random.RandomState(1), len(js) - 1)
    syn0 = ((np.random.Generator(np.random.PCG64(2)).random((V, D)) - 0.5) / D).astype(np.float32)
    eng = E.SGNSEngine(V, D, K)
    eng.set_vocab(counts, 1e-3)
    eng.set_weights(syn0, np.zeros((V, D), np.float32))
    eng.set_corpus(tok, sent_off=off)
    eng.train(js, al, sd, N.MODE_SEQUENTIAL)
    st = eng.read_stats()
    g0, g1 = eng.get_weights()
    a0, a1 = syn0.copy(), np.zeros((V, D), np.float32)
    ref = CO.train(tok, off, js, al.astype(np.float32), sd, CO.sample_int(counts, 1e-3), True,
                   CO.make_cum_table(counts), a0, a1, np.ones(V, np.float32), K)
    assert (st["effective_words"], st["examples"], st["raw_words"]) == (
        ref["effective_words"], ref["examples"], ref["raw_words"])
    np.testing.assert_allclose(g0, a0, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(g1, a1, rtol=1e-5, atol=1e-6)
    eng.close()


def test_fixed_length_over_batch_words():
    """sent_len > batch_words (no offsets): empty first job, one job per
    sentence, each truncated -- the same records as the CSR form"""
    rng = np.random.RandomState(5)
    V, L, n = 30000, 12001, 3
    tok = rng.randint(0, V, size=L * n).astype(np.int32)
    counts = np.sort(np.bincount(tok, minlength=V).astype(np.int64) + 1)[::-1].copy()
    js = E.plan_jobs(n_sent=n, sent_len=L)
    assert js.tolist() == [0, 0, 1, 2, 3]
    seeds = E.job_seeds(np.random.RandomState(1), len(js) - 1)
    eng = E.SGNSEngine(V, 8, 5)
    eng.set_vocab(counts, 0.0)
    eng.set_corpus(tok, sent_len=L)
    got = eng.debug_sample(js, seeds)
    off = np.arange(0, L * n + 1, L, dtype=np.int64)
    ref = CO.sample_records(tok, off, js, seeds, CO.sample_int(counts, 0.0), False,
                            CO.make_cum_table(counts), 5)
    assert len(got) == 3 * 2 * (10000 - 1) and np.array_equal(got, ref)
    eng.close()


def test_host_corpus_ids_checked():
    eng = E.SGNSEngine(10, 8, 5)
    eng.set_vocab(np.arange(10, 0, -1, dtype=np.int64), 1e-3)
    for bad in (10, -2, 2 ** 31 - 1):
        tok = np.array([1, 2, bad, 3], np.int32)
        with pytest.raises(N.G2VError) as e:
            eng.set_corpus(tok, sent_len=2)
        assert e.value.code == N.G2V_EINVAL
    with pytest.raises(N.G2VError):  # decreasing offsets
        eng.set_corpus(np.array([1, 2, 3], np.int32), sent_off=np.array([0, 2, 1, 3], np.int64))
    eng.set_corpus(np.array([1, -1, 9, 0], np.int32), sent_len=2)  # -1 = OOV is valid
    eng.close()


def test_device_corpus_fault_reported():
    """a device corpus is not host-checked: the sampler skips an id >= V like
    an OOV token (no out-of-bounds access) and latches a fault that the next
    g2v_sync / g2v_read_stats raises, then clears"""
    V = 50
    eng = E.SGNSEngine(V, 16, 5)
    eng.set_vocab(np.arange(V, 0, -1, dtype=np.int64), 1e-3)
    eng.set_weights(np.zeros((V, 16), np.float32), np.zeros((V, 16), np.float32))
    tok = torch.tensor([1, 2, 3, V + 7, 4, 5], dtype=torch.int32, device="cuda")
    eng.set_corpus_device(tok.data_ptr(), tok.numel(), sent_len=2, keepalive=tok)
    js = E.plan_jobs(n_sent=3, sent_len=2)
    eng.train(js, E.job_alphas(js, 3), E.job_seeds(np.random.RandomState(1), 1))
    with pytest.raises(N.G2VError) as e:
        eng.sync()
    assert e.value.code == N.G2V_EINVAL and "outside [-1, V)" in str(e.value)
    eng.sync()  # cleared
    # a device CSR whose job packs several sentences past 10000 raw words
    tok2 = torch.zeros(12000, dtype=torch.int32, device="cuda")
    off2 = torch.tensor([0, 6000, 12000], dtype=torch.int64, device="cuda")
    eng.set_corpus_device(tok2.data_ptr(), 12000, off_ptr=off2.data_ptr(), n_sent=2,
                          keepalive=(tok2, off2))
    eng.train(np.array([0, 2], np.int64), np.array([0.025]), E.job_seeds(np.random.RandomState(1), 1))
    with pytest.raises(N.G2VError) as e:
        eng.read_stats()
    assert "10000 raw words" in str(e.value)
    eng.close()
