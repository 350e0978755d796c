"""GPU: G2V_OPT_SAMPLE_OVERLAP -- the sampler of segment s+1 runs on a side
stream under segment s's update kernel, over two record workspaces.  The
segments still train in order, so a SEQUENTIAL multi-segment epoch is bit for
bit the serial one, across segment counts that exercise both workspaces,
their growth, and an odd last segment."""
import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd import engine as E
from tests.helpers import vocab_from_ids, zipf_pairs

pytestmark = pytest.mark.gpu


def _train(tok, counts, syn0, js, al, seeds, seg, overlap, mode):
    V, D = syn0.shape
    eng = E.SGNSEngine(V, D, 5)
    eng.set_option(N.OPT_SEG_JOBS, seg)
    eng.set_option(N.OPT_SAMPLE_OVERLAP, overlap)
    eng.set_vocab(counts, 1e-3)
    eng.set_weights(syn0, np.zeros_like(syn0))
    eng.set_corpus(tok, sent_len=2)
    eng.train(js, al, seeds, mode)
    s0, s1 = eng.get_weights()
    st = eng.read_stats()
    assert eng.get_option(N.OPT_SAMPLE_OVERLAP) == overlap
    eng.close()
    return s0, s1, st


@pytest.mark.parametrize("seg", [1, 3, 7])
def test_overlap_sequential_bit_exact(seg):
    pairs = zipf_pairs(100_003, 700, seed=31)
    flat = pairs.reshape(-1)
    _, remap, counts = vocab_from_ids(flat, 700)
    tok = remap[flat].astype(np.int32)
    V, D = len(counts), 48
    syn0 = ((np.random.Generator(np.random.PCG64(8)).random((V, D)) - 0.5) / D).astype(np.float32)
    js = E.plan_jobs(n_sent=len(tok) // 2, sent_len=2)
    al = E.job_alphas(js, len(tok) // 2)
    seeds = E.job_seeds(np.random.RandomState(4), len(js) - 1)
    a0, a1, sa = _train(tok, counts, syn0, js, al, seeds, seg, 0, N.MODE_SEQUENTIAL)
    b0, b1, sb = _train(tok, counts, syn0, js, al, seeds, seg, 1, N.MODE_SEQUENTIAL)
    assert np.array_equal(a0, b0) and np.array_equal(a1, b1)
    assert sa["examples"] == sb["examples"] and sa["effective_words"] == sb["effective_words"]
    assert sa["launches"] == sb["launches"] == -(-(len(js) - 1) // seg)


def test_overlap_hogwild_counts():
    pairs = zipf_pairs(300_000, 2000, seed=32)
    flat = pairs.reshape(-1)
    _, remap, counts = vocab_from_ids(flat, 2000)
    tok = remap[flat].astype(np.int32)
    V, D = len(counts), 64
    syn0 = ((np.random.Generator(np.random.PCG64(9)).random((V, D)) - 0.5) / D).astype(np.float32)
    js = E.plan_jobs(n_sent=len(tok) // 2, sent_len=2)
    al = E.job_alphas(js, len(tok) // 2)
    seeds = E.job_seeds(np.random.RandomState(5), len(js) - 1)
    _, _, sa = _train(tok, counts, syn0, js, al, seeds, 8, 0, N.MODE_HOGWILD)
    b0, b1, sb = _train(tok, counts, syn0, js, al, seeds, 8, 1, N.MODE_HOGWILD)
    # the sampled stream is the same; only the Hogwild update order may differ
    assert sa["examples"] == sb["examples"] and sa["effective_words"] == sb["effective_words"]
    assert np.isfinite(b0).all() and np.isfinite(b1).all()
