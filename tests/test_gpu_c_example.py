"""GPU: the C ABI driven from C alone (examples/g2v_train.c: no Python, no
torch in the process) trains exactly what the Python engine trains through
the same ABI -- sequential mode bit for bit -- and the Hogwild mode learns."""
import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd import engine as E
from tests.c_example import read_output, run, write_input
from tests.helpers import vocab_from_ids, zipf_pairs

pytestmark = pytest.mark.gpu


def _case(V0=500, n_pairs=60_000, D=64, K=5):
    pairs = zipf_pairs(n_pairs, V0, seed=21)
    flat = pairs.reshape(-1)
    _, remap, counts = vocab_from_ids(flat, V0)
    tok = remap[flat].astype(np.int32)
    V = len(counts)
    rng = np.random.Generator(np.random.PCG64(5))
    syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
    js = E.plan_jobs(n_sent=n_pairs, sent_len=2)
    seeds = E.job_seeds(np.random.RandomState(1), len(js) - 1)
    return V, D, K, counts, syn0, tok, js, seeds


def test_c_host_sequential_equals_python_engine(tmp_path):
    V, D, K, counts, syn0, tok, js, seeds = _case()
    inp, out = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    write_input(inp, V, D, K, N.MODE_SEQUENTIAL, counts, syn0, tok, seeds)
    r = run(inp, out)
    assert r.returncode == 0, r.stdout + r.stderr
    c0, c1, st = read_output(out, V, D)

    eng = E.SGNSEngine(V, D, K)
    eng.set_vocab(counts, 1e-3)
    eng.set_weights(syn0, np.zeros_like(syn0))
    eng.set_corpus(tok, sent_len=2)
    eng.train(js, E.job_alphas(js, len(tok) // 2), seeds, N.MODE_SEQUENTIAL)
    p0, p1 = eng.get_weights()
    pst = eng.read_stats()
    eng.close()
    assert np.array_equal(c0, p0) and np.array_equal(c1, p1)
    assert st["effective_words"] == pst["effective_words"] and st["examples"] == pst["examples"]
    assert st["jobs"] == len(js) - 1


def test_c_host_hogwild_learns(tmp_path):
    from oracle import sgns_oracle as O
    V, D, K, counts, syn0, tok, js, seeds = _case(n_pairs=200_000)
    inp, out = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    write_input(inp, V, D, K, N.MODE_HOGWILD, counts, syn0, tok, seeds)
    r = run(inp, out)
    assert r.returncode == 0, r.stdout + r.stderr
    c0, c1, st = read_output(out, V, D)
    assert np.isfinite(c0).all() and np.isfinite(c1).all()
    rg = np.random.Generator(np.random.PCG64(2))
    idx = rg.integers(0, len(tok) // 2, 5000)
    c, j = tok[2 * idx].astype(np.int64), tok[2 * idx + 1].astype(np.int64)
    p = counts.astype(np.float64) ** 0.75
    negs = rg.choice(V, size=(5000, K), p=p / p.sum())
    loss = O.sgns_loss(c0, c1, c, j, negs)
    assert loss < 0.9 * (K + 1) * np.log(2), loss
