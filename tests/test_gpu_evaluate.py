"""GPU: the target-function evaluator (src/evaluation_target_function.py)
against its numpy restatement, on a synthetic .gmt (MSigDB is absent)."""
import numpy as np
import pytest

from gene2vec_amd import KeyedVectors
from gene2vec_amd import evaluate as EV
from oracle import target_oracle as TO

pytestmark = pytest.mark.gpu


def _fixture(tmp_path, V=1500, D=200, n_path=60):
    rng = np.random.Generator(np.random.PCG64(4))
    kv = KeyedVectors(D)
    words = [f"G{i:05d}" for i in range(V)]
    kv.index2word = words
    from gene2vec_amd.word2vec import Vocab
    kv.vocab = {w: Vocab(count=V - i, index=i) for i, w in enumerate(words)}
    kv.vectors = (rng.standard_normal((V, D)) * 0.3 + 0.2).astype(np.float32)
    f = str(tmp_path / "emb_w2v.txt")
    kv.save_word2vec_format(f)
    lines = []
    for p in range(n_path):
        k = int(rng.integers(3, 60))  # some lines exceed 52 fields -> skipped
        genes = [words[int(i)] for i in rng.integers(0, V, k)]
        genes += ["NOT_A_GENE"] if p % 3 == 0 else []
        lines.append("\t".join([f"PATH{p}", "http://x"] + genes) + "\n")
    gmt = tmp_path / "p.gmt"
    gmt.write_text("".join(lines))
    return f, str(gmt), kv


def test_target_function_matches_oracle(tmp_path):
    f, gmt, kv = _fixture(tmp_path)
    got = EV.target_function(f, gmt, verbose=False)
    kv2 = KeyedVectors.load_word2vec_format(f)
    pm, rm, ratio = TO.target_function(kv2.index2word, kv2.vectors, EV.read_pathways(gmt))
    assert got["n_random_pairs"] == 499500
    assert got["path_mean"] == pytest.approx(pm, rel=1e-5)
    assert got["rand_mean"] == pytest.approx(rm, rel=1e-4, abs=1e-6)
    assert got["ratio"] == pytest.approx(ratio, rel=1e-4)


def test_cosine_pairs_matches_numpy(tmp_path):
    rng = np.random.Generator(np.random.PCG64(5))
    kv = KeyedVectors(200)
    kv.vectors = rng.standard_normal((300, 200)).astype(np.float32)
    a = rng.integers(0, 300, 5000)
    b = rng.integers(0, 300, 5000)
    got = EV.cosine_pairs(kv, a, b)
    ref = np.array([TO.similarity(kv.vectors, x, y) for x, y in zip(a, b)], np.float32)
    np.testing.assert_allclose(got, ref, rtol=2e-6, atol=1e-7)
    assert np.all(got[a == b] == pytest.approx(1.0, abs=1e-6))
