"""GPU: the CLI's ``--shuffle device`` (reshuffles of src/gene2vec.py:80 as a
keyed permutation of the HBM-resident pairs, g2v_permute_items8).  The first
shuffle stays CPython's (it fixes the vocabulary order), so iteration 1 is
the very run ``--shuffle python`` makes (bit for bit in sequential mode);
later iterations see another uniform order, so the 3-iteration model is
judged by its held-in SGNS objective against the Python-shuffle run."""
import numpy as np
import pytest

from gene2vec_amd import Word2Vec
from gene2vec_amd import synthetic as S
from gene2vec_amd.gene2vec import main as cli_main
from oracle import sgns_oracle as O

pytestmark = pytest.mark.gpu


def _corpus(tmp_path, V=2000, n_pairs=300_000):
    names = S.gene_names(V)
    pairs = S.zipf_gene_pairs(n_pairs, V, 1.0, seed=13)
    data = tmp_path / "data"
    data.mkdir()
    for k, part in enumerate(np.array_split(pairs, 3)):
        (data / f"pairs_{k}.txt").write_text(
            "\n".join(f"{names[a]} {names[b]}" for a, b in part) + "\n", encoding="windows-1252")
    return data, pairs, names


def _heldin(model, pairs, names, K=5, n=20000, seed=3):
    idx = {w: v.index for w, v in model.wv.vocab.items()}
    r = np.random.Generator(np.random.PCG64(seed))
    pick = pairs[r.integers(0, len(pairs), n)]
    c = np.array([idx[names[a]] for a in pick[:, 0]], np.int64)
    j = np.array([idx[names[b]] for b in pick[:, 1]], np.int64)
    counts = np.array([model.wv.vocab[w].count for w in model.wv.index2word], np.float64)
    p = counts ** 0.75
    negs = r.choice(len(counts), size=(n, K), p=p / p.sum())
    return O.sgns_loss(model.wv.vectors, model.syn1neg, c, j, negs)


def test_device_shuffle_iteration1_identical(tmp_path):
    data, _, _ = _corpus(tmp_path)
    base = ["--iters", "2", "--dim", "32", "--hash", "crc32", "--shuffle-seed", "9",
            "--native-ingest", "--no-txt", "--no-w2v", "--mode", "sequential"]
    cli_main([str(data), str(tmp_path / "py"), "txt", "--shuffle", "python"] + base)
    cli_main([str(data), str(tmp_path / "dev"), "txt", "--shuffle", "device"] + base)
    a = Word2Vec.load(str(tmp_path / "py" / "gene2vec_dim_32_iter_1"))
    b = Word2Vec.load(str(tmp_path / "dev" / "gene2vec_dim_32_iter_1"))
    assert a.wv.index2word == b.wv.index2word
    assert np.array_equal(a.wv.vectors, b.wv.vectors)
    assert np.array_equal(a.syn1neg, b.syn1neg)
    # iteration 2 trains every pair once more, in another order
    a2 = Word2Vec.load(str(tmp_path / "py" / "gene2vec_dim_32_iter_2"))
    b2 = Word2Vec.load(str(tmp_path / "dev" / "gene2vec_dim_32_iter_2"))
    assert not np.array_equal(a2.wv.vectors, b2.wv.vectors)


def test_device_shuffle_quality(tmp_path):
    data, pairs, names = _corpus(tmp_path)
    base = ["--iters", "3", "--dim", "64", "--hash", "crc32", "--shuffle-seed", "4",
            "--native-ingest", "--no-txt", "--no-w2v"]
    cli_main([str(data), str(tmp_path / "py"), "txt", "--shuffle", "python"] + base)
    cli_main([str(data), str(tmp_path / "dev"), "txt", "--shuffle", "device"] + base)
    a = Word2Vec.load(str(tmp_path / "py" / "gene2vec_dim_64_iter_3"))
    b = Word2Vec.load(str(tmp_path / "dev" / "gene2vec_dim_64_iter_3"))
    la, lb = _heldin(a, pairs, names), _heldin(b, pairs, names)
    print("held-in objective: python shuffle %.5f, device shuffle %.5f" % (la, lb))
    assert la < 0.9 * 6 * np.log(2)
    assert abs(lb - la) <= 0.005 * la, (la, lb)
