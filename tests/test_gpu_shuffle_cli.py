"""GPU: the CLI's ``--shuffle device``: the shuffles of src/gene2vec.py:52,80
(unseeded random.shuffle calls in the reference) as keyed permutations of
the HBM-resident pairs (g2v_permute_items8), the vocabulary scanned in the
first one's order on the device (g2v_first_occurrence_perm8).  Checked: the
vocabulary order against the numpy restatement, and the 3-iteration model's
held-in SGNS objective against the Python-shuffle run."""
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


def test_device_shuffle_vocabulary_order(tmp_path):
    """iteration 1's vocabulary: counts descending, ties in first-occurrence
    order of the device-shuffled corpus (the order g2v_permute_items8 gives
    with the seed the CLI draws after the file shuffle), restated here with
    the numpy oracle; iteration 2 trains the same vocabulary."""
    import os
    import random

    from gene2vec_amd import ingest
    from oracle import shuffle_oracle as SO
    data, _, _ = _corpus(tmp_path)
    base = ["--iters", "2", "--dim", "32", "--hash", "crc32", "--shuffle-seed", "9",
            "--native-ingest", "--no-txt", "--no-w2v", "--shuffle", "device"]
    cli_main([str(data), str(tmp_path / "dev"), "txt"] + base)
    rng = random.Random(9)
    files = os.listdir(data)
    rng.shuffle(files)
    seed = rng.getrandbits(64)
    corpus = ingest.read_corpus([os.path.join(data, f) for f in files if f.endswith("txt")])
    first = SO.first_occurrence(corpus.tokens.reshape(-1, 2), seed, len(corpus.words))
    order = sorted(np.nonzero(first >= 0)[0], key=lambda i: (-corpus.counts[i], first[i]))
    a = Word2Vec.load(str(tmp_path / "dev" / "gene2vec_dim_32_iter_1"))
    assert a.wv.index2word == [corpus.words[i] for i in order]
    b = Word2Vec.load(str(tmp_path / "dev" / "gene2vec_dim_32_iter_2"))
    assert b.wv.index2word == a.wv.index2word


def test_device_shuffle_quality(tmp_path):
    """the mean over four shuffle seeds of each mode's 3-iteration objective
    within 0.5 %: one run's own spread over seeds is ~0.6 % (python
    2.810-2.827, device 2.808-2.820 over seeds 4-7, profiles/r03/r03f_spread.log:
    sd ~0.25 %), so a single pair of runs cannot carry a sub-percent bar; the
    difference of two 4-run means has an sd of ~0.18 %, and the 0.5 % bar sits
    at ~2.8 of them (round 3 ran 2 seeds at 0.6 %)"""
    data, pairs, names = _corpus(tmp_path)
    loss = {"python": [], "device": []}
    for seed in ("4", "5", "6", "7"):
        base = ["--iters", "3", "--dim", "64", "--hash", "crc32", "--shuffle-seed", seed,
                "--native-ingest", "--no-txt", "--no-w2v"]
        for mode in loss:
            out = tmp_path / f"{mode}{seed}"
            cli_main([str(data), str(out), "txt", "--shuffle", mode] + base)
            loss[mode].append(_heldin(Word2Vec.load(str(out / "gene2vec_dim_64_iter_3")), pairs,
                                      names))
    la, lb = np.mean(loss["python"]), np.mean(loss["device"])
    print("held-in objective: python shuffle %s, device shuffle %s" % (loss["python"], loss["device"]))
    assert la < 0.9 * 6 * np.log(2)
    assert abs(lb - la) <= 0.005 * la, (la, lb)
