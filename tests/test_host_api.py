"""Host-side mirror of the reference interface (no GPU needed): vocabulary,
initial weights, persistence and the three output formats the reference's
consumers read (src/generateMatrix.py .txt, word2vec text/binary)."""
import os
import random

import numpy as np
import pytest

from gene2vec_amd import KeyedVectors, Word2Vec
from gene2vec_amd import generateMatrix as gM
from gene2vec_amd.gene2vec import read_gene_pairs
from oracle import sgns_oracle as O
from tests.conftest import GOLDEN
from tests.helpers import crc_hash


def _model(test_pairs, sample=1e-3):
    m = Word2Vec(size=200, window=1, min_count=1, workers=32, iter=1, sg=1, sample=sample,
                 hashfxn=crc_hash)
    m.build_vocab(test_pairs)
    return m


def test_vocab_and_init_match_oracle(test_pairs, golden):
    m = _model(test_pairs)
    g = golden["test_pairs"]
    assert m.wv.index2word == g["index2word"]
    assert list(m.wv.vocab.keys()) == g["first_order"]
    assert [m.wv.vocab[w].count for w in m.wv.index2word] == g["counts"]
    assert [m.wv.vocab[w].sample_int for w in m.wv.index2word] == g["sample_int"]
    assert m.corpus_count == 40 and m.corpus_total_words == 80
    syn0, syn1, lockf = O.reset_weights(m.wv.index2word, 200, 1, crc_hash)
    assert np.array_equal(m.wv.vectors, syn0)
    assert not m.syn1neg.any() and (m.vectors_lockf == 1).all()
    z = np.load(os.path.join(GOLDEN, "e2e_test_pairs_s1e-3.npz"))
    assert np.array_equal(m.wv.vectors, z["syn0_init"])


def test_unsupported_configs_raise():
    for kw in (dict(sg=0), dict(sg=1, hs=1), dict(sg=1, window=5), dict(sg=1, negative=21), dict(sg=1, negative=0),
               dict(sg=1, size=1000)):
        with pytest.raises(NotImplementedError):
            Word2Vec(**kw)


def test_similarity_and_lookup(test_pairs):
    m = _model(test_pairs)
    a, b = m.wv["TLE1"], m.wv["ALDOB"]
    ref = np.dot(a / np.linalg.norm(a), b / np.linalg.norm(b))
    assert m.wv.similarity("TLE1", "ALDOB") == pytest.approx(ref, rel=1e-6)
    assert "TLE1" in m.wv and "NOPE" not in m.wv
    assert m.wv[["TLE1", "ALDOB"]].shape == (2, 200)
    assert m.wv.most_similar("TLE1", topn=3)[0][0] != "TLE1"


def test_save_load_roundtrip(tmp_path, test_pairs):
    m = _model(test_pairs)
    m.syn1neg[:] = np.random.RandomState(0).rand(*m.syn1neg.shape).astype(np.float32)
    m.random.randint(0, 2 ** 24, size=7)
    f = str(tmp_path / "gene2vec_dim_200_iter_1")
    m.save(f)
    assert os.path.isfile(f)
    m2 = Word2Vec.load(f)
    assert m2.wv.index2word == m.wv.index2word
    assert list(m2.wv.vocab) == list(m.wv.vocab)
    assert np.array_equal(m2.wv.vectors, m.wv.vectors)
    assert np.array_equal(m2.syn1neg, m.syn1neg)
    assert m2.random.randint(0, 2 ** 24) == m.random.randint(0, 2 ** 24)
    assert m2.corpus_count == 40 and m2.iter == 1
    kv = KeyedVectors.load(f)  # src/generateMatrix.py:7-8 pattern
    assert np.array_equal(kv.wv["TLE1"], m.wv["TLE1"])


def test_generate_matrix_txt_format(tmp_path, test_pairs):
    m = _model(test_pairs)
    f = str(tmp_path / "m")
    m.save(f)
    out = gM.outputTxt(f)
    lines = open(out).read().split("\n")
    assert lines[-1] == "" and len(lines) == 80
    words = list(m.wv.vocab.keys())
    for line, w in zip(lines, words):
        name, rest = line.split("\t")
        assert name == w and rest.endswith(" ") and not rest.endswith("  ")
        vals = rest.split(" ")[:-1]
        assert len(vals) == 200
        assert vals == [str(np.float32(v)) for v in m.wv[w]]  # reference: str(elee) + " "
        # consumers: GGIPNN_util.py:9-11 / tsne_multi_core.py:12-14 read with split()
        parts = line.split()
        assert np.array_equal(np.asarray(parts[1:], dtype="float32"), m.wv[w])


@pytest.mark.parametrize("binary", [False, True])
def test_word2vec_format_roundtrip(tmp_path, test_pairs, binary):
    m = _model(test_pairs)
    f = str(tmp_path / "m_w2v.txt")
    m.wv.save_word2vec_format(f, binary=binary)
    raw = open(f, "rb").read()
    assert raw.startswith(b"79 200\n")
    kv = KeyedVectors.load_word2vec_format(f, binary=binary)
    assert kv.index2word == m.wv.index2word  # descending count order
    assert np.array_equal(kv.vectors, m.wv.vectors)
    if not binary:
        lines = raw.decode().split("\n")
        # evaluation_target_function.py:18-23 reads names with split(" ")
        names = [ln.split(" ")[0] for ln in lines[:-1] if len(ln.split(" ")) != 2]
        assert names == m.wv.index2word
        assert all(len(ln.split(" ")) == 201 for ln in lines[1:-1])


def test_word2vec_binary_reads_word2vec_c_newlines(tmp_path):
    f = tmp_path / "c.bin"
    rows = np.arange(6, dtype="<f4").reshape(2, 3)
    f.write_bytes(b"2 3\nA " + rows[0].tobytes() + b"\nBB " + rows[1].tobytes() + b"\n")
    kv = KeyedVectors.load_word2vec_format(str(f), binary=True)
    assert kv.index2word == ["A", "BB"] and np.array_equal(kv.vectors, rows)


def test_cli_ingest(tmp_path):
    d = tmp_path / "data"
    d.mkdir()
    (d / "a.txt").write_bytes("G1 G2\nG\xe9 G3\n\nG1 G3".encode("windows-1252"))
    (d / "b.txt").write_text("G4 G5\n")
    (d / "skip.csv").write_text("X Y\n")
    pairs = read_gene_pairs(str(d), "txt", random.Random(0))
    assert sorted(map(tuple, pairs)) == sorted(
        [("G1", "G2"), ("Gé", "G3"), (), ("G1", "G3"), ("G4", "G5")])


def _py_txt(words, rows):
    # src/generateMatrix.py:18-24 in pure Python
    return "".join(str(w) + "\t" + "".join(str(v) + " " for v in r) + "\n"
                   for w, r in zip(words, rows)).encode("utf-8")


def _py_w2v(words, rows):
    # [ext] save_word2vec_format(binary=False) row text
    return "".join(w + " " + " ".join(str(v) for v in r) + "\n"
                   for w, r in zip(words, rows)).encode("utf-8")


def test_native_row_formatter_matches_python_exporters():
    from gene2vec_amd import textio
    rng = np.random.default_rng(3)
    v = (rng.standard_normal((300, 37)) * rng.choice([1e-6, 0.3, 1e5], size=(300, 1)))
    v = v.astype(np.float32)
    v[0, :6] = [0.0, -0.0, np.inf, -np.inf, np.nan, 1e-4]
    words = [f"G{i}" for i in range(299)] + ["Gé"]
    order = rng.permutation(300)
    assert textio.format_rows(v, None, words, textio.TXT_MATRIX) == _py_txt(words, v)
    assert textio.format_rows(v, order, [words[i] for i in order], textio.TXT_W2V) == \
        _py_w2v([words[i] for i in order], v[order])
    assert textio.format_rows(v[:0], None, [], textio.TXT_W2V) == b""


def test_float32_formatter_on_random_bit_patterns():
    import ctypes as C

    from gene2vec_amd import _native as N
    bits = np.random.default_rng(5).integers(0, 2 ** 32, 300_000, dtype=np.uint64)
    x = bits.astype(np.uint32).view(np.float32)
    buf = np.empty(len(x) * 24, np.uint8)
    w = C.c_int64()
    N.check(N.lib().g2v_format_f32(N.ptr(x), len(x), N.ptr(buf), len(buf), C.byref(w)))
    got = bytes(buf[:w.value]).decode().split("\n")[:-1]
    assert got == x.astype(str).tolist()
