"""Native ingest == the reference's Python ingest (src/gene2vec.py:36-52)."""
import random

import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd.ingest import ShufflePipeline, count_lines, py_shuffle_perm, read_corpus


def _py_read(paths):
    out = []
    for p in paths:
        with open(p, "r", encoding="windows-1252") as f:
            for line in f:
                out.append(line.strip().split())
    return out


@pytest.fixture
def files(tmp_path):
    rng = np.random.RandomState(0)
    genes = ["TP53", "G\xe9ne", "ABC-1", "X", "hla_a"] + [f"G{i}" for i in range(300)]
    seps = [" ", "\t", "  ", "\xa0", "\x1c", " \x0b "]
    ends = ["\n", "\r\n", "\r"]
    paths = []
    for k in range(3):
        lines = []
        for _ in range(2000):
            n = rng.choice([0, 1, 2, 2, 2, 4])
            toks = [genes[int(i)] for i in rng.randint(0, len(genes), n)]
            sep = seps[rng.randint(len(seps))]
            lines.append((" " if rng.rand() < 0.1 else "") + sep.join(toks) +
                         ends[rng.randint(len(ends))])
        text = "".join(lines)
        if k == 1:
            text = text.rstrip("\r\n")  # no trailing newline
        p = tmp_path / f"f{k}.txt"
        p.write_bytes(text.encode("windows-1252"))
        paths.append(str(p))
    (tmp_path / "empty.txt").write_bytes(b"")
    paths.append(str(tmp_path / "empty.txt"))
    return paths


def test_native_reader_matches_python(files):
    ref = _py_read(files)
    for threads in (1, 4):
        c = read_corpus(files, threads=threads)
        assert c.n_sent == len(ref)
        assert c.sentences() == ref
        words_fo = []
        seen = set()
        for s in ref:
            for w in s:
                if w not in seen:
                    seen.add(w)
                    words_fo.append(w)
        assert c.words == words_fo
        assert int(c.counts.sum()) == sum(len(s) for s in ref)
        # the newline count the CLI starts its first shuffle from
        assert count_lines(files, threads=threads) == len(ref)


@pytest.mark.parametrize("text", [b"", b"A B", b"A B\n", b"A B\r\n\r\n", b"\r\r\n\n",
                                  b"A B\rC D", b"A B\n   ", b"\n", b"A\r", b"A B\r\nC"])
def test_count_lines_equals_reader(tmp_path, text):
    """universal newlines at the edges: lone CR, CRLF, unterminated or
    whitespace-only last line, empty file"""
    p = tmp_path / "t.txt"
    p.write_bytes(text)
    assert count_lines([str(p)], threads=2) == read_corpus([str(p)]).n_sent == len(_py_read([p]))


def test_pair_files_keep_offsets_implicit(tmp_path):
    p = tmp_path / "pairs.txt"
    p.write_text("A B\nC D\nB A\n")
    c = read_corpus([str(p)])
    assert c._sent_off is None and c.pairs_only and c.n_sent == 3
    np.testing.assert_array_equal(c.sent_off, [0, 2, 4, 6])
    assert c.sentences() == [["A", "B"], ["C", "D"], ["B", "A"]]
    q = tmp_path / "ragged.txt"
    q.write_text("A B\nC\n")
    r = read_corpus([str(q)])
    assert r._sent_off is not None and not r.pairs_only


def test_undefined_cp1252_byte_raises(tmp_path):
    p = tmp_path / "bad.txt"
    p.write_bytes(b"A B\nC \x81D\n")
    with pytest.raises(UnicodeDecodeError):
        open(p, encoding="windows-1252").read()
    with pytest.raises(UnicodeDecodeError):
        read_corpus([str(p)])


@pytest.mark.parametrize("n", [0, 1, 2, 10, 1000, 123457])
def test_py_shuffle_perm_bit_compatible(n):
    r1, r2 = random.Random(12345), random.Random(12345)
    data = list(range(n))
    r1.shuffle(data)
    perm = py_shuffle_perm(n, r2)
    assert perm.tolist() == data
    assert r1.getstate() == r2.getstate()
    assert r1.random() == r2.random()


@pytest.mark.parametrize("n", [0, 1, 2, 1000, 123457])
def test_py_shuffle_skip_leaves_shuffle_state(n):
    """g2v_py_shuffle_skip replays shuffle(n)'s draws without the swaps"""
    r1 = random.Random(2024)
    r1.shuffle(list(range(n)))
    st = np.array(random.Random(2024).getstate()[1][:624], dtype=np.uint32)
    pos = np.array([random.Random(2024).getstate()[1][624]], dtype=np.uint32)
    N.check(N.lib().g2v_py_shuffle_skip(N.ptr(st), N.ptr(pos), n))
    assert tuple(int(x) for x in st) + (int(pos[0]),) == r1.getstate()[1]


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_shuffle_pipeline_equals_in_place_shuffles(depth):
    """gene2vec.py's shuffle (:52) and per-iteration reshuffles (:80) drawn
    ahead on host threads (ShufflePipeline) == successive rng.shuffle calls."""
    n = 50021
    r1, r2 = random.Random(99), random.Random(99)
    data = list(range(n))
    cur = np.arange(n)
    pipe = ShufflePipeline(n, r2, 5, depth=depth)
    for _ in range(5):
        r1.shuffle(data)
        perm = pipe.next()
        cur = cur[perm]
        pipe.release(perm)
        assert cur.tolist() == data
        assert r1.getstate() == r2.getstate()
    with pytest.raises(IndexError):
        pipe.next()


def test_shuffle_pipeline_dropped_when_rng_drawn_meanwhile():
    r1, r2 = random.Random(5), random.Random(5)
    pipe = ShufflePipeline(1000, r2, 3)
    data = list(range(1000))
    r1.shuffle(data)
    assert pipe.next().tolist() == data
    r1.random()
    r2.random()  # a draw between two shuffles: the pipeline is stale
    for _ in range(2):
        data = list(range(1000))
        r1.shuffle(data)
        assert pipe.next().tolist() == data
    assert r1.getstate() == r2.getstate()


def test_permuted_corpus_and_vocab(files):
    ref = _py_read(files)
    c = read_corpus(files)
    r1, r2 = random.Random(7), random.Random(7)
    r1.shuffle(ref)
    c2 = c.permuted(py_shuffle_perm(c.n_sent, r2))
    assert c2.sentences() == ref
    raw = {}
    for s in ref:
        for w in s:
            raw[w] = raw.get(w, 0) + 1
    assert list(c2.vocab_raw_counts().items()) == list(raw.items())


def test_native_reader_long_words_table_growth_and_chunks(tmp_path):
    """words longer than a table slot's 16-byte prefix (and sharing it), more
    distinct words than the initial table holds, and a file larger than one
    16 MiB tokenizer chunk (ids must stay in global first-occurrence order)."""
    rng = np.random.RandomState(1)
    long_words = [f"ENSG0000000000{i:06d}|LONGNAME" for i in range(50)]
    many = [f"w{i}" for i in range(70000)]
    lines = []
    for i in range(70000):
        lines.append(f"{many[i]} {long_words[i % 50]}\n")
    big = "".join(lines)
    filler = "".join(f"{many[int(a)]} {many[int(b)]}\n"
                     for a, b in rng.randint(0, 70000, (1_300_000, 2)))
    p1, p2 = tmp_path / "a.txt", tmp_path / "b.txt"
    p1.write_bytes((big + filler).encode("windows-1252"))
    p2.write_bytes(("".join(f"{w} x\n" for w in long_words[::-1])).encode("windows-1252"))
    assert p1.stat().st_size > (16 << 20)
    ref = _py_read([str(p1), str(p2)])
    for threads in (1, 3):
        c = read_corpus([str(p1), str(p2)], threads=threads)
        assert c.n_sent == len(ref)
        assert c.sentences()[:1000] == ref[:1000]
        assert c.sentences()[-60:] == ref[-60:]
        seen, fo = set(), []
        for s in ref:
            for w in s:
                if w not in seen:
                    seen.add(w)
                    fo.append(w)
        assert c.words == fo
        idx = {w: i for i, w in enumerate(fo)}
        flat = np.array([idx[w] for s in ref for w in s], np.int32)
        assert np.array_equal(c.tokens, flat)


def test_pairs_permute_equals_csr_permute():
    """all-pairs corpora take the 8-byte pair gather (g2v_pairs_permute);
    the result equals the CSR gather, offsets untouched"""
    from gene2vec_amd.ingest import Corpus
    rs = np.random.RandomState(1)
    n = 200003
    tok = rs.randint(0, 5000, 2 * n).astype(np.int32)
    off = np.arange(0, 2 * n + 1, 2, dtype=np.int64)
    perm = py_shuffle_perm(n, random.Random(3))
    a = Corpus(tok.copy(), off.copy(), [], None)
    assert a.pairs_only
    a.permute_(perm)
    a.permute_(perm)  # second call reuses the spare buffer
    ref = tok.reshape(n, 2)[perm][perm].ravel()
    np.testing.assert_array_equal(a.tokens, ref)
    np.testing.assert_array_equal(a.sent_off, off)
    mixed = Corpus(np.arange(5, dtype=np.int32), np.array([0, 2, 5], dtype=np.int64), [], None)
    assert not mixed.pairs_only
    mixed.permute_(np.array([1, 0]))
    np.testing.assert_array_equal(mixed.tokens, [2, 3, 4, 0, 1])
    np.testing.assert_array_equal(mixed.sent_off, [0, 3, 5])
    with pytest.raises(N.G2VError):
        Corpus(tok.copy(), off.copy(), [], None).permute_(np.full(n, n, dtype=np.int64))


def test_shuffle_pipeline_close_wait_joins_threads():
    pipe = ShufflePipeline(100003, random.Random(1), 4, depth=2)
    pipe.next()
    pipe.close(wait=True)
    assert not pipe.driver.is_alive()
    assert all(not t.is_alive() for t in pipe.workers)


def test_adopt_vocab_ids_renumbers_corpus_once():
    """gene2vec.py renumbers the corpus into the model's vocabulary order at
    iteration 1 so later iterations skip the token remap"""
    from gene2vec_amd.gene2vec import _adopt_vocab_ids
    from gene2vec_amd.ingest import Corpus
    c = Corpus(np.array([0, 1, 2, 0], np.int32), np.array([0, 2, 4], np.int64),
               ["b", "a", "c"], np.array([2, 1, 1], np.int64))
    ids = np.array([1, 0, 2], np.int32)  # corpus id -> model index
    tok = ids[c.tokens]
    _adopt_vocab_ids(c, ids, tok)
    assert c.words == ["a", "b", "c"]
    np.testing.assert_array_equal(c.tokens, [1, 0, 2, 1])
    np.testing.assert_array_equal(c.counts, [1, 2, 1])
    assert c.sentences() == [["b", "a"], ["c", "b"]]
    # a word outside the vocabulary (-1) keeps the corpus numbering
    d = Corpus(np.array([0, 1], np.int32), np.array([0, 2], np.int64), ["x", "y"],
               np.array([1, 1], np.int64))
    _adopt_vocab_ids(d, np.array([0, -1], np.int32), np.array([0, -1], np.int32))
    assert d.words == ["x", "y"]
    np.testing.assert_array_equal(d.tokens, [0, 1])
