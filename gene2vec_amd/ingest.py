"""Native ingest of gene-pair files (§8(f) rank 3: tokenizer/vocab builder).

``read_corpus(paths)`` == the reference's
``for f in files: for line in open(f, encoding='windows-1252'): pairs.append(line.strip().split())``
(src/gene2vec.py:36-47) as CSR int32 ids (global first occurrence), with the
words decoded from windows-1252.  ``py_shuffle_perm(n, rng)`` applies exactly
the swaps ``rng.shuffle`` would (src/gene2vec.py:52,80) and leaves ``rng`` in
the same state, so native and Python ingest agree for a seeded generator.
"""
from __future__ import annotations

import ctypes as C
import os
import random

import numpy as np

from . import _native as N
from . import engine as E


class Corpus:
    def __init__(self, tokens, sent_off, words, counts):
        self.tokens = tokens        # int32[n_tokens], ids into words
        self.sent_off = sent_off    # int64[n_sent + 1]
        self.words = words          # list[str], first-occurrence order
        self.counts = counts        # int64[n_words]

    @property
    def n_sent(self):
        return len(self.sent_off) - 1

    def sentences(self):
        """materialise list[list[str]] (small corpora / tests)"""
        w = self.words
        t = self.tokens
        o = self.sent_off
        return [[w[i] for i in t[o[k]:o[k + 1]]] for k in range(self.n_sent)]

    def permuted(self, perm):
        perm = np.ascontiguousarray(perm, dtype=np.int64)
        tok = np.empty_like(self.tokens)
        off = np.empty_like(self.sent_off)
        N.check(N.lib().g2v_csr_permute(N.ptr(self.tokens), N.ptr(self.sent_off), self.n_sent,
                                        N.ptr(perm), N.ptr(tok), N.ptr(off)))
        return Corpus(tok, off, self.words, self.counts)

    def permute_(self, perm):
        """In-place form of ``permuted`` for the per-iteration reshuffle of
        src/gene2vec.py:80: the sentences are gathered into a spare pair of
        buffers kept from the previous call (no fresh 2 x 160 MB allocation
        and page faults per iteration at 20 M pairs), then the buffers swap."""
        perm = np.ascontiguousarray(perm, dtype=np.int64)
        spare = getattr(self, "_spare", None)
        if spare is None or spare[0].shape != self.tokens.shape:
            spare = (np.empty_like(self.tokens), np.empty_like(self.sent_off))
        tok, off = spare
        N.check(N.lib().g2v_csr_permute(N.ptr(self.tokens), N.ptr(self.sent_off), self.n_sent,
                                        N.ptr(perm), N.ptr(tok), N.ptr(off)))
        self._spare = (self.tokens, self.sent_off)
        self.tokens, self.sent_off = tok, off
        return self

    def vocab_raw_counts(self):
        """{word: count} in first-occurrence order of the CURRENT sentence order
        (what gensim's scan_vocab builds), plus ids remapped to that order."""
        counts, first = E.count_ids(self.tokens, len(self.words))
        present = np.nonzero(counts)[0]
        fo = present[np.argsort(first[present], kind="stable")]
        return {self.words[i]: int(counts[i]) for i in fo}


def read_corpus(paths, threads=None):
    L = N.lib()
    arr = (C.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
    h = C.c_void_p()
    rc = L.g2v_corpus_read(arr, len(paths), threads or min(16, os.cpu_count() or 1), C.byref(h))
    if rc != N.G2V_OK:
        raise UnicodeDecodeError("windows-1252", b"", 0, 1,
                                 "undefined byte or unreadable file (native ingest)") \
            if rc == N.G2V_EINVAL else N.G2VError(rc, "g2v_corpus_read")
    try:
        nt, ns, nw, nb = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        N.check(L.g2v_corpus_info(h, C.byref(nt), C.byref(ns), C.byref(nw), C.byref(nb)))
        tok = np.empty(nt.value, np.int32)
        off = np.empty(ns.value + 1, np.int64)
        counts = np.empty(nw.value, np.int64)
        wbytes = np.empty(max(nb.value, 1), np.uint8)
        woff = np.empty(nw.value + 1, np.int64)
        N.check(L.g2v_corpus_export(h, N.ptr(tok), N.ptr(off), N.ptr(counts), N.ptr(wbytes),
                                    N.ptr(woff)))
    finally:
        L.g2v_corpus_free(h)
    raw = wbytes.tobytes()
    words = [raw[woff[i]:woff[i + 1]].decode("windows-1252") for i in range(nw.value)]
    return Corpus(tok, off, words, counts)


def py_shuffle_perm(n, rng: random.Random, out=None):
    """permutation p with shuffled[i] = original[p[i]], consuming rng exactly
    as rng.shuffle(list_of_length_n) does (``out``: int64[n] buffer to reuse)."""
    version, internal, gauss = rng.getstate()
    state = np.array(internal[:624], dtype=np.uint32)
    pos = np.array([internal[624]], dtype=np.uint32)
    if out is None or out.shape != (n,) or out.dtype != np.int64:
        perm = np.empty(n, dtype=np.int64)
    else:
        perm = out
    N.check(N.lib().g2v_py_shuffle_range(N.ptr(state), N.ptr(pos), N.ptr(perm), n))
    rng.setstate((version, tuple(int(x) for x in state) + (int(pos[0]),), gauss))
    return perm


class ShufflePrefetch:
    """The next ``py_shuffle_perm(n, rng)``, computed on a host thread while the
    GPU trains the current iteration (src/gene2vec.py:80 reshuffles before every
    iteration >= 2; the Fisher-Yates swaps depend only on n and the Mersenne
    Twister state, not on the list's contents, so the permutation can be drawn
    one iteration early).  ``result()`` joins, hands ``rng`` the state
    ``rng.shuffle`` would have left and returns the permutation.  If anything
    drew from ``rng`` after ``start`` the prefetched permutation is discarded and
    recomputed from the live state, so the result is always what an in-place
    ``rng.shuffle`` at ``result()`` time gives.  ctypes releases the GIL for the
    native draw, so Python-side training and exports proceed meanwhile."""

    def __init__(self, n, rng: random.Random, out=None):
        import threading
        self.n, self.rng = n, rng
        self.snap = rng.getstate()
        version, internal, gauss = self.snap
        self.state = np.array(internal[:624], dtype=np.uint32)
        self.pos = np.array([internal[624]], dtype=np.uint32)
        if out is None or out.shape != (n,) or out.dtype != np.int64:
            out = np.empty(n, dtype=np.int64)
        self.perm = out
        self.rc = None
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    def _run(self):
        self.rc = N.lib().g2v_py_shuffle_range(N.ptr(self.state), N.ptr(self.pos),
                                               N.ptr(self.perm), self.n)
        if self.rc != N.G2V_OK:  # g2v_last_error is thread-local: read it here
            msg = N.lib().g2v_last_error()
            self.err = N.G2VError(self.rc, msg.decode() if msg else "")

    def result(self):
        self.th.join()
        if self.rc != N.G2V_OK:
            raise self.err
        if self.rng.getstate() != self.snap:  # rng was used meanwhile: redo from now
            return py_shuffle_perm(self.n, self.rng, out=self.perm)
        version, _, gauss = self.snap
        self.rng.setstate((version, tuple(int(x) for x in self.state) + (int(self.pos[0]),),
                           gauss))
        return self.perm
