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
    def __init__(self, tokens, sent_off, words, counts, sent_len=0):
        self.tokens = tokens        # int32[n_tokens], ids into words
        # int64[n_sent + 1]; None when every sentence has sent_len tokens (pair
        # files: the 8-byte offset per pair is never materialised)
        self._sent_off = sent_off
        self._sent_len = int(sent_len)
        self.words = words          # list[str], first-occurrence order
        self.counts = counts        # int64[n_words]

    @property
    def sent_off(self):
        if self._sent_off is None:
            n = len(self.tokens) // self._sent_len
            self._sent_off = np.arange(0, self._sent_len * n + 1, self._sent_len, dtype=np.int64)
        return self._sent_off

    @sent_off.setter
    def sent_off(self, v):
        self._sent_off = v

    @property
    def n_sent(self):
        if self._sent_off is None:
            return len(self.tokens) // self._sent_len
        return len(self._sent_off) - 1

    @property
    def pairs_only(self):
        """every sentence is exactly 2 tokens (the pair generator's output);
        checked once, permutations keep it"""
        if getattr(self, "_pairs_only", None) is None:
            if self._sent_off is None:
                self._pairs_only = self._sent_len == 2
            else:
                self._pairs_only = bool(np.array_equal(
                    self._sent_off, np.arange(0, 2 * self.n_sent + 1, 2, dtype=np.int64)))
        return self._pairs_only

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
        if self.pairs_only:
            if len(perm) != self.n_sent:
                raise ValueError("permutation length != number of sentences")
            spare = getattr(self, "_spare_tok", None)
            if spare is None or spare.shape != self.tokens.shape:
                spare = np.empty_like(self.tokens)
            N.check(N.lib().g2v_pairs_permute(N.ptr(self.tokens), self.n_sent, N.ptr(perm),
                                              N.ptr(spare)))
            self._spare_tok, self.tokens = self.tokens, spare
            return self
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


def count_lines(paths, threads=None):
    """sentences ``read_corpus(paths)`` will return (g2v_count_lines)"""
    arr = (C.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
    n = C.c_int64()
    rc = N.lib().g2v_count_lines(arr, len(paths), threads or min(16, os.cpu_count() or 1),
                                 C.byref(n))
    if rc != N.G2V_OK:
        raise N.G2VError(rc, "g2v_count_lines")
    return n.value


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
        sl = C.c_int64()
        N.check(L.g2v_corpus_sent_len(h, C.byref(sl)))
        tok = np.empty(nt.value, np.int32)
        # fixed-length sentences (pair files): offsets stay implicit
        off = None if sl.value == 2 else np.empty(ns.value + 1, np.int64)
        counts = np.empty(nw.value, np.int64)
        wbytes = np.empty(max(nb.value, 1), np.uint8)
        woff = np.empty(nw.value + 1, np.int64)
        N.check(L.g2v_corpus_export(h, N.ptr(tok), N.ptr(off) if off is not None else None,
                                    N.ptr(counts), N.ptr(wbytes), N.ptr(woff)))
    finally:
        L.g2v_corpus_free(h)
    raw = wbytes.tobytes()
    words = [raw[woff[i]:woff[i + 1]].decode("windows-1252") for i in range(nw.value)]
    return Corpus(tok, off, words, counts, sent_len=2 if off is None else 0)


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


class ShufflePipeline:
    """The ``count`` successive ``py_shuffle_perm(n, rng)`` of the CLI
    (src/gene2vec.py:52 once, :80 before every iteration >= 2), drawn ahead
    on host threads while the GPU trains.  Fisher-Yates swaps depend only on n
    and the Mersenne Twister state, never on the list, so shuffle k+1's state
    is known as soon as shuffle k's draws are replayed (``g2v_py_shuffle_skip``,
    no swaps): a driver thread replays the draws and starts each shuffle's
    memory-bound swaps on a thread of its own, at most ``depth`` permutations
    alive at once (``release`` hands one back).  ``next()`` returns the next
    permutation and leaves ``rng`` in the state ``rng.shuffle`` would; if
    anything else drew from ``rng`` meanwhile the pipeline is dropped and the
    permutation recomputed from the live state, so the results always equal
    in-place ``rng.shuffle`` calls.  ctypes releases the GIL for the native
    calls."""

    def __init__(self, n, rng: random.Random, count, depth=2):
        import queue
        import threading
        self.n, self.rng, self.count = n, rng, count
        self.expect = rng.getstate()
        version, internal, gauss = self.expect
        self.meta = (version, gauss)
        self.cond = threading.Condition()
        self.perm, self.after, self.err = {}, {}, None
        self.k = 0
        self.dead = False
        self.workers = []
        self.free = queue.Queue()
        for _ in range(depth):
            self.free.put(None)
        st = np.array(internal[:624], dtype=np.uint32)
        pos = np.array([internal[624]], dtype=np.uint32)
        self.driver = threading.Thread(target=self._drive, args=(st, pos), daemon=True)
        self.driver.start()

    def _fail(self, rc):
        msg = N.lib().g2v_last_error()  # thread-local: read it on this thread
        with self.cond:
            self.err = N.G2VError(rc, msg.decode() if msg else "")
            self.cond.notify_all()

    def _drive(self, st, pos):
        import threading
        L = N.lib()
        for k in range(self.count):
            buf = self.free.get()
            if self.dead:
                return
            th = threading.Thread(target=self._swaps, args=(k, st.copy(), pos.copy(), buf),
                                  daemon=True)
            self.workers.append(th)
            th.start()
            rc = L.g2v_py_shuffle_skip(N.ptr(st), N.ptr(pos), self.n)
            if rc != N.G2V_OK:
                return self._fail(rc)
            with self.cond:
                self.after[k] = (st.copy(), int(pos[0]))
                self.cond.notify_all()

    def _swaps(self, k, st, pos, buf):
        perm = buf if buf is not None else np.empty(self.n, dtype=np.int64)
        rc = N.lib().g2v_py_shuffle_range(N.ptr(st), N.ptr(pos), N.ptr(perm), self.n)
        if rc != N.G2V_OK:
            return self._fail(rc)
        with self.cond:
            self.perm[k] = perm
            self.cond.notify_all()

    def next(self):
        if self.k >= self.count:
            raise IndexError("ShufflePipeline: all permutations consumed")
        k = self.k
        self.k += 1
        if self.dead or self.rng.getstate() != self.expect:
            self.close()
            return py_shuffle_perm(self.n, self.rng)
        with self.cond:
            self.cond.wait_for(lambda: self.err is not None or (k in self.perm and k in self.after))
            if self.err is not None:
                raise self.err
            perm = self.perm.pop(k)
            st, pos = self.after.pop(k)
        version, gauss = self.meta
        self.rng.setstate((version, tuple(int(x) for x in st) + (pos,), gauss))
        self.expect = self.rng.getstate()
        return perm

    def release(self, perm):
        """perm (from next()) is no longer needed: its buffer serves a later shuffle"""
        if not self.dead:
            self.free.put(perm)

    def close(self, wait=False):
        """stop drawing ahead; ``wait``: also join the threads (no native call
        left running when the interpreter shuts down after an error)"""
        self.dead = True
        self.free.put(None)  # wakes a driver blocked on a buffer
        if wait:
            self.driver.join()
            for th in list(self.workers):
                th.join()
