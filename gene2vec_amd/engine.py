"""Thin Python owner of a ``g2v_ctx`` (libg2v.so) plus the host-side schedule.

``SGNSEngine`` is the device half of the Word2Vec model: it replaces the
arrays gensim keeps in the model object and the per-job Cython hook
(``train_batch_sg`` -> ``fast_sentence_sg_neg``) that ``src/gene2vec.py:70,87``
reach through ``Word2Vec(...)`` / ``model.train(...)``.

The schedule helpers restate gensim 3.4.0's job producer ([ext]
``BaseAny2VecModel._job_producer`` / ``_update_job_params``) vectorised:
``plan_jobs`` (greedy <= 10000 raw words per job, native), ``job_alphas``
(linear decay by pushed sentences, restarting every ``train()`` call) and
``job_seeds`` (``2**24*randint(2**24) + randint(2**24)`` from ``model.random``).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


# ---------------------------------------------------------------------------
# schedule (host)
# ---------------------------------------------------------------------------
def plan_jobs(sent_off=None, n_sent=None, sent_len=0, batch_words=N.BATCH_WORDS):
    """Job boundaries (sentence indices, int64[n_jobs+1]) of [ext] _job_producer."""
    L = N.lib()
    if sent_len > 0:
        assert n_sent is not None
        so = None
    else:
        so = np.ascontiguousarray(sent_off, dtype=np.int64)
        n_sent = len(so) - 1
    nj = C.c_int64(0)
    N.check(L.g2v_plan_jobs(N.ptr(so), n_sent, sent_len, batch_words, None, 0, C.byref(nj)))
    out = np.zeros(nj.value + 1, dtype=np.int64)
    N.check(L.g2v_plan_jobs(N.ptr(so), n_sent, sent_len, batch_words, N.ptr(out), len(out),
                            C.byref(nj)))
    return out


def job_alphas(job_sent, total_examples, alpha=0.025, min_alpha=0.0001, cur_epoch=0, epochs=1):
    """alpha per job, float64, in gensim's arithmetic order ([ext] _update_job_params)."""
    job_sent = np.asarray(job_sent, dtype=np.int64)
    n = len(job_sent) - 1
    out = np.empty(n, dtype=np.float64)
    if n == 0:
        return out
    out[0] = alpha - (alpha - min_alpha) * float(cur_epoch) / epochs
    pushed = (job_sent[1:n] - job_sent[0]).astype(np.float64)
    progress = (cur_epoch + 1.0 * pushed / total_examples) / epochs
    nxt = alpha - (alpha - min_alpha) * progress
    out[1:] = np.maximum(min_alpha, nxt)
    return out


def job_seeds(random_state: np.random.RandomState, n_jobs):
    """next_random per job: 2**24 * randint(0, 2**24) + randint(0, 2**24).
    (randint(0, window=1, n) for reduced_windows draws nothing.)"""
    r = random_state.randint(0, 2 ** 24, size=2 * n_jobs).astype(np.uint64)
    return (r[0::2] << np.uint64(24)) + r[1::2]


def seeded_vectors(seeds, dim):
    """[ext] seeded_vector for every row, native MT19937 (bit-identical to numpy)."""
    seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
    out = np.empty((len(seeds), dim), dtype=np.float32)
    N.check(N.lib().g2v_seeded_vectors(N.ptr(seeds), len(seeds), dim, N.ptr(out)))
    return out


def permute_items8(device, src_ptr, dst_ptr, n_items, first, count, seed, stream=None):
    """g2v_permute_items8: dst[i] = src[p(first + i)] for a device-resident
    corpus of 8-byte items (int32 pairs), p a keyed permutation of [0, n_items)
    (the per-iteration reshuffle of src/gene2vec.py:80 done in HBM).  Enqueued
    on ``stream`` (a HIP stream handle, None = null stream)."""
    N.check(N.lib().g2v_permute_items8(int(device), C.c_void_p(src_ptr), C.c_void_p(dst_ptr),
                                       int(n_items), int(first), int(count),
                                       int(seed) % 2 ** 64,
                                       C.c_void_p(stream) if stream else None))


def first_occurrence_perm8(device, items_ptr, n_items, seed, n_ids, first_ptr, stream=None):
    """g2v_first_occurrence_perm8: int64 first[n_ids] (device) = each id's first
    token position in the order permute_items8(seed) gives, -1 if absent."""
    N.check(N.lib().g2v_first_occurrence_perm8(int(device), C.c_void_p(items_ptr), int(n_items),
                                               int(seed) % 2 ** 64, int(n_ids),
                                               C.c_void_p(first_ptr),
                                               C.c_void_p(stream) if stream else None))


def kept_token_share(counts, sample):
    """each row's share of the tokens downsampling keeps ([ext] prepare_vocab's
    sample_int as a probability, Appendix A.2; the p_tok(r) g2v_set_vocab
    derives the Hogwild budgets and the tail-store rows from)"""
    v = np.asarray(counts, dtype=np.float64)
    total = v.sum()
    if 0.0 < sample < 1.0:
        thr = sample * total
    elif sample >= 1.0:
        thr = float(int(sample * (3.0 + np.sqrt(5.0)) / 2.0))
    else:
        thr = total
    kept = v * np.minimum(1.0, (np.sqrt(v / thr) + 1.0) * (thr / v))
    return kept / kept.sum()


TAIL_COLLISION = 0.15  # kTailCollision in g2v_api.hip


def tail_store_row(counts, sample, negative, waves, ns_exponent=0.75):
    """first syn1neg row the auto cold-row stores (G2V_OPT_TAIL_STORE -1,
    DESIGN.md 5e) write with plain stores: the first row r from which every
    row r' >= r has waves x u(r') <= TAIL_COLLISION, u = K p_neg + p_tok (a
    suffix max, so a negative ns_exponent or unsorted counts, which put hot
    rows late, store nothing after them); len(counts) = none"""
    v = np.asarray(counts, dtype=np.float64)
    pn = v ** ns_exponent
    u = negative * pn / pn.sum() + kept_token_share(v, sample)
    suffix = np.maximum.accumulate(u[::-1])[::-1]
    over = np.nonzero(waves * suffix > TAIL_COLLISION)[0]
    return int(over[-1]) + 1 if len(over) else 0


def count_ids(ids, V):
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    counts = np.zeros(V, dtype=np.int64)
    first = np.zeros(V, dtype=np.int64)
    N.check(N.lib().g2v_count_ids(N.ptr(ids), len(ids), V, N.ptr(counts), N.ptr(first)))
    return counts, first


# ---------------------------------------------------------------------------
# device context
# ---------------------------------------------------------------------------
class LocalGroup:
    """g2v_local_group: ``nranks`` replicas of one process on one GPU, each
    engine driven by its own thread, merging through a device sum in place of
    ncclAllReduce (the multi-replica merge path on a one-GPU box, where RCCL
    refuses two ranks).  Destroy it after its engines' last collective."""

    def __init__(self, nranks, timeout_s=0):
        h = C.c_void_p()
        N.check(N.lib().g2v_local_group_create(int(nranks), int(timeout_s), C.byref(h)))
        self._h = h
        self.nranks = nranks

    def close(self):
        if getattr(self, "_h", None):
            N.lib().g2v_local_group_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class SGNSEngine:
    """One g2v_ctx on one GPU (one host thread drives it)."""

    def __init__(self, vocab_size, vector_size, negative=5, window=1, device=0):
        self._lib = N.lib()
        h = C.c_void_p()
        N.check(self._lib.g2v_create(device, vocab_size, vector_size, negative, window,
                                     C.byref(h)))
        self._h = h
        self.V, self.D, self.K, self.window, self.device = (vocab_size, vector_size, negative,
                                                            window, device)
        ld = C.c_int64()
        N.check(self._lib.g2v_row_stride(h, C.byref(ld)))
        self.ld = ld.value
        self._keep = []  # device buffers borrowed by the context

    # -- lifecycle -----------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._lib.g2v_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, key, value):
        N.check(self._lib.g2v_set_option(self._h, key, int(value)))

    def get_option(self, key):
        v = C.c_int64()
        N.check(self._lib.g2v_get_option(self._h, key, C.byref(v)))
        return v.value

    def set_stream(self, stream_handle):
        N.check(self._lib.g2v_set_stream(self._h, C.c_void_p(stream_handle or 0)))

    # -- vocabulary ------------------------------------------------------------
    def set_vocab(self, counts, sample=1e-3, ns_exponent=0.75, return_tables=False):
        counts = np.ascontiguousarray(counts, dtype=np.int64)
        assert len(counts) == self.V
        cum = si = None
        if return_tables:
            cum = np.zeros(self.V, dtype=np.uint32)
            si = np.zeros(self.V, dtype=np.uint32)
        N.check(self._lib.g2v_set_vocab(self._h, N.ptr(counts), float(sample), float(ns_exponent),
                                        N.ptr(cum), N.ptr(si)))
        return cum, si

    # -- weights -----------------------------------------------------------------
    def set_weights(self, syn0=None, syn1neg=None, lockf=None):
        def prep(a, shape):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=np.float32)
            assert a.shape == shape, (a.shape, shape)
            return a
        syn0 = prep(syn0, (self.V, self.D))
        syn1neg = prep(syn1neg, (self.V, self.D))
        lockf = prep(lockf, (self.V,))
        N.check(self._lib.g2v_set_weights(self._h, N.ptr(syn0), N.ptr(syn1neg), N.ptr(lockf)))

    def get_weights(self):
        s0 = np.empty((self.V, self.D), dtype=np.float32)
        s1 = np.empty((self.V, self.D), dtype=np.float32)
        N.check(self._lib.g2v_get_weights(self._h, N.ptr(s0), N.ptr(s1)))
        return s0, s1

    def bind_tables(self, syn0_ptr, syn1neg_ptr, ld, keepalive=None):
        """Borrow device tables (e.g. torch tensors' data_ptr()); keepalive is
        held until unbound."""
        N.check(self._lib.g2v_bind_tables(self._h, C.c_void_p(syn0_ptr), C.c_void_p(syn1neg_ptr),
                                          ld))
        self.ld = ld if syn0_ptr else self.ld
        self._tables_keep = keepalive

    # -- corpus ----------------------------------------------------------------
    def set_corpus(self, tokens, sent_off=None, sent_len=0):
        tokens = np.ascontiguousarray(tokens, dtype=np.int32)
        so = None if sent_len > 0 else np.ascontiguousarray(sent_off, dtype=np.int64)
        n_sent = len(tokens) // sent_len if sent_len > 0 else len(so) - 1
        N.check(self._lib.g2v_set_corpus(self._h, N.ptr(tokens), len(tokens), N.ptr(so), n_sent,
                                         sent_len, 0))
        self.n_sent = n_sent

    def set_corpus_device(self, tok_ptr, n_tokens, off_ptr=None, n_sent=None, sent_len=0,
                          keepalive=None):
        if sent_len > 0:
            n_sent = n_tokens // sent_len
        N.check(self._lib.g2v_set_corpus(self._h, C.c_void_p(tok_ptr), n_tokens,
                                         C.c_void_p(off_ptr or 0), n_sent, sent_len,
                                         N.CORPUS_DEVICE))
        self._corpus_keep = keepalive
        self.n_sent = n_sent

    # -- training ----------------------------------------------------------------
    def train(self, job_sent, job_alpha, job_seed, mode=N.MODE_HOGWILD, timing=False,
              compute_loss=False):
        job_sent = np.ascontiguousarray(job_sent, dtype=np.int64)
        job_alpha = np.ascontiguousarray(job_alpha, dtype=np.float32)
        job_seed = np.ascontiguousarray(job_seed, dtype=np.uint64)
        n = len(job_sent) - 1
        assert len(job_alpha) == n and len(job_seed) == n
        flags = (mode | (N.FLAG_TIMING if timing else 0)
                 | (N.FLAG_COMPUTE_LOSS if compute_loss else 0))
        self._check_coll(self._lib.g2v_train(self._h, N.ptr(job_sent), N.ptr(job_alpha),
                                             N.ptr(job_seed), n, flags))

    def step_explicit(self, center, inp, negs, alpha, mode=N.MODE_SEQUENTIAL, timing=False,
                      compute_loss=False):
        center = np.ascontiguousarray(center, dtype=np.int32)
        inp = np.ascontiguousarray(inp, dtype=np.int32)
        negs = np.ascontiguousarray(negs, dtype=np.int32).reshape(len(center), self.K)
        flags = (mode | (N.FLAG_TIMING if timing else 0)
                 | (N.FLAG_COMPUTE_LOSS if compute_loss else 0))
        N.check(self._lib.g2v_sgns_step_explicit(self._h, N.ptr(center), N.ptr(inp), N.ptr(negs),
                                                 len(center), C.c_float(alpha), flags))

    def debug_sample(self, job_sent, job_seed):
        job_sent = np.ascontiguousarray(job_sent, dtype=np.int64)
        job_seed = np.ascontiguousarray(job_seed, dtype=np.uint64)
        n = len(job_sent) - 1
        cnt = C.c_int64(0)
        N.check(self._lib.g2v_debug_sample(self._h, N.ptr(job_sent), N.ptr(job_seed), n, None, 0,
                                           C.byref(cnt)))
        out = np.zeros((max(cnt.value, 1), self.K + 2), dtype=np.int32)
        N.check(self._lib.g2v_debug_sample(self._h, N.ptr(job_sent), N.ptr(job_seed), n,
                                           N.ptr(out), len(out), C.byref(cnt)))
        return out[:cnt.value]

    def reset_loss(self):
        N.check(self._lib.g2v_reset_loss(self._h))

    # -- replica averaging (multi-GPU) -----------------------------
    @staticmethod
    def comm_unique_id():
        """128-byte RCCL unique id (rank 0 draws it, every rank receives it)."""
        buf = (C.c_char * N.UNIQUE_ID_BYTES)()
        N.check(N.lib().g2v_comm_unique_id(buf, N.UNIQUE_ID_BYTES))
        return bytes(buf)

    def comm_init(self, unique_id, nranks, rank):
        self.host_collective = None
        buf = (C.c_char * N.UNIQUE_ID_BYTES).from_buffer_copy(unique_id)
        N.check(self._lib.g2v_comm_init(self._h, buf, nranks, rank))

    def average(self, rule=N.MERGE_TOUCH):
        self._check_coll(self._lib.g2v_average(self._h, rule))

    def merge_snapshot(self):
        N.check(self._lib.g2v_merge_snapshot(self._h))

    @staticmethod
    def average_local(engines, rule=N.MERGE_TOUCH):
        arr = (C.c_void_p * len(engines))(*[e._h.value for e in engines])
        N.check(N.lib().g2v_average_local(arr, len(engines), rule))

    def comm_init_local(self, group, rank):
        """Join an in-process replica group (g2v_comm_init_local; collective:
        every rank calls it from its own thread)."""
        N.check(self._lib.g2v_comm_init_local(self._h, group._h, rank))
        self._group = group

    def comm_init_host(self, collective, nranks, rank):
        """Merge over a host collective (g2v_comm_init_host).  ``collective(op,
        buf)`` performs op (N.COLL_SUM / N.COLL_BCAST0) in place on the float32
        numpy array ``buf`` across the ranks.  An exception inside it fails the
        libg2v call (G2V_ECOMM) and is re-raised from it."""
        def tramp(_user, op, buf, count):
            try:
                collective(op, np.ctypeslib.as_array(buf, shape=(count,)))
                return 0
            except BaseException as e:  # noqa: BLE001 - crosses the C ABI
                self._coll_error = e
                return 1
        self._coll_error = None
        self._coll_fn = N.COLLECTIVE_FN(tramp)  # kept alive with the engine
        # ReplicaTrainer's failure protocol reads it (distributed.HostCollective)
        self.host_collective = collective
        self._check_coll(self._lib.g2v_comm_init_host(self._h, self._coll_fn, None, nranks, rank))

    def _check_coll(self, rc):
        err, self._coll_error = getattr(self, "_coll_error", None), None
        if rc != N.G2V_OK and err is not None:
            raise err
        return N.check(rc)

    def comm_abort(self):
        N.check(self._lib.g2v_comm_abort(self._h))

    def sync(self):
        N.check(self._lib.g2v_sync(self._h))

    def read_stats(self):
        st = N.Stats()
        N.check(self._lib.g2v_read_stats(self._h, C.byref(st)))
        return st.as_dict()
