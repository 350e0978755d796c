"""ctypes binding of ``oracle/build/liboracle.so`` -- TEST INFRASTRUCTURE ONLY.

Builds the library on first use when it is missing (``make -C oracle``).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or (
                os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "sgns_oracle.c"))):
            build()
        _lib = C.CDLL(_LIB_PATH)
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def make_cum_table(counts, power=0.75):
    counts = np.ascontiguousarray(counts, dtype=np.int64)
    out = np.zeros(len(counts), dtype=np.uint32)
    lib().orc_make_cum_table(_p(counts), C.c_int32(len(counts)), C.c_double(power), _p(out))
    return out


def sample_int(counts, sample):
    counts = np.ascontiguousarray(counts, dtype=np.int64)
    out = np.zeros(len(counts), dtype=np.uint64)
    lib().orc_sample_int(_p(counts), C.c_int32(len(counts)), C.c_double(sample), _p(out))
    return out


def exp_table():
    out = np.zeros(1000, dtype=np.float32)
    lib().orc_exp_table(_p(out))
    return out


def log_table():
    out = np.zeros(1000, dtype=np.float32)
    lib().orc_log_table(_p(out))
    return out


def _u32_sample(sample_int):
    return np.minimum(np.asarray(sample_int, dtype=np.uint64), 0xFFFFFFFF).astype(np.uint32)


def train(tok, sent_off, job_sent, job_alpha, job_seed, sample_int, sample_on, cum, syn0,
          syn1neg, lockf, K, nthreads=0, loss=None, ld=None, loss_exact=None):
    """In-place training of syn0/syn1neg ([V][D] float32 C-order).
    nthreads == 0: sequential (workers=1 order); > 0: OpenMP Hogwild.
    loss: None, or a float32 array of one element holding gensim's running
    training loss (compute_loss=True), continued in place (sequential only);
    loss_exact: None, or a float64 array of one element: the same terms
    added in double (sequential only).
    ld: row stride in floats for the training copy (Hogwild: a multiple of 16
    keeps each row on cache lines of its own, so threads updating neighbouring
    hot rows do not falsely share lines); None = D, in place."""
    V, D = syn0.shape
    if ld is not None and ld != D:
        assert ld >= D
        p0 = np.zeros((V, ld), np.float32)
        p1 = np.zeros((V, ld), np.float32)
        p0[:, :D] = syn0
        p1[:, :D] = syn1neg
        st = _train(tok, sent_off, job_sent, job_alpha, job_seed, sample_int, sample_on, cum,
                    p0, p1, lockf, K, nthreads, loss, ld, D, loss_exact)
        syn0[:] = p0[:, :D]
        syn1neg[:] = p1[:, :D]
        return st
    return _train(tok, sent_off, job_sent, job_alpha, job_seed, sample_int, sample_on, cum,
                  syn0, syn1neg, lockf, K, nthreads, loss, D, D, loss_exact)


def _train(tok, sent_off, job_sent, job_alpha, job_seed, sample_int, sample_on, cum, syn0,
           syn1neg, lockf, K, nthreads, loss, ld, D, loss_exact=None):
    tok = np.ascontiguousarray(tok, dtype=np.int32)
    sent_off = np.ascontiguousarray(sent_off, dtype=np.int64)
    job_sent = np.ascontiguousarray(job_sent, dtype=np.int64)
    job_alpha = np.ascontiguousarray(job_alpha, dtype=np.float32)
    job_seed = np.ascontiguousarray(job_seed, dtype=np.uint64)
    si = _u32_sample(sample_int)
    cum = np.ascontiguousarray(cum, dtype=np.uint32)
    lockf = np.ascontiguousarray(lockf, dtype=np.float32)
    assert syn0.dtype == np.float32 and syn0.flags.c_contiguous
    assert syn1neg.dtype == np.float32 and syn1neg.flags.c_contiguous
    V = syn0.shape[0]
    stats = np.zeros(4, dtype=np.int64)
    n_jobs = len(job_sent) - 1
    args = [_p(tok), _p(sent_off), _p(job_sent), C.c_int64(n_jobs), _p(job_alpha), _p(job_seed),
            _p(si), C.c_int(int(bool(sample_on))), _p(cum), C.c_int32(V), _p(syn0), _p(syn1neg),
            _p(lockf), C.c_int64(ld), C.c_int32(D), C.c_int32(K)]
    if nthreads and nthreads > 0:
        assert loss is None and loss_exact is None, \
            "the oracle tallies the loss in sequential order only"
        lib().orc_train_hogwild(*args, C.c_int(nthreads), _p(stats))
    else:
        if loss is not None:
            assert loss.dtype == np.float32 and loss.size == 1
        if loss_exact is not None:
            assert loss_exact.dtype == np.float64 and loss_exact.size == 1
        lib().orc_train_sequential(*args, _p(stats), _p(loss), _p(loss_exact))
    return dict(raw_words=int(stats[0]), effective_words=int(stats[1]), examples=int(stats[2]),
                jobs=int(stats[3]))


def sample_records(tok, sent_off, job_sent, job_seed, sample_int, sample_on, cum, K):
    tok = np.ascontiguousarray(tok, dtype=np.int32)
    sent_off = np.ascontiguousarray(sent_off, dtype=np.int64)
    job_sent = np.ascontiguousarray(job_sent, dtype=np.int64)
    job_seed = np.ascontiguousarray(job_seed, dtype=np.uint64)
    si = _u32_sample(sample_int)
    cum = np.ascontiguousarray(cum, dtype=np.uint32)
    L = lib()
    L.orc_sample_records.restype = C.c_int64
    n_jobs = len(job_sent) - 1
    args = [_p(tok), _p(sent_off), _p(job_sent), C.c_int64(n_jobs), _p(job_seed), _p(si),
            C.c_int(int(bool(sample_on))), _p(cum), C.c_int32(len(cum)), C.c_int32(K)]
    n = L.orc_sample_records(*args, None, C.c_int64(0))
    out = np.zeros((max(n, 1), K + 2), dtype=np.int32)
    L.orc_sample_records(*args, _p(out), C.c_int64(n))
    return out[:n]


def sgns_step_sequential(syn0, syn1neg, lockf, center, inp, negs, alpha, loss=None):
    V, D = syn0.shape
    center = np.ascontiguousarray(center, dtype=np.int32)
    inp = np.ascontiguousarray(inp, dtype=np.int32)
    negs = np.ascontiguousarray(negs, dtype=np.int32)
    lockf = np.ascontiguousarray(lockf, dtype=np.float32)
    lib().orc_sgns_step_sequential(_p(syn0), _p(syn1neg), _p(lockf), C.c_int64(D), C.c_int32(D),
                                   C.c_int32(negs.shape[1]), _p(center), _p(inp), _p(negs),
                                   C.c_int64(len(center)), C.c_float(alpha), _p(loss))


def count_records(tok, sent_off, job_sent, job_seed, sample_int, sample_on, cum, K):
    """number of directed examples the jobs produce (no records materialised)"""
    tok = np.ascontiguousarray(tok, dtype=np.int32)
    sent_off = np.ascontiguousarray(sent_off, dtype=np.int64)
    job_sent = np.ascontiguousarray(job_sent, dtype=np.int64)
    job_seed = np.ascontiguousarray(job_seed, dtype=np.uint64)
    si = _u32_sample(sample_int)
    cum = np.ascontiguousarray(cum, dtype=np.uint32)
    L = lib()
    L.orc_sample_records.restype = C.c_int64
    return int(L.orc_sample_records(_p(tok), _p(sent_off), _p(job_sent),
                                    C.c_int64(len(job_sent) - 1), _p(job_seed), _p(si),
                                    C.c_int(int(bool(sample_on))), _p(cum), C.c_int32(len(cum)),
                                    C.c_int32(K), None, C.c_int64(0)))


def atomic_one_wave(syn0, syn1neg, lockf, center, inp, negs, alpha, stripe_rows=0,
                    stripe_copies=1, stripe2_rows=0, stripe2_copies=1, chunk=32):
    """k_sgns_atomic's update order on one wave (orc_atomic_one_wave): in place
    on [V][D] float32 tables.  stripe_* describe the hot-row copies the kernel
    used (g2v_stats.stripe_*)."""
    V, D = syn0.shape
    center = np.ascontiguousarray(center, dtype=np.int32)
    inp = np.ascontiguousarray(inp, dtype=np.int32)
    negs = np.ascontiguousarray(negs, dtype=np.int32)
    lockf = np.ascontiguousarray(lockf, dtype=np.float32)
    assert syn0.dtype == np.float32 and syn0.flags.c_contiguous
    assert syn1neg.dtype == np.float32 and syn1neg.flags.c_contiguous
    lib().orc_atomic_one_wave(_p(syn0), _p(syn1neg), _p(lockf), C.c_int64(D), C.c_int32(D),
                              C.c_int32(negs.shape[1]), _p(center), _p(inp), _p(negs),
                              C.c_int64(len(center)), C.c_float(alpha), C.c_int32(stripe_rows),
                              C.c_int32(stripe_copies), C.c_int32(stripe2_rows),
                              C.c_int32(stripe2_copies), C.c_int32(chunk))
