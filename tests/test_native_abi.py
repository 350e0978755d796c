"""libg2v.so loads here (no GPU), exports every symbol include/g2v.h
declares, and its host-only helpers match the oracle / numpy."""
import os
import re

import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd import engine as E
from oracle import sgns_oracle as O
from tests.conftest import ROOT
from tests.helpers import crc_hash


def header_symbols():
    src = open(os.path.join(ROOT, "include", "g2v.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(g2v_[a-z_0-9]+)\s*\(", src)))


def test_library_loads_and_exports_header():
    L = N.lib()
    syms = header_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(L, s), s
        assert s in N.SIGNATURES, f"{s} missing from the ctypes signature table"
    assert set(N.SIGNATURES) == set(syms)
    assert L.g2v_abi_version() == N.ABI_VERSION == 5


def test_error_path_without_gpu_is_loud():
    # creating a context needs a device; on a CPU box it must fail with a
    # status code and a message, never crash
    import ctypes as C
    h = C.c_void_p()
    rc = N.lib().g2v_create(0, 10, 8, 5, 2, C.byref(h))  # window=2 rejected up front
    assert rc == N.G2V_EINVAL
    assert b"window" in N.lib().g2v_last_error()
    rc = N.lib().g2v_create(0, 10, 8, 21, 1, C.byref(h))  # negative=21 not compiled
    assert rc == N.G2V_EINVAL
    rc = N.lib().g2v_create(0, 10, 513, 5, 1, C.byref(h))  # wider than one wave's 2 float4s
    assert rc == N.G2V_EINVAL
    rc = N.lib().g2v_create(0, 3_000_000, 200, 5, 1, C.byref(h))  # > 2 GiB per table
    assert rc == N.G2V_EINVAL and b"2 GiB" in N.lib().g2v_last_error()


def test_local_group_arguments_without_gpu():
    """g2v_local_group_create / _destroy are host-only: argument checks and a
    create/destroy round trip need no device"""
    import ctypes as C
    L = N.lib()
    h = C.c_void_p()
    assert L.g2v_local_group_create(0, 0, C.byref(h)) == N.G2V_EINVAL
    assert L.g2v_local_group_create(17, 0, C.byref(h)) == N.G2V_EINVAL  # > kMaxLocalReplicas
    assert L.g2v_local_group_create(2, -1, C.byref(h)) == N.G2V_EINVAL
    assert L.g2v_local_group_create(4, 0, C.byref(h)) == N.G2V_OK and h.value
    assert L.g2v_local_group_destroy(h) == N.G2V_OK
    assert L.g2v_local_group_destroy(None) == N.G2V_OK
    # a context is required for the collectives themselves
    assert L.g2v_comm_init_local(None, None, 0) == N.G2V_EINVAL
    assert L.g2v_comm_abort(None) == N.G2V_EINVAL


def test_stats_struct_matches_header():
    """g2v_stats as the header declares it: the ctypes mirror has the same
    fields in the same order (ABI 3 appended the launch layout)"""
    src = open(os.path.join(ROOT, "include", "g2v.h")).read()
    body = re.search(r"typedef struct g2v_stats \{(.*?)\} g2v_stats;", src, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = []
    for decl in body.split(";"):
        decl = decl.strip()
        if decl:
            names += [x.strip() for x in decl.split(None, 1)[1].split(",")]
    assert names == [f for f, _ in N.Stats._fields_]


@pytest.mark.parametrize("lengths", [[2] * 40, [2] * 12345, [2, 4, 0, 2, 3, 9997, 2, 10000, 1] * 3,
                                     [], [0, 0, 0], [10000, 10000], [5000, 5000, 1],
                                     # sentences over batch_words: a job each, and an
                                     # empty first job when the first one is long
                                     [10001], [25000, 2, 2], [2, 30000, 2, 10001, 0, 3],
                                     [0, 10001], [10001, 10001, 10001]])
def test_plan_jobs_matches_oracle(lengths):
    ref = O.plan_jobs(lengths)
    off = np.cumsum([0] + lengths).astype(np.int64)
    js = E.plan_jobs(sent_off=off)
    expect = [ref[0][0]] + [j[1] for j in ref] if ref else [0]
    assert js.tolist() == expect


def test_plan_jobs_uniform_and_long_sentences():
    js = E.plan_jobs(n_sent=12345, sent_len=2)
    assert js.tolist() == [j[0] for j in O.plan_jobs([2] * 12345)] + [12345]
    # [ext] _job_producer: a first sentence over batch_words queues the empty
    # batch first (a job of its own, two model.random draws), then trains alone
    assert E.plan_jobs(sent_off=np.array([0, 10001], np.int64)).tolist() == [0, 0, 1]
    assert O.plan_jobs([10001]) == [(0, 0), (0, 1)]


def test_job_alphas_and_seeds(golden):
    s = golden["schedule"]
    js = E.plan_jobs(n_sent=1000000, sent_len=2)
    a = E.job_alphas(js, 1000000)
    assert a[:5].tolist() == s["alphas1m_head"] and a[-5:].tolist() == s["alphas1m_tail"]
    js40 = E.plan_jobs(n_sent=40, sent_len=2)
    assert E.job_alphas(js40, 40, cur_epoch=1, epochs=3).tolist() == s["epoch2of3"]
    assert E.job_seeds(np.random.RandomState(1), 5).tolist() == s["seeds_rs1"]
    # vectorised == the oracle's per-job Python loop on an irregular corpus
    lengths = list(np.random.RandomState(3).randint(0, 7, 30000))
    jobs = O.plan_jobs(lengths)
    js = E.plan_jobs(sent_off=np.cumsum([0] + lengths))
    assert E.job_alphas(js, len(lengths)).tolist() == O.job_alphas(jobs, len(lengths))


def test_seeded_vectors_native_is_numpy_randomstate():
    words = ["TLE1", "ALDOB", "G00017", "x" * 40]
    seeds = np.array([crc_hash(w + "1") & 0xFFFFFFFF for w in words], np.uint32)
    for dim in (1, 7, 200, 512):
        got = E.seeded_vectors(seeds, dim)
        for i, w in enumerate(words):
            ref = O.seeded_vector(w + "1", dim, crc_hash).astype(np.float32)
            assert np.array_equal(got[i], ref)


def test_count_ids():
    ids = np.array([3, 1, 3, 0, 3, 1], np.int32)
    c, f = E.count_ids(ids, 5)
    assert c.tolist() == [1, 2, 0, 3, 0] and f.tolist() == [3, 1, -1, 0, -1]


@pytest.mark.parametrize("sent_len", [1, 2, 3, 7, 10000])
@pytest.mark.parametrize("n", [0, 1, 4999, 5000, 5001, 123457])
def test_plan_jobs_fixed_length_equal_csr(n, sent_len):
    """Fixed-length sentences (the CLI trains an all-pairs corpus with
    sent_len=2) take a closed form; its gensim jobs must equal the CSR loop's."""
    csr = E.plan_jobs(sent_off=np.arange(0, sent_len * n + 1, sent_len, dtype=np.int64))
    fixed = E.plan_jobs(n_sent=n, sent_len=sent_len)
    np.testing.assert_array_equal(csr, fixed)


@pytest.mark.parametrize("n", [0, 1, 3])
def test_plan_jobs_fixed_length_over_batch_words(n):
    L = N.BATCH_WORDS + 1
    fixed = E.plan_jobs(n_sent=n, sent_len=L)
    csr = E.plan_jobs(sent_off=np.arange(0, L * n + 1, L, dtype=np.int64))
    np.testing.assert_array_equal(fixed, csr)
    ref = O.plan_jobs([L] * n)
    assert fixed.tolist() == ([ref[0][0]] + [j[1] for j in ref] if ref else [0])
