"""GPU: the cold-row stores at C4's shape (verdict r5 item 2).

At BASELINE configs[3] (60,000 genes, dim 512, neg 15) the default
G2V_OPT_TAIL_STORE (-1, the collision budget) writes about 38 %
of the update bytes as plain read-modify-write stores -- gensim's own
unsynchronised Hogwild write-back -- instead of float atomics.  This gate
trains the reference's 10-iteration flow (src/gene2vec.py:67-92: a fresh
permutation of the pairs and the alpha sawtooth restarting every train()
call) on a planted-module corpus of that shape, once with the default stores
and once with every row atomic (G2V_OPT_TAIL_STORE 0), and requires the
manuscript target function (src/evaluation_target_function.py:16-60, the
modules as pathways) and the held-in SGNS objective within north_star's 1 %
(measured: -0.66 % and +0.38 %, a systematic shift beyond the seeds' own
spread of 0.02 % / 0.35 %; storing fewer rows shrinks it, at a cost in
throughput: DESIGN.md 5e).
The full-size comparison against the C restatement's 16-thread Hogwild is
scripts/e2e_parity.py (profiles/r06/e2e_c4/).
"""
import zlib

import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd import engine as E
from gene2vec_amd import replica_study as RQ
from gene2vec_amd import synthetic as S

pytestmark = pytest.mark.gpu

V0, D, K, MODULES = 60000, 512, 15, 2000


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    # scripts/e2e_parity.py's C4 corpus (profiles/r06/e2e_c4/): 10 M planted
    # pairs + the reference's GGIPNN positive pairs x3 (at 3 M pairs the
    # modules are barely learned, target function 1.37)
    mod = RQ.module_of(V0, MODULES)
    pairs = RQ.planted_pairs(10_000_000, V0, mod, MODULES, 0.5, 0)
    names = S.gene_names(V0)
    gid = {}
    pos = RQ.positives()
    for x, y in pos:
        for g in (x, y):
            if g not in gid:
                gid[g] = V0 + len(gid)
    names += list(gid)
    pp = np.array([[gid[x], gid[y]] for x, y in pos], np.int32)
    pairs = np.concatenate([pairs] + [pp] * 3)
    n = len(pairs)
    flat = pairs.reshape(-1)
    counts, first = E.count_ids(flat, len(names))
    order, remap = S.vocab_order(counts, first)
    tok0 = remap[flat].astype(np.int32)
    vc = counts[order].astype(np.int64)
    index2word = [names[i] for i in order]
    gmt = str(tmp_path_factory.mktemp("c4e2e") / "modules.gmt")
    RQ.module_gmt(gmt, mod, MODULES, names, n_paths=300)
    seeds = np.array([zlib.crc32((w + "1").encode()) for w in index2word], np.uint32)
    syn0 = E.seeded_vectors(seeds, D)
    rs = np.random.RandomState(11)
    perms = [rs.permutation(n) for _ in range(10)]
    return tok0, vc, index2word, gmt, syn0, perms


def _train(corpus, tail, seed):
    tok0, vc, _, _, syn0, perms = corpus
    n = len(tok0) // 2
    V = len(vc)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    al = E.job_alphas(js, n)
    eng = E.SGNSEngine(V, D, K)
    try:
        if tail is not None:
            eng.set_option(N.OPT_TAIL_STORE, tail)
        eng.set_vocab(vc, 1e-3)
        eng.set_weights(syn0, np.zeros_like(syn0))
        rs = np.random.RandomState(seed)
        for p in perms:
            eng.set_corpus(np.ascontiguousarray(tok0.reshape(n, 2)[p].reshape(-1)), sent_len=2)
            eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD)
        eng.sync()
        st = eng.read_stats()
        s0, s1 = eng.get_weights()
        return s0, s1, st
    finally:
        eng.close()


def test_c4_cold_row_stores_keep_target_function(corpus):
    tok0, vc, index2word, gmt, _, _ = corpus
    V = len(vc)
    res = {}
    for arm, tail in (("stores", None), ("atomic", 0)):
        tg, hi = [], []
        for seed in (1, 2):
            s0, s1, st = _train(corpus, tail, seed)
            if arm == "stores":  # the default stores syn1neg's cold rows at this shape
                assert 0 < st["tail_row_syn1neg"] < V, st
            else:
                assert st["tail_row_syn1neg"] == -1, st
            assert st["tail_row_syn0"] == -1
            assert np.isfinite(s0).all() and np.isfinite(s1).all()
            tg.append(RQ.target_of(s0, index2word, vc, gmt, D)["ratio"])
            hi.append(RQ.heldin(s0, s1, tok0, vc, K))
        res[arm] = (float(np.mean(tg)), float(np.mean(hi)))
    (t_s, h_s), (t_a, h_a) = res["stores"], res["atomic"]
    assert t_a > 2.0, res  # the modules are learned (measured 2.43)
    # measured at this corpus (three seeds each, profiles/r06/e2e_c4_tail/):
    # stores vs atomics target -0.66 %, objective +0.38 %; the seeds' own
    # spread 0.02 % / 0.35 %; north_star's bar is 1 %
    assert abs(t_s - t_a) / t_a < 0.01, res
    assert abs(h_s - h_a) / h_a < 0.01, res
