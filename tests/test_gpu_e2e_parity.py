"""GPU: the north-star metrics end to end (SURVEY.md 8(c) "final-epoch loss,
target function ... within a stated tolerance of gensim on the same input").

gensim is absent, so its stand-in is oracle/sgns_oracle.c's sequential
trainer (gensim workers=1 order), whose results on this corpus are committed
in tests/golden/e2e_parity.json (tests/golden/make_e2e_golden.py).  The GPU
runs the production path -- libg2v's Hogwild kernel at the default grid --
through the reference's flow (src/gene2vec.py:67-92): 10 iterations, the
pairs reshuffled before each (the same permutations as the golden run), the
alpha sawtooth restarting per train() call, compute_loss on the last one.
Means over the same three model.random seeds; bars 1 % (north star) for the
final-iteration loss and the manuscript target function
(src/evaluation_target_function.py, planted modules as pathways) and 0.5 %
for the SGNS objective on corpus pairs.  The Hogwild staleness shows in the
target function most (round 5, the production kernel
with its cold syn1neg rows stored: -0.5 % here, -0.3 % at the C2 vocabulary,
-0.8 % on the dense 5,000-gene corpus with syn0 stores too, which is why syn0
stays atomic; round 4, all atomics: -0.25 / -0.09 / -0.46 %; gensim's own
32-thread Hogwild, restated, sits 0.1-0.8 % below its sequential order)."""
import json
import os
import zlib

import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd import engine as E
from gene2vec_amd import evaluate as EV
from gene2vec_amd.word2vec import KeyedVectors, Vocab
from tests.conftest import GOLDEN
from tests.helpers import E2E, E2E_C2, E2E_V5K, e2e_corpus, e2e_heldin

pytestmark = pytest.mark.gpu
# experiment hook (verdict r4 item 4): G2V_TEST_TAIL_STORE=n
# runs these gates with G2V_OPT_TAIL_STORE n (cold rows stored, not added)
_ts = os.environ.get("G2V_TEST_TAIL_STORE")  # unset: the library's default (-1, auto)
TAIL_STORE = int(_ts) if _ts not in (None, "") else None


def _train_e2e(tmp_path, sample, grid=None, cfg=E2E):
    """the reference's 10-iteration flow on the GPU, every seed of the golden
    run; returns per-seed metrics and the grids (set_vocab's, last call's)"""
    tok, counts, index2word, lines, perms, wseeds = e2e_corpus(cfg)
    n = len(tok) // 2
    D, K = cfg["D"], cfg["K"]
    V = len(counts)
    syn0 = E.seeded_vectors(wseeds, D)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    al = E.job_alphas(js, n)
    got = {"loss": [], "heldin": [], "target_ratio": [], "grid": [], "waves": []}
    for seed in cfg["seeds"]:
        eng = E.SGNSEngine(V, D, K)
        if grid:
            eng.set_option(N.OPT_GRID, grid)
        if TAIL_STORE is not None:
            eng.set_option(N.OPT_TAIL_STORE, min(TAIL_STORE, V))
        eng.set_vocab(counts, sample)
        eng.set_weights(syn0, np.zeros_like(syn0))
        rs = np.random.RandomState(seed)
        for it in range(cfg["iters"]):
            last = it == cfg["iters"] - 1
            eng.set_corpus(np.ascontiguousarray(tok.reshape(n, 2)[perms[it]].reshape(-1)),
                           sent_len=2)
            if last:
                eng.reset_loss()
            eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD, compute_loss=last)
        eng.sync()
        st = eng.read_stats()
        got["grid"].append(int(eng.get_option(N.OPT_GRID)))
        got["waves"].append(int(st["sgns_waves"]))  # the last launch's, after the cap
        s0, s1 = eng.get_weights()
        eng.close()
        kv = KeyedVectors(D)
        kv.index2word = list(index2word)
        kv.vocab = {w: Vocab(count=int(counts[i]), index=i) for i, w in enumerate(index2word)}
        kv.vectors = np.ascontiguousarray(s0)
        w2v = str(tmp_path / f"seed{seed}_w2v.txt")
        kv.save_word2vec_format(w2v)
        t = EV.target_function(w2v, pathways=lines, strict=False, verbose=False)
        got["loss"].append(float(st["training_loss"]))
        got["heldin"].append(e2e_heldin(s0, s1, tok, counts, K))
        got["target_ratio"].append(float(t["ratio"]))
    return got


def _gaps(got, ref):
    return {k: (np.mean(got[k]) - ref[k + "_mean"]) / ref[k + "_mean"]
            for k in ("loss", "heldin", "target_ratio")}


def _golden(name="e2e_parity.json", cfg=E2E):
    with open(os.path.join(GOLDEN, name)) as f:
        ref = json.load(f)
    tok = e2e_corpus(cfg)[0]
    assert zlib.crc32(tok.tobytes()) == ref["corpus_crc32"]
    return ref


def test_gpu_hogwild_end_to_end_metrics_within_one_percent_of_sequential(tmp_path):
    ref = _golden()
    got = _train_e2e(tmp_path, E2E["sample"])
    gaps = _gaps(got, ref)
    print("gpu", got, "gaps vs sequential oracle", gaps)
    assert abs(gaps["loss"]) < 0.01, gaps
    assert abs(gaps["heldin"]) < 0.005, gaps
    assert abs(gaps["target_ratio"]) < 0.01, gaps


def test_gpu_hogwild_sample0_stays_stable(tmp_path):
    """sample = 0 keeps the hottest genes' syn0 rows busy: past a staleness
    that grows with the vectors' norms a hot syn0 row overshoots at a
    sawtooth restart and freezes (|f| >= 6 skips every later update; DESIGN.md
    5c).  k_sgns_atomic caps the waves that train in every launch for it (from
    |syn1neg|^2 measured on the device just before the launch): the objective
    and the final loss track the sequential oracle's, and the cap has engaged
    by the last launch.  The target function is reported, not
    gated: at sample 0 the Hogwild staleness moves it a few percent on
    structured corpora."""
    ref = _golden()["sample0"]
    got = _train_e2e(tmp_path, 0.0)
    gaps = _gaps(got, ref)
    print("gpu sample 0", got, "gaps vs sequential oracle", gaps)
    assert all(w < 4 * g for w, g in zip(got["waves"], got["grid"])), got
    assert abs(gaps["heldin"]) < 0.005, gaps
    assert abs(gaps["loss"]) < 0.01, gaps


def test_gpu_end_to_end_at_the_c2_vocabulary(tmp_path):
    """the same gate at the bench's vocabulary (24,447 Zipf genes, 1,000
    planted modules, 10 M pairs, sample 1e-3), the production defaults (one
    workgroup per CU); golden from the sequential oracle, two seeds
    (tests/golden/make_e2e_golden.py --c2).  The only e2e corpus with
    syn1neg rows cold enough for the default tail stores.
    Measured, round 5: loss +0.4 %, objective +0.29 %, target function
    -0.3 % (all atomics, round 4: +0.07 / -0.05 / -0.09 %)."""
    ref = _golden("e2e_parity_c2.json", E2E_C2)
    got = _train_e2e(tmp_path, E2E_C2["sample"], cfg=E2E_C2)
    gaps = _gaps(got, ref)
    print("gpu C2 vocabulary", got, "gaps vs sequential oracle", gaps)
    assert abs(gaps["loss"]) < 0.01, gaps
    assert abs(gaps["heldin"]) < 0.005, gaps
    assert abs(gaps["target_ratio"]) < 0.01, gaps


def test_gpu_end_to_end_dense_5k_genes(tmp_path):
    """the dense corpus where Hogwild staleness moves the target function most
    (5,000 genes, 200 planted modules, 4 M pairs: every gene in ~1,600 pairs;
    DESIGN.md 8 measured -0.97 % at the default one-workgroup-per-CU grid with
    GGIPNN pairs added, -1.39 % at the 295 workgroups the staleness budget
    alone allowed; rounds 4 and 5 -0.46 % with all rows atomic, -0.84 % when
    syn0 rows were stored too).  Golden: the sequential oracle, three seeds
    (tests/golden/make_e2e_golden.py --v5k).  North-star bar: 1 % on the loss
    and the target function, 0.5 % on the SGNS objective."""
    ref = _golden("e2e_parity_v5k.json", E2E_V5K)
    got = _train_e2e(tmp_path, E2E_V5K["sample"], cfg=E2E_V5K)
    gaps = _gaps(got, ref)
    print("gpu dense 5k genes", got, "gaps vs sequential oracle", gaps)
    assert abs(gaps["loss"]) < 0.01, gaps
    assert abs(gaps["heldin"]) < 0.005, gaps
    assert abs(gaps["target_ratio"]) < 0.01, gaps
