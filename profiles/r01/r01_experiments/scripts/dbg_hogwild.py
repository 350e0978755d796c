import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
from gene2vec_amd import _native as N, engine as E
from tests.helpers import zipf_pairs, vocab_from_ids
pairs = zipf_pairs(40000, 2000, seed=20250114)
flat = pairs.reshape(-1); order, remap, counts = vocab_from_ids(flat, 2000); tok = remap[flat]
V = len(counts); D, K = 200, 5
rng = np.random.Generator(np.random.PCG64(1)); syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
js = E.plan_jobs(n_sent=len(tok)//2, sent_len=2); al = E.job_alphas(js, len(tok)//2)
sd = E.job_seeds(np.random.RandomState(1), len(js)-1)
res = {}
for mode in (N.MODE_SEQUENTIAL, N.MODE_HOGWILD):
    eng = E.SGNSEngine(V, D, K); eng.set_vocab(counts, 1e-3)
    eng.set_weights(syn0, np.zeros((V, D), np.float32)); eng.set_corpus(tok, sent_len=2)
    eng.train(js, al, sd, mode, timing=True); st = eng.read_stats()
    g0, g1 = eng.get_weights(); res[mode] = (g0, g1)
    print(mode, st, np.abs(g1).max(), np.abs(g0 - syn0).max(), flush=True)
print("diff", np.abs(res[0][1] - res[1][1]).max())
# explicit hogwild with overlapping rows
recs = None
eng = E.SGNSEngine(V, D, K); eng.set_vocab(counts, 1e-3); eng.set_corpus(tok, sent_len=2)
recs = eng.debug_sample(js, sd)
print("recs", recs.shape, recs[:3])
for mode in (N.MODE_SEQUENTIAL, N.MODE_HOGWILD):
    eng.set_weights(syn0, np.zeros((V, D), np.float32))
    eng.step_explicit(recs[:, 0], recs[:, 1], recs[:, 2:], 0.025, mode)
    g0, g1 = eng.get_weights(); print("explicit", mode, np.abs(g1).max(), np.abs(g0 - syn0).max())
