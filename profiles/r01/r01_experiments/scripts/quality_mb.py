import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np
from gene2vec_amd import _native as N, engine as E
from oracle import sgns_oracle as O
from tests.helpers import zipf_pairs, vocab_from_ids
NP = 4_000_000; V0, D, K, sample = 24447, 200, 5, 1e-3
pairs = zipf_pairs(NP, V0, seed=20250114)
flat = pairs.reshape(-1); order, remap, counts = vocab_from_ids(flat, V0); tok = remap[flat]; V = len(counts)
rng = np.random.Generator(np.random.PCG64(1)); syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
js = E.plan_jobs(n_sent=NP, sent_len=2); al = E.job_alphas(js, NP)
def evl(s0, s1, n_eval=50000, seed=99):
    r = np.random.Generator(np.random.PCG64(seed)); idx = r.integers(0, NP, n_eval)
    c, j = tok[2 * idx], tok[2 * idx + 1]; p = counts.astype(np.float64) ** 0.75
    negs = r.choice(V, size=(n_eval, K), p=p / p.sum()); return O.sgns_loss(s0, s1, c, j, negs)
eng = E.SGNSEngine(V, D, K); eng.set_vocab(counts, sample); eng.set_corpus(tok, sent_len=2)
rs = np.random.RandomState(1)
recs = [eng.debug_sample(js, E.job_seeds(rs, len(js) - 1)) for _ in range(2)]
# alpha per record: records are in job order; job of record = searchsorted on per-job counts
for B in [int(b) for b in sys.argv[1].split(",")]:
    eng.set_weights(syn0, np.zeros((V, D), np.float32))
    for it in range(2):
        R = recs[it]; n = len(R); t = time.time()
        for b0 in range(0, n, B):
            r = R[b0:b0 + B]
            a = float(al[min(len(al) - 1, int(b0 / n * len(al)))])
            eng.step_explicit(r[:, 0], r[:, 1], r[:, 2:], a, N.MODE_MINIBATCH)
        g0, g1 = eng.get_weights()
        print("minibatch B", B, "iter", it, "loss", evl(g0, g1), "t", time.time() - t, flush=True)
