"""delta16 (packed-f16 delta tables) quality + speed: the reference's
10-iteration schedule over 4M Zipf pairs at C2's vocabulary; held-in SGNS
loss per iteration (sequential oracle, profiles/r01_quality_10iter.log:
2.7655 ... 2.5791).  variants: d16rows:grid:segjobs (d16rows -1 = f32 atomics)"""
import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np
from gene2vec_amd import _native as N, engine as E
from oracle import sgns_oracle as O
from tests.helpers import zipf_pairs, vocab_from_ids
NP = int(sys.argv[1]); ITERS = int(sys.argv[2])
V0, D, K, sample = 24447, 200, 5, 1e-3
pairs = zipf_pairs(NP, V0, seed=20250114)
flat = pairs.reshape(-1); order, remap, counts = vocab_from_ids(flat, V0); tok = remap[flat]
V = len(counts)
rng = np.random.Generator(np.random.PCG64(1)); syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
js = E.plan_jobs(n_sent=NP, sent_len=2); al = E.job_alphas(js, NP)
def evl(s0, s1, n_eval=50000, seed=99):
    r = np.random.Generator(np.random.PCG64(seed)); idx = r.integers(0, NP, n_eval)
    c, j = tok[2 * idx], tok[2 * idx + 1]; p = counts.astype(np.float64) ** 0.75
    negs = r.choice(V, size=(n_eval, K), p=p / p.sum()); return O.sgns_loss(s0, s1, c, j, negs)
for var in sys.argv[3].split(","):
    d16, grid, seg = (list(map(int, var.split(":"))) + [0, 0])[:3]
    eng = E.SGNSEngine(V, D, K); eng.set_vocab(counts, sample)
    eng.set_option(N.OPT_GRID, grid); eng.set_option(N.OPT_DELTA16_ROWS, d16)
    if seg:
        eng.set_option(N.OPT_SEG_JOBS, seg)
    eng.set_weights(syn0, np.zeros((V, D), np.float32)); eng.set_corpus(tok, sent_len=2)
    rs = np.random.RandomState(1)
    for it in range(ITERS):
        eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD, timing=True); st = eng.read_stats()
        g0, g1 = eng.get_weights()
        ok = np.isfinite(g0).all() and np.isfinite(g1).all()
        print("var", var, "iter", it, "sgns ms %.2f ex/s %.3g" % (st["sgns_kernel_ms"], st["examples"] / st["sgns_kernel_ms"] * 1e3),
              "loss %.5f" % evl(g0, g1), "finite", ok, flush=True)
    eng.close()
