import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np
from gene2vec_amd import _native as N, engine as E
from oracle import c_oracle as CO, sgns_oracle as O
from tests.helpers import zipf_pairs, vocab_from_ids
NP = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
V0, D, K, sample = 24447, 200, 5, 1e-3
t = time.time()
pairs = zipf_pairs(NP, V0, seed=20250114)
flat = pairs.reshape(-1); order, remap, counts = vocab_from_ids(flat, V0); tok = remap[flat]
V = len(counts); print("corpus", NP, V, time.time() - t, flush=True)
rng = np.random.Generator(np.random.PCG64(1)); syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
js = E.plan_jobs(n_sent=NP, sent_len=2); al = E.job_alphas(js, NP)
off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)
def evl(s0, s1, n_eval=50000, seed=99):
    r = np.random.Generator(np.random.PCG64(seed)); idx = r.integers(0, NP, n_eval)
    c, j = tok[2 * idx], tok[2 * idx + 1]; p = counts.astype(np.float64) ** 0.75
    negs = r.choice(V, size=(n_eval, K), p=p / p.sum()); return O.sgns_loss(s0, s1, c, j, negs)
print("init loss", evl(syn0, np.zeros((V, D), np.float32)), flush=True)
res = {}
a0, a1 = syn0.copy(), np.zeros((V, D), np.float32); rs = np.random.RandomState(1)
si = CO.sample_int(counts, sample); cum = CO.make_cum_table(counts)
for it in range(ITERS):
    t = time.time(); st = CO.train(tok, off, js, al.astype(np.float32), E.job_seeds(rs, len(js) - 1), si, True, cum, a0, a1, np.ones(V, np.float32), K)
    print("oracle seq iter", it, time.time() - t, st, "loss", evl(a0, a1), flush=True)
for var in (sys.argv[3].split(",") if len(sys.argv) > 3 else ["-1:1"]):
    hot, pol, mem, grid = (list(map(int, var.split(":"))) + [0, 0])[:4]; mode = N.MODE_HOGWILD
    eng = E.SGNSEngine(V, D, K); eng.set_vocab(counts, sample); eng.set_option(N.OPT_TABLE_MEM, mem)
    eng.set_option(N.OPT_GRID, grid)
    eng.set_option(N.OPT_HOT_ROWS, hot); eng.set_option(N.OPT_CACHE_POLICY, pol)
    eng.set_weights(syn0, np.zeros((V, D), np.float32)); eng.set_corpus(tok, sent_len=2)
    rs = np.random.RandomState(1)
    for it in range(ITERS):
        eng.train(js, al, E.job_seeds(rs, len(js) - 1), mode, timing=True); st = eng.read_stats()
        g0, g1 = eng.get_weights()
        print("gpu hot:pol", var, "iter", it, "sgns ms %.2f samp ms %.2f ex/s %.3g" % (st["sgns_kernel_ms"], st["sample_kernel_ms"], st["examples"] / st["sgns_kernel_ms"] * 1e3), "loss", evl(g0, g1), flush=True)
    eng.close()
