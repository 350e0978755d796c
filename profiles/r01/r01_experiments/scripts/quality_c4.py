import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np
from gene2vec_amd import _native as N, engine as E, synthetic as S
from oracle import c_oracle as CO, sgns_oracle as O
NP = int(sys.argv[1]); ITERS = int(sys.argv[2]); V0, D, K, sample = 60000, 512, 15, 1e-3
pairs = S.zipf_gene_pairs(NP, V0, 1.0); flat = pairs.reshape(-1)
counts, first = E.count_ids(flat, V0); order, remap = S.vocab_order(counts, first)
V = len(order); vc = counts[order]; tok = remap[flat]
rng = np.random.Generator(np.random.PCG64(1)); syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
js = E.plan_jobs(n_sent=NP, sent_len=2); al = E.job_alphas(js, NP); off = np.arange(0, 2 * NP + 1, 2, dtype=np.int64)
def evl(s0, s1, n_eval=30000, seed=99):
    r = np.random.Generator(np.random.PCG64(seed)); idx = r.integers(0, NP, n_eval)
    c, j = tok[2 * idx], tok[2 * idx + 1]; p = vc.astype(np.float64) ** 0.75
    negs = r.choice(V, size=(n_eval, K), p=p / p.sum()); return O.sgns_loss(s0, s1, c, j, negs)
if "--oracle" in sys.argv:
    a0, a1 = syn0.copy(), np.zeros((V, D), np.float32); rs = np.random.RandomState(1)
    for it in range(ITERS):
        t = time.time(); CO.train(tok, off, js, al.astype(np.float32), E.job_seeds(rs, len(js) - 1), CO.sample_int(vc, sample), True, CO.make_cum_table(vc), a0, a1, np.ones(V, np.float32), K)
        print("oracle iter", it, "%.1fs" % (time.time() - t), "loss", evl(a0, a1), flush=True)
for grid in [int(g) for g in sys.argv[3].split(",")]:
    eng = E.SGNSEngine(V, D, K); eng.set_vocab(vc, sample); eng.set_corpus(tok, sent_len=2)
    eng.set_weights(syn0, np.zeros((V, D), np.float32)); eng.set_option(N.OPT_GRID, grid)
    rs = np.random.RandomState(1)
    for it in range(ITERS):
        eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD, timing=True); st = eng.read_stats()
        g0, g1 = eng.get_weights()
        print("grid", grid, "iter", it, "ex/s %.3g pairs/s %.3g" % (st["examples"] / st["sgns_kernel_ms"] * 1e3, NP / (st["sgns_kernel_ms"] + st["sample_kernel_ms"]) * 1e3), "loss", evl(g0, g1), flush=True)
    eng.close()
