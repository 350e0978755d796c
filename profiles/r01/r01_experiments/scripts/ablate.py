import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np
from gene2vec_amd import _native as N, engine as E
from gene2vec_amd import synthetic as S
NP = 20_000_000; V0, D, K = 24447, 200, 5
ZS = float(os.environ.get("ZIPF", "1.0")); pairs = S.zipf_gene_pairs(NP, V0, ZS); flat = pairs.reshape(-1)
counts, first = E.count_ids(flat, V0); order, remap = S.vocab_order(counts, first)
V = len(order); vc = counts[order]; tok = remap[flat]
js = E.plan_jobs(n_sent=NP, sent_len=2); al = E.job_alphas(js, NP)
rng = np.random.Generator(np.random.PCG64(1)); syn0 = ((rng.random((V, D)) - 0.5) / D).astype(np.float32)
for spec in sys.argv[1].split(","):
    wr, grid, H, R = (list(map(int, spec.split(":"))) + [8, 8][len(spec.split(":")) - 2:])[:4]
    eng = E.SGNSEngine(V, D, K); eng.set_vocab(vc, float(os.environ.get("SAMPLE", "1e-3"))); eng.set_corpus(tok, sent_len=2)
    eng.set_weights(syn0, np.zeros((V, D), np.float32)); eng.set_option(N.OPT_DEBUG_WRITE, wr); eng.set_option(N.OPT_GRID, grid); eng.set_option(N.OPT_STRIPE_ROWS, H); eng.set_option(N.OPT_STRIPE_COPIES, R)
    rs = np.random.RandomState(1)
    for it in range(2):
        eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD, timing=True); st = eng.read_stats()
    print("write", wr, "grid", grid, "H", H, "R", R, "ex/s %.3g" % (st["examples"] / st["sgns_kernel_ms"] * 1e3), "launch ms %.2f" % (st["sgns_kernel_ms"] / st["launches"]), flush=True)
    eng.close()
