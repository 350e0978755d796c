"""sampler kernel time per segment at C2 (k_job_sample x2 + k_scan_jobs)"""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
from gene2vec_amd import _native as N, engine as E, synthetic as S
NP = 20_000_000; V0, D, K = 24447, 200, 5
pairs = S.zipf_gene_pairs(NP, V0, 1.0, seed=20250114); flat = pairs.reshape(-1)
counts, first = E.count_ids(flat, V0); order, remap = S.vocab_order(counts, first)
V = len(order); tok = remap[flat]
js = E.plan_jobs(n_sent=NP, sent_len=2); al = E.job_alphas(js, NP)
eng = E.SGNSEngine(V, D, K); eng.set_vocab(counts[order].astype(np.int64), 1e-3); eng.set_corpus(tok, sent_len=2)
eng.set_weights(((np.random.rand(V, D) - 0.5) / D).astype(np.float32), np.zeros((V, D), np.float32))
rs = np.random.RandomState(1)
for it in range(3):
    eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD, timing=True); st = eng.read_stats()
    print("iter", it, "segments", st["launches"], "sample ms/segment %.3f" % (st["sample_kernel_ms"] / max(1, st["launches"])),
          "sgns ms/segment %.3f" % (st["sgns_kernel_ms"] / max(1, st["launches"])), flush=True)
