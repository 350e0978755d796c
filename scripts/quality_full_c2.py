"""Quality at the benchmark's full size: the reference's 10-iteration schedule
(alpha sawtooth, reshuffle-free) over C2 (24,447 genes, 100 M Zipf pairs) on
one MI355X (production HOGWILD kernel) against the CPU restatement run the way
gensim runs it (Hogwild threads, oracle/sgns_oracle.c), same initial tables,
same job seeds.  Prints the held-in SGNS objective after every iteration and
one JSON summary line.

    python scripts/quality_full_c2.py [--pairs 100000000] [--iters 10] [--threads 16]
    python scripts/quality_full_c2.py --vocab 60000 --dim 512 --negative 15 --pairs 20000000  # C4
"""
import argparse
import json
import os
import sys
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gene2vec_amd import _native as N  # noqa: E402
from gene2vec_amd import engine as E  # noqa: E402
from gene2vec_amd import synthetic as S  # noqa: E402
from oracle import c_oracle as CO  # noqa: E402
from oracle import sgns_oracle as O  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=100_000_000)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--vocab", type=int, default=24447)
    p.add_argument("--dim", type=int, default=200)
    p.add_argument("--negative", type=int, default=5)
    p.add_argument("--sample", type=float, default=1e-3)
    p.add_argument("--grid", type=int, default=0, help="SGNS workgroups (0 = library default)")
    a = p.parse_args()
    V0, D, K, sample = a.vocab, a.dim, a.negative, a.sample
    n = a.pairs
    pairs = S.zipf_gene_pairs(n, V0, 1.0, seed=20250114)
    flat = pairs.reshape(-1)
    del pairs
    counts, first = E.count_ids(flat, V0)
    order, remap = S.vocab_order(counts, first)
    tok = remap[flat]
    del flat
    vc = counts[order].astype(np.int64)
    V = len(order)
    names = S.gene_names(V0)
    seeds = np.array([zlib.crc32((names[i] + "1").encode()) for i in order], np.uint32)
    syn0 = E.seeded_vectors(seeds, D)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    al = E.job_alphas(js, n)
    off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)

    rng = np.random.Generator(np.random.PCG64(99))
    idx = rng.integers(0, n, 50000)
    ec, ej = tok[2 * idx], tok[2 * idx + 1]
    pw = vc.astype(np.float64) ** 0.75
    negs = rng.choice(V, size=(50000, K), p=pw / pw.sum())

    def loss(s0, s1):
        return float(O.sgns_loss(s0, s1, ec, ej, negs))

    eng = E.SGNSEngine(V, D, K)
    if a.grid:
        eng.set_option(N.OPT_GRID, a.grid)
    eng.set_vocab(vc, sample)
    eng.set_weights(syn0, np.zeros((V, D), np.float32))
    eng.set_corpus(tok, sent_len=2)
    c0, c1 = syn0.copy(), np.zeros((V, D), np.float32)
    si, cum = CO.sample_int(vc, sample), CO.make_cum_table(vc)
    rs_g, rs_c = np.random.RandomState(1), np.random.RandomState(1)
    out = {"gpu": [], "cpu": [], "gpu_s": 0.0, "cpu_s": 0.0}
    print("init loss %.5f" % loss(syn0, np.zeros((V, D), np.float32)), flush=True)
    for it in range(a.iters):
        t = time.time()
        eng.train(js, al, E.job_seeds(rs_g, len(js) - 1), N.MODE_HOGWILD)
        eng.sync()
        out["gpu_s"] += time.time() - t
        g0, g1 = eng.get_weights()
        t = time.time()
        CO.train(tok, off, js, al.astype(np.float32), E.job_seeds(rs_c, len(js) - 1), si, True,
                 cum, c0, c1, np.ones(V, np.float32), K, nthreads=a.threads, ld=(D + 15) // 16 * 16)
        out["cpu_s"] += time.time() - t
        out["gpu"].append(round(loss(g0, g1), 5))
        out["cpu"].append(round(loss(c0, c1), 5))
        print("iter", it, "gpu", out["gpu"][-1], "cpu hogwild", out["cpu"][-1], flush=True)
    out.update({"pairs": n, "iters": a.iters, "cpu_threads": a.threads, "vocab": V0, "dim": D,
                "negative": K, "sample": sample, "grid": eng.get_option(N.OPT_GRID),
                "rel_gap_final": round((out["gpu"][-1] - out["cpu"][-1]) / out["cpu"][-1], 5)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
