"""Hogwild-vs-sequential deviation per kernel configuration (the quantity
tests/test_gpu_parity.py::test_train_hogwild_objective_matches_oracle bounds):
the C oracle trains the same jobs/seeds sequentially once, then every GPU
configuration trains from the same init and the held-in SGNS objective is
compared.  Experiment script, not product code.

    python scripts/hogwild_dev.py --vocab 3000 --pairs 200000 --configs grid=300 grid=200,ov=1
"""
import argparse
import json
import os
import sys
import time

ROOT = os.environ.get("G2V_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=200_000)
    p.add_argument("--vocab", type=int, default=3000)
    p.add_argument("--dim", type=int, default=200)
    p.add_argument("--negative", type=int, default=5)
    p.add_argument("--sample", type=float, default=1e-3)
    p.add_argument("--iters", type=int, default=3)
    p.add_argument("--configs", nargs="+", default=["grid=0"])
    p.add_argument("--seeds", type=int, default=1, help="job-seed streams (RandomState(1..n))")
    p.add_argument("--repeat", type=int, default=1, help="GPU runs per seed (Hogwild is timing-dependent)")
    p.add_argument("--n-eval", type=int, default=20000)
    a = p.parse_args()

    from gene2vec_amd import _native as N
    from gene2vec_amd import engine as E
    from oracle import c_oracle as CO
    from tests.helpers import crc_hash, vocab_from_ids, zipf_pairs
    from tests.test_gpu_parity import _corpus_from_pairs, _eval_loss, _zipf_setup

    D, K, sample = a.dim, a.negative, a.sample
    tok, counts, syn0 = _zipf_setup(a.pairs, a.vocab, D, K, sample)
    V = len(counts)
    n = len(tok) // 2
    off = np.arange(0, len(tok) + 1, 2, dtype=np.int64)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    refs = []
    for seed in range(1, a.seeds + 1):
        a0, a1 = syn0.copy(), np.zeros((V, D), np.float32)
        rs_c = np.random.RandomState(seed)
        for _ in range(a.iters):
            al = E.job_alphas(js, n)
            CO.train(tok, off, js, al.astype(np.float32), E.job_seeds(rs_c, len(js) - 1),
                     CO.sample_int(counts, sample), sample != 0, CO.make_cum_table(counts), a0,
                     a1, np.ones(V, np.float32), K)
        refs.append(_eval_loss(a0, a1, tok, counts, K, n_eval=a.n_eval))
    refs = np.array(refs)
    print(json.dumps({"oracle": [round(x, 5) for x in refs], "mean": round(refs.mean(), 5),
                      "V": V, "pairs": n}), flush=True)
    for text in a.configs:
        cfg = dict(kv.split("=") for kv in text.split(",") if kv)
        out = []
        for seed in [s for s in range(1, a.seeds + 1) for _ in range(a.repeat)]:
            eng = E.SGNSEngine(V, D, K)
            if int(cfg.get("ov", 0)):
                eng.set_option(N.OPT_ATOMIC_OVERLAP, 1)
            eng.set_vocab(counts, sample)
            if int(cfg.get("grid", 0)):
                eng.set_option(N.OPT_GRID, int(cfg["grid"]))
            eng.set_weights(syn0, np.zeros((V, D), np.float32))
            eng.set_corpus(tok, sent_len=2)
            rs_g = np.random.RandomState(seed)
            for _ in range(a.iters):
                al = E.job_alphas(js, n)
                eng.train(js, al, E.job_seeds(rs_g, len(js) - 1), N.MODE_HOGWILD)
            g0, g1 = eng.get_weights()
            grid = eng.get_option(N.OPT_GRID)
            eng.close()
            out.append(_eval_loss(g0, g1, tok, counts, K, n_eval=a.n_eval))
        out = np.array(out)
        dev = (out - np.repeat(refs, a.repeat)) / np.repeat(refs, a.repeat)
        print(json.dumps({"config": text, "grid": grid, "loss": [round(x, 5) for x in out],
                          "rel_dev": [round(x, 5) for x in dev],
                          "mean_dev": round(float((out.mean() - refs.mean()) / refs.mean()), 5),
                          "max_abs_dev": round(float(np.abs(dev).max()), 5)}),
              flush=True)


if __name__ == "__main__":
    t = time.time()
    main()
    print(f"# {time.time() - t:.1f} s", flush=True)
