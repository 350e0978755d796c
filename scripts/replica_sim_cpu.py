"""CPU simulation of data-parallel replica merging (merge-rule exploration
without a GPU): R replicas trained window by window with the C oracle
(oracle/sgns_oracle.c, sequential gensim order) on their shards of each
iteration's shuffle, merged with numpy restatements of libg2v's rules, vs one
model on the same shuffles.  Planted co-expression modules give the target
function (pathways = modules) meaning.  Test infrastructure: it drives the
oracle, not the product.

    python scripts/replica_sim_cpu.py --rules touch,align --every 2
"""
import argparse
import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from gene2vec_amd import engine as E  # noqa: E402
from gene2vec_amd import synthetic as S  # noqa: E402
from oracle import c_oracle as CO  # noqa: E402
from gene2vec_amd import replica_study as RQ  # noqa: E402


def merge(rule, ts, olds, beta=1.0, gamma=1.0):
    d = [t - o for t, o in zip(ts, olds)]
    k = sum((x != 0).any(axis=1).astype(np.float32) for x in d)
    s = np.zeros_like(d[0])
    for x in d:
        s = s + x
    if rule == "align":
        nsq = sum((x.astype(np.float64) ** 2).sum(1) for x in d)
        tsq = (s.astype(np.float64) ** 2).sum(1)
        div = np.where(nsq > 0, np.clip(tsq / np.maximum(nsq, 1e-300), 1, np.maximum(k, 1)), 1)
        div = np.maximum(1.0, div ** beta / gamma)
    elif rule == "sum":
        div = np.ones(len(k))
    else:
        div = np.maximum(1.0, np.maximum(k, 1) ** beta / gamma)
    return olds[0] + s / div.astype(np.float32)[:, None]


def target(vec, mod, modules, rng_seed=35):
    u = vec / np.linalg.norm(vec, axis=1, keepdims=True)
    paths = []
    for m in range(min(modules, 300)):
        g = np.nonzero(mod == m)[0]
        if len(g) < 2:
            continue
        c = u[g] @ u[g].T
        iu = np.triu_indices(len(g), 1)
        paths.append(c[iu].mean())
    r = np.random.RandomState(rng_seed).permutation(len(vec))[:1000]
    c = u[r] @ u[r].T
    iu = np.triu_indices(len(r), 1)
    rm = c[iu].mean()
    return float(np.mean(paths) / rm), float(np.mean(paths)), float(rm)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--per", type=int, default=200_000)
    ap.add_argument("--vocab", type=int, default=3000)
    ap.add_argument("--modules", type=int, default=100)
    ap.add_argument("--p-module", type=float, default=0.5)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--every", type=int, default=2)
    ap.add_argument("--rules", default="touch,align")
    a = ap.parse_args()
    R, V0, D, K = a.replicas, a.vocab, a.dim, 5
    mod = RQ.module_of(V0, a.modules)
    pairs = np.concatenate([RQ.planted_pairs(a.per, V0, mod, a.modules, a.p_module, r)
                            for r in range(R)])
    n = len(pairs)
    flat = pairs.reshape(-1)
    counts, first = E.count_ids(flat, V0)
    order, remap = S.vocab_order(counts, first)
    tok = remap[flat]
    vc = counts[order].astype(np.int64)
    V = len(order)
    mod_v = mod[order]
    names = S.gene_names(V0)
    syn0 = E.seeded_vectors(np.array([zlib.crc32((names[i] + "1").encode()) for i in order],
                                     np.uint32), D)
    si, cum = CO.sample_int(vc, 1e-3), CO.make_cum_table(vc)
    lockf = np.ones(V, np.float32)
    ho = RQ.planted_pairs(20000, V0, mod, a.modules, a.p_module, 99)
    hc, hj = remap[ho[:, 0]], remap[ho[:, 1]]
    perms = [np.random.RandomState(100 + it).permutation(n) for it in range(a.iters)]

    def evaluate(s0, s1):
        r = np.random.Generator(np.random.PCG64(98))
        idx = r.integers(0, n, 20000)
        hi = RQ.objective(s0, s1, tok[2 * idx], tok[2 * idx + 1], vc, K, r)
        hoo = RQ.objective(s0, s1, hc, hj, vc, K, np.random.Generator(np.random.PCG64(97)))
        tr, pm, rm = target(s0, mod_v, a.modules)
        return {"heldin": round(hi, 5), "heldout": round(hoo, 5), "target": round(tr, 4),
                "path": round(pm, 4), "rand": round(rm, 4)}

    out = {}
    s0, s1 = syn0.copy(), np.zeros_like(syn0)
    rs = np.random.RandomState(1)
    for it in range(a.iters):
        t = tok.reshape(-1, 2)[perms[it]].reshape(-1)
        js = E.plan_jobs(n_sent=n, sent_len=2)
        CO.train(t, np.arange(0, 2 * n + 1, 2, dtype=np.int64), js,
                 E.job_alphas(js, n).astype(np.float32), E.job_seeds(rs, len(js) - 1), si, True,
                 cum, s0, s1, lockf, K)
    out["single"] = evaluate(s0, s1)
    print("single", out["single"], flush=True)
    for rule in a.rules.split(","):
        beta, gamma = 1.0, 1.0
        name = rule
        if ":" in rule:
            rule, b, g = rule.split(":")
            beta, gamma = float(b), float(g)
        reps = [[syn0.copy(), np.zeros_like(syn0)] for _ in range(R)]
        old = [syn0.copy(), np.zeros_like(syn0)]
        rs = np.random.RandomState(1)
        for it in range(a.iters):
            t = tok.reshape(-1, 2)[perms[it]].reshape(-1)
            base = int(rs.randint(0, 2 ** 31 - 1))
            shards = []
            for r in range(R):
                s0r, s1r = np.array_split(np.arange(n), R)[r][[0, -1]]
                tr = t[2 * s0r:2 * (s1r + 1)]
                jr = E.plan_jobs(n_sent=len(tr) // 2, sent_len=2)
                shards.append((tr, jr, E.job_alphas(jr, len(tr) // 2).astype(np.float32),
                               E.job_seeds(np.random.RandomState((base + 7919 * r) % 2 ** 32),
                                           len(jr) - 1)))
            nw = max((len(x[1]) - 1 + a.every - 1) // a.every for x in shards)
            for w in range(nw):
                for r, (tr, jr, al, sd) in enumerate(shards):
                    j0, j1 = w * a.every, min(len(jr) - 1, (w + 1) * a.every)
                    if j0 >= len(jr) - 1:
                        continue
                    off = np.arange(0, len(tr) + 1, 2, dtype=np.int64)
                    CO.train(tr, off, jr[j0:j1 + 1], al[j0:j1], sd[j0:j1], si, True, cum,
                             reps[r][0], reps[r][1], lockf, K)
                for tb in (0, 1):
                    m = merge(rule, [x[tb] for x in reps], [old[tb]] * R, beta, gamma)
                    old[tb] = m.copy()
                    for x in reps:
                        x[tb] = m.copy()
        out[name] = evaluate(*reps[0])
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
