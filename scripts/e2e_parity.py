"""End-to-end parity of the north-star metrics (verdict row n1):
the GPU trainer vs the gensim restatement on the same input, through the
reference's whole training flow.

gensim 3.4 is absent, so "gensim" here is oracle/sgns_oracle.c's sequential
trainer: gensim's workers=1 order (Appendix A), bit-compatible with the GPU's
sequential mode and its sampled stream.  The GPU side is the production path
(libg2v, k_sgns_atomic Hogwild).  Both train the reference's flow
(src/gene2vec.py:67-92): 10 iterations, the pairs reshuffled before every
iteration (one permutation per iteration, shared by both engines), the alpha
sawtooth restarting at every train() call, per-job seeds from model.random,
compute_loss on the last iteration.

Corpus: Zipf(1) gene pairs over --vocab genes with --modules planted
co-expression modules (gene2vec_amd/replica_study.planted_pairs: half the pairs
rewired inside the first gene's module) plus the reference's GGIPNN positive
pairs (data/predictionData, all three splits, label-leaky as in
scripts/ggipnn_e2e.py) repeated --ggipnn-repeat times.

Metrics after the 10th iteration:
  loss     gensim's get_latest_training_loss() of the last train() call (the
           GPU's Hogwild tally vs the oracle's terms summed in double; the
           oracle's float32 running sum is reported as well)
  heldin   SGNS objective on 50,000 corpus pairs
  target   the manuscript target function (gene2vec_amd/evaluate.py) with the
           planted modules as pathways
  auc      GGIPNN test AUC (gene2vec_amd/ggipnn.py), mean over classifier seeds
Each engine runs with --seeds model.random seeds (its own run-to-run spread).

    python scripts/e2e_parity.py --out gpurun_out/e2e_parity
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
from gene2vec_amd import replica_study as RQ  # noqa: E402
from gene2vec_amd import engine as E  # noqa: E402
from gene2vec_amd import synthetic as S  # noqa: E402
from oracle import c_oracle as CO  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=4_000_000)
    ap.add_argument("--vocab", type=int, default=5000)
    ap.add_argument("--modules", type=int, default=200)
    ap.add_argument("--p-module", type=float, default=0.5)
    ap.add_argument("--ggipnn-repeat", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dim", type=int, default=200)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--sample", type=float, default=1e-3)
    ap.add_argument("--seeds", default="1,2")
    ap.add_argument("--auc-seeds", default="0,1,2")
    ap.add_argument("--engines", default="gpu,oracle",
                    help="gpu (libg2v Hogwild), gpu_seq (libg2v sequential mode), gpu_gridN "
                         "(Hogwild on N workgroups), gpu_uncapped (Hogwild fixed at set_vocab's "
                         "default grid: no per-call stability cap), gpu_tailN (Hogwild with "
                         "G2V_OPT_TAIL_STORE N: gpu_tail0 every row atomic; gpu = the default, "
                         "the collision budget), oracle (sequential), "
                         "oracle_hogN (the C restatement's OpenMP Hogwild on N threads: gensim "
                         "workers=N)")
    ap.add_argument("--reference-engine", default="oracle",
                    help="the engine the summary's gaps are taken against (oracle, oracle_hogN)")
    ap.add_argument("--per-iter", action="store_true", help="print the GPU runs' objective per iteration")
    ap.add_argument("--out", default="gpurun_out/e2e_parity")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    D, K = a.dim, a.negative
    t0 = time.time()
    mod = RQ.module_of(a.vocab, a.modules)
    pairs = RQ.planted_pairs(a.pairs, a.vocab, mod, a.modules, a.p_module, 0)
    names = S.gene_names(a.vocab)
    pos = RQ.positives()
    gid = {}
    for x, y in pos:
        for g in (x, y):
            if g not in gid:
                gid[g] = a.vocab + len(gid)
    names += list(gid)
    pp = np.array([[gid[x], gid[y]] for x, y in pos], np.int32)
    pairs = np.concatenate([pairs] + [pp] * a.ggipnn_repeat)
    n = len(pairs)
    flat = pairs.reshape(-1)
    counts, first = E.count_ids(flat, len(names))
    order, remap = S.vocab_order(counts, first)
    tok0 = remap[flat].astype(np.int32)
    vc = counts[order].astype(np.int64)
    V = len(order)
    index2word = [names[i] for i in order]
    pos_genes = {g for p in pos for g in p}
    gmt = os.path.join(a.out, "modules.gmt")
    RQ.module_gmt(gmt, mod, a.modules, names, n_paths=min(300, a.modules))
    seeds_w = np.array([zlib.crc32((w + "1").encode()) for w in index2word], np.uint32)
    syn0 = E.seeded_vectors(seeds_w, D)
    # one permutation of the pairs per iteration, shared by both engines
    # (src/gene2vec.py:52,80 reshuffle before every train() call)
    rs_perm = np.random.RandomState(11)
    perms = [rs_perm.permutation(n) for _ in range(a.iters)]
    js = E.plan_jobs(n_sent=n, sent_len=2)
    al = E.job_alphas(js, n)
    off = np.arange(0, 2 * n + 1, 2, dtype=np.int64)
    si, cum = CO.sample_int(vc, a.sample), CO.make_cum_table(vc)
    lockf = np.ones(V, np.float32)
    log = {"config": {"pairs_total": n, "vocab": V, "modules": a.modules, "p_tok_max": None,
                      "ggipnn_repeat": a.ggipnn_repeat, "iters": a.iters, "dim": D,
                      "negative": K, "sample": a.sample},
           "corpus_s": round(time.time() - t0, 1), "runs": {}}
    print(json.dumps(log["config"]), flush=True)

    def tokens(it):
        return np.ascontiguousarray(tok0.reshape(n, 2)[perms[it]].reshape(-1))

    # the stability cap's product (g2v_api.hip stability_grid): waves x p_tok_max
    # x (K+1) x alpha x max |syn1neg[r]|^2, capped at 100
    tot = float(vc.sum())
    thr = a.sample * tot if 0 < a.sample < 1 else tot
    pt = vc * np.minimum(1.0, (np.sqrt(vc / thr) + 1.0) * (thr / vc))
    p_tok_max = float((pt / pt.sum()).max())
    log["config"]["p_tok_max"] = p_tok_max

    def train_gpu(seed, mode=N.MODE_HOGWILD, grid=0, overlap=None, tail=None):
        eng = E.SGNSEngine(V, D, K)
        if tail is not None:
            eng.set_option(N.OPT_TAIL_STORE, tail)
        if grid == -1:  # set_vocab's default, fixed (no per-call cap)
            probe = E.SGNSEngine(V, D, K)
            probe.set_vocab(vc, a.sample)
            grid = int(probe.get_option(N.OPT_GRID))
            probe.close()
        if grid:
            eng.set_option(N.OPT_GRID, grid)
        if overlap is not None:
            eng.set_option(N.OPT_ATOMIC_OVERLAP, overlap)
        eng.set_vocab(vc, a.sample)
        eng.set_weights(syn0, np.zeros_like(syn0))
        rs = np.random.RandomState(seed)
        for it in range(a.iters):
            last = it == a.iters - 1
            eng.set_corpus(tokens(it), sent_len=2)
            if last:
                eng.reset_loss()
            eng.train(js, al, E.job_seeds(rs, len(js) - 1), mode, compute_loss=last)
            eng.sync()
            if a.per_iter:
                g0, g1 = eng.get_weights()
                n0 = (g0.astype(np.float64) ** 2).sum(1)
                n1 = (g1.astype(np.float64) ** 2).sum(1)
                cw = eng.read_stats()['sgns_waves']
                prod = cw * p_tok_max * (K + 1) * float(al.max()) * n1.max()
                print(f"  gpu grid {grid} (last launch {cw} waves, cap product at the call's "
                      f"end {prod:.1f}) seed {seed} "
                      f"iteration {it + 1} heldin "
                      f"{RQ.heldin(g0, g1, tok0, vc, K, n=20000):.5f} |syn0|^2 max/top20 "
                      f"{n0.max():.2f}/{n0[:20].max():.2f} |syn1neg|^2 max/top20 "
                      f"{n1.max():.2f}/{n1[:20].max():.2f}", flush=True)
        st = eng.read_stats()
        extra = {"grid": int(eng.get_option(N.OPT_GRID)), "last_launch_waves": int(st["sgns_waves"]),
                 "tail_row_syn1neg": int(st["tail_row_syn1neg"]),
                 "tail_row_syn0": int(st["tail_row_syn0"])}
        s0, s1 = eng.get_weights()
        eng.close()
        return s0, s1, {"loss": float(st["training_loss"]), **extra}

    def train_oracle(seed, threads=0):
        a0, a1 = syn0.copy(), np.zeros_like(syn0)
        rs = np.random.RandomState(seed)
        extra = {}
        for it in range(a.iters):
            last = it == a.iters - 1
            loss = np.zeros(1, np.float32) if last and not threads else None
            lex = np.zeros(1, np.float64) if last and not threads else None
            CO.train(tokens(it), off, js, al.astype(np.float32), E.job_seeds(rs, len(js) - 1), si,
                     a.sample != 0, cum, a0, a1, lockf, K, nthreads=threads, loss=loss,
                     loss_exact=lex)
            if last and not threads:
                extra = {"loss": float(lex[0]), "loss_float32_running": float(loss[0])}
            print(f"  oracle threads {threads} seed {seed} iteration {it + 1} done", flush=True)
        return a0, a1, extra

    for eng_name in a.engines.split(","):
        for seed in (int(x) for x in a.seeds.split(",")):
            t = time.time()
            if eng_name == "gpu":
                s0, s1, extra = train_gpu(seed)
            elif eng_name == "gpu_seq":
                s0, s1, extra = train_gpu(seed, N.MODE_SEQUENTIAL)
            elif eng_name.startswith("gpu_ov"):
                s0, s1, extra = train_gpu(seed, overlap=int(eng_name[6:]))
            elif eng_name.startswith("gpu_grid"):
                s0, s1, extra = train_gpu(seed, grid=int(eng_name[8:]))
            elif eng_name.startswith("gpu_tail"):
                s0, s1, extra = train_gpu(seed, tail=int(eng_name[8:]))
            elif eng_name == "gpu_uncapped":
                s0, s1, extra = train_gpu(seed, grid=-1)
            elif eng_name.startswith("oracle_hog"):
                s0, s1, extra = train_oracle(seed, int(eng_name[10:]))
            else:
                s0, s1, extra = train_oracle(seed)
            tr = time.time() - t
            res = {"train_s": round(tr, 1), **extra,
                   "heldin": round(RQ.heldin(s0, s1, tok0, vc, K), 5)}
            t = RQ.target_of(s0, index2word, vc, gmt, D)
            res.update({"target_ratio": t["ratio"], "path_mean": t["path_mean"],
                        "rand_mean": t["rand_mean"], "n_pathways": t["n_pathways"]})
            auc_seeds = [int(x) for x in a.auc_seeds.split(",") if x]
            if auc_seeds:
                aucs = RQ.ggipnn_auc(s0, index2word, pos_genes, auc_seeds)
                res.update({"auc": aucs, "auc_mean": float(np.mean(aucs))})
            log["runs"][f"{eng_name}_seed{seed}"] = res
            print(eng_name, seed, json.dumps(res), flush=True)
            json.dump(log, open(os.path.join(a.out, "e2e_parity.json"), "w"), indent=1)

    # gaps of the GPU runs to the oracle runs' mean, beside the oracle's own spread
    def mean(engine, key):
        v = [r[key] for t, r in log["runs"].items() if t.startswith(engine + "_seed") and key in r]
        return float(np.mean(v)) if v else None
    summ = {}
    ref = a.reference_engine
    others = [x for x in a.engines.split(",") if x != ref]
    summ["reference"] = ref
    for key in ("loss", "heldin", "target_ratio", "auc_mean"):
        o = mean(ref, key)
        ov = [r[key] for t, r in log["runs"].items() if t.startswith(ref + "_seed") and key in r]
        summ[key] = {"oracle": o,
                     "oracle_spread": round((max(ov) - min(ov)) / abs(np.mean(ov)), 5)
                     if len(ov) > 1 else None}
        for eng_name in others:
            g = mean(eng_name, key)
            summ[key][eng_name] = g
            summ[key][eng_name + "_gap"] = (None if g is None or o is None
                                            else round((g - o) / o, 5))
        if "gpu" in others:  # (the field name earlier rounds' files use)
            summ[key]["gap"] = summ[key]["gpu_gap"]
    log["summary"] = summ
    json.dump(log, open(os.path.join(a.out, "e2e_parity.json"), "w"), indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
