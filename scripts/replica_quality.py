"""Data-parallel quality at the configuration C3 runs (verdict r2 item 1).

The reference trains ONE model with 32 Hogwild threads (src/gene2vec.py:59,70);
C3 trains 8 replicas on 8 x 125 M pairs and merges them with libg2v's touch
rule every --merge-every jobs.  This script runs both on ONE GPU and compares
them on the same corpus, the same per-iteration shuffles and the reference's
10-iteration alpha sawtooth (src/gene2vec.py:67-92):

  replicas  R engines, one host thread each, an in-process replica group
            (g2v_comm_init_local: libg2v's delta/apply kernels and in-call
            merges, the all-reduce a device sum) -- the production merge path
            of the data-parallel CLI (word2vec.Word2Vec._bind_replica /
            distributed.ReplicaTrainer), rank r training the r-th contiguous
            1/R of each iteration's permutation with its own job seeds and its
            shard's alpha schedule (word2vec.Word2Vec.train_ids)
  single    one engine over the whole permutation (gensim's one model)

Corpus ("C3q"): C3's synthetic Zipf(1) pairs over 24,447 genes (R shards of
bench.py's generator) plus the positive pairs of the reference's GGIPNN splits
(data/predictionData, all three) repeated --ggipnn-repeat times, so the run
also carries real gene-pair structure: a label-leaky harness (test positives
are trained on) that measures data-parallel vs single-model parity only, as
scripts/ggipnn_e2e.py does.  Metrics after the last iteration:
  heldin   SGNS objective on 50,000 corpus pairs (K unigram^0.75 negatives)
  auc      GGIPNN test AUC (gene2vec_amd/ggipnn.py) on the exported .txt,
           mean over --auc-seeds classifier seeds
  target   the manuscript target function (gene2vec_amd/evaluate.py) on a
           synthetic .gmt: neighbourhoods of the positive-pair graph
           (MSigDB is absent)

    python scripts/replica_quality.py --merge-every 1024,4096 --out gpurun_out/rq
"""
import argparse
import json
import os
import sys
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gene2vec_amd import _native as N  # noqa: E402
from gene2vec_amd import distributed as Dd  # noqa: E402
from gene2vec_amd import engine as E  # noqa: E402
from gene2vec_amd import synthetic as S  # noqa: E402

DATA = os.path.join(ROOT, "data", "predictionData")


def positives():
    out = []
    for part in ("train", "valid", "test"):
        text = open(os.path.join(DATA, f"{part}_text.txt")).read().splitlines()
        lab = open(os.path.join(DATA, f"{part}_label.txt")).read().splitlines()
        out += [t.split() for t, l in zip(text, lab) if l == "1" and len(t.split()) == 2]
    return out


def module_of(V0, modules, seed=3):
    """planted co-expression modules: gene g -> module (a random balanced split)"""
    perm = np.random.RandomState(seed).permutation(V0)
    mod = np.empty(V0, np.int64)
    mod[perm] = np.arange(V0) % modules
    return mod


def planted_pairs(n, V0, mod, modules, p_in, shard):
    """C3's Zipf(1) pairs, a fraction p_in of them rewired inside the first
    gene's module (the second gene uniform among its module mates): every gene
    keeps a Zipf-like degree and gains co-expression partners, so the target
    function's pathways (= the modules) and its random pairs both mean something"""
    pairs = S.zipf_gene_pairs(n, V0, 1.0, seed=20250114, shard=shard)
    rng = np.random.Generator(np.random.PCG64(9000 + shard))
    order = np.argsort(mod, kind="stable")
    start = np.searchsorted(mod[order], np.arange(modules))
    size = np.bincount(mod, minlength=modules)
    sel = np.nonzero(rng.random(n) < p_in)[0]
    a = pairs[sel, 0]
    m = mod[a]
    b = order[start[m] + (rng.random(len(sel)) * size[m]).astype(np.int64)]
    bad = b == a
    while bad.any():
        mb = m[bad]
        b[bad] = order[start[mb] + (rng.random(int(bad.sum())) * size[mb]).astype(np.int64)]
        bad = b == a
    pairs[sel, 1] = b
    return pairs


def build_corpus(R, per, V0, rep, seed, modules=0, p_in=0.0):
    """(pairs int32[N][2] in id space, names by id, positive pairs by name)"""
    mod = module_of(V0, modules) if modules else None

    def shard(r):
        if modules:
            return planted_pairs(per, V0, mod, modules, p_in, r)
        return S.zipf_gene_pairs(per, V0, 1.0, seed=20250114, shard=r)
    with ThreadPoolExecutor(max_workers=min(R, 16)) as ex:
        shards = list(ex.map(shard, range(R)))
    names = S.gene_names(V0)
    pos = positives()
    gid = {}
    for a, b in pos:
        for g in (a, b):
            if g not in gid:
                gid[g] = V0 + len(gid)
    names += list(gid)
    pp = np.array([[gid[a], gid[b]] for a, b in pos], np.int32)
    parts = shards + [np.tile(pp, (rep, 1))] if rep else shards
    pairs = np.concatenate(parts)
    del shards, parts
    return pairs, names, pos


def module_gmt(path, mod, modules, names, n_paths=300, seed=0):
    """pathways = planted modules (random 300 of them)"""
    rng = np.random.RandomState(seed)
    with open(path, "w") as f:
        for k, m in enumerate(rng.choice(modules, size=min(n_paths, modules), replace=False)):
            genes = [names[g] for g in np.nonzero(mod == m)[0]]
            f.write("\t".join([f"MODULE{m}", "http://synthetic"] + genes) + "\n")


def synthetic_gmt(path, pos, n_paths=300, max_genes=40, seed=0):
    """pathways = a gene and its positive-pair neighbours (>= 4 of them)"""
    nb = {}
    for a, b in pos:
        nb.setdefault(a, set()).add(b)
        nb.setdefault(b, set()).add(a)
    rng = np.random.RandomState(seed)
    cands = sorted(g for g, s in nb.items() if len(s) >= 4)
    pick = rng.choice(len(cands), size=min(n_paths, len(cands)), replace=False)
    with open(path, "w") as f:
        for k, i in enumerate(pick):
            g = cands[i]
            genes = [g] + sorted(nb[g])[:max_genes - 1]
            f.write("\t".join([f"PATH{k}", "http://synthetic"] + genes) + "\n")


def heldin(s0, s1, tok, counts, K, n=50000, seed=99):
    rng = np.random.Generator(np.random.PCG64(seed))
    idx = rng.integers(0, len(tok) // 2, n)
    return objective(s0, s1, tok[2 * idx], tok[2 * idx + 1], counts, K, rng)


def objective(s0, s1, c, j, counts, K, rng):
    """mean SGNS objective of pairs (c, j) with K unigram^0.75 negatives"""
    p = counts.astype(np.float64) ** 0.75
    negs = rng.choice(len(counts), size=(len(c), K), p=p / p.sum())
    u = s0[j].astype(np.float64)
    pos = np.einsum("nd,nd->n", u, s1[c].astype(np.float64))
    neg = np.einsum("nd,nkd->nk", u, s1[negs].astype(np.float64))
    return float((np.logaddexp(0, -pos) + np.logaddexp(0, neg).sum(1)).mean())


def export_and_score(tag, s0, index2word, counts, pos_genes, gmt, out, auc_seeds, D):
    """exports (_w2v.txt, .txt) to a scratch directory, scored, then deleted
    (tens of MB each: they stay out of gpurun_out)"""
    import shutil
    import tempfile
    out = tempfile.mkdtemp(prefix="rq_")
    try:
        return _export_and_score(tag, s0, index2word, counts, pos_genes, gmt, out, auc_seeds, D)
    finally:
        shutil.rmtree(out, ignore_errors=True)


def _export_and_score(tag, s0, index2word, counts, pos_genes, gmt, out, auc_seeds, D):
    from gene2vec_amd import evaluate as EV
    from gene2vec_amd import ggipnn as G
    from gene2vec_amd.word2vec import KeyedVectors, Vocab
    kv = KeyedVectors(D)
    kv.index2word = list(index2word)
    kv.vocab = {w: Vocab(count=int(counts[i]), index=i) for i, w in enumerate(index2word)}
    kv.vectors = np.ascontiguousarray(s0, np.float32)
    w2v = os.path.join(out, f"{tag}_w2v.txt")
    kv.save_word2vec_format(w2v)
    t = EV.target_function(w2v, gmt, strict=False, verbose=False)
    txt = os.path.join(out, f"{tag}.txt")
    with open(txt, "w") as f:  # generateMatrix layout, the GGIPNN genes only
        for i, w in enumerate(index2word):
            if w in pos_genes:
                f.write(w + "\t" + "".join(v + " " for v in s0[i].astype(np.float32).astype(str))
                        + "\n")
    aucs = [G.train_and_auc(txt, DATA, seed=s, device="cuda") for s in auc_seeds]
    return {"target_ratio": t["ratio"], "path_mean": t["path_mean"], "rand_mean": t["rand_mean"],
            "n_pathways": t["n_pathways"], "auc": aucs, "auc_mean": float(np.mean(aucs))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--pairs-per-replica", type=int, default=125_000_000)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--merge-every", default="1024", help="comma-separated job cadences")
    ap.add_argument("--rules", default="1000:1000",
                    help="comma-separated merge rules: 'align', 'mean', or a touch-rule shape "
                         "beta:gamma x 1000 (G2V_OPT_MERGE_BETA_MILLI / _GAMMA_MILLI)")
    ap.add_argument("--no-eval", action="store_true",
                    help="held-in objective only (no exports, target function, GGIPNN)")
    ap.add_argument("--vocab", type=int, default=24447)
    ap.add_argument("--dim", type=int, default=200)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--sample", type=float, default=1e-3)
    ap.add_argument("--ggipnn-repeat", type=int, default=30)
    ap.add_argument("--modules", type=int, default=0,
                    help="plant this many co-expression modules in the Zipf pairs (the "
                         "target function's pathways are then the modules)")
    ap.add_argument("--p-module", type=float, default=0.5)
    ap.add_argument("--auc-seeds", default="0,1,2")
    ap.add_argument("--no-single", action="store_true")
    ap.add_argument("--single-seeds", default="1",
                    help="model.random seeds of the one-model runs (several: the one model's "
                         "own run-to-run spread, the yardstick for the replica gaps)")
    ap.add_argument("--oracle", action="store_true",
                    help="also train the sequential C oracle (gensim workers=1 order) on the same "
                         "permutations and job seeds as the first one-model run")
    ap.add_argument("--out", default="gpurun_out/replica_quality")
    a = ap.parse_args()
    import torch
    os.makedirs(a.out, exist_ok=True)
    R, D, K = a.replicas, a.dim, a.negative
    t0 = time.time()
    pairs, names, pos = build_corpus(R, a.pairs_per_replica, a.vocab, a.ggipnn_repeat, 5,
                                     a.modules, a.p_module)
    n = len(pairs)
    flat = pairs.reshape(-1)
    del pairs
    counts, first = E.count_ids(flat, len(names))
    order, remap = S.vocab_order(counts, first)
    tok = remap[flat]
    del flat
    vc = counts[order].astype(np.int64)
    V = len(order)
    index2word = [names[i] for i in order]
    pos_genes = {g for p in pos for g in p}
    gmt = os.path.join(a.out, "synthetic.gmt")
    if a.modules:
        module_gmt(gmt, module_of(a.vocab, a.modules), a.modules, names)
    else:
        synthetic_gmt(gmt, pos)
    seeds = np.array([zlib.crc32((w + "1").encode()) for w in index2word], np.uint32)
    syn0 = E.seeded_vectors(seeds, D)
    dev = torch.device("cuda", 0)
    base = torch.from_numpy(tok.view(np.int64)).to(dev)  # one pair per 8-byte item
    perm = torch.empty_like(base)
    rs_perm = np.random.RandomState(11)
    perm_seeds = [int(rs_perm.randint(0, 2 ** 62)) for _ in range(a.iters)]
    log = {"config": {"replicas": R, "pairs_per_replica": a.pairs_per_replica,
                      "ggipnn_repeat": a.ggipnn_repeat, "modules": a.modules,
                      "p_module": a.p_module if a.modules else 0.0, "pairs_total": n, "vocab": V,
                      "dim": D, "negative": K, "sample": a.sample, "iters": a.iters},
           "corpus_s": round(time.time() - t0, 1), "runs": {}}
    print(json.dumps(log["config"]), flush=True)
    st = torch.cuda.current_stream(dev)

    def permute(it):
        E.permute_items8(0, base.data_ptr(), perm.data_ptr(), n, 0, n, perm_seeds[it],
                         st.cuda_stream)
        st.synchronize()

    # held-out pairs: a fresh draw of C3's Zipf generator (another seed), so
    # memorising the training pairs does not count as quality
    ho = S.zipf_gene_pairs(50000, a.vocab, 1.0, seed=777)
    ho_c, ho_j = remap[ho[:, 0]], remap[ho[:, 1]]
    keep = (ho_c >= 0) & (ho_j >= 0)
    ho_c, ho_j = ho_c[keep], ho_j[keep]

    def heldout(s0, s1):
        return objective(s0, s1, ho_c, ho_j, vc, K, np.random.Generator(np.random.PCG64(98)))

    def finish(tag, s0, s1, extra):
        res = {"heldin": round(heldin(s0, s1, tok, vc, K), 5),
               "heldout": round(heldout(s0, s1), 5)}
        if not a.no_eval:
            res.update(export_and_score(tag, s0, index2word, vc, pos_genes, gmt, a.out,
                                        [int(x) for x in a.auc_seeds.split(",")], D))
        res.update(extra)
        log["runs"][tag] = res
        print(tag, json.dumps(res), flush=True)
        json.dump(log, open(os.path.join(a.out, "replica_quality.json"), "w"), indent=1)

    # ---- one model over the whole corpus ----------------------------------------
    for si, sseed in enumerate(int(x) for x in a.single_seeds.split(",")):
        if a.no_single:
            break
        eng = E.SGNSEngine(V, D, K)
        eng.set_vocab(vc, a.sample)
        eng.set_weights(syn0, np.zeros_like(syn0))
        rs = np.random.RandomState(sseed)
        js = E.plan_jobs(n_sent=n, sent_len=2)
        al = E.job_alphas(js, n)
        t = time.time()
        per_it = []
        for it in range(a.iters):
            permute(it)
            eng.set_corpus_device(perm.data_ptr(), 2 * n, sent_len=2, keepalive=perm)
            eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD)
            eng.sync()
            g0, g1 = eng.get_weights()
            per_it.append((round(heldin(g0, g1, tok, vc, K, n=20000), 5), round(heldout(g0, g1), 5)))
            print("single", sseed, "iter", it, per_it[-1], flush=True)
        s0, s1 = eng.get_weights()
        eng.close()
        finish("single" if si == 0 else f"single_seed{sseed}", s0, s1,
               {"train_s": round(time.time() - t, 1), "heldin_per_iter": per_it})

    # ---- the sequential oracle (gensim's workers=1 order) -----------------------------
    if a.oracle:
        from oracle import c_oracle as CO
        a0, a1 = syn0.copy(), np.zeros_like(syn0)
        rs = np.random.RandomState(int(a.single_seeds.split(",")[0]))
        js = E.plan_jobs(n_sent=n, sent_len=2)
        al = E.job_alphas(js, n).astype(np.float32)
        off = np.arange(0, 2 * n + 1, 2, dtype=np.int64)
        si, cum = CO.sample_int(vc, a.sample), CO.make_cum_table(vc)
        t = time.time()
        for it in range(a.iters):
            permute(it)
            tk = perm.cpu().numpy().view(np.int32)
            CO.train(tk, off, js, al, E.job_seeds(rs, len(js) - 1), si, a.sample != 0, cum, a0,
                     a1, np.ones(V, np.float32), K)
            print("oracle iter", it, round(heldin(a0, a1, tok, vc, K, n=20000), 5), flush=True)
        finish("oracle", a0, a1, {"train_s": round(time.time() - t, 1)})

    # ---- R replicas, libg2v merge every c jobs ---------------------------------------
    def parse_rule(r):
        """'mean', 'touch:B:G', 'align:B:G' (B, G = beta, gamma x 1000) or 'B:G' (touch)"""
        parts = r.split(":")
        if parts[0] in ("align", "mean", "touch"):
            name, parts = parts[0], parts[1:]
        else:
            name = "touch"
        b, g = (int(parts[0]), int(parts[1])) if parts else (1000, 1000)
        return name, b, g
    combos = [(int(e),) + parse_rule(r) for e in a.merge_every.split(",")
              for r in a.rules.split(",")]
    for every, rule, beta, gamma in combos:
        grp = E.LocalGroup(R)
        agree = Dd.ThreadAgreement(R)
        engs = []
        for r in range(R):
            e = E.SGNSEngine(V, D, K)
            e.set_vocab(vc, a.sample)
            e.set_weights(syn0, np.zeros_like(syn0))
            e.set_option(N.OPT_MERGE_BETA_MILLI, beta)
            e.set_option(N.OPT_MERGE_GAMMA_MILLI, gamma)
            engs.append(e)
        with ThreadPoolExecutor(max_workers=R) as ex:
            list(ex.map(lambda r: engs[r].comm_init_local(grp, r), range(R)))
        trainers = [Dd.ReplicaTrainer(engs[r], (), every, N.MODE_HOGWILD, merge=rule,
                                      backend="libg2v", world=R, agree=agree.for_rank(r))
                    for r in range(R)]
        rs = np.random.RandomState(1)  # model.random, identical on every rank
        t = time.time()
        per_it = []
        for it in range(a.iters):
            permute(it)
            base_seed = int(rs.randint(0, 2 ** 31 - 1))

            def rank(r):
                s0r, s1r = Dd.shard_range(n, r, R)
                e = engs[r]
                e.set_corpus_device(perm.data_ptr() + 8 * s0r, 2 * (s1r - s0r), sent_len=2,
                                    keepalive=perm)
                js = E.plan_jobs(n_sent=s1r - s0r, sent_len=2)
                al = E.job_alphas(js, s1r - s0r)
                sd = E.job_seeds(np.random.RandomState((base_seed + 7919 * r) % 2 ** 32),
                                 len(js) - 1)
                trainers[r].train_epoch(js, al, sd)
                e.sync()
            with ThreadPoolExecutor(max_workers=R) as ex:
                list(ex.map(rank, range(R)))
            g0, g1 = engs[0].get_weights()
            per_it.append((round(heldin(g0, g1, tok, vc, K, n=20000), 5), round(heldout(g0, g1), 5)))
            print(f"replicas x{R} every {every} {rule} beta {beta} gamma {gamma} iter {it} "
                  f"{per_it[-1]}", flush=True)
        s0, s1 = engs[0].get_weights()
        same = all(np.array_equal(e.get_weights()[0], s0) for e in engs[1:])
        merges = trainers[0].averages
        for e in engs:
            e.close()
        grp.close()
        finish(f"replicas{R}_every{every}" + (f"_{rule}" if rule != "touch" else "")
               + (f"_beta{beta}" if beta != 1000 else "")
               + (f"_gamma{gamma}" if gamma != 1000 else ""), s0, s1,
               {"train_s": round(time.time() - t, 1), "heldin_per_iter": per_it,
                "merges_total": merges, "replicas_identical": same})
    for ref_tag in ("single", "oracle"):
        if ref_tag not in log["runs"]:
            continue
        ref = log["runs"][ref_tag]
        sfx = "" if ref_tag == "single" else "_vs_oracle"
        for tag, r in log["runs"].items():
            if tag != ref_tag:  # gaps to the reference run
                r["heldin_gap" + sfx] = round((r["heldin"] - ref["heldin"]) / ref["heldin"], 5)
                r["heldout_gap" + sfx] = round((r["heldout"] - ref["heldout"]) / ref["heldout"],
                                               5)
                if "auc_mean" in r and "auc_mean" in ref:
                    r["auc_gap" + sfx] = round((r["auc_mean"] - ref["auc_mean"])
                                               / ref["auc_mean"], 5)
                    r["target_gap" + sfx] = round((r["target_ratio"] - ref["target_ratio"])
                                                  / ref["target_ratio"], 5)
        json.dump(log, open(os.path.join(a.out, "replica_quality.json"), "w"), indent=1)
    for tag, r in log["runs"].items():
        print(tag, {k: r[k] for k in ("heldin", "heldin_gap", "heldin_gap_vs_oracle", "heldout",
                                      "heldout_gap", "heldout_gap_vs_oracle", "auc_mean",
                                      "auc_gap", "auc_gap_vs_oracle", "target_ratio",
                                      "target_gap", "target_gap_vs_oracle") if k in r})
    print(json.dumps(log))


if __name__ == "__main__":
    main()
