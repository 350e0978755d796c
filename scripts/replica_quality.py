"""Data-parallel quality at the configuration C3 runs.

The reference trains ONE model with 32 Hogwild threads (src/gene2vec.py:59,70);
C3 trains 8 replicas on 8 x 125 M pairs and merges them with libg2v's touch
rule every --merge-every jobs.  This script runs both on ONE GPU over the same
corpus, per-iteration shuffles and alpha sawtooth (src/gene2vec.py:67-92); the
harness (corpus, arms, metrics) is gene2vec_amd/replica_study.py, shared with
tests/test_gpu_c3_quality.py.

    python scripts/replica_quality.py --merge-every 1024,4096 --out gpurun_out/rq
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gene2vec_amd import engine as E  # noqa: E402
from gene2vec_amd import replica_study as RQ  # noqa: E402


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
                    help="held-in / held-out objectives only (no target function, GGIPNN)")
    ap.add_argument("--no-auc", action="store_true", help="skip GGIPNN AUC")
    ap.add_argument("--vocab", type=int, default=24447)
    ap.add_argument("--dim", type=int, default=200)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--sample", type=float, default=1e-3)
    ap.add_argument("--ggipnn-repeat", type=int, default=30)
    ap.add_argument("--modules", type=int, default=0,
                    help="plant this many co-expression modules in the Zipf pairs (the "
                         "target function's pathways are then the modules)")
    ap.add_argument("--p-module", type=float, default=0.5)
    ap.add_argument("--zipf", type=float, default=1.0, help="Zipf exponent of the pair endpoints")
    ap.add_argument("--auc-seeds", default="0,1,2")
    ap.add_argument("--no-single", action="store_true")
    ap.add_argument("--single-seeds", default="1",
                    help="model.random seeds of the one-model runs (several: the one model's "
                         "own run-to-run spread, the yardstick for the replica gaps)")
    ap.add_argument("--replica-seeds", default="1",
                    help="model.random seeds of the replica runs (each gives the ranks' job-seed "
                         "streams); several: every cadence / rule runs once per seed")
    ap.add_argument("--oracle", action="store_true",
                    help="also train the sequential C oracle (gensim workers=1 order) on the same "
                         "permutations and job seeds as the first one-model run")
    ap.add_argument("--ensemble-singles", action="store_true",
                    help="also score the plain average of the one-model runs' tables (the "
                         "ensemble effect of averaging independently trained models)")
    ap.add_argument("--tail-store", type=int, default=0,
                    help="G2V_OPT_TAIL_STORE on every engine (experiment, DESIGN.md 5e)")
    ap.add_argument("--out", default="gpurun_out/replica_quality")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    K, D = a.negative, a.dim
    t0 = time.time()
    from gene2vec_amd import _native as N
    st = RQ.Study(a.replicas, a.pairs_per_replica, a.vocab, a.ggipnn_repeat, a.modules,
                  a.p_module, a.zipf, a.iters, D, K, a.sample,
                  engine_options={N.OPT_TAIL_STORE: a.tail_store} if a.tail_store else None)
    gmt = st.gmt(os.path.join(a.out, "synthetic.gmt"))
    log = {"config": {"replicas": a.replicas, "pairs_per_replica": a.pairs_per_replica,
                      "ggipnn_repeat": a.ggipnn_repeat, "modules": a.modules,
                      "p_module": a.p_module if a.modules else 0.0, "zipf": a.zipf,
                      "pairs_total": st.n, "vocab": st.V, "dim": D, "negative": K,
                      "sample": a.sample, "iters": a.iters, "tail_store": a.tail_store},
           "corpus_s": round(time.time() - t0, 1), "runs": {}}
    print(json.dumps(log["config"]), flush=True)
    auc_seeds = [int(x) for x in a.auc_seeds.split(",")]

    def progress(tag):
        per_it = []

        def cb(kind, it, eng):
            g0, g1 = eng.get_weights()
            r = (round(st.heldin(g0, g1, n=20000), 5), round(st.heldout(g0, g1), 5))
            per_it.append(r)
            print(tag, "iter", it, r, flush=True)
        return cb, per_it

    def finish(tag, s0, s1, extra):
        res = {"heldin": round(st.heldin(s0, s1), 5), "heldout": round(st.heldout(s0, s1), 5)}
        if not a.no_eval:
            t = RQ.target_of(s0, st.index2word, st.vc, gmt, D)
            res.update({"target_ratio": t["ratio"], "path_mean": t["path_mean"],
                        "rand_mean": t["rand_mean"], "n_pathways": t["n_pathways"]})
            if not a.no_auc:
                aucs = RQ.ggipnn_auc(s0, st.index2word, st.pos_genes, auc_seeds)
                res.update({"auc": aucs, "auc_mean": float(np.mean(aucs))})
        res.update(extra)
        log["runs"][tag] = res
        print(tag, json.dumps(res), flush=True)
        json.dump(log, open(os.path.join(a.out, "replica_quality.json"), "w"), indent=1)

    # ---- one model over the whole corpus ----------------------------------------
    singles = []
    for si, sseed in enumerate(int(x) for x in a.single_seeds.split(",")):
        if a.no_single:
            break
        tag = "single" if si == 0 else f"single_seed{sseed}"
        cb, per_it = progress(f"single {sseed}")
        t = time.time()
        s0, s1 = st.train_single(sseed, progress=cb)
        finish(tag, s0, s1, {"train_s": round(time.time() - t, 1), "heldin_per_iter": per_it})
        if a.ensemble_singles:
            singles.append((s0, s1))
    if len(singles) > 1:
        # the models trained independently (their own job seeds, the same
        # permutations), averaged once at the end: no merge during training
        e0 = np.mean([x[0] for x in singles], axis=0, dtype=np.float64).astype(np.float32)
        e1 = np.mean([x[1] for x in singles], axis=0, dtype=np.float64).astype(np.float32)
        finish("single_ensemble", e0, e1, {"members": len(singles)})

    # ---- the sequential oracle (gensim's workers=1 order) -----------------------------
    if a.oracle:
        from oracle import c_oracle as CO
        a0, a1 = st.syn0.copy(), np.zeros_like(st.syn0)
        rs = np.random.RandomState(int(a.single_seeds.split(",")[0]))
        js = E.plan_jobs(n_sent=st.n, sent_len=2)
        al = E.job_alphas(js, st.n).astype(np.float32)
        off = np.arange(0, 2 * st.n + 1, 2, dtype=np.int64)
        si_, cum = CO.sample_int(st.vc, a.sample), CO.make_cum_table(st.vc)
        t = time.time()
        for it in range(a.iters):
            st.permute(it)
            tk = st.perm.cpu().numpy().view(np.int32)
            CO.train(tk, off, js, al, E.job_seeds(rs, len(js) - 1), si_, a.sample != 0, cum, a0,
                     a1, np.ones(st.V, np.float32), K)
            print("oracle iter", it, round(st.heldin(a0, a1, n=20000), 5), flush=True)
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
    combos = [(int(e),) + parse_rule(r) + (int(sd),) for e in a.merge_every.split(",")
              for r in a.rules.split(",") for sd in a.replica_seeds.split(",")]
    R = a.replicas
    for every, rule, beta, gamma, rseed in combos:
        tag = (f"replicas{R}_every{every}" + (f"_{rule}" if rule != "touch" else "")
               + (f"_beta{beta}" if beta != 1000 else "")
               + (f"_gamma{gamma}" if gamma != 1000 else "")
               + (f"_seed{rseed}" if rseed != 1 else ""))
        cb, per_it = progress(tag)
        t = time.time()
        s0, s1, merges, same = st.train_replicas(every, rule, beta, gamma, rseed, progress=cb)
        finish(tag, s0, s1, {"train_s": round(time.time() - t, 1), "heldin_per_iter": per_it,
                             "merges_total": merges, "replicas_identical": same})
    for ref_tag in ("single", "oracle"):
        if ref_tag not in log["runs"]:
            continue
        ref = log["runs"][ref_tag]
        sfx = "" if ref_tag == "single" else "_vs_oracle"
        for tag, r in log["runs"].items():
            if tag != ref_tag:  # gaps to the reference run
                for k in ("heldin", "heldout", "auc_mean", "target_ratio"):
                    if k in r and k in ref:
                        name = {"auc_mean": "auc", "target_ratio": "target"}.get(k, k)
                        r[f"{name}_gap{sfx}"] = round((r[k] - ref[k]) / ref[k], 5)
        json.dump(log, open(os.path.join(a.out, "replica_quality.json"), "w"), indent=1)
    for tag, r in log["runs"].items():
        print(tag, {k: r[k] for k in ("heldin", "heldin_gap", "heldin_gap_vs_oracle", "heldout",
                                      "heldout_gap", "heldout_gap_vs_oracle", "auc_mean",
                                      "auc_gap", "auc_gap_vs_oracle", "target_ratio",
                                      "target_gap", "target_gap_vs_oracle") if k in r})
    print(json.dumps(log))


if __name__ == "__main__":
    main()
