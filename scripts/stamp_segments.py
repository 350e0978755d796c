"""Where a k_sgns_atomic wave spends its cycles (verdict r3 item 5): the
production kernel rebuilt with s_memtime stamps per loop segment
(G2V_OPT_DEBUG_WRITE 8, g2v_debug_stamps), on the bench's corpus shape.

Segments per example (g2v.h g2v_debug_stamps): rows (waiting for the
example's rows), compute (dots, sigmoid, gradients, LDS staging), land
(waiting for the previous example's atomics to land before the prefetch),
prefetch (issuing the next example's loads, summing striped copies), atomics
(issuing this example's atomics); chunk = the rest of the loop (record
staging, work queue).  Shares of the stamped build, not its run time
(cdna_hip_programming.md 7).  The in-kernel clock is memtime / memrealtime x
100 MHz (MI355X_MICROARCH.md DVFS item 6).

    python scripts/stamp_segments.py --sample 0 --pairs 20000000
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=20_000_000)
    ap.add_argument("--vocab", type=int, default=24447)
    ap.add_argument("--sample", type=float, default=1e-3)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--arms", default="production,stamped,production_again",
                    help="production, stamped (debug write 8), notail (debug write 9: each "
                         "row's last atomic instruction dropped, a throughput probe), copiesN "
                         "(production with G2V_OPT_STRIPE_COPIES N), tailN (production with "
                         "G2V_OPT_TAIL_STORE N), stamped_tailN, any suffix _again; notail "
                         "needs the ablation build (--ablations)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--library", default=None,
                    help="load this libg2v build instead (an experiment build, "
                         "gene2vec_amd.build.build(tag=..., defines=...))")
    ap.add_argument("--ablations", action="store_true",
                    help="load the -DG2V_ABLATIONS build (debug write modes 1, 3-7, 9)")
    a = ap.parse_args()
    if a.ablations:
        from gene2vec_amd import build as B
        N.use_library(B.build(ablations=True))
    elif a.library:
        N.use_library(a.library)
    D, K = 200, 5
    pairs = S.zipf_gene_pairs(a.pairs, a.vocab, 1.0, seed=20250114)
    flat = pairs.reshape(-1)
    counts, first = E.count_ids(flat, a.vocab)
    order, remap = S.vocab_order(counts, first)
    tok = remap[flat]
    vc = counts[order].astype(np.int64)
    V = len(order)
    names = S.gene_names(a.vocab)
    syn0 = E.seeded_vectors(np.array([zlib.crc32((names[i] + "1").encode()) for i in order],
                                     np.uint32), D)
    eng = E.SGNSEngine(V, D, K)
    if a.grid:
        eng.set_option(N.OPT_GRID, a.grid)
    eng.set_vocab(vc, a.sample)
    eng.set_weights(syn0, np.zeros_like(syn0))
    eng.set_corpus(tok, sent_len=2)
    js = E.plan_jobs(n_sent=a.pairs, sent_len=2)
    al = E.job_alphas(js, a.pairs)
    rs = np.random.RandomState(1)
    out = {"config": {"pairs": a.pairs, "vocab": a.vocab, "sample": a.sample, "D": D, "K": K},
           "arms": {}}
    buf = np.zeros(16, np.uint64)
    for arm in a.arms.split(","):
        base = arm.replace("_again", "")
        dbg = 8 if base.startswith("stamped") else {"notail": 9}.get(base, 0)
        eng.set_option(N.OPT_DEBUG_WRITE, dbg)
        eng.set_option(N.OPT_STRIPE_COPIES, int(base[6:]) if base.startswith("copies") else 0)
        # tailN: G2V_OPT_TAIL_STORE N (tail0 = all atomic); otherwise the
        # library's default (-1, the collision budget)
        tail = base.split("tail")[-1] if "tail" in base and base != "notail" else "-1"
        eng.set_option(N.OPT_TAIL_STORE, int(tail))
        eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD)  # warm (and |syn1| grows)
        eng.read_stats()
        eng._lib.g2v_debug_stamps(eng._h, N.ptr(buf), 16)
        t = time.time()
        for _ in range(a.epochs):
            eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD, timing=True)
        st = eng.read_stats()
        wall = time.time() - t
        N.check(eng._lib.g2v_debug_stamps(eng._h, N.ptr(buf), 16))
        res = {"grid": st["sgns_grid"], "waves": st["sgns_waves"],
               "stripes": f"{st['stripe_rows']}x{st['stripe_copies']}", "examples": st["examples"],
               "sgns_ms": round(st["sgns_kernel_ms"], 2), "wall_s": round(wall, 3),
               "examples_per_s": round(st["examples"] / (st["sgns_kernel_ms"] / 1e3), 1)}
        if dbg == 8:
            b = [int(x) for x in buf]
            n_ex, waves = b[6], b[9]
            names_ = ["rows", "compute", "land", "prefetch", "atomics"]
            seg = {k: b[i] / n_ex for i, k in enumerate(names_)}
            seg["chunk"] = (b[5] - sum(b[:5])) / n_ex
            seg["compute.dots_reduce"] = b[10] / n_ex
            seg["compute.lut_grad_update"] = b[11] / n_ex
            seg["compute.staging"] = (b[1] - b[10] - b[11]) / n_ex
            seg["atomics.first16"] = b[12] / n_ex
            seg["atomics.last12"] = (b[4] - b[12]) / n_ex
            seg["prefetch.stripe_copies"] = b[13] / n_ex
            seg["prefetch.main_loads"] = (b[3] - b[13]) / n_ex
            tot = b[5] / n_ex
            clock_mhz = b[7] / b[8] * 100.0
            res.update({"cycles_per_example_per_wave": round(tot, 1),
                        "segments_cycles": {k: round(v, 1) for k, v in seg.items()},
                        "segments_share": {k: round(v / tot, 4) for k, v in seg.items()},
                        "clock_MHz": round(clock_mhz, 1),
                        "period_us": round(tot / clock_mhz, 3),
                        "wave_launches": waves, "stamped_examples": n_ex})
        out["arms"][arm] = res
        print(arm, json.dumps(res), flush=True)
    eng.close()
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
