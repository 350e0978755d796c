"""Lost-update rate of the cold-row plain stores (G2V_OPT_TAIL_STORE; DESIGN.md
5e, verdict r4 item 4).

Runs the -DG2V_ABLATIONS build's G2V_OPT_DEBUG_WRITE 10: the production
kernel with, before every cold-row store, a write-through-fresh re-read of
the row's first 64 floats compared with what the wave read for its update.
A difference means another wave wrote the row inside this wave's read-to-
store window, so the store overwrites that update: one lost update
(g2v_debug_stamps [14] stores, [15] such rows).  The probe's extra load
lengthens each wave's window a little, so the rates are upper-ish estimates
for the production kernel.  The reference's gensim Hogwild loses updates the
same way with 32 threads (src/gene2vec.py:59) -- at far fewer in flight.

    python scripts/lost_updates.py --tails auto,8192,4096,2048 --out gpurun_out/lost.json
"""
import argparse
import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=20_000_000)
    ap.add_argument("--vocab", type=int, default=24447)
    ap.add_argument("--sample", type=float, default=1e-3)
    ap.add_argument("--dim", type=int, default=200)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--tails", default="auto,8192,4096,2048")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch  # noqa: F401  (torch's HIP runtime first, as _native.lib() does)

    from gene2vec_amd import _native as N
    from gene2vec_amd import build as B
    N.use_library(B.build(ablations=True))
    from gene2vec_amd import engine as E
    from gene2vec_amd import synthetic as S

    D, K = a.dim, a.negative
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
    js = E.plan_jobs(n_sent=a.pairs, sent_len=2)
    al = E.job_alphas(js, a.pairs)
    out = {"config": {"pairs": a.pairs, "vocab": a.vocab, "sample": a.sample, "epochs": a.epochs,
                      "D": D, "K": K}, "arms": {}}
    buf = np.zeros(16, np.uint64)
    for arm in a.tails.split(","):
        eng = E.SGNSEngine(V, D, K)
        eng.set_vocab(vc, a.sample)
        eng.set_weights(syn0, np.zeros_like(syn0))
        eng.set_corpus(tok, sent_len=2)
        eng.set_option(N.OPT_TAIL_STORE, -1 if arm == "auto" else int(arm))
        eng.set_option(N.OPT_DEBUG_WRITE, 10)
        rs = np.random.RandomState(1)
        per_epoch = []
        for ep in range(a.epochs):
            eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD)
            st = eng.read_stats()
            N.check(eng._lib.g2v_debug_stamps(eng._h, N.ptr(buf), 16))
            stores, changed = int(buf[14]), int(buf[15])
            per_epoch.append({"stores": stores, "lost": changed,
                              "lost_rate": changed / max(1, stores),
                              "row_updates": (K + 2) * st["examples"],
                              "stored_share": stores / max(1, (K + 2) * st["examples"]),
                              "tail_row_syn0": st["tail_row_syn0"],
                              "tail_row_syn1neg": st["tail_row_syn1neg"]})
            print(arm, ep, per_epoch[-1], flush=True)
        out["arms"][arm] = per_epoch
        eng.close()
    print(json.dumps(out))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
