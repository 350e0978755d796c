"""Kernel experiment sweep at C2 (V 24,447 Zipf, D 200, K 5, sample 1e-3):
SGNS-kernel examples/s per configuration (row stride, hot-row stripes, grid)
on one MI355X, plus the held-in objective after the run so a fast-but-wrong
setting shows.  Each config trains the same 20 M pairs from the same init.

    python scripts/exp_sweep.py --configs "ld=224" "ld=256" "stripe=16x8" "grid=640"
"""
import argparse
import json
import os
import sys
import time
import zlib

ROOT = os.environ.get("G2V_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def parse_cfg(text):
    cfg = {}
    for part in text.split(","):
        if not part:
            continue
        k, v = part.split("=")
        cfg[k] = v
    return cfg


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=20_000_000)
    p.add_argument("--vocab", type=int, default=24447)
    p.add_argument("--dim", type=int, default=200)
    p.add_argument("--negative", type=int, default=5)
    p.add_argument("--sample", type=float, default=1e-3)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--configs", nargs="+", default=["ld=224"])
    p.add_argument("--epochs-eval", action="store_true",
                   help="print the held-in objective after every epoch")
    p.add_argument("--ablations", action="store_true",
                   help="load the -DG2V_ABLATIONS build (debug write modes 1, 3-7, 9)")
    a = p.parse_args()
    import torch

    from gene2vec_amd import _native as N
    if a.ablations:
        from gene2vec_amd import build as B
        N.use_library(B.build(ablations=True))
    from gene2vec_amd import engine as E
    from gene2vec_amd import synthetic as S
    from oracle import sgns_oracle as O

    n, V0, D, K = a.pairs, a.vocab, a.dim, a.negative
    pairs = S.zipf_gene_pairs(n, V0, 1.0, seed=20250114)
    flat = pairs.reshape(-1)
    counts, first = E.count_ids(flat, V0)
    order, remap = S.vocab_order(counts, first)
    tok = remap[flat]
    vc = counts[order].astype(np.int64)
    V = len(order)
    names = S.gene_names(V0)
    seeds = np.array([zlib.crc32((names[i] + "1").encode()) for i in order], np.uint32)
    syn0_h = E.seeded_vectors(seeds, D)
    js = E.plan_jobs(n_sent=n, sent_len=2)
    al = E.job_alphas(js, n)
    dev = torch.device("cuda", 0)
    tok_d = torch.from_numpy(tok).to(dev)
    rng = np.random.Generator(np.random.PCG64(99))
    idx = rng.integers(0, n, 20000)
    ec, ej = tok[2 * idx], tok[2 * idx + 1]
    pw = vc.astype(np.float64) ** 0.75
    enegs = rng.choice(V, size=(20000, K), p=pw / pw.sum())
    for text in a.configs:
        cfg = parse_cfg(text)
        ld = int(cfg.get("ld", (D + 31) // 32 * 32))
        eng = E.SGNSEngine(V, D, K)
        if "grid" in cfg:
            eng.set_option(N.OPT_GRID, int(cfg["grid"]))
        if "stripe" in cfg:
            r, c = cfg["stripe"].split("x")
            eng.set_option(N.OPT_STRIPE_ROWS, int(r))
            eng.set_option(N.OPT_STRIPE_COPIES, int(c))
        if "stripe2" in cfg:  # second tier: END_ROWxCOPIES
            r, c = cfg["stripe2"].split("x")
            eng.set_option(N.OPT_STRIPE2_ROWS, int(r))
            eng.set_option(N.OPT_STRIPE2_COPIES, int(c))
        if "seg" in cfg:
            eng.set_option(N.OPT_SEG_JOBS, int(cfg["seg"]))
        if "dbg" in cfg:
            eng.set_option(N.OPT_DEBUG_WRITE, int(cfg["dbg"]))
        if "aw" in cfg:  # waves per workgroup that train (grid spreads them over more CUs)
            eng.set_option(N.OPT_ACTIVE_WAVES, int(cfg["aw"]))
        if "ov" in cfg:
            eng.set_option(N.OPT_ATOMIC_OVERLAP, int(cfg["ov"]))
        mode = N.MODE_SEQUENTIAL if cfg.get("mode") == "seq" else N.MODE_HOGWILD
        stream = torch.cuda.Stream(dev)
        eng.set_stream(stream.cuda_stream)
        tables = torch.zeros((2, V, ld), dtype=torch.float32, device=dev)
        tables[0, :, :D] = torch.from_numpy(syn0_h).to(dev)
        eng.bind_tables(tables[0].data_ptr(), tables[1].data_ptr(), ld, keepalive=(tables,))
        eng.set_vocab(vc, a.sample)
        eng.set_corpus_device(tok_d.data_ptr(), tok_d.numel(), sent_len=2, keepalive=tok_d)
        rs = np.random.RandomState(1)
        rates = []
        per_epoch = []
        for rep in range(a.reps):
            eng.train(js, al, E.job_seeds(rs, len(js) - 1), mode, timing=True)
            st = eng.read_stats()
            rates.append(st["examples"] / (st["sgns_kernel_ms"] / 1e3))
            if a.epochs_eval:
                torch.cuda.synchronize()
                per_epoch.append(round(O.sgns_loss(tables[0, :, :D].cpu().numpy(),
                                                   tables[1, :, :D].cpu().numpy(), ec, ej,
                                                   enegs), 4))
        torch.cuda.synchronize()
        s0 = tables[0, :, :D].cpu().numpy()
        s1 = tables[1, :, :D].cpu().numpy()
        loss = O.sgns_loss(s0, s1, ec, ej, enegs)
        try:
            grid = eng.get_option(N.OPT_GRID)
        except AttributeError:  # round-1 library
            grid = None
        print(json.dumps({"config": text, "ld": ld, "grid": grid, "per_epoch": per_epoch,
                          "ex_per_s": [round(r / 1e6, 2) for r in rates],
                          "launch_ms": round(st["sgns_kernel_ms"] / max(1, st["launches"]), 3),
                          "heldin_loss_after": round(loss, 4)}), flush=True)
        eng.close()
        del tables


if __name__ == "__main__":
    t = time.time()
    main()
    print(f"# {time.time() - t:.1f} s", flush=True)
