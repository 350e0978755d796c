"""Co-expression producer timing (src/generate_gene_pairs.py coexpr) on one
MI355X vs pandas on the host.

    python scripts/bench_coexpr.py [--genes 20000] [--samples 100]

GPU: g2v_coexpr_pairs end to end (H2D copy of the study matrix, stats, fused
correlation+threshold, scan, ordered emission, D2H of the pairs), best of 3
after a warm-up.  CPU baseline: pandas DataFrame.corr (the reference's own
call) on a --cpu-genes subset, scaled by (G / subset)^2 (the work is O(G^2 n)).
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gene2vec_amd import generate_gene_pairs as GP  # noqa: E402
from tests.helpers import planted_expression  # noqa: E402


FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 matrix (= vector) peak, spec


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--genes", type=int, default=20000)
    p.add_argument("--samples", type=int, default=100)
    p.add_argument("--threshold", type=float, default=0.9)
    p.add_argument("--cpu-genes", type=int, default=2000)
    a = p.parse_args()
    x = np.log2(planted_expression(a.samples, a.genes, n_groups=a.genes // 20, noise=0.4, seed=1))
    GP.coexpr_indices(x[:, :256], a.threshold)
    best = 1e9
    n_pairs = 0
    mask_ms = []
    for _ in range(3):
        t = time.perf_counter()
        n_pairs = len(GP.coexpr_indices(x, a.threshold))
        best = min(best, time.perf_counter() - t)
        mask_ms.append(GP.last_timing()[0])
    # roofline of the dominant kernel (k_coexpr_mask_mfma): algorithmic flops
    # = 2n per distinct correlation, G(G+1)/2 of them (pandas' nancorr also
    # fills only i <= j and mirrors), against the MI355X fp64 matrix peak
    mask = sum(mask_ms) / len(mask_ms)
    G, n = a.genes, a.samples
    flops_launch = float(G) * (G + 1) * n
    achieved = flops_launch / (mask / 1e3) / 1e12
    roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 4),
                "traffic": None, "kernel": "k_coexpr_mask_mfma",
                "avg_launch_ms": round(mask, 4), "flops_per_launch": flops_launch,
                "note": "upper-triangle 64x64 tiles only; the transposed bits are mirrored "
                        "in the epilogue"}
    import pandas as pd
    sub = pd.DataFrame(x[:, :a.cpu_genes])
    t = time.perf_counter()
    c = sub.corr().abs()
    (c > a.threshold).values.nonzero()
    cpu_sub = time.perf_counter() - t
    cpu_full = cpu_sub * (a.genes / a.cpu_genes) ** 2
    print(json.dumps({"metric": "co-expression gene-pair generation (one study)",
                      "genes": a.genes, "samples": a.samples, "pairs": n_pairs,
                      "gpu_s": round(best, 4), "gpu_fp64_tflops_end_to_end": round(flops_launch / best / 1e12, 2),
                      "cpu_pandas_s_scaled": round(cpu_full, 2),
                      "cpu_sample": f"pandas corr on {a.cpu_genes} genes ({cpu_sub:.2f} s), x (G/sub)^2",
                      "speedup": round(cpu_full / best, 1), "roofline": roofline}))


if __name__ == "__main__":
    main()
