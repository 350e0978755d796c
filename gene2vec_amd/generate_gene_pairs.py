"""Co-expression gene-pair generator with the correlation on the GPU.

Mirror of ``src/generate_gene_pairs.py`` (the producer of gene2vec's pair
corpus): same command line, same per-study cleaning
and naming, same output bytes -- including the reference's join quirk
(``src/generate_gene_pairs.py:206-209``: each study's pairs are joined with
'\\n' and written with no separator after them, so the last pair of one study
and the first of the next share a line, which ``gene2vec.py`` reads as a
4-token sentence).

The hot loop, ``coexpr`` (``src/generate_gene_pairs.py:45-65``: pandas
``DataFrame.corr().abs() > threshold``, ``nonzero()``, ``row != col``), runs
in ``libg2v.so`` (``g2v_coexpr_pairs``: fp64 standardisation, tiled fp64
Z^T Z with the threshold fused into the epilogue, ordered pair emission).  Ray
(``--parallel``) is replaced by the GPU: studies run one after another, each
on the whole device.  The rest -- CSV loading, low-expression filter, half-min
zero replacement, log2, gene-name restriction -- is host pandas code like the
reference's.
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
from copy import deepcopy

import numpy as np

from . import _native as N

CORR_THRESHOLD = 0.9  # src/generate_gene_pairs.py:20-24 default


def coexpr_indices(values: np.ndarray, corr_threshold: float, device: int = 0) -> np.ndarray:
    """(row, col) column-index pairs with |pearson| > threshold, row != col, in
    ``nonzero()`` order; values is [samples][genes].  GPU only (no fallback)."""
    x = np.ascontiguousarray(values, dtype=np.float64)
    if x.ndim != 2:
        raise ValueError("expected a 2-D [samples][genes] matrix")
    n, g = x.shape
    if g == 0:
        return np.zeros((0, 2), np.int32)
    if n < 1:
        raise ValueError("need at least one sample")
    if not np.isfinite(x.sum()) and not np.isfinite(x).all():  # sum: one cheap pass
        raise ValueError("non-finite expression values: pandas' pairwise-NaN correlation is not "
                         "implemented on the GPU path")
    L = N.lib()
    cnt = C.c_int64(0)
    cap = min(g * (g - 1), 1 << 22)
    out = np.empty((max(cap, 1), 2), np.int32)
    rc = L.g2v_coexpr_pairs(device, N.ptr(x), n, g, float(corr_threshold), N.ptr(out), cap,
                            C.byref(cnt))
    if rc == N.G2V_ERANGE:
        out = np.empty((cnt.value, 2), np.int32)
        N.check(L.g2v_coexpr_pairs(device, N.ptr(x), n, g, float(corr_threshold), N.ptr(out),
                                   cnt.value, C.byref(cnt)))
    else:
        N.check(rc)
    return out[:cnt.value]


def last_timing() -> tuple:
    """(fused correlation kernel ms, whole call ms) of this thread's last
    ``coexpr_indices`` call, from HIP events on its stream."""
    m, t = C.c_double(0), C.c_double(0)
    N.check(N.lib().g2v_coexpr_last_timing(C.byref(m), C.byref(t)))
    return m.value, t.value


def coexpr(data, corr_threshold: float | None = None, device: int = 0) -> list:
    """``src/generate_gene_pairs.py:45-65``: "name_a name_b" strings."""
    thr = CORR_THRESHOLD if corr_threshold is None else corr_threshold
    print("Computing gene correlations...")
    idx = coexpr_indices(data.values, thr, device)
    print(f"Computing gene co-expressions with correlation threshold={thr}...")
    names = [str(c) for c in data.columns]
    return [f"{names[r]} {names[c]}" for r, c in idx.tolist()]


def gene_name(gene_fields: list) -> str:
    """``src/generate_gene_pairs.py:67-71``: second '|' field or ''."""
    return gene_fields[1] if len(gene_fields) > 1 else ""


def half_min(x):
    """``src/generate_gene_pairs.py:73-79``: half the smallest positive value
    (per column for a DataFrame)."""
    return x[x > 0].min() / 2


def clean_and_normalize(data, gene_counts, sample_ids=None):
    """``src/generate_gene_pairs.py:81-100``: drop genes with total count < 10
    over the study's samples, replace 0 by the half-minimum of the FULL data,
    log2."""
    if sample_ids is None:
        sample_ids = data.index.tolist()
    print("Computing low expression genes (total counts ≤ 10)...")
    ensembl_ids = [g.split("|")[0] for g in gene_counts["gene_id"]]
    import pandas as pd
    totals = pd.Series(index=ensembl_ids, data=gene_counts.loc[:, sample_ids].sum(axis=1).values)
    print("Removing low expression genes...")
    normed = deepcopy(data.loc[sample_ids, totals >= 10])
    print("Replacing 0 with non-zero half-minimum...")
    normed = normed.replace(0.0, half_min(data))
    print("log2 normalizing data...")
    return normed.apply(np.log2)


def gene_annotated_data(data, gene_counts, sample_ids=None):
    """``src/generate_gene_pairs.py:102-125``: columns renamed to gene names,
    unnamed and duplicated names dropped."""
    normed = clean_and_normalize(data, gene_counts, sample_ids)
    names = {g.split("|")[0]: gene_name(g.split("|")) for g in gene_counts["gene_id"]}
    print("Restricting data to genes with unique gene names...")
    normed = normed.rename(columns=names)
    normed = normed.loc[:, normed.columns != ""]
    vc = normed.columns.value_counts()
    return normed.loc[:, vc.index[vc == 1]]


def study_pairs(data, gene_counts, sample_ids, ensembl: bool, corr_threshold: float,
                device: int = 0) -> list:
    """One study: ``generate_gene_{name,ensembl}_pairs`` without Ray."""
    if ensembl:
        return coexpr(clean_and_normalize(data, gene_counts, sample_ids), corr_threshold, device)
    return coexpr(gene_annotated_data(data, gene_counts, sample_ids), corr_threshold, device)


def write_pairs(path: str, results: list) -> int:
    """``src/generate_gene_pairs.py:203-209`` byte for byte (no separator
    between studies)."""
    with open(path, "w+") as f:
        for gene_pairs in results:
            f.write("\n".join(gene_pairs))
    return sum(len(p) for p in results)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Generate gene co-expression pairs from a processed "
                                            "query for a downstream gene2vec model (GPU).")
    p.add_argument("--query", type=str, help="File path of the directory containing the query.")
    p.add_argument("--out", type=str, default="../data/gene_pairs.txt",
                   help="File path of output gene pairs.")
    p.add_argument("--corr-threshold", type=float, dest="corr_threshold", default=0.9,
                   help="Value to threshold correlation at for gene co-expression.")
    p.add_argument("--min-study-samples", type=int, dest="min_study_samples", default=20,
                   help="Minimum number of samples which must be present in each study.")
    p.add_argument("--parallel", dest="parallel", action="store_true",
                   help="Accepted for compatibility; studies run on the GPU one by one.")
    p.add_argument("--ensembl", dest="ensembl", action="store_true",
                   help="Indicates to use ensembl id over gene name.")
    p.add_argument("--device", type=int, default=0)
    p.set_defaults(parallel=False, ensembl=False)
    return p.parse_args(argv)


def main(argv=None) -> int:
    import pandas as pd

    a = parse_args(argv)
    print("\nRunning:")
    print("\t[*] Loading SRA Run Table...")
    run_table = pd.read_csv(os.path.join(a.query, "data/SRARunTable.csv"), index_col=0)
    print("\t[*] Loading TPM data...")
    data = pd.read_csv(os.path.join(a.query, "data/gene_counts_TPM.csv"), index_col=0)
    print("\t[*] Loading gene counts for filtering...")
    gene_counts = pd.read_csv(os.path.join(a.query, "data/gene_counts.csv"))
    data = data.loc[run_table.index.tolist()]
    study_counts = run_table["SRA Study"].value_counts()
    studies = study_counts.index[(study_counts >= a.min_study_samples).values].tolist()
    results = []
    for study in studies:
        sample_ids = run_table.index[(run_table["SRA Study"] == study)].tolist()
        results.append(study_pairs(data, gene_counts, sample_ids, a.ensembl, a.corr_threshold,
                                   a.device))
    print(f"\t[*] Writing gene pairs to file: {os.path.abspath(a.out)}...")
    total = write_pairs(a.out, results)
    print(f"\t[*] {'{:,}'.format(total)} total co-expression gene pairs computed.")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
