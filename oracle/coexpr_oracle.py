"""Restatement of src/generate_gene_pairs.py:45-65 (coexpr) -- TEST
INFRASTRUCTURE ONLY.

The reference's hot loop is pandas' own Pearson correlation
(``data.corr()``: Welford fp64 per column pair, pairwise-complete, NaN for
zero variance) followed by ``abs() > threshold``, ``values.nonzero()``
(row-major order) and ``row != col``.  pandas is the reference's dependency
and is importable here, so this oracle calls it exactly as the reference does
-- parity for this path is pinned by the reference's own library, not by a
re-derivation.  ``near_threshold`` reports pairs whose |r| lies within eps of
the threshold (the only place an fp64 re-association can flip a decision).
"""
import numpy as np


def coexpr_indices(data, corr_threshold):
    """(row, col) pairs in the order src/generate_gene_pairs.py:53-63 emits them."""
    corr = data.corr().abs()                                    # :50
    rows, cols = (corr > corr_threshold).values.nonzero()       # :53
    keep = rows != cols                                         # :61
    return np.stack([rows[keep], cols[keep]], axis=1).astype(np.int32)


def coexpr_strings(data, corr_threshold):
    """:56-63 -- "name_a name_b" for each pair."""
    idx = data.columns
    return [f"{idx[r]} {idx[c]}" for r, c in coexpr_indices(data, corr_threshold).tolist()]


def near_threshold(data, corr_threshold, eps=1e-9):
    """number of off-diagonal |r| within eps of the threshold"""
    a = data.corr().abs().values
    np.fill_diagonal(a, np.nan)
    return int(np.sum(np.abs(a - corr_threshold) < eps))


def reference_pipeline(query_dir, corr_threshold=0.9, min_study_samples=20, ensembl=False):
    """src/generate_gene_pairs.py:73-125,143-210 (serial branch) restated;
    returns the bytes the reference writes to --out."""
    import os
    from copy import deepcopy

    import pandas as pd

    run_table = pd.read_csv(os.path.join(query_dir, "data/SRARunTable.csv"), index_col=0)
    data = pd.read_csv(os.path.join(query_dir, "data/gene_counts_TPM.csv"), index_col=0)
    gene_counts = pd.read_csv(os.path.join(query_dir, "data/gene_counts.csv"))
    data = data.loc[run_table.index.tolist()]

    def half_min(x):
        y = x[x > 0]
        return y.min() / 2

    def clean(sample_ids):
        split = gene_counts["gene_id"].str.split("|")
        ens = [g[0] for g in split]
        tot = pd.Series(index=ens, data=gene_counts.loc[:, sample_ids].sum(axis=1).values)
        d = deepcopy(data.loc[sample_ids, tot >= 10])
        d = d.replace(0.0, half_min(data))
        return d.apply(np.log2)

    def annotated(sample_ids):
        d = clean(sample_ids)
        split = gene_counts["gene_id"].str.split("|")
        names = {g[0]: (g[1] if len(g) > 1 else "") for g in split}
        d.rename(columns=names, inplace=True)
        d = d.loc[:, d.columns != ""]
        counts = d.columns.value_counts()
        return d.loc[:, counts.index[(counts == 1)]]

    study_counts = run_table["SRA Study"].value_counts()
    studies = study_counts.index[(study_counts >= min_study_samples).values].tolist()
    out = []
    for study in studies:
        ids = run_table.index[(run_table["SRA Study"] == study)].tolist()
        d = clean(ids) if ensembl else annotated(ids)
        out.append("\n".join(coexpr_strings(d, corr_threshold)))
    return "".join(out)
