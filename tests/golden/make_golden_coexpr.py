"""Regenerate the co-expression golden fixtures (src/generate_gene_pairs.py).

    python tests/golden/make_golden_coexpr.py

Outputs are produced by pandas' own DataFrame.corr (the reference's library,
through oracle/coexpr_oracle.py) on seeded synthetic inputs:

* coexpr_small.npz  -- x [30][130] planted co-expression (+3 constant columns),
                       threshold 0.9, the (row, col) pairs pandas selects
* coexpr_query_name.txt / coexpr_query_ensembl.txt -- the bytes the reference
                       pipeline writes for tests.helpers.make_query(seed=0)
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import coexpr_oracle as O  # noqa: E402
from tests.helpers import make_query, planted_expression  # noqa: E402


def small():
    import pandas as pd
    x = planted_expression(30, 130, n_groups=5, noise=0.2, seed=7)
    x = np.log2(x)
    x[:, [4, 50, 129]] = 1.25                       # zero-variance genes
    d = pd.DataFrame(x, columns=[f"G{k}" for k in range(x.shape[1])])
    assert O.near_threshold(d, 0.9, 1e-9) == 0
    pairs = O.coexpr_indices(d, 0.9)
    np.savez_compressed(os.path.join(HERE, "coexpr_small.npz"), x=x, threshold=0.9, pairs=pairs)
    print("coexpr_small: pairs", len(pairs))


def query():
    with tempfile.TemporaryDirectory() as d:
        make_query(d, seed=0)
        for mode, ens in (("name", False), ("ensembl", True)):
            s = O.reference_pipeline(d, 0.9, 20, ens)
            with open(os.path.join(HERE, f"coexpr_query_{mode}.txt"), "w") as f:
                f.write(s)
            print("query", mode, len(s), "bytes")


if __name__ == "__main__":
    small()
    query()
