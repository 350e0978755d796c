"""Synthetic Zipf-degree gene-pair corpora.

The reference's corpus is "GENE_A GENE_B" lines of co-expressed genes
(src/generate_gene_pairs.py:59-63, never a self-pair).  The benchmark corpus
replaces it with V genes named G00000.. whose pair endpoints are drawn iid
from Zipf(s) over rank (p(r) ~ r^-s, r = 1..V) with
numpy.random.Generator(PCG64(seed)), rejecting a == b.  Rank r is gene
G{r-1:05d}.  Shard k of a multi-GPU run uses PCG64(seed).jumped(k).
"""
from __future__ import annotations

import numpy as np

_BUCKETS = 1 << 20


def gene_names(V):
    return [f"G{i:05d}" for i in range(V)]


class _ZipfSampler:
    def __init__(self, V, s):
        p = 1.0 / np.arange(1, V + 1, dtype=np.float64) ** s
        cdf = np.cumsum(p)
        cdf /= cdf[-1]
        self.cdf = cdf
        self.V = V
        # bucketed inverse CDF: start index per 2^-20 slice of [0, 1)
        self.lo = np.searchsorted(cdf, np.arange(_BUCKETS) / _BUCKETS, side="right").astype(np.int64)

    def __call__(self, u):
        """ranks-1 (0-based ids) for uniforms u: searchsorted(cdf, u, 'right')"""
        idx = self.lo[(u * _BUCKETS).astype(np.int64)]
        V = self.V
        while True:
            m = self.cdf[np.minimum(idx, V - 1)] <= u
            if not m.any():
                break
            idx[m] += 1
        return np.minimum(idx, V - 1).astype(np.int32)


def zipf_gene_pairs(n_pairs, V=24447, s=1.0, seed=20250114, shard=0, chunk=1 << 24):
    """int32[n_pairs, 2] gene ids (0-based rank), a != b."""
    bitgen = np.random.PCG64(seed)
    if shard:
        bitgen = bitgen.jumped(shard)
    rng = np.random.Generator(bitgen)
    zs = _ZipfSampler(V, s)
    out = np.empty((n_pairs, 2), dtype=np.int32)
    for b0 in range(0, n_pairs, chunk):
        n = min(chunk, n_pairs - b0)
        a = zs(rng.random(n))
        b = zs(rng.random(n))
        bad = np.nonzero(a == b)[0]
        while len(bad):
            b[bad] = zs(rng.random(len(bad)))
            bad = bad[a[bad] == b[bad]]
        out[b0:b0 + n, 0] = a
        out[b0:b0 + n, 1] = b
    return out


def vocab_order(counts, first):
    """gensim index order over ids: stable sort by descending count over
    first-occurrence order ([ext] sort_vocab).  Returns (order, remap)."""
    counts = np.asarray(counts)
    first = np.asarray(first)
    present = np.nonzero(counts > 0)[0]
    fo = present[np.argsort(first[present], kind="stable")]
    order = fo[np.argsort(-counts[fo], kind="stable")]
    remap = np.full(len(counts), -1, dtype=np.int32)
    remap[order] = np.arange(len(order), dtype=np.int32)
    return order, remap
