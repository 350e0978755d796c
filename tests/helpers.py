"""shared test helpers (synthetic corpora, crc hash)"""
import zlib

import numpy as np


def crc_hash(s):
    return zlib.crc32(s.encode("utf-8"))


def zipf_pairs(n_pairs, V, s=1.0, seed=20250114):
    """SURVEY 8(d) synthetic corpus: endpoints iid Zipf(s) over ranks, a != b."""
    rng = np.random.Generator(np.random.PCG64(seed))
    p = 1.0 / np.arange(1, V + 1, dtype=np.float64) ** s
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    a = np.searchsorted(cdf, rng.random(n_pairs), side="right").astype(np.int32)
    b = np.searchsorted(cdf, rng.random(n_pairs), side="right").astype(np.int32)
    bad = a == b
    while bad.any():
        b[bad] = np.searchsorted(cdf, rng.random(int(bad.sum())), side="right")
        bad = a == b
    np.minimum(a, V - 1, out=a)
    np.minimum(b, V - 1, out=b)
    return np.stack([a, b], axis=1)


def vocab_from_ids(pairs_flat, V):
    """gensim vocab order for integer-id corpora: stable sort by -count over
    first occurrence.  Returns (order: vocab index -> raw id, remap raw id ->
    vocab index, counts in index order); ids that never occur are dropped."""
    counts = np.bincount(pairs_flat, minlength=V)
    present = np.nonzero(counts)[0]
    first = np.full(V, len(pairs_flat), dtype=np.int64)
    uniq, idx = np.unique(pairs_flat, return_index=True)
    first[uniq] = idx
    fo = present[np.argsort(first[present], kind="stable")]   # first-occurrence order
    order = fo[np.argsort(-counts[fo], kind="stable")]
    remap = np.full(V, -1, dtype=np.int32)
    remap[order] = np.arange(len(order), dtype=np.int32)
    return order, remap, counts[order].astype(np.int64)
