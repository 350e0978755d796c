"""Restatement of libg2v's device reshuffle (g2v_permute_items8) in numpy --
TEST INFRASTRUCTURE ONLY.

The reference reshuffles its pair list with an unseeded ``random.shuffle``
before training and before every later iteration (src/gene2vec.py:52,80), so
no particular permutation is "the" reference result: any uniform permutation
is as faithful.  The device path uses a keyed pseudo-random permutation that
every GPU can evaluate for any position without the others: a 6-round
balanced Feistel network on 2h bits (the smallest h >= 1 with 4^h >= n),
round function ``mix64(R ^ k_r) & (2^h - 1)`` (the splitmix64 finalizer),
round keys ``k_r = mix64(seed + 0x9e3779b97f4a7c15 * (r + 1))``, cycle-walked
into [0, n) (apply the network again while the value is >= n).

This module is the bit-level checker of that definition; it has no reference
counterpart (parity of the *distribution* is the claim, tested by the
bijection and uniformity properties in tests/).
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z ^ (z >> np.uint64(30))
        z = z * np.uint64(0xBF58476D1CE4E5B9)
        z = z ^ (z >> np.uint64(27))
        z = z * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def perm_key(n, seed):
    half = 1
    while half < 31 and (1 << (2 * half)) < n:
        half += 1
    with np.errstate(over="ignore"):
        keys = [mix64(np.uint64(seed % 2 ** 64) + np.uint64(0x9E3779B97F4A7C15)
                      * np.uint64(r + 1)) for r in range(6)]
    return half, keys


def feistel(y, half, keys):
    mask = np.uint64((1 << half) - 1)
    h = np.uint64(half)
    L = y >> h
    R = y & mask
    for k in keys:
        L, R = R, L ^ (mix64(R ^ k) & mask)
    return (L << h) | R


def perm_at(n, seed, idx):
    """p(idx) for an array of positions idx in [0, n)."""
    half, keys = perm_key(n, seed)
    y = np.asarray(idx, dtype=np.uint64).copy()
    todo = np.ones(y.shape, dtype=bool)
    nn = np.uint64(n)
    while todo.any():
        y[todo] = feistel(y[todo], half, keys)
        todo = y >= nn
    return y.astype(np.int64)


def permute_items(src, seed, first=0, count=None):
    """dst[i] = src[p(first + i)] (g2v_permute_items8 on host arrays)."""
    n = len(src)
    if count is None:
        count = n - first
    if count == 0:
        return src[:0].copy()
    return src[perm_at(n, seed, np.arange(first, first + count, dtype=np.uint64))]


def first_occurrence(pairs, seed, n_ids):
    """g2v_first_occurrence_perm8 restated: pairs int32[n][2]; first token
    position of every id in [0, n_ids) in the permuted order, -1 if absent."""
    n = len(pairs)
    first = np.full(n_ids, -1, dtype=np.int64)
    if n == 0:
        return first
    flat = np.asarray(pairs)[perm_at(n, seed, np.arange(n, dtype=np.uint64))].reshape(-1)
    ok = (flat >= 0) & (flat < n_ids)
    ids, pos = np.unique(flat[ok], return_index=True)
    first[ids] = np.nonzero(ok)[0][pos]
    return first
