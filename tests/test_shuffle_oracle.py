"""CPU: the restated device reshuffle (oracle/shuffle_oracle.py, the
definition g2v_permute_items8 implements) is a permutation of [0, n) for
every size the Feistel domain rounds up from, is reproducible from its seed,
and spreads positions uniformly.  The reference's own shuffle
(src/gene2vec.py:52,80) is an unseeded random.shuffle, so uniformity -- not a
particular permutation -- is the property to keep."""
import numpy as np
import pytest

from oracle import shuffle_oracle as S


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 15, 16, 17, 1000, 4097, 65536, 65537, 300_001])
def test_bijection(n):
    p = S.perm_at(n, 20250114, np.arange(n, dtype=np.uint64)) if n else np.zeros(0, np.int64)
    assert np.array_equal(np.sort(p), np.arange(n))


def test_seeded_and_sharded():
    n = 10_007
    a = S.perm_at(n, 1, np.arange(n, dtype=np.uint64))
    assert np.array_equal(a, S.perm_at(n, 1, np.arange(n, dtype=np.uint64)))
    b = S.perm_at(n, 2, np.arange(n, dtype=np.uint64))
    assert (a != b).mean() > 0.99
    # shards of one permutation (data-parallel ranks) cover every item once
    src = np.arange(n, dtype=np.int64) * 3
    parts = [S.permute_items(src, 5, lo, hi - lo)
             for lo, hi in [(0, 2500), (2500, 5003), (5003, 7777), (7777, n)]]
    assert np.array_equal(np.concatenate(parts), S.permute_items(src, 5))
    assert np.array_equal(np.sort(np.concatenate(parts)), src)


def test_uniform_positions():
    # where item 0 lands, over 4,000 seeds, n = 40: chi-square over 40 cells
    n, trials = 40, 4000
    hits = np.zeros(n)
    for s in range(trials):
        p = S.perm_at(n, s, np.arange(n, dtype=np.uint64))
        hits[p[0]] += 1  # position 0 of the output takes item p[0]
    exp = trials / n
    chi2 = ((hits - exp) ** 2 / exp).sum()
    assert chi2 < 80, chi2  # 39 dof: p < 1e-4 above ~80
    # neighbours stay apart: consecutive outputs are not consecutive inputs
    p = S.perm_at(100_000, 9, np.arange(100_000, dtype=np.uint64))
    assert np.mean(np.abs(np.diff(p)) == 1) < 1e-3


def test_matches_committed_anchors():
    """the restated permutation equals the committed anchors (including a
    2^40-item domain: 21-bit halves, cycle-walking at scale)"""
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "device_shuffle.json")))
    for c in g["cases"]:
        got = S.perm_at(c["n"], c["seed"], np.array(c["idx"], np.uint64))
        assert [int(v) for v in got] == c["perm"], c
    fo = g["first_occurrence"]
    assert [int(v) for v in S.first_occurrence(np.array(fo["pairs"], np.int32), fo["seed"],
                                               fo["n_ids"])] == fo["first"]
