"""GPU: the production Hogwild kernel's arithmetic on REPEATED rows
(verdict r2 weak #1 / next #3).

k_sgns_atomic (gene2vec_amd/csrc/g2v_sgns_atomic.hip) deliberately lags a
wave's own updates by one example -- example e+1's rows are loaded before e's
atomics issue -- and spreads the hottest rows' deltas over stripe copies.  The
exact-value checks of test_gpu_parity.py use disjoint rows, where neither is
visible.  Here the kernel runs on ONE wave (G2V_OPT_GRID 1,
G2V_OPT_ACTIVE_WAVES 1: its chunks then train in record order) over a
40-gene vocabulary, so every example shares rows with the previous ones, and
its tables must match oracle/sgns_oracle.c's orc_atomic_one_wave -- the
restatement of that documented order -- at 1e-5 relative (the measured gap is
the double-sum order of the dots, ~1e-7).  The plain sequential (gensim
workers=1) result differs from both by ~0.5 %, so the check discriminates."""
import numpy as np
import pytest

from gene2vec_amd import _native as N
from gene2vec_amd import engine as E
from oracle import c_oracle as CO

pytestmark = pytest.mark.gpu

STRIPES = {
    "off": {N.OPT_STRIPE_COPIES: 1},
    # the library's default at one workgroup (< CUs): 4 rows x 16 copies at
    # D <= 256, x 8 above, no tier 2
    "default": {},
    "two_tier": {N.OPT_STRIPE_ROWS: 8, N.OPT_STRIPE_COPIES: 16, N.OPT_STRIPE2_ROWS: 20,
                 N.OPT_STRIPE2_COPIES: 4},
}


def _examples(V, K, n, seed):
    rng = np.random.RandomState(seed)
    # Zipf-like reuse: the head rows recur within every chunk
    p = 1.0 / np.arange(1, V + 1)
    p /= p.sum()
    c = rng.choice(V, n, p=p).astype(np.int32)
    i = rng.choice(V, n, p=p).astype(np.int32)
    negs = rng.choice(V, (n, K), p=p).astype(np.int32)
    negs[negs == c[:, None]] = -1        # gensim skips a negative equal to the centre
    negs[rng.rand(n, K) < 0.05] = -1     # and explicit skips
    return c, i, negs


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("D,K", [(200, 5), (512, 15), (37, 3)])
@pytest.mark.parametrize("stripes", ["off", "default", "two_tier"])
def test_one_wave_atomic_kernel_matches_restatement(D, K, stripes):
    V, n, alpha = 40, 3000, 0.025
    rng = np.random.RandomState(1)
    syn0 = ((rng.rand(V, D) - 0.5) / D).astype(np.float32)
    syn1 = ((rng.rand(V, D) - 0.5) / D * 0.1).astype(np.float32)
    lockf = np.ones(V, np.float32)
    c, i, negs = _examples(V, K, n, seed=D + K)
    e = E.SGNSEngine(V, D, K)
    e.set_weights(syn0, syn1)
    e.set_option(N.OPT_GRID, 1)
    e.set_option(N.OPT_ACTIVE_WAVES, 1)
    for k, v in STRIPES[stripes].items():
        e.set_option(k, v)
    e.step_explicit(c, i, negs, alpha, mode=N.MODE_HOGWILD)
    g0, g1 = e.get_weights()
    st = e.read_stats()
    assert st["sgns_grid"] == 1
    if stripes == "off":
        assert st["stripe_copies"] == 1
    if stripes == "default":
        assert (st["stripe_rows"], st["stripe_copies"], st["stripe2_rows"]) == \
            (4, 16 if D <= 256 else 8, 4)
    if stripes == "two_tier":
        assert (st["stripe_rows"], st["stripe_copies"], st["stripe2_rows"],
                st["stripe2_copies"]) == (8, 16, 20, 4)
    e.close()

    r0, r1 = syn0.copy(), syn1.copy()
    CO.atomic_one_wave(r0, r1, lockf, c, i, negs, alpha, st["stripe_rows"], st["stripe_copies"],
                       st["stripe2_rows"], st["stripe2_copies"])
    assert _rel(g0, r0) < 1e-5 and _rel(g1, r1) < 1e-5, (_rel(g0, r0), _rel(g1, r1))
    # the restated order is what the kernel does: gensim's plain sequential
    # order is measurably elsewhere
    s0, s1 = syn0.copy(), syn1.copy()
    CO.sgns_step_sequential(s0, s1, lockf, c, i, negs, alpha)
    assert max(_rel(g0, s0), _rel(g1, s1)) > 20 * max(_rel(g0, r0), _rel(g1, r1), 1e-7)


def test_one_wave_chunk_boundaries_and_short_tail():
    """n not a multiple of the 32-example chunk and a single-example launch:
    the first example of every chunk sees all earlier updates"""
    V, D, K, alpha = 12, 64, 5, 0.05
    rng = np.random.RandomState(4)
    syn0 = ((rng.rand(V, D) - 0.5) / D).astype(np.float32)
    syn1 = np.zeros((V, D), np.float32)
    lockf = np.ones(V, np.float32)
    for n in (1, 31, 33, 97):
        c, i, negs = _examples(V, K, n, seed=n)
        e = E.SGNSEngine(V, D, K)
        e.set_weights(syn0, syn1)
        e.set_option(N.OPT_GRID, 1)
        e.set_option(N.OPT_ACTIVE_WAVES, 1)
        e.step_explicit(c, i, negs, alpha, mode=N.MODE_HOGWILD)
        g0, g1 = e.get_weights()
        st = e.read_stats()
        e.close()
        r0, r1 = syn0.copy(), syn1.copy()
        CO.atomic_one_wave(r0, r1, lockf, c, i, negs, alpha, st["stripe_rows"],
                           st["stripe_copies"], st["stripe2_rows"], st["stripe2_copies"])
        assert _rel(g0, r0) < 1e-5 and _rel(g1, r1) < 1e-5, (n, _rel(g0, r0), _rel(g1, r1))


def _no_consecutive_share(V, K, n, seed, zipf=True):
    """Zipf (or uniform) examples in which no row of either table recurs in
    the NEXT example (the one whose loads overtake this example's writes)"""
    rng = np.random.RandomState(seed)
    p = 1.0 / np.arange(1, V + 1) if zipf else np.ones(V)
    p /= p.sum()
    c = np.empty(n, np.int32)
    i = np.empty(n, np.int32)
    negs = np.empty((n, K), np.int32)
    prev1, prev0 = set(), set()
    for e in range(n):
        while True:
            ce, ie = rng.choice(V, 2, p=p)
            ne = rng.choice(V, K, p=p)
            s1 = {int(ce), *map(int, ne)}
            if not (s1 & prev1) and int(ie) not in prev0:
                break
        ne[ne == ce] = -1
        c[e], i[e], negs[e] = ce, ie, ne
        prev1, prev0 = s1, {int(ie)}
    return c, i, negs


@pytest.mark.parametrize("tail,D,K", [(100, 200, 5), (1, 200, 5), (1, 512, 15), (1, 37, 3)])
def test_one_wave_tail_stores_match_restatement(tail, D, K):
    """G2V_OPT_TAIL_STORE: on one wave, with no row shared by
    consecutive examples, a cold row's plain store of (row as read + delta)
    leaves the same value as the atomic (row + delta): the kernel still
    matches orc_atomic_one_wave at 1e-5, repeated targets (atomics) included;
    tail 1 = every unstriped row stored (at negative 15 more cold rows than
    the 8 staging slots: the rest take atomics; at D 37 the 16-B stores also
    write the last float4's zero padding, which must stay zero); syn0_lockf
    0 / 0.5 / 1 per row"""
    V, n, alpha = (2000, 1500, 0.025) if K == 5 else (6000, 800, 0.025)
    rng = np.random.RandomState(3)
    syn0 = ((rng.rand(V, D) - 0.5) / D).astype(np.float32)
    syn1 = ((rng.rand(V, D) - 0.5) / D * 0.1).astype(np.float32)
    # locked, half-locked and free syn0 rows: a stored syn0 row is l1 + lockf * work
    lockf = np.random.RandomState(7).choice([0.0, 0.5, 1.0], V).astype(np.float32)
    c, i, negs = _no_consecutive_share(V, K, n, seed=tail + K, zipf=K == 5)
    negs[5::97, 1] = negs[5::97, 0]  # some repeated targets: those examples keep atomics
    e = E.SGNSEngine(V, D, K)
    e.set_weights(syn0, syn1, lockf)
    e.set_option(N.OPT_GRID, 1)
    e.set_option(N.OPT_ACTIVE_WAVES, 1)
    for k, v in STRIPES["two_tier"].items():
        e.set_option(k, v)
    e.set_option(N.OPT_TAIL_STORE, tail)
    assert e.get_option(N.OPT_TAIL_STORE) == tail
    e.step_explicit(c, i, negs, alpha, mode=N.MODE_HOGWILD)
    g0, g1 = e.get_weights()
    st = e.read_stats()
    e.close()
    r0, r1 = syn0.copy(), syn1.copy()
    CO.atomic_one_wave(r0, r1, lockf, c, i, negs, alpha, st["stripe_rows"], st["stripe_copies"],
                       st["stripe2_rows"], st["stripe2_copies"])
    assert _rel(g0, r0) < 1e-5 and _rel(g1, r1) < 1e-5, (_rel(g0, r0), _rel(g1, r1))
    assert np.abs(g1 - syn1).max() > 0


def test_retired_and_unsupported_options_refused():
    """ABI 5: the measured-slower kernel variants are gone (keys 19 / 20), a
    debug build on a shape the library does not compile it for is
    G2V_EINVAL, not a silent production run, and tail-store rows
    lie in [-1, V]"""
    e = E.SGNSEngine(100, 512, 15)
    try:
        for key, val in ((19, 1), (20, 1), (N.OPT_DEBUG_WRITE, 8), (N.OPT_DEBUG_WRITE, 2),
                         (N.OPT_DEBUG_WRITE, 1), (N.OPT_TAIL_STORE, 101), (N.OPT_TAIL_STORE, -2)):
            with pytest.raises(N.G2VError):
                e.set_option(key, val)
    finally:
        e.close()
    e = E.SGNSEngine(100, 200, 5)
    try:
        e.set_option(N.OPT_DEBUG_WRITE, 8)
        e.set_option(N.OPT_DEBUG_WRITE, 2)
        e.set_option(N.OPT_DEBUG_WRITE, 0)
        for bad in (1, 3, 4, 5, 6, 7, 9):  # ablations: -DG2V_ABLATIONS build only
            with pytest.raises(N.G2VError):
                e.set_option(N.OPT_DEBUG_WRITE, bad)
    finally:
        e.close()
