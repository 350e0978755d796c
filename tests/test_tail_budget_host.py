"""CPU: the host-side arithmetic behind the cold-row stores and
bench.py's composite roofline.

engine.kept_token_share is the keep probability of [ext] prepare_vocab's
sample_int (Appendix A.2, restated in oracle/sgns_oracle.py) times the count,
normalised -- the p_tok(r) that g2v_set_vocab derives the Hogwild budgets and
the tail-store rows from.  The collision budget's first stored row at the C2
vocabulary and bench.py's stored share per example follow from it."""
import numpy as np

from gene2vec_amd import engine as E
from oracle import sgns_oracle as O


def _zipf_counts(V, n_tokens, s=1.0):
    p = 1.0 / np.arange(1, V + 1) ** s
    return np.maximum(1, np.round(n_tokens * p / p.sum())).astype(np.int64)


def test_kept_token_share_is_sample_int_as_probability():
    for V, sample in ((300, 1e-3), (5000, 1e-3), (2000, 0.0), (1000, 5.0)):
        c = _zipf_counts(V, 2_000_000)
        si = O.sample_int_from_counts(c, sample).astype(np.float64) / 2 ** 32
        ref = c * np.minimum(si, 1.0)
        ref /= ref.sum()
        np.testing.assert_allclose(E.kept_token_share(c, sample), ref, rtol=1e-6, atol=0)


def test_collision_budget_rows_at_c2():
    """1,024 waves (256 workgroups x 4) and a budget of 0.15: syn1neg rows are
    stored from ~7,700 at the C2 vocabulary, 1.49 of the 7 rows an example
    updates (the lost-update probe counted 1.476: it skips repeat examples)"""
    c = _zipf_counts(24447, 200_000_000)
    pt = E.kept_token_share(c, 1e-3)
    pn = c.astype(np.float64) ** 0.75
    pn /= pn.sum()
    u = 5 * pn + pt
    t1 = int(np.argmax(1024 * u <= 0.15))
    assert 7000 < t1 < 8500
    stored = pt[t1:].sum() + 5 * pn[t1:].sum()
    assert 1.4 < stored < 1.6
    # the budget is monotone: u(r) is non-increasing over the sorted counts
    assert np.all(np.diff(u) <= 1e-15)


def test_tail_row_is_a_suffix_max_boundary():
    """the auto boundary must hold for u(r) that is not
    non-increasing -- a negative ns_exponent (rare genes drawn most as
    negatives) or unsorted counts put hot rows late, and no row before the
    last hot one may take plain stores"""
    c = _zipf_counts(24447, 200_000_000)
    t_sorted = E.tail_store_row(c, 1e-3, 5, 1024)
    assert 7000 < t_sorted < 8500
    # reversed counts: the hottest row is last, so nothing is stored
    assert E.tail_store_row(c[::-1].copy(), 1e-3, 5, 1024) == len(c)
    # negative exponent: the rarest rows carry the most negatives
    t_neg = E.tail_store_row(c, 1e-3, 5, 1024, ns_exponent=-0.75)
    pn = c.astype(np.float64) ** -0.75
    u = 5 * pn / pn.sum() + E.kept_token_share(c, 1e-3)
    assert np.all(1024 * u[t_neg:] <= 0.15)
    assert t_neg == len(c) or 1024 * u[t_neg - 1:].max() > 0.15
    # one hot row planted in the cold tail moves the boundary past it
    c2 = c.copy()
    c2[20000] = c2[0]
    assert E.tail_store_row(c2, 1e-3, 5, 1024) == 20001
    # a small vocabulary stores nothing at this budget
    assert E.tail_store_row(_zipf_counts(3000, 2_000_000), 1e-3, 5, 1024) == 3000
