"""CPU: bench.py's roofline arithmetic -- the composite
atomic + store roof and the expected stored rows per example -- and the
committed round-5 bench line recomputed from its own fields."""
import json
import os

import numpy as np
import pytest

import bench
from gene2vec_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_composite_roof_limits():
    t = 1e-9
    _, peak, _ = bench.composite_roofline(5600, 0.0, t)
    assert peak == pytest.approx(bench.ATOMIC_PEAK_GBPS)
    _, peak, _ = bench.composite_roofline(5600, 5600.0, t)
    assert peak == pytest.approx(bench.STORE_PEAK_GBPS)
    ach, peak, frac = bench.composite_roofline(5600, 1400.0, 5600 / 1e12)  # 1 TB/s
    assert ach == pytest.approx(1000.0)
    assert peak == pytest.approx(5600 / (4200 / 1300 + 1400 / 6100))
    assert frac == pytest.approx(ach / peak)


def test_stored_rows_per_example():
    c = np.maximum(1, np.round(2e8 / np.arange(1, 24448) / 10.6)).astype(np.int64)
    pt = E.kept_token_share(c, 1e-3)
    pn = c ** 0.75 / (c ** 0.75).sum()
    r1 = bench.stored_rows_per_example(c, 1e-3, 5, -1, 7734)
    assert r1 == pytest.approx(pt[7734:].sum() + 5 * pn[7734:].sum())
    assert bench.stored_rows_per_example(c, 1e-3, 5, 900, 7734) == pytest.approx(r1 + pt[900:].sum())
    assert bench.stored_rows_per_example(c, 1e-3, 5, -1, -1) == 0.0


def test_committed_bench_line_recomputes():
    """profiles/r05/final_bench_c2.json: achieved = update bytes per example /
    the kernel's seconds per example; peak and frac follow from its stored
    bytes through composite_roofline"""
    line = json.load(open(os.path.join(ROOT, "profiles", "r05", "final_bench_c2.json")))
    r = line["roofline"]
    upd, stored = r["update_bytes_per_example"], r["stored_bytes_per_example"]
    assert stored == pytest.approx(r["stored_rows_per_example"] * line["config"]["dim"] * 4,
                                   rel=1e-4)
    t_ex = upd / (r["achieved"] * 1e9)
    ach, peak, frac = bench.composite_roofline(upd, stored, t_ex)
    assert peak == pytest.approx(r["peak"], rel=1e-3)
    assert frac == pytest.approx(r["frac"], rel=1e-3)
    assert r["atomic_achieved_GBps"] == pytest.approx((upd - stored) / t_ex / 1e9, rel=1e-3)
