"""CPU: CLI option handling that needs no GPU (gene2vec_amd/gene2vec.py): the
defaults the data-parallel gates run with, and the --sample 0 warning."""
from unittest import mock

import pytest

from gene2vec_amd import gene2vec as G


def _parsed(argv):
    seen = {}

    def fake_init(args):
        seen.update(vars(args))
        raise SystemExit(0)
    with mock.patch.object(G, "_init_dp", fake_init), pytest.raises(SystemExit):
        G.main(argv)
    return seen


def test_cli_defaults_match_the_c3_gate():
    """tests/test_gpu_c3_quality.py runs the CLI's defaults: a merge every 3,584
    jobs from 125 M pairs per rank, sharding only in the measured windows
    (distributed.DP_DEFAULT_WINDOWS); the reference's own settings
    (src/gene2vec.py:57-63) stay the CLI's"""
    a = _parsed(["d", "o", "txt"])
    assert a["merge_every_jobs"] is None and a["dp_min_pairs_per_rank"] is None
    assert a["merge_rule"] == "auto"
    assert (a["dim"], a["negative"], a["window"], a["sample"], a["iters"], a["workers"]) == \
        (200, 5, 1, 1e-3, 10, 32)
    assert a["grid"] == 0


def test_sample0_warns_about_the_target_function(capsys):
    _parsed(["d", "o", "txt", "--sample", "0"])
    err = capsys.readouterr().err
    assert "--sample 0" in err and "--grid 16" in err
    _parsed(["d", "o", "txt", "--sample", "0", "--grid", "16"])
    assert "--sample 0" not in capsys.readouterr().err
    _parsed(["d", "o", "txt"])
    assert "warning" not in capsys.readouterr().err


def test_dp_merge_plan_by_shard_size():
    """distributed.dp_merge_plan: touch every 3,584 jobs from 125 M pairs per
    rank (C3, tests/test_gpu_c3_quality.py), touch at 7 merges per epoch from
    80 M, align at 7 merges per epoch from 50 M (tests/test_gpu_c3_quality.py's
    50 M gate); explicit rules keep the cadence"""
    from gene2vec_amd import distributed as Dd
    assert Dd.dp_merge_plan(125_000_000) == ("touch", 3584)
    assert Dd.dp_merge_plan(1_000_000_000, 1024) == ("touch", 1024)
    # 50 M pairs = 10,000 jobs of 5,000 pairs -> every 1,429 jobs = 7 merges
    assert Dd.dp_merge_plan(50_000_000) == ("align", 1429)
    rule, every = Dd.dp_merge_plan(79_999_999)
    assert rule == "align" and -(-16_000 // every) == 7
    rule, every = Dd.dp_merge_plan(80_000_000)
    assert rule == "touch" and every == 2286 and -(-16_000 // every) == 7
    assert Dd.dp_merge_plan(100_000_000) == ("touch", 2858)
    assert Dd.dp_merge_plan(100_000_000, 1000) == ("touch", 1000)
    assert Dd.dp_merge_plan(50_000_000, 4096, "touch") == ("touch", 4096)
    assert Dd.dp_merge_plan(60_000_000, 333, "mean") == ("mean", 333)
    assert Dd.dp_merge_plan(60_000_000, None, "mean") == ("mean", 3584)


def test_dp_merge_plan_by_world_size():
    """up to 4 ranks the plan merges once per epoch (DESIGN.md 7a, round 5:
    the least target-function lead over one model at 2 and 4 ranks); 8 ranks
    keep the C3 plan; an explicit cadence wins"""
    from gene2vec_amd import distributed as Dd
    for w in (2, 3, 4):
        assert Dd.dp_merge_plan(125_000_000, world=w) == ("touch", 25_000)
        assert Dd.dp_merge_plan(80_000_000, world=w) == ("touch", 16_000)
        assert Dd.dp_merge_plan(125_000_000, 3584, world=w) == ("touch", 3584)
    assert Dd.dp_merge_plan(125_000_000, world=5) == ("touch", 3584)
    assert Dd.dp_merge_plan(125_000_000, world=8) == ("touch", 3584)
    assert Dd.dp_merge_plan(125_000_000, jobs_per_rank=25_088, world=4) == ("touch", 25_088)


def test_default_shard_windows():
    """verdict r5 item 1: the CLI shards by default only at the world sizes and
    pairs per rank where the merge plan was measured within 1 % of one model
    on both test corpora; --dp-min-pairs-per-rank opts in"""
    from gene2vec_amd import distributed as Dd
    M = 1_000_000
    # 2 ranks: 80-200 M pairs per rank with the damped divisor k^beta(shard)
    for per in (50 * M, 79 * M, 201 * M, 500 * M):
        assert not Dd.dp_default_shard(2 * per, 2)
    for per in (80 * M, 125 * M, 200 * M):
        assert Dd.dp_default_shard(2 * per, 2)
    assert Dd.dp_merge_beta(80 * M, 2) == 1.5 and Dd.dp_merge_beta(125 * M, 2) == 1.7
    assert abs(Dd.dp_merge_beta(112.5 * M, 2) - 1.625) < 1e-9  # interpolated
    assert Dd.dp_merge_beta(300 * M, 2) == 1.85
    assert Dd.dp_merge_beta(50 * M, 2) == 1.0  # below the window: undamped (opt-in shards)
    assert Dd.dp_merge_beta(125 * M, 2, rule="touch") == 1.0  # an explicit rule: undamped
    assert Dd.dp_merge_beta(125 * M, 8) == 1.0
    # 3 ranks: 80-100 M pairs per rank; 4 ranks: 80-250 M (damped from 100 M)
    for w, hi in ((3, 100), (4, 250)):
        assert not Dd.dp_default_shard(w * 79 * M, w)
        assert Dd.dp_default_shard(w * 80 * M, w) and Dd.dp_default_shard(w * hi * M, w)
        assert not Dd.dp_default_shard(w * (hi + 1) * M, w)
    assert Dd.dp_default_shard(4 * 125 * M, 4) and not Dd.dp_default_shard(3 * 125 * M, 3)
    assert Dd.dp_merge_beta(90 * M, 4) == 1.0 and Dd.dp_merge_beta(125 * M, 4) == 1.1
    assert Dd.dp_merge_beta(150 * M, 4) == 1.15 and Dd.dp_merge_beta(100 * M, 3) == 1.0
    assert Dd.dp_merge_beta(250 * M, 4) == 1.3 and Dd.dp_default_shard(10 ** 9, 4)  # C3 over 4
    # 5-7 ranks: never by default; 8 ranks with 150-200 M pairs per rank (not
    # C3's 125 M, where corpus B reads -1.1..-1.2 %)
    for w in (5, 6, 7):
        assert not Dd.dp_default_shard(w * 200 * M, w)
    assert not Dd.dp_default_shard(10 ** 9, 8)
    for per in (80, 125, 149, 201, 250, 500):
        assert not Dd.dp_default_shard(8 * per * M, 8), per
    for per in (150, 175, 200):
        assert Dd.dp_default_shard(8 * per * M, 8), per
    assert not Dd.dp_default_shard(10 ** 9, 1) and not Dd.dp_default_shard(16 * 125 * M, 16)
    # the explicit threshold: any world size from that many pairs per rank
    assert Dd.dp_default_shard(2 * 125 * M, 2, 50 * M)
    assert Dd.dp_default_shard(6 * 10, 6, 0)
    assert not Dd.dp_default_shard(2 * 40 * M, 2, 50 * M)
    # the plans the windows were measured with
    assert Dd.dp_merge_plan(100 * M, world=4) == ("touch", 20000)
    assert Dd.dp_merge_plan(80 * M, world=3) == ("touch", 16000)
    assert Dd.dp_merge_plan(125 * M, world=8) == ("touch", 3584)
    # wide shards: round(750 M / pairs per rank) merges per epoch
    assert Dd.dp_merge_plan(150 * M, world=8) == ("touch", 6000)       # 5
    assert Dd.dp_merge_plan(200 * M, world=8) == ("touch", 10000)      # 4
    assert Dd.dp_merge_plan(250 * M, world=8) == ("touch", 16667)      # 3
    assert Dd.dp_merge_plan(150 * M, 2048, world=8) == ("touch", 2048)  # explicit kept
