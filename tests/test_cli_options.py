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
    jobs from 125 M pairs per rank and sharding from 50 M; the reference's own settings
    (src/gene2vec.py:57-63) stay the CLI's"""
    a = _parsed(["d", "o", "txt"])
    assert a["merge_every_jobs"] is None and a["dp_min_pairs_per_rank"] == 80_000_000
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
