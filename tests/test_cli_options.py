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
    """tests/test_gpu_c3_quality.py runs the CLI's defaults: a merge every 4,096
    jobs and sharding from 125 M pairs per rank; the reference's own settings
    (src/gene2vec.py:57-63) stay the CLI's"""
    a = _parsed(["d", "o", "txt"])
    assert a["merge_every_jobs"] == 4096 and a["dp_min_pairs_per_rank"] == 125_000_000
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
