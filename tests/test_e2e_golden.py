"""CPU: the end-to-end parity corpus (tests.helpers.e2e_corpus) is the one
tests/golden/e2e_parity.json was generated on, and the golden run's own
seed-to-seed spread is below the bars test_gpu_e2e_parity.py applies."""
import json
import os
import zlib

from tests.conftest import GOLDEN
from tests.helpers import e2e_corpus


def test_e2e_golden_matches_corpus_and_spread_is_small():
    with open(os.path.join(GOLDEN, "e2e_parity.json")) as f:
        ref = json.load(f)
    tok, counts, index2word, lines, perms, seeds = e2e_corpus()
    assert zlib.crc32(tok.tobytes()) == ref["corpus_crc32"]
    assert len(counts) == ref["vocab"] and len(lines) == ref["config"]["modules"]
    for key, bar in (("loss", 0.01), ("heldin", 0.005), ("target_ratio", 0.01)):
        v = [r[key] for r in ref["runs"].values()]
        assert (max(v) - min(v)) / ref[key + "_mean"] < bar / 2, (key, v)


def test_e2e_c2_golden_matches_corpus():
    from tests.helpers import E2E_C2
    with open(os.path.join(GOLDEN, "e2e_parity_c2.json")) as f:
        ref = json.load(f)
    tok, counts, index2word, lines, perms, seeds = e2e_corpus(E2E_C2)
    assert zlib.crc32(tok.tobytes()) == ref["corpus_crc32"]
    assert len(counts) == ref["vocab"] and len(lines) == ref["config"]["modules"]
    for key, bar in (("loss", 0.01), ("heldin", 0.005), ("target_ratio", 0.01)):
        v = [r[key] for r in ref["runs"].values()]
        assert (max(v) - min(v)) / ref[key + "_mean"] < bar / 2, (key, v)
