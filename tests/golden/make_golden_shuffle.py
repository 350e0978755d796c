"""Regenerate tests/golden/device_shuffle.json from oracle/shuffle_oracle.py:
anchors of the keyed permutation g2v_permute_items8 implements (the device
reshuffle; no reference counterpart -- the reference's shuffles are unseeded),
so the definition cannot drift in the oracle and the kernel together.

    python tests/golden/make_golden_shuffle.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import shuffle_oracle as S  # noqa: E402


def main():
    out = {"cases": []}
    for n, seed in ((1, 0), (7, 1), (1000, 20250114), (100_000_000, 99), (2 ** 40 + 3, 2 ** 64 - 1)):
        idx = [0, 1, 2, n // 2, n - 1] if n > 2 else list(range(n))
        idx = sorted(set(i for i in idx if 0 <= i < n))
        out["cases"].append({"n": n, "seed": seed, "idx": idx,
                             "perm": [int(v) for v in S.perm_at(n, seed, np.array(idx, np.uint64))]})
    pairs = np.array([[0, 1], [2, 0], [3, -1], [1, 4], [4, 2], [5, 5], [-1, 3], [2, 6]], np.int32)
    out["first_occurrence"] = {"pairs": pairs.tolist(), "seed": 11, "n_ids": 8,
                               "first": [int(v) for v in S.first_occurrence(pairs, 11, 8)]}
    with open(os.path.join(HERE, "device_shuffle.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
