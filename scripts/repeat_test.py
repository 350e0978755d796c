"""Run one GPU test function several times in one process and report each
outcome (Hogwild results are timing-dependent).  Experiment script.

    python scripts/repeat_test.py tests.test_gpu_parity test_train_hogwild_full_vocab_tracks_oracle 5
"""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    mod, fn, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    f = getattr(importlib.import_module(mod), fn)
    for i in range(n):
        t = time.time()
        try:
            f()
            print(f"{fn} run {i}: ok ({time.time() - t:.1f} s)", flush=True)
        except AssertionError as e:
            print(f"{fn} run {i}: FAIL {e}", flush=True)


if __name__ == "__main__":
    main()
