"""CPU: examples/g2v_train.c -- a Python-free host of the C ABI -- compiles
against include/g2v.h with plain gcc, links libg2v.so and reports its usage
without touching a GPU (the GPU run is tests/test_gpu_c_example.py)."""
import os
import subprocess

from gene2vec_amd import build as B
from tests.c_example import EXE


def test_c_example_builds_and_links(tmp_path):
    out = B.build_examples()
    assert out == EXE and os.access(EXE, os.X_OK)
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "usage" in r.stderr
