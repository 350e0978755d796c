"""shared by the C-example tests: the in.bin / out.bin format of
examples/g2v_train.c"""
import os
import struct
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "g2v_train")


def write_input(path, V, D, K, mode, counts, syn0, tok, seeds, alpha=0.025, min_alpha=1e-4,
                sample=1e-3):
    n_pairs = len(tok) // 2
    with open(path, "wb") as f:
        f.write(struct.pack("<4i", V, D, K, mode))
        f.write(struct.pack("<2q", n_pairs, len(seeds)))
        f.write(struct.pack("<3d", alpha, min_alpha, sample))
        f.write(np.ascontiguousarray(counts, np.int64).tobytes())
        f.write(np.ascontiguousarray(syn0, np.float32).tobytes())
        f.write(np.ascontiguousarray(tok, np.int32).tobytes())
        f.write(np.ascontiguousarray(seeds, np.uint64).tobytes())


def read_output(path, V, D):
    raw = open(path, "rb").read()
    n = V * D * 4
    s0 = np.frombuffer(raw[:n], np.float32).reshape(V, D)
    s1 = np.frombuffer(raw[n:2 * n], np.float32).reshape(V, D)
    st = struct.unpack("<5q2dd", raw[2 * n:2 * n + 64])
    return s0, s1, dict(zip(["raw_words", "effective_words", "examples", "jobs", "launches",
                             "sgns_kernel_ms", "sample_kernel_ms", "training_loss"], st))


def run(inp, out, timeout=120):
    return subprocess.run([EXE, inp, out], capture_output=True, text=True, timeout=timeout)
