"""Tokenizer / shuffle timing (SURVEY.md 8(f) rank 3, 8(d) "a text copy of C2
is used only to time the tokenizer separately").

    python scripts/bench_ingest.py [--pairs 100000000] [--files 8] [--py-pairs 5000000]

Writes the C2 corpus (Zipf gene pairs, "Gxxxxx Gyyyyy" lines) as text files,
then times
  * native: ``ingest.read_corpus`` (g2v_corpus_read, multi-threaded C++) over
    all of it, and the per-iteration reshuffle (CPython-exact Fisher-Yates
    permutation + CSR gather, src/gene2vec.py:80);
  * reference: the reference's own loop (src/gene2vec.py:36-47, re-stated in
    ``gene2vec_amd.gene2vec.read_gene_pairs``) and ``random.shuffle`` on a
    bounded prefix (--py-pairs), scaled linearly.
Both read the files from the page cache (each file is read once untimed
first).  Prints one JSON line.  Host-only: no GPU work.
"""
import argparse
import json
import os
import random
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gene2vec_amd import gene2vec as G  # noqa: E402
from gene2vec_amd import ingest  # noqa: E402
from gene2vec_amd import synthetic as S  # noqa: E402


def write_corpus(d, pairs, n_files, names, tag="pairs"):
    sizes = []
    for k, part in enumerate(np.array_split(np.arange(len(pairs)), n_files)):
        a, b = pairs[part, 0], pairs[part, 1]
        lines = np.char.add(np.char.add(names[a], " "), names[b])
        path = os.path.join(d, f"{tag}_{k}.txt")
        with open(path, "w", encoding="windows-1252") as f:
            f.write("\n".join(lines.tolist()))
            f.write("\n")
        sizes.append(os.path.getsize(path))
        print(f"wrote {path} ({sizes[-1]} B)", flush=True)
    return sum(sizes)


def warm(d):
    for f in os.listdir(d):
        with open(os.path.join(d, f), "rb") as fh:
            while fh.read(1 << 24):
                pass


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=100_000_000)
    p.add_argument("--files", type=int, default=8)
    p.add_argument("--py-pairs", type=int, default=5_000_000)
    p.add_argument("--vocab", type=int, default=24447)
    p.add_argument("--threads", type=int, default=16)
    a = p.parse_args()
    names = np.array(S.gene_names(a.vocab))
    work = tempfile.mkdtemp(prefix="g2v_ingest_")
    try:
        full, small = os.path.join(work, "full"), os.path.join(work, "small")
        os.makedirs(full)
        os.makedirs(small)
        t = time.perf_counter()
        pairs = S.zipf_gene_pairs(a.pairs, a.vocab, 1.0, seed=20250114)
        nbytes = write_corpus(full, pairs, a.files, names)
        sbytes = write_corpus(small, pairs[:a.py_pairs], 1, names)
        del pairs
        t_write = time.perf_counter() - t
        warm(full)
        warm(small)
        paths = sorted(os.path.join(full, f) for f in os.listdir(full))

        t = time.perf_counter()
        corpus = ingest.read_corpus(paths, threads=a.threads)
        t_read = time.perf_counter() - t
        assert corpus.n_sent == a.pairs, corpus.n_sent
        rng = random.Random(7)
        t = time.perf_counter()
        perm = ingest.py_shuffle_perm(corpus.n_sent, rng)
        t_perm = time.perf_counter() - t
        t = time.perf_counter()
        corpus.permute_(perm)
        t_gather = time.perf_counter() - t
        del corpus, perm

        t = time.perf_counter()
        gp = G.read_gene_pairs(small, "txt", random.Random(7))
        t_py_read = time.perf_counter() - t
        assert len(gp) == a.py_pairs
        t = time.perf_counter()
        random.Random(7).shuffle(gp)
        t_py_shuf = time.perf_counter() - t
        del gp
        scale = a.pairs / a.py_pairs
        out = {
            "metric": "pair-file ingest (tokenize + vocab ids) and per-iteration reshuffle",
            "pairs": a.pairs, "text_bytes": nbytes, "files": a.files, "threads": a.threads,
            "native_read_s": round(t_read, 3),
            "native_read_GBps": round(nbytes / t_read / 1e9, 3),
            "native_read_pairs_per_s": round(a.pairs / t_read, 1),
            "native_shuffle_perm_s": round(t_perm, 3),
            "native_csr_gather_s": round(t_gather, 3),
            "reference_read_s_scaled": round(t_py_read * scale, 2),
            "reference_shuffle_s_scaled": round(t_py_shuf * scale, 2),
            "reference_sample": f"src/gene2vec.py:36-47 loop and random.shuffle on the first "
                                f"{a.py_pairs} pairs ({sbytes} B): {t_py_read:.2f} s + "
                                f"{t_py_shuf:.2f} s, x {scale:g}",
            "read_speedup": round(t_py_read * scale / t_read, 1),
            "shuffle_speedup": round(t_py_shuf * scale / (t_perm + t_gather), 1),
            "corpus_write_s_excluded": round(t_write, 2),
        }
        print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
