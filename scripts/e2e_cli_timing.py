"""End-to-end timing of the gene2vec CLI mirror (src/gene2vec.py) on a
synthetic pair corpus: ingest -> 10 iterations (train, checkpoint, .txt,
_w2v.txt) on one MI355X.

    python scripts/e2e_cli_timing.py [--pairs 20000000] [--files 4] [--iters 10]

Writes the corpus as text files like the reference's data_dir (one "A B" pair
per line), runs ``gene2vec_amd.gene2vec.main`` with --native-ingest, and prints
one JSON line with the wall-clock split (corpus write excluded).
"""
import argparse
import contextlib
import io
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gene2vec_amd import gene2vec as G  # noqa: E402
from gene2vec_amd import synthetic as S  # noqa: E402


def write_corpus(d, n_pairs, n_files, vocab):
    names = np.array(S.gene_names(vocab))
    pairs = S.zipf_gene_pairs(n_pairs, vocab, 1.0, seed=20250114)
    for k, (a, b) in enumerate(zip(np.array_split(pairs[:, 0], n_files),
                                   np.array_split(pairs[:, 1], n_files))):
        lines = np.char.add(np.char.add(names[a], " "), names[b])
        with open(os.path.join(d, f"pairs_{k}.txt"), "w", encoding="windows-1252") as f:
            f.write("\n".join(lines.tolist()))
            f.write("\n")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pairs", type=int, default=20_000_000)
    p.add_argument("--files", type=int, default=4)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--vocab", type=int, default=24447)
    p.add_argument("--keep", action="store_true")
    p.add_argument("--shuffle", choices=("python", "device"), default="python",
                   help="the CLI's --shuffle (reshuffles of iterations >= 2)")
    a = p.parse_args()
    work = tempfile.mkdtemp(prefix="g2v_e2e_")
    data, out = os.path.join(work, "data"), os.path.join(work, "out")
    os.makedirs(data)
    t = time.perf_counter()
    write_corpus(data, a.pairs, a.files, a.vocab)
    t_write = time.perf_counter() - t
    log = io.StringIO()
    t = time.perf_counter()
    with contextlib.redirect_stdout(log):
        outs = G.main([data, out, "txt", "--native-ingest", "--hash", "crc32",
                       "--shuffle-seed", "7", "--iters", str(a.iters), "--shuffle", a.shuffle,
                       "--timing", os.path.join(work, "phases.json")])
    total = time.perf_counter() - t
    sizes = {os.path.basename(f): os.path.getsize(f) for f in
             [outs[-1] + ".txt", outs[-1] + "_w2v.txt"]}
    res = {"metric": "gene2vec CLI end to end (native ingest + %d iterations + exports)" % a.iters,
           "pairs": a.pairs, "files": a.files, "shuffle": a.shuffle, "wall_s": round(total, 2),
           "pairs_per_s_incl_io": round(a.pairs * a.iters / total, 1),
           "corpus_write_s_excluded": round(t_write, 2), "outputs": sizes,
           "phases_s": json.load(open(os.path.join(work, "phases.json")))}
    print(json.dumps(res))
    if not a.keep:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
