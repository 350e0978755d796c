"""Manuscript target function -- mirror of src/evaluation_target_function.py.

    target = mean over MSigDB pathways (<= 50 genes) of the mean pairwise
             cosine of the pathway's in-vocabulary genes
           / mean pairwise cosine of the first 1000 genes after
             random.seed(35); random.shuffle(gene list in file order)

Reproduced exactly, quirks included (reference line numbers):
  * pathways: lines of the .gmt with <= 52 tab fields (:8-14), genes are
    fields 2.. of ``line.split("\\t")`` -- the last field keeps its "\\n", so
    the last gene of every newline-terminated line never matches (:30-33);
  * gene list = first token of every line of the _w2v.txt except the
    header (``len(line.split(" ")) == 2``, :18-23), in file order;
  * similarities are gensim's float32 ``wv.similarity`` (:38,:49), computed
    on the GPU by ``g2v_cosine_pairs``; ``sum(list)`` of numpy float32 values
    is a sequential float32 accumulation, reproduced with ``np.cumsum``;
  * a pathway with < 2 in-vocabulary genes divides by zero (:40) -- raised
    as in the reference unless ``strict=False`` (then skipped).
"""
from __future__ import annotations

import itertools
import random

import numpy as np

from . import _native as N
from .word2vec import KeyedVectors


def read_pathways(gmt_file):
    out = []
    with open(gmt_file, "r") as f:
        for line in f:
            if len(line.split("\t")) > 52:
                continue
            out.append(line)
    return out


def read_gene_list(emb_w2v_file):
    genes = []
    with open(emb_w2v_file, "r") as f:
        for line in f:
            if len(line.split(" ")) == 2:
                continue
            genes.append(line.split(" ")[0])
    return genes


def cosine_pairs(kv, pairs_a, pairs_b, device=0):
    """gensim wv.similarity for index pairs, on the GPU (no CPU fallback)."""
    a = np.ascontiguousarray(pairs_a, dtype=np.int32)
    b = np.ascontiguousarray(pairs_b, dtype=np.int32)
    out = np.zeros(len(a), dtype=np.float32)
    vec = np.ascontiguousarray(kv.vectors, dtype=np.float32)
    N.check(N.lib().g2v_cosine_pairs(device, N.ptr(vec), vec.shape[0], vec.shape[1], N.ptr(a),
                                     N.ptr(b), len(a), N.ptr(out)))
    return out


def _f32_sum(x):
    """Python's sum() over numpy float32 scalars: sequential float32 adds"""
    x = np.asarray(x, dtype=np.float32)
    return np.cumsum(x, dtype=np.float32)[-1] if len(x) else np.float32(0)


def target_function(emb_w2v_file, gmt_file=None, pathways=None, strict=True, device=0,
                    verbose=True):
    gene_list = read_gene_list(emb_w2v_file)
    kv = KeyedVectors.load_word2vec_format(emb_w2v_file)
    if pathways is None:
        pathways = read_pathways(gmt_file)
    in_vocab = set(gene_list)
    idx = {w: kv.vocab[w].index for w in kv.vocab}
    # numerator: all pathway pairs in one GPU call
    pa, pb, bounds = [], [], []
    for pw in pathways:
        tmp = pw.split("\t")
        genes = [tmp[i] for i in range(2, len(tmp)) if tmp[i] in in_vocab]
        n0 = len(pa)
        for x, y in itertools.combinations(genes, 2):
            pa.append(idx[x])
            pb.append(idx[y])
        bounds.append((n0, len(pa)))
    sims = cosine_pairs(kv, pa, pb, device) if pa else np.zeros(0, np.float32)
    paths = []
    for n0, n1 in bounds:
        if n1 == n0:
            if strict:
                raise ZeroDivisionError("pathway with fewer than 2 in-vocabulary genes "
                                        "(src/evaluation_target_function.py:40)")
            continue
        # sum(tmp_arr)/len(tmp_arr) (:40): float32 adds, then a float32 scalar
        # over a Python int, which NumPy 1.x (the gensim 3.4 era) promotes to
        # float64; the mean of means (:54-55) and the ratio stay float64
        paths.append(np.float64(_f32_sum(sims[n0:n1])) / (n1 - n0))
    # denominator: random.seed(35); shuffle; first 1000 genes, all pairs
    rng = random.Random(35)
    shuffled = list(gene_list)
    rng.shuffle(shuffled)
    top = [idx[w] for w in shuffled[:1000]]
    ra, rb = zip(*itertools.combinations(top, 2)) if len(top) > 1 else ((), ())
    rsims = cosine_pairs(kv, ra, rb, device)
    path_mean = np.float64(sum(paths)) / len(paths)
    rand_mean = np.float64(_f32_sum(rsims)) / len(rsims)
    ratio = path_mean / rand_mean
    if verbose:
        print("------------")
        print(emb_w2v_file)
        print(path_mean, end="")
        print("\t", rand_mean)
        print(ratio)
        print("------------")
    return {"path_mean": float(path_mean), "rand_mean": float(rand_mean), "ratio": float(ratio),
            "n_pathways": len(paths), "n_random_pairs": len(rsims)}
