"""Restatement of src/evaluation_target_function.py on numpy/gensim semantics
-- TEST INFRASTRUCTURE ONLY.  wv.similarity = float32 dot of gensim
unitvec(v) = sscal(1/snrm2(v), v); Python sum() of float32 scalars is a
sequential float32 accumulation; dividing that float32 by a Python int is
float64 under NumPy 1.x (the gensim 3.4 era), so the pathway means, their
mean and the ratio are float64.  Parity unpinned (gensim absent)."""
import itertools
import random

import numpy as np


def _unit(v):
    v = np.asarray(v, dtype=np.float32)
    n = np.float32(np.sqrt(np.dot(v.astype(np.float64), v.astype(np.float64))))
    return v * np.float32(1.0 / float(n))


def similarity(vecs, a, b):
    return np.float32(np.dot(_unit(vecs[a]).astype(np.float64), _unit(vecs[b]).astype(np.float64)))


def target_function(words, vecs, pathways):
    """words: names in _w2v.txt row order; vecs: rows; pathways: raw gmt lines"""
    idx = {w: i for i, w in enumerate(words)}
    units = np.stack([_unit(v) for v in vecs]).astype(np.float64)

    def similarity(_, a, b):  # noqa: F811 -- same math, unit vectors cached
        return np.float32(np.dot(units[a], units[b]))

    paths = []
    for pw in pathways:
        tmp = pw.split("\t")
        genes = [tmp[i] for i in range(2, len(tmp)) if tmp[i] in idx]
        arr = np.float32(0)
        cnt = 0
        for x, y in itertools.combinations(genes, 2):
            arr = np.float32(arr + similarity(vecs, idx[x], idx[y]))
            cnt += 1
        paths.append(np.float64(arr) / cnt)  # cnt == 0: nan (the reference raises: sum([]) is int 0)
    gl = list(words)
    random.seed(35)
    random.shuffle(gl)
    rs = np.float32(0)
    cnt = 0
    for x, y in itertools.combinations(gl[:1000], 2):
        rs = np.float32(rs + similarity(vecs, idx[x], idx[y]))
        cnt += 1
    pm = 0.0
    for p in paths:
        pm = pm + p
    pm = pm / len(paths)
    rm = np.float64(rs) / cnt
    return float(pm), float(rm), float(pm / rm)
