#!/usr/bin/env python
"""End-to-end parity harness (SURVEY.md §8(f) ranks 1-2 on real reference data).

The paper-scale co-expression corpus and MSigDB are absent, so the
reference's own labelled GGIPNN splits supply both sides.  The splits are
gene-disjoint (no test gene occurs in train), so the corpus must include the
test positives: the harness is LABEL-LEAKY by construction and only measures
engine parity (GPU vs oracle on identical inputs), not gene2vec's AUC.
  corpus  the positive pairs of all three splits (label 1),
          ingested the gene2vec.py way (seeded shuffle, 10 sawtooth iterations,
          dim 200, window 1, sample 1e-3, neg 5);
  metric  GGIPNN test AUC (gene2vec_amd/ggipnn.py, TF1 model restated in torch)
          on those embeddings, mean over several classifier seeds.

    python scripts/ggipnn_e2e.py train --engine gpu    --out runs/gpu     # MI355X, libg2v
    python scripts/ggipnn_e2e.py train --engine oracle --out runs/oracle  # C oracle, CPU
    python scripts/ggipnn_e2e.py auc --emb runs/gpu/emb.txt --seeds 0,1,2,3,4
"""
import argparse
import json
import os
import random
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

DATA = os.path.join(ROOT, "data", "predictionData")


def crc(s):
    return zlib.crc32(s.encode("utf-8"))


def positive_pairs(parts=("train", "valid", "test")):
    out = []
    for part in parts:
        text = open(os.path.join(DATA, f"{part}_text.txt")).read().splitlines()
        lab = open(os.path.join(DATA, f"{part}_label.txt")).read().splitlines()
        out += [t.strip().split() for t, l in zip(text, lab) if l == "1"]
    return out


def write_txt(path, words_first_order, vec_of):
    rows = np.array([vec_of(w) for w in words_first_order], np.float32).astype(str)
    with open(path, "w") as f:
        for w, r in zip(words_first_order, rows):
            f.write(w + "\t" + "".join(v + " " for v in r) + "\n")


def train(engine, out, iters, seed):
    os.makedirs(out, exist_ok=True)
    pairs = positive_pairs()
    rng = random.Random(seed)
    rng.shuffle(pairs)
    t0 = time.time()
    if engine == "gpu":
        from gene2vec_amd import Word2Vec
        m = Word2Vec(pairs, size=200, window=1, min_count=1, workers=32, iter=1, sg=1,
                     hashfxn=crc)
        for _ in range(1, iters):
            rng.shuffle(pairs)
            m.train(pairs, total_examples=m.corpus_count, epochs=m.iter)
        words = list(m.wv.vocab.keys())
        write_txt(os.path.join(out, "emb.txt"), words, lambda w: m.wv[w])
    else:
        from oracle import c_oracle as CO
        from oracle import sgns_oracle as O
        voc = O.build_vocab(pairs, 1, 1e-3)
        syn0, syn1, lockf = O.reset_weights(voc.index2word, 200, 1, crc)
        cum = O.make_cum_table(voc.counts)
        rs = np.random.RandomState(1)
        for it in range(iters):
            if it:
                rng.shuffle(pairs)
            ids = O.sentences_to_ids(pairs, voc.word2index)
            tok = np.array([w for s in ids for w in s], np.int32)
            off = np.cumsum([0] + [len(s) for s in ids]).astype(np.int64)
            jobs = O.plan_jobs([len(s) for s in ids])
            js = np.array([jobs[0][0]] + [j[1] for j in jobs], np.int64)
            al = np.array(O.job_alphas(jobs, len(ids)), np.float32)
            sd = np.array(O.job_seeds(rs, len(jobs)), np.uint64)
            CO.train(tok, off, js, al, sd, voc.sample_int, True, cum, syn0, syn1, lockf, 5)
        write_txt(os.path.join(out, "emb.txt"), voc.first_order,
                  lambda w: syn0[voc.word2index[w]])
    info = {"engine": engine, "pairs": len(pairs), "iters": iters, "seed": seed,
            "train_s": round(time.time() - t0, 2)}
    json.dump(info, open(os.path.join(out, "train.json"), "w"))
    print(json.dumps(info))


def cosine_auc(emb):
    """AUC of the plain embedding cosine on the test pairs (no classifier)"""
    from sklearn import metrics
    vec = {}
    for line in open(emb):
        v = line.split()
        vec[v[0]] = np.asarray(v[1:], np.float32)
    text = open(os.path.join(DATA, "test_text.txt")).read().splitlines()
    lab = np.array(open(os.path.join(DATA, "test_label.txt")).read().splitlines(), int)
    s = []
    for t in text:
        a, b = t.split()
        if a in vec and b in vec:
            x, y = vec[a], vec[b]
            s.append(float(x @ y / (np.linalg.norm(x) * np.linalg.norm(y))))
        else:
            s.append(0.0)
    return float(metrics.roc_auc_score(lab, s))


def auc(emb, seeds):
    from gene2vec_amd import ggipnn as G
    vals = [G.train_and_auc(emb, DATA, seed=s) for s in seeds]
    out = {"emb": emb, "seeds": seeds, "auc": vals, "mean": float(np.mean(vals)),
           "std": float(np.std(vals)), "cosine_auc": cosine_auc(emb)}
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("cmd", choices=("train", "auc"))
    p.add_argument("--engine", choices=("gpu", "oracle"), default="gpu")
    p.add_argument("--out", default="runs/e2e")
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--seed", type=int, default=7)
    p.add_argument("--emb")
    p.add_argument("--seeds", default="0,1,2,3,4")
    a = p.parse_args()
    if a.cmd == "train":
        train(a.engine, a.out, a.iters, a.seed)
    else:
        auc(a.emb, [int(s) for s in a.seeds.split(",")])
