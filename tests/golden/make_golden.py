"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle.

    python tests/golden/make_golden.py

Inputs: ``test_pairs.txt`` is the reference's own smoke corpus
(``/root/reference/data/test.txt``, 40 gene pairs, copied verbatim as data).
Everything else is synthetic with fixed seeds.  Outputs are produced by
``oracle/sgns_oracle.py`` (gensim 3.4.0 restatement; parity unpinned upstream,
see oracle/__init__.py) and are the regression anchors the CPU and GPU tests
compare against.
"""
from __future__ import annotations

import json
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import sgns_oracle as O  # noqa: E402


def crc_hash(s: str) -> int:
    """deterministic stand-in for Python's randomised str hash (gensim hashfxn)"""
    return zlib.crc32(s.encode("utf-8"))


def read_pairs(path):
    with open(path, "r", encoding="windows-1252") as f:
        return [line.strip().split() for line in f]


def zipf_counts(V, s, total, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    p = 1.0 / np.arange(1, V + 1) ** s
    p /= p.sum()
    c = rng.multinomial(total, p)
    c[c == 0] = 1
    return np.sort(c)[::-1].astype(np.int64)


def main():
    out = {}
    sents = read_pairs(os.path.join(HERE, "test_pairs.txt"))
    voc = O.build_vocab(sents, min_count=1, sample=1e-3)
    out["test_pairs"] = dict(
        corpus_count=voc.corpus_count, total_words=voc.total_words,
        index2word=voc.index2word, first_order=voc.first_order,
        counts=voc.counts.tolist(), sample_int=[int(x) for x in voc.sample_int],
        sample_int_s0=[int(x) for x in O.sample_int_from_counts(voc.counts, 0.0)],
        cum_table=[int(x) for x in O.make_cum_table(voc.counts)])
    # synthetic Zipf cum tables (bit-exact targets)
    for V, s in ((1000, 1.0), (24447, 1.0), (60000, 0.8)):
        c = zipf_counts(V, s, 50 * V, 20250114)
        np.savez_compressed(os.path.join(HERE, f"zipf{V}_tables.npz"), counts=c,
                            cum=O.make_cum_table(c),
                            sample_int=O.sample_int_from_counts(c, 1e-3).astype(np.uint64))
    # LUT + LCG stream + negative draws
    np.save(os.path.join(HERE, "exp_table.npy"), O.exp_table())
    nr = 123456789012345
    stream = []
    cum = np.load(os.path.join(HERE, "zipf1000_tables.npz"))["cum"]
    negs = []
    x = nr
    for _ in range(1000):
        stream.append(x >> 16)
        t, x = O.draw_negative(cum, x)
        negs.append(t)
    out["lcg"] = dict(seed=nr, outputs=stream[:1000], negatives_zipf1000=negs,
                      jump_1000=O.lcg_jump(nr, 1000), jump_123457=O.lcg_jump(nr, 123457))
    # alpha schedule / job boundaries
    jobs40 = O.plan_jobs([2] * 40)
    jobs1m = O.plan_jobs([2] * 1000000)
    a1m = O.job_alphas(jobs1m, 1000000)
    mixed = [2, 4, 0, 2, 3, 9997, 2, 10000, 1] * 3
    out["schedule"] = dict(
        jobs40=jobs40, alphas40=O.job_alphas(jobs40, 40),
        jobs1m_n=len(jobs1m), jobs1m_first=jobs1m[:3], alphas1m_head=a1m[:5],
        alphas1m_tail=a1m[-5:], mixed_lengths=mixed, mixed_jobs=O.plan_jobs(mixed),
        epoch2of3=O.job_alphas(jobs40, 40, cur_epoch=1, epochs=3),
        seeds_rs1=[int(v) for v in O.job_seeds(np.random.RandomState(1), 5)])
    # seeded_vector with crc hash (numpy RandomState)
    out["seeded_vector"] = dict(word="TLE1", seed=1, dim=8,
                                values=[float(v) for v in
                                        O.seeded_vector("TLE11", 8, crc_hash).astype(np.float32)])
    # explicit-negative SGNS steps (sequential gensim order)
    for (V, D, K) in ((60, 200, 5), (40, 512, 15)):
        rng = np.random.Generator(np.random.PCG64(7 + D))
        syn0 = ((rng.random((V, D)) - 0.5) / D * 50).astype(np.float32)
        syn1 = ((rng.random((V, D)) - 0.5) / D * 50).astype(np.float32)
        lockf = np.ones(V, dtype=np.float32)
        B = 256
        center = rng.integers(0, V, B).astype(np.int32)
        inp = rng.integers(0, V, B).astype(np.int32)
        negs = rng.integers(-1, V, (B, K)).astype(np.int32)
        negs[negs == center[:, None]] = -1
        a0, a1 = syn0.copy(), syn1.copy()
        O.sgns_step_sequential(a0, a1, lockf, center, inp, negs, 0.025)
        np.savez_compressed(os.path.join(HERE, f"step_V{V}_D{D}_K{K}.npz"), syn0=syn0,
                            syn1neg=syn1, center=center, input=inp, negs=negs, alpha=0.025,
                            syn0_out=a0, syn1neg_out=a1)
    # tiny end-to-end run on the reference corpus, workers=1 order
    for sample in (0.0, 1e-3):
        voc = O.build_vocab(sents, 1, sample)
        ids = O.sentences_to_ids(sents, voc.word2index)
        syn0, syn1, lockf = O.reset_weights(voc.index2word, 200, 1, crc_hash)
        a0, a1 = syn0.copy(), syn1.copy()
        rs = np.random.RandomState(1)
        cum = O.make_cum_table(voc.counts)
        stats = []
        for it in range(3):  # three gene2vec "iterations" (sawtooth alpha)
            stats.append(O.train_epoch_sequential(ids, voc, a0, a1, lockf, cum, 5, rs,
                                                  sample=sample))
        tag = "s0" if sample == 0 else "s1e-3"
        np.savez_compressed(os.path.join(HERE, f"e2e_test_pairs_{tag}.npz"), syn0_init=syn0,
                            syn0=a0, syn1neg=a1, stats=json.dumps(stats))
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, default=lambda o: o.item() if hasattr(o, "item") else list(o))
    print("wrote", HERE)


if __name__ == "__main__":
    main()
