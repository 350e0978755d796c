"""Replica-vs-one-model quality harness: the
evaluation side of data parallelism, shared by scripts/replica_quality.py (the
studies) and tests/test_gpu_c3_quality.py (the C3 gate).

The reference trains ONE model with 32 Hogwild threads (src/gene2vec.py:59,70)
over the reference's 10-iteration alpha sawtooth (src/gene2vec.py:67-92).
Data parallelism (C3: 8 ranks x 125 M pairs) trains R replicas on contiguous
shards of each iteration's permutation and merges them with libg2v's rule
every `every` jobs.  Here both run on ONE GPU on the same permutations:

  train_single    one engine over the whole permutation
  train_replicas  R engines, one host thread each, an in-process replica
                  group (g2v_comm_init_local: libg2v's merge kernels and
                  in-call merges -- the production merge path of
                  distributed.ReplicaTrainer), rank r training the r-th
                  contiguous 1/R of each permutation with its own job seeds

Corpus ("C3q"): Zipf(s) pairs over V genes, optionally with planted
co-expression modules (a fraction p_in of the pairs rewired inside the first
gene's module) and the reference's GGIPNN positive pairs
(data/predictionData) repeated.  Metrics: the SGNS objective on training pairs
(held-in) and on fresh pairs of the generator (held-out), the manuscript
target function (gene2vec_amd/evaluate.py) with the planted modules as
pathways, and optionally GGIPNN test AUC."""
from __future__ import annotations

import os
import shutil
import tempfile
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _native as N
from . import distributed as Dd
from . import engine as E
from . import synthetic as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "data", "predictionData")


def positives():
    """the GGIPNN splits' positive pairs (all three), as gene-name pairs"""
    out = []
    for part in ("train", "valid", "test"):
        text = open(os.path.join(DATA, f"{part}_text.txt")).read().splitlines()
        lab = open(os.path.join(DATA, f"{part}_label.txt")).read().splitlines()
        out += [t.split() for t, l in zip(text, lab) if l == "1" and len(t.split()) == 2]
    return out


def module_of(V0, modules, seed=3):
    """planted co-expression modules: gene g -> module (a random balanced split)"""
    perm = np.random.RandomState(seed).permutation(V0)
    mod = np.empty(V0, np.int64)
    mod[perm] = np.arange(V0) % modules
    return mod


def planted_pairs(n, V0, mod, modules, p_in, shard, zipf=1.0):
    """Zipf(zipf) pairs, a fraction p_in of them rewired inside the first
    gene's module (the second gene uniform among its module mates): every gene
    keeps a Zipf-like degree and gains co-expression partners, so the target
    function's pathways (= the modules) and its random pairs both mean something"""
    pairs = S.zipf_gene_pairs(n, V0, zipf, seed=20250114, shard=shard)
    rng = np.random.Generator(np.random.PCG64(9000 + shard))
    order = np.argsort(mod, kind="stable")
    start = np.searchsorted(mod[order], np.arange(modules))
    size = np.bincount(mod, minlength=modules)
    sel = np.nonzero(rng.random(n) < p_in)[0]
    a = pairs[sel, 0]
    m = mod[a]
    b = order[start[m] + (rng.random(len(sel)) * size[m]).astype(np.int64)]
    bad = b == a
    while bad.any():
        mb = m[bad]
        b[bad] = order[start[mb] + (rng.random(int(bad.sum())) * size[mb]).astype(np.int64)]
        bad = b == a
    pairs[sel, 1] = b
    return pairs


def build_corpus(R, per, V0, rep, modules=0, p_in=0.0, zipf=1.0):
    """(pairs int32[N][2] in id space, names by id, positive pairs by name)"""
    mod = module_of(V0, modules) if modules else None

    def shard(r):
        if modules:
            return planted_pairs(per, V0, mod, modules, p_in, r, zipf)
        return S.zipf_gene_pairs(per, V0, zipf, seed=20250114, shard=r)
    with ThreadPoolExecutor(max_workers=min(R, 16)) as ex:
        shards = list(ex.map(shard, range(R)))
    names = S.gene_names(V0)
    pos = positives()
    gid = {}
    for a, b in pos:
        for g in (a, b):
            if g not in gid:
                gid[g] = V0 + len(gid)
    names += list(gid)
    if rep:
        pp = np.array([[gid[a], gid[b]] for a, b in pos], np.int32)
        shards.append(np.tile(pp, (rep, 1)))
    pairs = np.concatenate(shards)
    del shards
    return pairs, names, pos


def module_gmt(path, mod, modules, names, n_paths=300, seed=0):
    """pathways = planted modules (a random n_paths of them)"""
    rng = np.random.RandomState(seed)
    with open(path, "w") as f:
        for m in rng.choice(modules, size=min(n_paths, modules), replace=False):
            genes = [names[g] for g in np.nonzero(mod == m)[0]]
            f.write("\t".join([f"MODULE{m}", "http://synthetic"] + genes) + "\n")


def synthetic_gmt(path, pos, n_paths=300, max_genes=40, seed=0):
    """pathways = a gene and its positive-pair neighbours (>= 4 of them)"""
    nb = {}
    for a, b in pos:
        nb.setdefault(a, set()).add(b)
        nb.setdefault(b, set()).add(a)
    rng = np.random.RandomState(seed)
    cands = sorted(g for g, s in nb.items() if len(s) >= 4)
    pick = rng.choice(len(cands), size=min(n_paths, len(cands)), replace=False)
    with open(path, "w") as f:
        for k, i in enumerate(pick):
            g = cands[i]
            genes = [g] + sorted(nb[g])[:max_genes - 1]
            f.write("\t".join([f"PATH{k}", "http://synthetic"] + genes) + "\n")


def objective(s0, s1, c, j, counts, K, rng):
    """mean SGNS objective of pairs (c, j) with K unigram^0.75 negatives"""
    p = counts.astype(np.float64) ** 0.75
    negs = rng.choice(len(counts), size=(len(c), K), p=p / p.sum())
    u = s0[j].astype(np.float64)
    pos = np.einsum("nd,nd->n", u, s1[c].astype(np.float64))
    neg = np.einsum("nd,nkd->nk", u, s1[negs].astype(np.float64))
    return float((np.logaddexp(0, -pos) + np.logaddexp(0, neg).sum(1)).mean())


def heldin(s0, s1, tok, counts, K, n=50000, seed=99):
    rng = np.random.Generator(np.random.PCG64(seed))
    idx = rng.integers(0, len(tok) // 2, n)
    return objective(s0, s1, tok[2 * idx], tok[2 * idx + 1], counts, K, rng)


def target_of(s0, index2word, counts, gmt, D):
    """the manuscript target function of the vectors (exported to a scratch
    _w2v.txt, as src/evaluation_target_function.py:18-25 reads it)"""
    from . import evaluate as EV
    from .word2vec import KeyedVectors, Vocab
    out = tempfile.mkdtemp(prefix="rq_")
    try:
        kv = KeyedVectors(D)
        kv.index2word = list(index2word)
        kv.vocab = {w: Vocab(count=int(counts[i]), index=i) for i, w in enumerate(index2word)}
        kv.vectors = np.ascontiguousarray(s0, np.float32)
        w2v = os.path.join(out, "model_w2v.txt")
        kv.save_word2vec_format(w2v)
        return EV.target_function(w2v, gmt, strict=False, verbose=False)
    finally:
        shutil.rmtree(out, ignore_errors=True)


def ggipnn_auc(s0, index2word, pos_genes, seeds, device="cuda"):
    """GGIPNN test AUC (gene2vec_amd/ggipnn.py) on a generateMatrix-layout .txt
    of the GGIPNN genes, mean over classifier seeds"""
    from . import ggipnn as G
    out = tempfile.mkdtemp(prefix="rq_")
    try:
        txt = os.path.join(out, "model.txt")
        with open(txt, "w") as f:
            for i, w in enumerate(index2word):
                if w in pos_genes:
                    f.write(w + "\t" + "".join(v + " " for v in s0[i].astype(np.float32)
                                               .astype(str)) + "\n")
        # the reference's classifier takes dim 200 (src/GGIPNN.py); other
        # dims (C4: 512) size its embedding layer to the vectors
        return [G.train_and_auc(txt, DATA, seed=s, device=device, embedding_size=s0.shape[1])
                for s in seeds]
    finally:
        shutil.rmtree(out, ignore_errors=True)


class Study:
    """One corpus on the GPU (token ids + a permutation buffer) and the
    per-iteration permutations every arm shares."""

    def __init__(self, R, per, V0, rep=3, modules=0, p_in=0.0, zipf=1.0, iters=10, D=200, K=5,
                 sample=1e-3, perm_seed=11, device=0, engine_options=None):
        import torch
        self.R, self.D, self.K, self.sample, self.iters = R, D, K, sample, iters
        # {g2v option key: value} set on every engine of both arms (e.g. the
        # G2V_OPT_TAIL_STORE experiment)
        self.engine_options = dict(engine_options or {})
        self.V0, self.modules, self.zipf = V0, modules, zipf
        pairs, names, pos = build_corpus(R, per, V0, rep, modules, p_in, zipf)
        self.n = n = len(pairs)
        flat = pairs.reshape(-1)
        del pairs
        counts, first = E.count_ids(flat, len(names))
        order, self.remap = S.vocab_order(counts, first)
        self.tok = self.remap[flat]
        del flat
        self.vc = counts[order].astype(np.int64)
        self.V = len(order)
        self.index2word = [names[i] for i in order]
        self.names = names
        self.pos = pos
        self.pos_genes = {g for p in pos for g in p}
        seeds = np.array([zlib.crc32((w + "1").encode()) for w in self.index2word], np.uint32)
        self.syn0 = E.seeded_vectors(seeds, D)
        self.dev = torch.device("cuda", device)
        self.base = torch.from_numpy(self.tok.view(np.int64)).to(self.dev)  # a pair per 8 bytes
        self.perm = torch.empty_like(self.base)
        rs = np.random.RandomState(perm_seed)
        self.perm_seeds = [int(rs.randint(0, 2 ** 62)) for _ in range(iters)]
        self.stream = torch.cuda.current_stream(self.dev)
        # held-out pairs: a fresh draw of the generator (another seed), so
        # memorising the training pairs does not count as quality
        ho = S.zipf_gene_pairs(50000, V0, zipf, seed=777)
        hc, hj = self.remap[ho[:, 0]], self.remap[ho[:, 1]]
        keep = (hc >= 0) & (hj >= 0)
        self.ho_c, self.ho_j = hc[keep], hj[keep]

    def gmt(self, path):
        if self.modules and self.V0 / self.modules > 50:
            # src/evaluation_target_function.py:8-14 drops pathways of > 50 genes
            raise ValueError(f"{self.V0} genes in {self.modules} modules: > 50 genes per module, "
                             "every pathway would be dropped by the target function")
        if self.modules:
            module_gmt(path, module_of(self.V0, self.modules), self.modules, self.names)
        else:
            synthetic_gmt(path, self.pos)
        return path

    def permute(self, it):
        E.permute_items8(0, self.base.data_ptr(), self.perm.data_ptr(), self.n, 0, self.n,
                         self.perm_seeds[it], self.stream.cuda_stream)
        self.stream.synchronize()

    def heldin(self, s0, s1, n=50000):
        return heldin(s0, s1, self.tok, self.vc, self.K, n=n)

    def heldout(self, s0, s1):
        return objective(s0, s1, self.ho_c, self.ho_j, self.vc, self.K,
                         np.random.Generator(np.random.PCG64(98)))

    def train_single(self, seed=1, progress=None):
        eng = E.SGNSEngine(self.V, self.D, self.K)
        try:
            for k, v in self.engine_options.items():
                eng.set_option(k, v)
            eng.set_vocab(self.vc, self.sample)
            eng.set_weights(self.syn0, np.zeros_like(self.syn0))
            rs = np.random.RandomState(seed)
            js = E.plan_jobs(n_sent=self.n, sent_len=2)
            al = E.job_alphas(js, self.n)
            for it in range(self.iters):
                self.permute(it)
                eng.set_corpus_device(self.perm.data_ptr(), 2 * self.n, sent_len=2,
                                      keepalive=self.perm)
                eng.train(js, al, E.job_seeds(rs, len(js) - 1), N.MODE_HOGWILD)
                eng.sync()
                if progress:
                    progress("single", it, eng)
            return eng.get_weights()
        finally:
            eng.close()

    def train_replicas(self, every, rule="touch", beta=1000, gamma=1000, seed=1, progress=None):
        """(syn0, syn1neg, merges, replicas identical?)"""
        R = self.R
        grp = E.LocalGroup(R)
        agree = Dd.ThreadAgreement(R)
        engs = []
        try:
            for _ in range(R):
                e = E.SGNSEngine(self.V, self.D, self.K)
                for k, v in self.engine_options.items():
                    e.set_option(k, v)
                e.set_vocab(self.vc, self.sample)
                e.set_weights(self.syn0, np.zeros_like(self.syn0))
                e.set_option(N.OPT_MERGE_BETA_MILLI, beta)
                e.set_option(N.OPT_MERGE_GAMMA_MILLI, gamma)
                engs.append(e)
            with ThreadPoolExecutor(max_workers=R) as ex:
                list(ex.map(lambda r: engs[r].comm_init_local(grp, r), range(R)))
            trainers = [Dd.ReplicaTrainer(engs[r], (), every, N.MODE_HOGWILD, merge=rule,
                                          backend="libg2v", world=R, agree=agree.for_rank(r))
                        for r in range(R)]
            rs = np.random.RandomState(seed)  # model.random, identical on every rank
            n = self.n
            for it in range(self.iters):
                self.permute(it)
                base_seed = int(rs.randint(0, 2 ** 31 - 1))

                def rank(r):
                    s0r, s1r = Dd.shard_range(n, r, R)
                    e = engs[r]
                    e.set_corpus_device(self.perm.data_ptr() + 8 * s0r, 2 * (s1r - s0r),
                                        sent_len=2, keepalive=self.perm)
                    js = E.plan_jobs(n_sent=s1r - s0r, sent_len=2)
                    al = E.job_alphas(js, s1r - s0r)
                    sd = E.job_seeds(np.random.RandomState((base_seed + 7919 * r) % 2 ** 32),
                                     len(js) - 1)
                    trainers[r].train_epoch(js, al, sd)
                    e.sync()
                with ThreadPoolExecutor(max_workers=R) as ex:
                    list(ex.map(rank, range(R)))
                if progress:
                    progress("replicas", it, engs[0])
            s0, s1 = engs[0].get_weights()
            same = all(np.array_equal(e.get_weights()[0], s0) for e in engs[1:])
            return s0, s1, trainers[0].averages, same
        finally:
            for e in engs:
                e.close()
            grp.close()
