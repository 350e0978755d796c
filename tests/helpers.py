"""shared test helpers (synthetic corpora, crc hash)"""
import zlib

import numpy as np


def crc_hash(s):
    return zlib.crc32(s.encode("utf-8"))


def zipf_pairs(n_pairs, V, s=1.0, seed=20250114):
    """SURVEY 8(d) synthetic corpus: endpoints iid Zipf(s) over ranks, a != b."""
    rng = np.random.Generator(np.random.PCG64(seed))
    p = 1.0 / np.arange(1, V + 1, dtype=np.float64) ** s
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    a = np.searchsorted(cdf, rng.random(n_pairs), side="right").astype(np.int32)
    b = np.searchsorted(cdf, rng.random(n_pairs), side="right").astype(np.int32)
    bad = a == b
    while bad.any():
        b[bad] = np.searchsorted(cdf, rng.random(int(bad.sum())), side="right")
        bad = a == b
    np.minimum(a, V - 1, out=a)
    np.minimum(b, V - 1, out=b)
    return np.stack([a, b], axis=1)


def vocab_from_ids(pairs_flat, V):
    """gensim vocab order for integer-id corpora: stable sort by -count over
    first occurrence.  Returns (order: vocab index -> raw id, remap raw id ->
    vocab index, counts in index order); ids that never occur are dropped."""
    counts = np.bincount(pairs_flat, minlength=V)
    present = np.nonzero(counts)[0]
    first = np.full(V, len(pairs_flat), dtype=np.int64)
    uniq, idx = np.unique(pairs_flat, return_index=True)
    first[uniq] = idx
    fo = present[np.argsort(first[present], kind="stable")]   # first-occurrence order
    order = fo[np.argsort(-counts[fo], kind="stable")]
    remap = np.full(V, -1, dtype=np.int32)
    remap[order] = np.arange(len(order), dtype=np.int32)
    return order, remap, counts[order].astype(np.int64)


def planted_expression(n_samples, n_genes, n_groups=4, noise=0.15, seed=0, zeros=0.0):
    """[samples][genes] positive expression with planted co-expressed groups:
    gene g follows latent factor g % n_groups with loading and noise; a
    fraction `zeros` of entries set to 0 (TPM dropouts)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    f = rng.normal(size=(n_samples, n_groups))
    load = rng.uniform(0.5, 2.0, size=n_genes) * rng.choice([-1.0, 1.0], size=n_genes)
    x = f[:, np.arange(n_genes) % n_groups] * load + noise * rng.normal(size=(n_samples, n_genes))
    x = np.exp(x)
    if zeros:
        x[rng.random(x.shape) < zeros] = 0.0
    return x


def make_query(root, seed=0, studies=(("SRP1", 24), ("SRP2", 30), ("SRP3", 5)), n_genes=150):
    """Synthetic processed query in the layout src/generate_gene_pairs.py:143-155
    reads: data/SRARunTable.csv, data/gene_counts_TPM.csv, data/gene_counts.csv.
    Gene ids 'ENSG<k>|NAME<k>' with some unnamed, some duplicated names and
    some low-count genes."""
    import os

    import pandas as pd

    rng = np.random.Generator(np.random.PCG64(seed + 1000))
    runs, study_of = [], []
    for s, n in studies:
        for i in range(n):
            runs.append(f"{s}_R{i:03d}")
            study_of.append(s)
    x = planted_expression(len(runs), n_genes, seed=seed, zeros=0.05)
    ens = [f"ENSG{k:05d}" for k in range(n_genes)]
    ids = []
    for k, e in enumerate(ens):
        if k % 17 == 3:
            ids.append(e)                       # no name -> dropped by name mode
        elif k % 23 == 5:
            ids.append(f"{e}|DUP{k % 2}")        # duplicated names -> dropped
        else:
            ids.append(f"{e}|G{k}")
    counts = rng.integers(0, 40, size=(n_genes, len(runs)))
    counts[::11] = 0                             # low-expression genes
    os.makedirs(os.path.join(root, "data"), exist_ok=True)
    pd.DataFrame({"SRA Study": study_of}, index=pd.Index(runs, name="Run")).to_csv(
        os.path.join(root, "data/SRARunTable.csv"))
    pd.DataFrame(x, index=pd.Index(runs, name="Run"), columns=ens).to_csv(
        os.path.join(root, "data/gene_counts_TPM.csv"))
    gc = pd.DataFrame(counts, columns=runs)
    gc.insert(0, "gene_id", ids)
    gc.to_csv(os.path.join(root, "data/gene_counts.csv"), index=False)
    return root


def long_sentence_corpus(seed=0):
    """sentences over gensim's batch_words (40000 tokens first, so the job
    producer queues an empty job; 12000; 10001) beside short and empty ones,
    a downsampling-heavy word in the long head, OOV tokens.  Returns (tok,
    sent_off, counts) in vocabulary index order."""
    rng = np.random.RandomState(seed)
    V = 20000
    lengths = [40000, 3, 2, 12000, 0, 10001, 10000, 7]
    tok = rng.randint(-1, V, size=sum(lengths)).astype(np.int32)
    tok[:30000][rng.rand(30000) < 0.6] = 0           # a very frequent word: heavy downsampling
    counts = np.bincount(tok[tok >= 0], minlength=V).astype(np.int64)
    order = np.argsort(-counts, kind="stable")
    order = order[counts[order] > 0]                  # words that occur
    remap = np.full(V, -1, np.int32)
    remap[order] = np.arange(len(order), dtype=np.int32)
    tok = np.where(tok >= 0, remap[np.maximum(tok, 0)], -1).astype(np.int32)
    off = np.cumsum([0] + lengths).astype(np.int64)
    return tok, off, counts[order]


# ---------------------------------------------------------------------------
# end-to-end parity corpus (tests/test_gpu_e2e_parity.py,
# tests/golden/make_e2e_golden.py): Zipf(1) pairs with planted co-expression
# modules, the reference's 10-iteration flow, one permutation per iteration
E2E = {"V0": 3000, "modules": 100, "p_in": 0.5, "pairs": 2_000_000, "iters": 10, "D": 200,
       "K": 5, "sample": 1e-3, "seeds": (1, 2, 3)}


# the same flow at the C2 bench vocabulary (tests/golden/e2e_parity_c2.json)
E2E_C2 = dict(E2E, V0=24447, modules=1000, pairs=10_000_000, seeds=(1, 2))

# a dense corpus (5,000 genes, 200 modules, 4 M pairs: every gene in ~1,600
# pairs), where the Hogwild staleness moves the target function most
# (tests/golden/e2e_parity_v5k.json)
E2E_V5K = dict(E2E, V0=5000, modules=200, pairs=4_000_000, seeds=(1, 2, 3))


def e2e_corpus(c=None):
    """(tok int32[2n] in vocab index order, vocab counts, index2word, pathway
    lines (gmt text, newline kept as the reference reads them), per-iteration
    permutations, seeded syn0 hashes)"""
    c = c or E2E
    V0, M = c["V0"], c["modules"]
    pairs = zipf_pairs(c["pairs"], V0, 1.0, seed=20250114)
    mod = np.empty(V0, np.int64)
    mod[np.random.RandomState(3).permutation(V0)] = np.arange(V0) % M
    rng = np.random.Generator(np.random.PCG64(9000))
    order_m = np.argsort(mod, kind="stable")
    start = np.searchsorted(mod[order_m], np.arange(M))
    size = np.bincount(mod, minlength=M)
    sel = np.nonzero(rng.random(len(pairs)) < c["p_in"])[0]
    a = pairs[sel, 0]
    m = mod[a]
    b = order_m[start[m] + (rng.random(len(sel)) * size[m]).astype(np.int64)]
    bad = b == a
    while bad.any():
        b[bad] = order_m[start[m[bad]] + (rng.random(int(bad.sum())) * size[m[bad]]).astype(np.int64)]
        bad = b == a
    pairs[sel, 1] = b
    order, remap, counts = vocab_from_ids(pairs.reshape(-1), V0)
    tok = remap[pairs.reshape(-1)].astype(np.int32)
    names = [f"G{i:05d}" for i in range(V0)]
    index2word = [names[i] for i in order]
    lines = []
    for k in range(M):
        genes = [names[g] for g in np.nonzero(mod == k)[0]]
        lines.append("\t".join([f"MODULE{k}", "http://synthetic"] + genes) + "\n")
    n = len(pairs)
    rs = np.random.RandomState(11)
    perms = [rs.permutation(n) for _ in range(c["iters"])]
    seeds = np.array([crc_hash(w + "1") for w in index2word], np.uint32)
    return tok, counts, index2word, lines, perms, seeds


def e2e_heldin(s0, s1, tok, counts, K, n=40000, seed=99):
    """SGNS objective on n corpus pairs with K unigram^0.75 negatives"""
    rng = np.random.Generator(np.random.PCG64(seed))
    idx = rng.integers(0, len(tok) // 2, n)
    c, j = tok[2 * idx], tok[2 * idx + 1]
    p = counts.astype(np.float64) ** 0.75
    negs = rng.choice(len(counts), size=(n, K), p=p / p.sum())
    u = s0[j].astype(np.float64)
    pos = np.einsum("nd,nd->n", u, s1[c].astype(np.float64))
    neg = np.einsum("nd,nkd->nk", u, s1[negs].astype(np.float64))
    return float((np.logaddexp(0, -pos) + np.logaddexp(0, neg).sum(1)).mean())
