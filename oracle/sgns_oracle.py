"""NumPy / pure-Python restatement of gensim 3.4.0 skip-gram negative sampling.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Parity unpinned: gensim
is absent offline and the reference has no tests; every function cites the
reference call site it serves and the gensim 3.4.0 routine it restates
([ext] = upstream gensim).

Reference call sites served:
  * ``src/gene2vec.py:45``      -- ``line.strip().split()`` tokenisation
  * ``src/gene2vec.py:70``      -- ``Word2Vec(pairs, size=200, window=1,
                                   min_count=1, workers=32, iter=1, sg=1)``
  * ``src/gene2vec.py:86-88``   -- ``load`` + ``train(total_examples=corpus_count,
                                   epochs=model.iter)`` (alpha restarts: sawtooth)
  * ``src/generateMatrix.py:12-24`` -- ``.txt`` matrix export
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

REAL = np.float32
MAX_EXP = 6
EXP_TABLE_SIZE = 1000
# word2vec_inner.pyx: int((f + MAX_EXP) * (EXP_TABLE_SIZE / MAX_EXP / 2)) with
# C integer division of the DEF constants -> 83 (the word2vec.c quirk).
LUT_SCALE = EXP_TABLE_SIZE // MAX_EXP // 2
MAX_SENTENCE_LEN = 10000
LCG_MUL = 25214903917
LCG_ADD = 11
LCG_MASK = (1 << 48) - 1
DOMAIN = 2 ** 31 - 1


# --------------------------------------------------------------------------
# A.1 / A.2 vocabulary  ([ext] Word2VecVocab.scan_vocab / prepare_vocab /
# sort_vocab; reference call site src/gene2vec.py:70)
# --------------------------------------------------------------------------
@dataclass
class Vocab:
    index2word: list            # index order (stable sort by -count)
    counts: np.ndarray          # int64, index order
    sample_int: np.ndarray      # uint64 holding values in [0, 2**32], index order
    first_order: list           # words in first-occurrence order (wv.vocab dict order)
    word2index: dict = field(default_factory=dict)
    corpus_count: int = 0       # number of sentences scanned
    total_words: int = 0        # raw words scanned


def scan_vocab(sentences):
    """[ext] scan_vocab: counts in first-occurrence (dict insertion) order."""
    raw = {}
    total = 0
    n = 0
    for n, sent in enumerate(sentences, 1):
        for w in sent:
            raw[w] = raw.get(w, 0) + 1
            total += 1
    return raw, n, total


def prepare_vocab(raw_vocab, min_count=1, sample=1e-3):
    """[ext] prepare_vocab + sort_vocab (gensim 3.4.0).

    sample_int = int(round(p * 2**32)), p = min(1, (sqrt(c/thr) + 1) * thr / c),
    thr = sample * retain_total (sample < 1), = retain_total if sample == 0,
    = int(sample * (3 + sqrt(5)) / 2) if sample >= 1.
    """
    retain = [w for w, c in raw_vocab.items() if c >= min_count]
    retain_total = sum(raw_vocab[w] for w in retain)
    if not sample:
        thr = retain_total
    elif sample < 1.0:
        thr = sample * retain_total
    else:
        thr = int(sample * (3 + math.sqrt(5)) / 2)
    sample_int = {}
    for w in retain:
        v = raw_vocab[w]
        p = (math.sqrt(v / thr) + 1) * (thr / v)
        if p >= 1.0:
            p = 1.0
        sample_int[w] = int(round(p * 2 ** 32))
    # sort_vocab: list.sort(key=count, reverse=True) is stable
    index2word = sorted(retain, key=lambda w: raw_vocab[w], reverse=True)
    counts = np.array([raw_vocab[w] for w in index2word], dtype=np.int64)
    sint = np.array([sample_int[w] for w in index2word], dtype=np.uint64)
    return Vocab(index2word=index2word, counts=counts, sample_int=sint,
                 first_order=retain,
                 word2index={w: i for i, w in enumerate(index2word)})


def build_vocab(sentences, min_count=1, sample=1e-3):
    raw, n, total = scan_vocab(sentences)
    voc = prepare_vocab(raw, min_count, sample)
    voc.corpus_count = n
    voc.total_words = total
    return voc


def sample_int_from_counts(counts, sample):
    """Vectorisable restatement of the sample_int formula on an index-ordered
    count array (same arithmetic, same order-independence)."""
    counts = [int(c) for c in counts]
    total = sum(counts)
    if not sample:
        thr = total
    elif sample < 1.0:
        thr = sample * total
    else:
        thr = int(sample * (3 + math.sqrt(5)) / 2)
    out = np.empty(len(counts), dtype=np.uint64)
    for i, v in enumerate(counts):
        p = (math.sqrt(v / thr) + 1) * (thr / v)
        out[i] = int(round(min(p, 1.0) * 2 ** 32))
    return out


# --------------------------------------------------------------------------
# A.3 cum_table ([ext] Word2VecVocab.make_cum_table)
# --------------------------------------------------------------------------
def make_cum_table(counts, power=0.75, domain=DOMAIN):
    """Sequential double accumulation in index order, Python round() (half-even)."""
    counts = [int(c) for c in counts]
    z = 0.0
    for c in counts:
        z += c ** power
    cum = np.zeros(len(counts), dtype=np.uint32)
    acc = 0.0
    for i, c in enumerate(counts):
        acc += c ** power
        cum[i] = round(acc / z * domain)
    if len(cum):
        assert int(cum[-1]) == domain
    return cum


# --------------------------------------------------------------------------
# A.5 sigmoid LUT, LCG, bisect ([ext] word2vec_inner.pyx init(),
# random_int32, bisect_left)
# --------------------------------------------------------------------------
def exp_table():
    i = np.arange(EXP_TABLE_SIZE, dtype=np.float32)
    x = (i / np.float32(EXP_TABLE_SIZE) * np.float32(2) - np.float32(1)) * np.float32(MAX_EXP)
    e = np.exp(x.astype(np.float64)).astype(np.float32)          # C exp(double)
    return (e / (e + np.float32(1))).astype(np.float32)


def log_table():
    """[ext] init(): LOG_TABLE[i] = <REAL_t>log(EXP_TABLE[i]) (C log of the float)."""
    return np.log(exp_table().astype(np.float64)).astype(np.float32)


def lcg_next(nr):
    return (nr * LCG_MUL + LCG_ADD) & LCG_MASK


def random_int32(nr):
    """returns (value, new_state)"""
    return nr >> 16, lcg_next(nr)


def lcg_jump(nr, n):
    """state after n LCG steps (affine power by squaring)."""
    a, c = 1, 0                       # accumulated map x -> a*x + c
    ma, mc = LCG_MUL, LCG_ADD         # map for 2**k steps
    while n:
        if n & 1:
            a, c = (ma * a) & LCG_MASK, (ma * c + mc) & LCG_MASK
        ma, mc = (ma * ma) & LCG_MASK, (ma * mc + mc) & LCG_MASK
        n >>= 1
    return (a * nr + c) & LCG_MASK


def bisect_left(a, x, lo, hi):
    while hi > lo:
        mid = (lo + hi) >> 1
        if a[mid] >= x:
            hi = mid
        else:
            lo = mid + 1
    return lo


def draw_negative(cum, nr):
    """one negative: t = bisect_left(cum, (nr>>16) % cum[-1]); nr advances."""
    t = bisect_left(cum, (nr >> 16) % int(cum[-1]), 0, len(cum))
    return t, lcg_next(nr)


# --------------------------------------------------------------------------
# A.4 weight init ([ext] Word2VecTrainables.reset_weights / seeded_vector)
# --------------------------------------------------------------------------
def seeded_vector(seed_string, size, hashfxn=hash):
    once = np.random.RandomState(hashfxn(seed_string) & 0xffffffff)
    return (once.rand(size) - 0.5) / size


def reset_weights(index2word, size, seed=1, hashfxn=hash):
    syn0 = np.empty((len(index2word), size), dtype=REAL)
    for i, w in enumerate(index2word):
        syn0[i] = seeded_vector(w + str(seed), size, hashfxn)
    syn1neg = np.zeros((len(index2word), size), dtype=REAL)
    lockf = np.ones(len(index2word), dtype=REAL)
    return syn0, syn1neg, lockf


# --------------------------------------------------------------------------
# A.6 job producer / alpha schedule ([ext] BaseAny2VecModel._job_producer,
# _get_job_params, _update_job_params)
# --------------------------------------------------------------------------
def plan_jobs(sentence_lengths, batch_words=10000):
    """Greedy packing: returns list of (first_sentence, end_sentence)."""
    jobs = []
    start, size = 0, 0
    for i, ln in enumerate(sentence_lengths):
        if size + ln <= batch_words:
            size += ln
        else:
            jobs.append((start, i))
            start, size = i, ln
    if len(sentence_lengths) > start:
        jobs.append((start, len(sentence_lengths)))
    return jobs


def job_alphas(jobs, total_examples, alpha=0.025, min_alpha=0.0001, cur_epoch=0, epochs=1):
    """alpha per job as a Python float (double); examples = sentences."""
    out = []
    a = alpha - (alpha - min_alpha) * float(cur_epoch) / epochs
    pushed = 0
    for (s0, s1) in jobs:
        out.append(a)
        pushed += s1 - s0
        progress = (cur_epoch + 1.0 * pushed / total_examples) / epochs
        a = max(min_alpha, alpha - (alpha - min_alpha) * progress)
    return out


def job_seeds(rs: np.random.RandomState, n_jobs):
    """next_random = 2**24 * randint(0, 2**24) + randint(0, 2**24) per job
    (train_batch_sg).  randint(0, window=1, n) draws nothing."""
    out = []
    for _ in range(n_jobs):
        a = int(rs.randint(0, 2 ** 24))
        b = int(rs.randint(0, 2 ** 24))
        out.append((2 ** 24) * a + b)
    return out


# --------------------------------------------------------------------------
# A.5 the kernel ([ext] fast_sentence_sg_neg / train_batch_sg)
# --------------------------------------------------------------------------
def _dot(a, b):
    """dsdot: float32 products accumulated in double, cast to float."""
    return np.float32(np.dot(a.astype(np.float64), b.astype(np.float64)))


def _axpy(g, x, y):
    """y <- g*x + y with a single rounding (FMA, as a modern BLAS saxpy)."""
    y[:] = (np.float64(g) * x.astype(np.float64) + y.astype(np.float64)).astype(np.float32)


def fast_sentence_sg_neg(K, cum, syn0, syn1neg, word_index, word2_index, alpha, nr,
                         lockf, exp_tab, explicit_negs=None, loss=None):
    """One directed example; returns the advanced LCG state.

    If ``explicit_negs`` (length K, -1 = skipped) is given, the LCG/bisect
    draw is replaced by those targets (deterministic step API).  ``loss``
    (compute_loss=True): a one-element float32 array holding the running
    training loss; every applied target subtracts
    LOG_TABLE[int((f_dot + 6) * 83)], f_dot = +f for the positive and -f for a
    negative, in float32 (train_batch_sg's REAL_t _running_training_loss)."""
    alpha = np.float32(alpha)
    l1 = syn0[word2_index]               # view; frozen until the end
    work = np.zeros(syn0.shape[1], dtype=np.float32)
    l1c = l1.copy()
    for d in range(K + 1):
        if d == 0:
            t = word_index
            label = np.float32(1.0)
        else:
            if explicit_negs is None:
                t, nr = draw_negative(cum, nr)
            else:
                t = int(explicit_negs[d - 1])
                if t < 0:
                    continue
            if t == word_index:
                continue
            label = np.float32(0.0)
        row = syn1neg[t]
        f = _dot(l1c, row)
        if f <= -MAX_EXP or f >= MAX_EXP:
            continue
        idx = int((f + np.float32(MAX_EXP)) * np.float32(LUT_SCALE))
        g = (label - exp_tab[idx]) * alpha
        if loss is not None:
            fl = f if d == 0 else -f
            li = int((fl + np.float32(MAX_EXP)) * np.float32(LUT_SCALE))
            loss[0] = np.float32(loss[0] - _LOG_TABLE[li])
        _axpy(g, row, work)
        _axpy(g, l1c, row)
    _axpy(lockf[word2_index], work, syn0[word2_index])
    return nr


_LOG_TABLE = log_table()


def downsample_job(tok_rows, sample_int, nr, sample_on):
    """train_batch_sg pre-pass over one job.

    tok_rows: list of int lists (vocab index, -1 = OOV).  Returns (sentences of
    kept indices, nr after the downsampling draws, effective words)."""
    out = []
    eff = 0
    for sent in tok_rows:
        if len(sent) == 0:
            continue
        cur = []
        for w in sent:
            if w < 0:
                continue
            if sample_on:
                r, nr = random_int32(nr)
                if int(sample_int[w]) < r:
                    continue
            cur.append(w)
            eff += 1
            if eff == MAX_SENTENCE_LEN:
                break
        out.append(cur)
        if eff == MAX_SENTENCE_LEN:
            break
    return out, nr, eff


def job_examples(kept_sents, window=1, reduced_windows=None):
    """(center i, input j) index pairs in gensim loop order."""
    ex = []
    pos = 0
    for sent in kept_sents:
        L = len(sent)
        for i in range(L):
            b = reduced_windows[pos + i] if reduced_windows is not None else 0
            j0 = max(i - window + b, 0)
            j1 = min(i + window + 1 - b, L)
            for j in range(j0, j1):
                if j != i:
                    ex.append((sent[i], sent[j]))
        pos += L
    return ex


def train_job(tok_rows, alpha, seed, vocab_sample_int, sample_on, cum, syn0, syn1neg,
              lockf, K, exp_tab, window=1, loss=None):
    kept, nr, eff = downsample_job(tok_rows, vocab_sample_int, seed, sample_on)
    for c, j in job_examples(kept, window):
        nr = fast_sentence_sg_neg(K, cum, syn0, syn1neg, c, j, alpha, nr, lockf, exp_tab,
                                  loss=loss)
    n_ex = len(job_examples(kept, window))
    return eff, n_ex


def sample_job_records(tok_rows, seed, sample_int, sample_on, cum, K, window=1):
    """The (center, input, negs[K]) records the GPU sampler must reproduce
    bit-exactly (negative == center encoded as -1)."""
    kept, nr, _ = downsample_job(tok_rows, sample_int, seed, sample_on)
    recs = []
    for c, j in job_examples(kept, window):
        negs = []
        for _ in range(K):
            t, nr = draw_negative(cum, nr)
            negs.append(-1 if t == c else t)
        recs.append((c, j, negs))
    return recs


def sentences_to_ids(sentences, word2index):
    return [[word2index.get(w, -1) for w in s] for s in sentences]


def train_epoch_sequential(id_sentences, vocab: Vocab, syn0, syn1neg, lockf, cum, K,
                           rs: np.random.RandomState, alpha=0.025, min_alpha=0.0001,
                           sample=1e-3, total_examples=None, cur_epoch=0, epochs=1,
                           batch_words=10000, window=1, loss=None):
    """One epoch in gensim workers=1 order (jobs in order, seeds in order);
    ``loss`` as in fast_sentence_sg_neg (compute_loss=True)."""
    if window != 1:
        raise NotImplementedError("oracle restates window=1 (src/gene2vec.py:62)")
    total_examples = total_examples or len(id_sentences)
    lengths = [len(s) for s in id_sentences]
    jobs = plan_jobs(lengths, batch_words)
    alphas = job_alphas(jobs, total_examples, alpha, min_alpha, cur_epoch, epochs)
    seeds = job_seeds(rs, len(jobs))
    exp_tab = exp_table()
    sample_on = bool(sample)
    eff_tot = ex_tot = 0
    for (s0, s1), a, sd in zip(jobs, alphas, seeds):
        eff, nex = train_job(id_sentences[s0:s1], a, sd, vocab.sample_int, sample_on,
                             cum, syn0, syn1neg, lockf, K, exp_tab, loss=loss)
        eff_tot += eff
        ex_tot += nex
    return dict(jobs=len(jobs), effective_words=eff_tot, examples=ex_tot,
                raw_words=sum(lengths))


# --------------------------------------------------------------------------
# Deterministic step APIs (explicit negatives)
# --------------------------------------------------------------------------
def sgns_step_sequential(syn0, syn1neg, lockf, center, inp, negs, alpha, loss=None):
    """Examples applied one after another (gensim semantics)."""
    exp_tab = exp_table()
    K = negs.shape[1]
    for e in range(len(center)):
        fast_sentence_sg_neg(K, None, syn0, syn1neg, int(center[e]), int(inp[e]),
                             alpha, 0, lockf, exp_tab, explicit_negs=negs[e], loss=loss)


def sgns_step_minibatch(syn0, syn1neg, lockf, center, inp, negs, alpha):
    """Synchronous minibatch: every example reads the pre-step tables; the
    per-example deltas (same per-example math as fast_sentence_sg_neg,
    sequential within the example) are summed and applied at the end."""
    exp_tab = exp_table()
    K = negs.shape[1]
    s0 = syn0.copy()
    s1 = syn1neg.copy()
    d0 = np.zeros(syn0.shape, dtype=np.float64)
    d1 = np.zeros(syn1neg.shape, dtype=np.float64)
    for e in range(len(center)):
        a0 = s0.copy()
        a1 = s1.copy()
        fast_sentence_sg_neg(K, None, a0, a1, int(center[e]), int(inp[e]), alpha, 0,
                             lockf, exp_tab, explicit_negs=negs[e])
        d0 += a0.astype(np.float64) - s0
        d1 += a1.astype(np.float64) - s1
    syn0[:] = (s0 + d0).astype(np.float32)
    syn1neg[:] = (s1 + d1).astype(np.float32)


# --------------------------------------------------------------------------
# Objective used for end-to-end quality comparisons (not in the reference:
# gensim 3.4 reports no loss with compute_loss=False)
# --------------------------------------------------------------------------
def sgns_loss(syn0, syn1neg, center, inp, negs):
    """mean over examples of -log s(v_c.u_j) - sum_k log s(-v_nk.u_j), float64."""
    u = syn0[inp].astype(np.float64)
    pos = np.einsum("nd,nd->n", u, syn1neg[center].astype(np.float64))
    neg = np.einsum("nd,nkd->nk", u, syn1neg[negs].astype(np.float64))
    lp = -np.logaddexp(0.0, -pos)
    ln = -np.logaddexp(0.0, neg).sum(axis=1)
    return float(-(lp + ln).mean())
