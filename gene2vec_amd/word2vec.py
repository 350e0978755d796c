"""gensim-3.4-shaped ``Word2Vec`` / ``KeyedVectors`` over the MI355X engine.

This is the host-side mirror of the reference interface the hot path sits
behind (src/gene2vec.py:70 ``gensim.models.Word2Vec(gene_pairs, size=200,
window=1, min_count=1, workers=32, iter=1, sg=1)``, :86 ``Word2Vec.load``,
:87 ``model.train(gene_pairs, total_examples=model.corpus_count,
epochs=model.iter)``, :71/:88 ``model.save``; src/generateMatrix.py:7-9
``KeyedVectors.load(f).wv.vocab`` / ``wv[word]``;
src/evaluation_target_function.py:25,38 ``load_word2vec_format`` /
``wv.similarity``).  Names, argument meaning and defaults follow gensim 3.4.0;
configurations the engine does not implement (CBOW, hierarchical softmax,
window != 1) raise ``NotImplementedError`` instead of silently training
something else.

Training runs in libg2v.so on the GPU; there is no CPU fallback.
"""
from __future__ import annotations

import io
import json
import logging
import math
import os
import time
import zipfile
import zlib

import numpy as np

from . import _native as N
from . import distributed as Dd
from . import engine as E

logger = logging.getLogger(__name__)
REAL = np.float32
_FORMAT = "gene2vec_amd/1"


# ---------------------------------------------------------------------------
# vocabulary ([ext] Word2VecVocab.scan_vocab / prepare_vocab / sort_vocab)
# ---------------------------------------------------------------------------
class Vocab:
    """gensim ``Vocab`` entry: count, index, sample_int."""
    __slots__ = ("count", "index", "sample_int")

    def __init__(self, count=0, index=0, sample_int=2 ** 32):
        self.count = count
        self.index = index
        self.sample_int = sample_int

    def __repr__(self):
        return f"Vocab(count={self.count}, index={self.index}, sample_int={self.sample_int})"


def scan_vocab(sentences):
    """raw counts in first-occurrence order, number of sentences, raw words."""
    raw = {}
    total = 0
    n = 0
    for n, sent in enumerate(sentences, 1):
        for w in sent:
            raw[w] = raw.get(w, 0) + 1
        total += len(sent)
    return raw, n, total


def sample_ints(counts, sample):
    """[ext] prepare_vocab sample_int per count (index order), Python ints."""
    total = int(sum(int(c) for c in counts))
    if not sample:
        thr = total
    elif sample < 1.0:
        thr = sample * total
    else:
        thr = int(sample * (3 + math.sqrt(5)) / 2)
    out = []
    for v in counts:
        v = int(v)
        p = (math.sqrt(v / thr) + 1) * (thr / v)
        out.append(int(round(min(p, 1.0) * 2 ** 32)))
    return out


# ---------------------------------------------------------------------------
# KeyedVectors
# ---------------------------------------------------------------------------
class KeyedVectors:
    """``wv``: vectors [V][D] float32 (index order), ``vocab`` dict in
    first-occurrence order (the row order of generateMatrix's .txt),
    ``index2word`` in index (descending count) order."""

    def __init__(self, vector_size):
        self.vector_size = vector_size
        self.vectors = np.zeros((0, vector_size), dtype=REAL)
        self.vocab = {}
        self.index2word = []
        self.vectors_norm = None

    # gensim 3.x: model.wv on a KeyedVectors is the object itself
    @property
    def wv(self):
        return self

    @property
    def syn0(self):
        return self.vectors

    def __len__(self):
        return len(self.index2word)

    def __contains__(self, word):
        return word in self.vocab

    def __getitem__(self, words):
        if isinstance(words, str):
            return self.vectors[self.vocab[words].index]
        return np.vstack([self.vectors[self.vocab[w].index] for w in words])

    def word_vec(self, word, use_norm=False):
        v = self[word]
        if use_norm:
            return v / np.sqrt((v.astype(np.float64) ** 2).sum()).astype(REAL)
        return v

    @staticmethod
    def _unitvec(v):
        v = np.asarray(v, dtype=REAL)
        n = np.sqrt(np.dot(v, v))
        return v / n if n > 0 else v

    def similarity(self, w1, w2):
        """cosine: dot(unitvec(a), unitvec(b)) (src/evaluation_target_function.py:38)"""
        return np.dot(self._unitvec(self[w1]), self._unitvec(self[w2]))

    def init_sims(self):
        v = self.vectors.astype(np.float64)
        n = np.sqrt((v * v).sum(axis=1, keepdims=True))
        n[n == 0] = 1.0
        self.vectors_norm = (v / n).astype(REAL)

    def most_similar(self, positive, topn=10):
        if isinstance(positive, str):
            positive = [positive]
        if self.vectors_norm is None:
            self.init_sims()
        mean = np.mean([self.vectors_norm[self.vocab[w].index] for w in positive], axis=0)
        mean = self._unitvec(mean)
        dists = self.vectors_norm @ mean
        excl = {self.vocab[w].index for w in positive}
        best = np.argsort(-dists)
        out = [(self.index2word[i], float(dists[i])) for i in best if i not in excl]
        return out[:topn]

    # -- word2vec formats ([ext] KeyedVectors.save_word2vec_format, 3.4) ---------
    def save_word2vec_format(self, fname, binary=False, total_vec=None):
        """Header "V D", then rows in descending-count order ([ext] sorted by
        -count over vocab order == index order).  Text rows: word, space, the
        float32 values' shortest repr joined by single spaces.  Binary rows:
        word, space, D little-endian float32 (no newline, as gensim 3.x)."""
        V = len(self.index2word)
        total_vec = V if total_vec is None else total_vec
        order = sorted(self.vocab.items(), key=lambda item: -item[1].count)
        with open(fname, "wb") as f:
            f.write(f"{total_vec} {self.vector_size}\n".encode("utf-8"))
            if binary:
                for word, voc in order:
                    row = self.vectors[voc.index].astype("<f4")
                    f.write(word.encode("utf-8") + b" " + row.tobytes())
            else:
                from . import textio
                f.write(textio.format_rows(self.vectors.astype(REAL, copy=False),
                                           [voc.index for _, voc in order],
                                           [word for word, _ in order], textio.TXT_W2V))

    @classmethod
    def load_word2vec_format(cls, fname, binary=False, encoding="utf8",
                             unicode_errors="strict", limit=None, datatype=REAL):
        with open(fname, "rb") as f:
            header = f.readline().decode(encoding, errors=unicode_errors)
            vocab_size, vector_size = (int(x) for x in header.split())
            if limit:
                vocab_size = min(vocab_size, limit)
            kv = cls(vector_size)
            kv.vectors = np.zeros((vocab_size, vector_size), dtype=datatype)

            def add(word, weights):
                word_id = len(kv.index2word)
                if word in kv.vocab:
                    logger.warning("duplicate word '%s' in %s, ignoring all but first", word,
                                   fname)
                    return
                kv.vocab[word] = Vocab(index=word_id, count=vocab_size - word_id)
                kv.vectors[word_id] = weights
                kv.index2word.append(word)

            if binary:
                binlen = np.dtype(REAL).itemsize * vector_size
                for _ in range(vocab_size):
                    word = []
                    while True:
                        ch = f.read(1)
                        if ch == b" ":
                            break
                        if ch == b"":
                            raise EOFError("unexpected end of input; is count incorrect?")
                        if ch != b"\n":  # word2vec.c writes a newline, gensim 3.x does not
                            word.append(ch)
                    w = b"".join(word).decode(encoding, errors=unicode_errors)
                    add(w, np.frombuffer(f.read(binlen), dtype=REAL))
            else:
                for line_no in range(vocab_size):
                    line = f.readline()
                    if line == b"":
                        raise EOFError("unexpected end of input; is count incorrect?")
                    parts = line.decode(encoding, errors=unicode_errors).rstrip().split(" ")
                    if len(parts) != vector_size + 1:
                        raise ValueError(
                            f"invalid vector on line {line_no} (is this really the text format?)")
                    add(parts[0], [REAL(x) for x in parts[1:]])
        if kv.vectors.shape[0] != len(kv.index2word):
            kv.vectors = np.ascontiguousarray(kv.vectors[:len(kv.index2word)])
        return kv

    # -- own persistence -------------------------------------------------------------
    def save(self, fname):
        _save_npz(fname, {"kind": "KeyedVectors", "vector_size": self.vector_size},
                  _kv_arrays(self))

    @classmethod
    def load(cls, fname, mmap=None):
        """Loads a KeyedVectors or Word2Vec file written by this package; a
        Word2Vec file yields the model itself (as gensim 3.4's SaveLoad does,
        so ``KeyedVectors.load(f).wv`` works -- src/generateMatrix.py:7-8)."""
        meta, arrs = _load_npz(fname)
        if meta["kind"] == "Word2Vec":
            return Word2Vec._from_saved(meta, arrs)
        kv = cls(meta["vector_size"])
        _kv_restore(kv, arrs)
        return kv


def _kv_arrays(kv):
    words = kv.index2word
    first = list(kv.vocab.keys())
    pos = {w: i for i, w in enumerate(words)}
    return {
        "vectors": np.ascontiguousarray(kv.vectors, dtype=REAL),
        "index2word": np.array(words, dtype=str) if words else np.zeros(0, dtype="<U1"),
        "first_order": np.array([pos[w] for w in first], dtype=np.int64),
        "counts": np.array([kv.vocab[w].count for w in words], dtype=np.int64),
        "sample_int": np.array([kv.vocab[w].sample_int for w in words], dtype=np.uint64),
    }


def _kv_restore(kv, arrs):
    words = [str(w) for w in arrs["index2word"]]
    counts = arrs["counts"]
    si = arrs["sample_int"]
    kv.index2word = words
    kv.vectors = np.ascontiguousarray(arrs["vectors"], dtype=REAL)
    kv.vocab = {}
    for i in arrs["first_order"]:
        i = int(i)
        kv.vocab[words[i]] = Vocab(count=int(counts[i]), index=i, sample_int=int(si[i]))


def _save_npz(fname, meta, arrays):
    """One file at exactly ``fname`` (gensim's model.save(fname) contract):
    a zip of .npy members + meta.json; readable without unpickling."""
    tmp = fname + ".tmp"
    with zipfile.ZipFile(tmp, "w", compression=zipfile.ZIP_STORED) as z:
        z.writestr("meta.json", json.dumps(dict(meta, format=_FORMAT)))
        for k, v in arrays.items():
            buf = io.BytesIO()
            np.save(buf, v, allow_pickle=False)
            z.writestr(k + ".npy", buf.getvalue())
    os.replace(tmp, fname)


def _load_npz(fname):
    with zipfile.ZipFile(fname, "r") as z:
        meta = json.loads(z.read("meta.json"))
        if meta.get("format") != _FORMAT:
            raise ValueError(f"{fname}: not a gene2vec_amd file")
        arrs = {}
        for name in z.namelist():
            if name.endswith(".npy"):
                arrs[name[:-4]] = np.load(io.BytesIO(z.read(name)), allow_pickle=False)
    return meta, arrs


# ---------------------------------------------------------------------------
# Word2Vec
# ---------------------------------------------------------------------------
# replica merge cadence for data-parallel training (gensim jobs per rank): the
# largest that kept 8 replicas within 1 % of one model on every measured metric
# at C3's size (SGNS objective held-in / held-out, GGIPNN AUC, target function;
# DESIGN.md section 7a, profiles/r03/replica_quality_c3*.json)
DP_MERGE_EVERY_JOBS = 3584
# merge transport under torch.distributed: "auto" = libg2v over RCCL for nccl,
# libg2v over the host collective for gloo; "torch" = torch-owned tables merged
# by torch.distributed (the CLI's --merge-transport)
DP_MERGE_TRANSPORT = "auto"
# merge rule of data-parallel training (the CLI picks it by shard size:
# distributed.dp_merge_plan)
DP_MERGE_RULE = "touch"
# touch divisor shape k^beta of the merges (distributed.dp_merge_beta: 1 but
# at 2 ranks, where the damped divisor keeps the merged model on one model's
# target function; G2V_OPT_MERGE_BETA_MILLI)
DP_MERGE_BETA = 1.0


def crc32_hash(s):
    """deterministic seeded_vector hash (the CLI's --hash crc32)"""
    return zlib.crc32(s.encode("utf-8"))


# hashfxn <-> name in the checkpoint (gensim pickles the function itself)
_HASH_NAMES = {"python": hash, "crc32": crc32_hash}


def _hash_name(fn):
    for k, v in _HASH_NAMES.items():
        if fn is v:
            return k
    return "custom"


class Word2Vec:
    """Skip-gram negative-sampling Word2Vec trained on an MI355X.

    gensim 3.4.0 signature; the reference calls it with size=200, window=1,
    min_count=1, workers=32, iter=1, sg=1 (src/gene2vec.py:70).  ``workers``
    is accepted for compatibility (the GPU kernel replaces the thread pool).
    Extra keyword ``device`` picks the GPU; ``mode`` = "hogwild" (default,
    all SGNS updates as memory-side atomics) or "sequential" (one wave,
    gensim workers=1 order, for parity checks); ``data_parallel`` = True
    shards the corpus over an initialised torch.distributed group and merges
    the replicas (opt-in: the gene2vec CLI sets it under torchrun; a model
    trained inside some unrelated process group stays single-GPU); ``grid``
    fixes the Hogwild kernel's workgroups (G2V_OPT_GRID; 0 = the library's
    staleness-bounded default with its per-call stability cap).
    ``compute_loss`` follows gensim 3.4: the running loss of the latest
    train() call, ``get_latest_training_loss()``."""

    def __init__(self, sentences=None, size=100, alpha=0.025, window=5, min_count=5,
                 max_vocab_size=None, sample=1e-3, seed=1, workers=3, min_alpha=0.0001,
                 sg=0, hs=0, negative=5, cbow_mean=1, hashfxn=hash, iter=5, null_word=0,
                 trim_rule=None, sorted_vocab=1, batch_words=N.BATCH_WORDS, compute_loss=False,
                 callbacks=(), ns_exponent=0.75, device=0, mode="hogwild", data_parallel=False,
                 grid=0):
        if sg != 1:
            raise NotImplementedError("only skip-gram (sg=1) is implemented (src/gene2vec.py:60)")
        if hs:
            raise NotImplementedError("hierarchical softmax (hs=1) is not implemented")
        if negative not in N.SUPPORTED_NEGATIVE:
            raise NotImplementedError(f"negative={negative}: compiled {N.SUPPORTED_NEGATIVE}")
        if window != 1:
            raise NotImplementedError("only window=1 is implemented (src/gene2vec.py:62)")
        if batch_words != N.BATCH_WORDS:
            raise NotImplementedError("batch_words is fixed at 10000 (gensim MAX_WORDS_IN_BATCH)")
        if not 1 <= size <= N.MAX_DIM:
            raise NotImplementedError(f"size must be in [1, {N.MAX_DIM}]")
        if max_vocab_size is not None or trim_rule is not None or not sorted_vocab:
            raise NotImplementedError("max_vocab_size / trim_rule / sorted_vocab=0 unsupported")
        self.vector_size = size
        self.alpha = float(alpha)
        self.min_alpha = float(min_alpha)
        self.min_alpha_yet_reached = float(alpha)
        self.window = window
        self.min_count = min_count
        self.sample = sample
        self.seed = seed
        self.workers = workers
        self.sg = sg
        self.hs = hs
        self.negative = negative
        self.ns_exponent = ns_exponent
        self.hashfxn = hashfxn
        self.iter = iter
        self.epochs = iter
        self.batch_words = batch_words
        self.compute_loss = compute_loss
        self.callbacks = callbacks
        self.device = device
        self.mode = mode
        self.data_parallel = data_parallel
        self.grid = int(grid)
        self.merge_every_jobs = DP_MERGE_EVERY_JOBS
        self.merge_rule = DP_MERGE_RULE
        self.merge_beta = DP_MERGE_BETA
        self.random = np.random.RandomState(seed)
        self.corpus_count = 0
        self.corpus_total_words = 0
        self.train_count = 0
        self.total_train_time = 0.0
        self.running_training_loss = 0.0
        self.wv = KeyedVectors(size)
        self.syn1neg = None
        self.vectors_lockf = None
        self.cum_table = None
        self.last_stats = None
        self._engine = None
        self._replica = None
        self._dev_dirty = False  # device tables newer than host copies
        if sentences is not None:
            self.build_vocab(sentences)
            self.train(sentences, total_examples=self.corpus_count, epochs=self.iter,
                       start_alpha=self.alpha, end_alpha=self.min_alpha,
                       compute_loss=compute_loss)

    # -- vocabulary ----------------------------------------------------------------
    def build_vocab(self, sentences, update=False, progress_per=10000, keep_raw_vocab=False,
                    trim_rule=None):
        if update:
            raise NotImplementedError("online vocabulary update is not implemented")
        raw, n, total = scan_vocab(sentences)
        self.corpus_count = n
        self.corpus_total_words = total
        self._build_from_counts(raw)

    def build_vocab_from_freq(self, word_freq):
        self._build_from_counts(dict(word_freq))

    def _build_from_counts(self, raw):
        retain = [w for w, c in raw.items() if c >= self.min_count]
        if not retain:
            raise RuntimeError("you must first build vocabulary before training the model")
        index2word = sorted(retain, key=lambda w: raw[w], reverse=True)  # stable
        counts = [raw[w] for w in index2word]
        si = sample_ints(counts, self.sample)
        wv = self.wv
        wv.index2word = index2word
        pos = {w: i for i, w in enumerate(index2word)}
        wv.vocab = {w: Vocab(count=raw[w], index=pos[w], sample_int=si[pos[w]]) for w in retain}
        self._reset_weights()

    def _reset_weights(self):
        """[ext] Word2VecTrainables.reset_weights: syn0 row i =
        seeded_vector(index2word[i] + str(seed)), syn1neg = 0, lockf = 1."""
        wv = self.wv
        seeds = np.array([self.hashfxn(w + str(self.seed)) & 0xFFFFFFFF for w in wv.index2word],
                         dtype=np.uint32)
        wv.vectors = E.seeded_vectors(seeds, self.vector_size)
        wv.vectors_norm = None
        self.syn1neg = np.zeros_like(wv.vectors)
        self.vectors_lockf = np.ones(len(wv.index2word), dtype=REAL)
        self._close_engine()

    # -- engine -----------------------------------------------------------------------
    def _close_engine(self):
        if self._engine is not None:
            self._engine.close()
        self._engine = None
        self._replica = None
        self._dev_dirty = False

    def _dp_world(self):
        """(rank, world) of the initialised torch.distributed group when this
        model trains data-parallel (opt-in), else (0, 1)."""
        if not getattr(self, "data_parallel", False):
            return 0, 1
        try:
            import torch.distributed as dist
        except ImportError:  # pragma: no cover
            return 0, 1
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            return dist.get_rank(), dist.get_world_size()
        return 0, 1

    def _bind_replica(self, eng):
        """Data-parallel replica (no reference equivalent: gensim is one process,
        src/gene2vec.py:59).  Backend "nccl": libg2v joins an RCCL communicator
        (unique id broadcast over the process group), takes rank 0's tables
        (Python's hash() seeds the init differently in every process) and
        merges the replicas itself every ``merge_every_jobs`` jobs (fused HIP
        kernels + ncclAllReduce over xGMI).  Backend "gloo" (ranks sharing one
        GPU, which RCCL refuses): the same libg2v merge with its all-reduce
        carried by gloo through the host (g2v_comm_init_host); with
        ``DP_MERGE_TRANSPORT = "torch"``, torch-owned tables merged by
        torch.distributed."""
        import torch
        import torch.distributed as dist
        mode = N.MODE_SEQUENTIAL if self.mode == "sequential" else N.MODE_HOGWILD
        rank, world = dist.get_rank(), dist.get_world_size()
        beta = float(getattr(self, "merge_beta", 1.0))
        if beta != 1.0:
            eng.set_option(N.OPT_MERGE_BETA_MILLI, int(round(beta * 1000)))
        transport = DP_MERGE_TRANSPORT
        if transport == "auto":
            transport = "rccl" if dist.get_backend() == "nccl" else "host"
        if transport == "rccl":
            box = [eng.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            eng.comm_init(box[0], world, rank)
            self._replica = Dd.ReplicaTrainer(eng, (), self.merge_every_jobs, mode,
                                              merge=self.merge_rule, backend="libg2v")
            return
        if transport == "host":
            eng.comm_init_host(Dd.host_collective(), world, rank)
            self._replica = Dd.ReplicaTrainer(eng, (), self.merge_every_jobs, mode,
                                              merge=self.merge_rule, backend="libg2v")
            return
        if transport != "torch":
            raise ValueError(f"merge transport {transport!r}")
        dev = torch.device("cuda", self.device)
        # engine launches, merges and collectives ordered on one non-default stream
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        eng.set_stream(stream.cuda_stream)
        V, D = len(self.wv.index2word), self.vector_size
        tables = torch.zeros((2, V, eng.ld), dtype=torch.float32, device=dev)
        tables[0, :, :D] = torch.from_numpy(np.ascontiguousarray(self.wv.vectors)).to(dev)
        tables[1, :, :D] = torch.from_numpy(np.ascontiguousarray(self.syn1neg)).to(dev)
        dist.broadcast(tables, src=0)
        eng.bind_tables(tables[0].data_ptr(), tables[1].data_ptr(), eng.ld, keepalive=(tables,))
        self._replica = Dd.ReplicaTrainer(eng, (tables,), self.merge_every_jobs, mode,
                                          merge=self.merge_rule, backend="torch", beta=beta)

    def _ensure_engine(self):
        if self._engine is not None:
            return self._engine
        wv = self.wv
        eng = E.SGNSEngine(len(wv.index2word), self.vector_size, self.negative, self.window,
                           device=self.device)
        counts = np.array([wv.vocab[w].count for w in wv.index2word], dtype=np.int64)
        cum, si = eng.set_vocab(counts, self.sample, self.ns_exponent, return_tables=True)
        self.cum_table = cum
        expect = np.minimum(np.array([wv.vocab[w].sample_int for w in wv.index2word],
                                     dtype=np.uint64), 2 ** 32 - 1).astype(np.uint32)
        if not np.array_equal(si, expect):
            raise RuntimeError("device sample_int differs from the host vocabulary")
        if getattr(self, "grid", 0):
            eng.set_option(N.OPT_GRID, self.grid)
        eng.set_weights(wv.vectors, self.syn1neg, self.vectors_lockf)
        self._replica = None
        if self._dp_world()[1] > 1:
            self._bind_replica(eng)
        self._engine = eng
        return eng

    def _sync_host(self):
        if self._engine is not None and self._dev_dirty:
            self.wv.vectors, self.syn1neg = self._engine.get_weights()
            self.wv.vectors_norm = None
            self._dev_dirty = False

    # -- training ------------------------------------------------------------------------
    def _corpus_ids(self, sentences):
        w2i = {w: v.index for w, v in self.wv.vocab.items()}
        lengths = []
        toks = []
        for s in sentences:
            lengths.append(len(s))
            toks.extend(w2i.get(w, -1) for w in s)
        tok = np.array(toks, dtype=np.int32)
        off = np.zeros(len(lengths) + 1, dtype=np.int64)
        np.cumsum(lengths, out=off[1:])
        return tok, off

    def train(self, sentences, total_examples=None, total_words=None, epochs=None,
              start_alpha=None, end_alpha=None, word_count=0, queue_factor=2, report_delay=1.0,
              compute_loss=False, callbacks=()):
        """[ext] BaseWordEmbeddingsModel.train: one job schedule per epoch,
        alpha restarting at start_alpha each call (the sawtooth of
        src/gene2vec.py:67-92)."""
        if not self.wv.vocab:
            raise RuntimeError("you must first build vocabulary before training the model")
        if epochs is None:
            raise ValueError("You must specify an explicit epochs count.")
        if total_examples is None and total_words is None:
            raise ValueError("You must specify either total_examples or total_words")
        tok, off = self._corpus_ids(sentences)
        return self.train_ids(tok, off, total_examples=total_examples, total_words=total_words,
                              epochs=epochs, start_alpha=start_alpha, end_alpha=end_alpha,
                              compute_loss=compute_loss)

    def train_ids(self, tokens, sent_off=None, sent_len=0, total_examples=None,
                  total_words=None, epochs=1, start_alpha=None, end_alpha=None,
                  compute_loss=False, device_tokens=None):
        """Fast path: pre-tokenised corpus (int32 vocabulary indices, -1 = OOV)
        as CSR sentence offsets or fixed-length sentences (pairs: sent_len=2).

        ``device_tokens = (ptr, n_tokens, keepalive)``: the pairs already sit
        in this GPU's memory (``tokens`` is then ignored, sent_len must be 2)
        and, under data parallelism, are already this rank's shard (the CLI's
        ``--shuffle device`` gathers each rank's shard of the reshuffled order
        on the device, g2v_permute_items8)."""
        self.alpha = float(start_alpha or self.alpha)
        self.min_alpha = float(end_alpha or self.min_alpha)
        self.epochs = epochs
        # [ext] BaseWordEmbeddingsModel.train: compute_loss is per call and the
        # running loss restarts at 0.0 every train()
        self.compute_loss = bool(compute_loss)
        self.running_training_loss = 0.0
        eng = self._ensure_engine()
        eng.reset_loss()
        rank, world = self._dp_world()
        if device_tokens is not None:
            if sent_len != 2:
                raise ValueError("device_tokens carry fixed-length pairs (sent_len=2)")
            if world > 1:
                total_examples, total_words = device_tokens[1] // 2, None
        elif world > 1:
            # contiguous shard of the (shuffled) sentences per rank; alpha follows
            # the shard's own progress, which is the global progress (all ranks
            # advance together)
            n_all = len(tokens) // sent_len if sent_len > 0 else len(sent_off) - 1
            s0, s1 = Dd.shard_range(n_all, rank, world)
            if sent_len > 0:
                tokens = tokens[s0 * sent_len:s1 * sent_len]
            else:
                so = np.asarray(sent_off, dtype=np.int64)
                tokens = tokens[so[s0]:so[s1]]
                sent_off = so[s0:s1 + 1] - so[s0]
            total_examples, total_words = s1 - s0, None
        if device_tokens is not None:
            ptr, n_tok, keep = device_tokens
            n_sent = n_tok // 2
            eng.set_corpus_device(ptr, n_tok, sent_len=2, keepalive=keep)
            js = E.plan_jobs(n_sent=n_sent, sent_len=2)
            lengths_total = n_tok
        elif sent_len > 0:
            n_sent = len(tokens) // sent_len
            eng.set_corpus(tokens, sent_len=sent_len)
            js = E.plan_jobs(n_sent=n_sent, sent_len=sent_len)
            lengths_total = len(tokens)
        else:
            n_sent = len(sent_off) - 1
            eng.set_corpus(tokens, sent_off=sent_off)
            js = E.plan_jobs(sent_off=sent_off)
            lengths_total = int(sent_off[-1])
        if total_examples is None:
            # words-based decay ([ext] _job_producer with total_words)
            total = total_words
            pushed = np.zeros(len(js) - 1)
            if sent_len > 0:
                pushed = (js[:-1] - js[0]) * sent_len
            else:
                pushed = (np.asarray(sent_off)[js[:-1]] - sent_off[js[0]]).astype(np.float64)
        mode = N.MODE_SEQUENTIAL if self.mode == "sequential" else N.MODE_HOGWILD
        t0 = time.time()
        stats = []
        for cur_epoch in range(epochs):
            if total_examples is not None:
                al = E.job_alphas(js, total_examples, self.alpha, self.min_alpha, cur_epoch,
                                  epochs)
            else:
                al = np.empty(len(js) - 1)
                al[0] = self.alpha - (self.alpha - self.min_alpha) * cur_epoch / epochs
                prog = (cur_epoch + pushed[1:] / total) / epochs
                al[1:] = np.maximum(self.min_alpha,
                                    self.alpha - (self.alpha - self.min_alpha) * prog)
            if world > 1:
                # every rank draws the same base from model.random (kept in step
                # across ranks), then a stream of its own
                base = int(self.random.randint(0, 2 ** 31 - 1))
                seeds = E.job_seeds(np.random.RandomState((base + 7919 * rank) % 2 ** 32),
                                    len(js) - 1)
                self._replica.train_epoch(js, al, seeds, compute_loss=self.compute_loss)
            else:
                seeds = E.job_seeds(self.random, len(js) - 1)
                eng.train(js, al, seeds, mode, compute_loss=self.compute_loss)
            st = eng.read_stats()
            stats.append(st)
            if len(al):
                self.min_alpha_yet_reached = float(al[-1])
            logger.info("EPOCH %d: trained %d raw words (%d effective words, %d examples)",
                        cur_epoch + 1, st["raw_words"], st["effective_words"], st["examples"])
        self._dev_dirty = True
        self._sync_host()
        if self.compute_loss and stats:
            loss = stats[-1]["training_loss"]  # running since the reset above
            # data parallel: the loss over every rank's shard
            self.running_training_loss = Dd.allreduce_sum_float(loss) if world > 1 else loss
        elapsed = time.time() - t0
        self.total_train_time += elapsed
        self.train_count += 1
        eff = sum(s["effective_words"] for s in stats)
        raw = sum(s["raw_words"] for s in stats)
        self.last_stats = {"raw_words": raw, "effective_words": eff,
                           "examples": sum(s["examples"] for s in stats),
                           "jobs": sum(s["jobs"] for s in stats), "seconds": elapsed,
                           "corpus_words": lengths_total}
        logger.info("training on %d raw words (%d effective words) took %.1fs, %.0f effective "
                    "words/s", raw, eff, elapsed, eff / max(elapsed, 1e-9))
        return eff, raw

    def get_latest_training_loss(self):
        """[ext] Word2Vec.get_latest_training_loss: the running loss of the
        latest train() call with compute_loss=True (0.0 otherwise)."""
        return self.running_training_loss

    # -- persistence --------------------------------------------------------------------------
    def save(self, fname):
        """Own checkpoint (replaces gensim's pickle; src/gene2vec.py:71,88): tables,
        vocabulary, counts, cum_table, RNG state, hyper-parameters."""
        self._sync_host()
        st = self.random.get_state()
        meta = {"kind": "Word2Vec", "vector_size": self.vector_size, "alpha": self.alpha,
                "min_alpha": self.min_alpha, "window": self.window, "min_count": self.min_count,
                "sample": self.sample, "seed": self.seed, "workers": self.workers, "sg": self.sg,
                "hs": self.hs, "negative": self.negative, "ns_exponent": self.ns_exponent,
                "iter": self.iter, "epochs": self.epochs, "batch_words": self.batch_words,
                "corpus_count": self.corpus_count, "corpus_total_words": self.corpus_total_words,
                "train_count": self.train_count, "mode": self.mode,
                "hashfxn": _hash_name(self.hashfxn),
                "running_training_loss": float(self.running_training_loss),
                "min_alpha_yet_reached": self.min_alpha_yet_reached,
                "rng_pos": int(st[2]), "rng_has_gauss": int(st[3]),
                "rng_cached_gaussian": float(st[4])}
        arrs = _kv_arrays(self.wv)
        arrs["syn1neg"] = np.ascontiguousarray(self.syn1neg, dtype=REAL)
        arrs["vectors_lockf"] = np.ascontiguousarray(self.vectors_lockf, dtype=REAL)
        arrs["rng_keys"] = np.asarray(st[1], dtype=np.uint32)
        if self.cum_table is not None:
            arrs["cum_table"] = self.cum_table
        _save_npz(fname, meta, arrs)

    @classmethod
    def load(cls, fname, device=None, **kw):
        meta, arrs = _load_npz(fname)
        if meta["kind"] != "Word2Vec":
            raise ValueError(f"{fname} holds {meta['kind']}, not Word2Vec")
        m = cls._from_saved(meta, arrs)
        if device is not None:
            m.device = device
        return m

    @classmethod
    def _from_saved(cls, meta, arrs):
        m = cls.__new__(cls)
        m.vector_size = meta["vector_size"]
        for k in ("alpha", "min_alpha", "window", "min_count", "sample", "seed", "workers", "sg",
                  "hs", "negative", "ns_exponent", "iter", "epochs", "batch_words",
                  "corpus_count", "corpus_total_words", "train_count", "mode",
                  "min_alpha_yet_reached"):
            setattr(m, k, meta[k])
        name = meta.get("hashfxn", "python")
        if name not in _HASH_NAMES:
            logger.warning("model was trained with a custom hashfxn; reloading with hash()")
        m.hashfxn = _HASH_NAMES.get(name, hash)
        m.compute_loss = False
        m.callbacks = ()
        m.device = 0
        m.data_parallel = False
        m.grid = 0
        m.merge_every_jobs = DP_MERGE_EVERY_JOBS
        m.merge_rule = DP_MERGE_RULE
        m.merge_beta = DP_MERGE_BETA
        m.total_train_time = 0.0
        m.running_training_loss = float(meta.get("running_training_loss", 0.0))
        m.random = np.random.RandomState()
        m.random.set_state(("MT19937", arrs["rng_keys"], meta["rng_pos"], meta["rng_has_gauss"],
                            meta["rng_cached_gaussian"]))
        m.wv = KeyedVectors(m.vector_size)
        _kv_restore(m.wv, arrs)
        m.syn1neg = np.ascontiguousarray(arrs["syn1neg"], dtype=REAL)
        m.vectors_lockf = np.ascontiguousarray(arrs["vectors_lockf"], dtype=REAL)
        m.cum_table = arrs.get("cum_table")
        m.last_stats = None
        m._engine = None
        m._replica = None
        m._dev_dirty = False
        return m

    def __getitem__(self, word):
        return self.wv[word]

    def __contains__(self, word):
        return word in self.wv

    def __del__(self):  # pragma: no cover
        try:
            self._close_engine()
        except Exception:
            pass
