"""CLI mirror of the reference's src/gene2vec.py.

    python -m gene2vec_amd.gene2vec <data_dir> <export_dir> <ending_pattern> [options]

Same positional arguments (src/gene2vec.py:8-15), same ingest (shuffled
listdir, files ending with the pattern, windows-1252, line.strip().split(),
one global shuffle; :29-55), same hyper-parameters (dim 200, 32 workers,
skip-gram, 10 iterations, window 1; :57-63) and the same 10-iteration loop:
iteration 1 builds the model with iter=1 (:70), iterations >= 2 reshuffle,
reload the previous iteration's file and train one more epoch with alpha
restarting at 0.025 (:76-92).  Every iteration writes
``gene2vec_dim_<dim>_iter_<n>`` (own checkpoint format, replacing gensim's
pickle), ``..._iter_<n>.txt`` (generateMatrix) and ``..._iter_<n>_w2v.txt``
(word2vec text format read by evaluation_target_function.py).  Training runs
on the GPU through libg2v.so.
"""
from __future__ import annotations

import argparse
import contextlib
import copy
import datetime
import json
import logging
import os
import random
import sys
import time

import numpy as np

from . import engine as E
from . import generateMatrix as gM
from . import ingest
from .word2vec import Word2Vec


def read_gene_pairs(source_dir, ending_pattern, rng=random):
    """src/gene2vec.py:29-47: shuffled file order, windows-1252, strip().split()."""
    files = os.listdir(source_dir)
    size = len(files)
    rng.shuffle(files)
    gene_pairs = []
    num_db = 0
    for fname in files:
        if not fname.endswith(ending_pattern):
            continue
        num_db += 1
        print(datetime.datetime.now())
        print("current file " + fname + " num: " + str(num_db) + " total files " + str(size))
        with open(os.path.join(source_dir, fname), "r", encoding="windows-1252") as f:
            for line in f:
                gene_pairs.append(line.strip().split())
    return gene_pairs


def _hashfxn(name):
    from .word2vec import crc32_hash
    if name == "python":
        return hash
    if name == "crc32":
        return crc32_hash
    raise ValueError(name)


def _vocab_ids(model, corpus):
    """corpus word id -> model vocabulary index (-1 when not in the vocabulary)"""
    import numpy as np
    voc = model.wv.vocab
    return np.array([voc[w].index if w in voc else -1 for w in corpus.words] or [0],
                    dtype=np.int32)


def _adopt_vocab_ids(corpus, ids, tok):
    """Renumber the corpus in the model's vocabulary order once (iteration 1),
    when every corpus word is in the vocabulary (min_count = 1): the reloaded
    model of iterations >= 2 keeps that vocabulary (src/gene2vec.py:86), so the
    per-iteration 200 M-token remap becomes an O(V) identity check."""
    import numpy as np
    if len(ids) != len(corpus.words) or (ids < 0).any():
        return
    if len(np.unique(ids)) != len(ids):
        return
    words = [None] * len(ids)
    for i, w in enumerate(corpus.words):
        words[ids[i]] = w
    counts = np.empty_like(corpus.counts)
    counts[ids] = corpus.counts
    corpus.tokens, corpus.words, corpus.counts = tok, words, counts


def _sentences(corpus, pairs_only):
    """train_ids' sentence layout: (None, 2) for an all-pairs corpus (same jobs
    and sampled stream as its CSR form), else the CSR offsets"""
    return (None, 2) if pairs_only else (corpus.sent_off, 0)


def _device_raw_counts(corpus, seed, device):
    """{word: count} in first-occurrence order of the corpus as
    g2v_permute_items8(seed) orders it ([ext] scan_vocab after the first
    shuffle, src/gene2vec.py:52), scanned on the GPU without materialising
    that order (g2v_first_occurrence_perm8)"""
    import torch
    dev = torch.device("cuda", device)
    raw = torch.from_numpy(np.ascontiguousarray(corpus.tokens).view(np.int64)).to(dev)
    first = torch.empty(len(corpus.words), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)
    E.first_occurrence_perm8(device, raw.data_ptr(), raw.numel(), seed, len(corpus.words),
                             first.data_ptr(), st.cuda_stream)
    f = first.cpu().numpy()
    del raw
    present = np.nonzero(f >= 0)[0]
    fo = present[np.argsort(f[present], kind="stable")]
    return {corpus.words[i]: int(corpus.counts[i]) for i in fo}


class _DeviceOrder:
    """``--shuffle device``: the pair corpus stays in HBM in file order, and
    every shuffle of the reference -- the first (src/gene2vec.py:52) and the
    reshuffle before each later iteration (:80), unseeded random.shuffle
    calls, so any uniform permutation is as faithful -- is a keyed permutation
    of it evaluated on the GPU, each data-parallel rank gathering only its own
    shard (g2v_permute_items8).  Replaces a serial host Fisher-Yates over the
    whole corpus per iteration on every rank and the per-iteration
    host-to-device copy of the tokens."""

    def __init__(self, tok, ids, device, rank, world):
        import torch
        from . import distributed as Dd
        self.torch = torch
        self.device = device
        self.dev = torch.device("cuda", device)
        self.ids = ids
        flat = np.ascontiguousarray(tok, dtype=np.int32)
        self.base = torch.from_numpy(flat.view(np.int64)).to(self.dev)  # one pair per item
        self.n = self.base.numel()
        self.s0, self.s1 = Dd.shard_range(self.n, rank, world)
        self.buf = None

    def shard(self, seed):
        """(ptr, n_tokens, keepalive) of this rank's pairs in the order of
        permutation `seed`"""
        torch = self.torch
        if self.buf is None:
            self.buf = torch.empty(self.s1 - self.s0, dtype=torch.int64, device=self.dev)
        st = torch.cuda.current_stream(self.dev)
        E.permute_items8(self.device, self.base.data_ptr(), self.buf.data_ptr(), self.n, self.s0,
                         self.s1 - self.s0, seed, st.cuda_stream)
        st.synchronize()  # the engine reads it on its own stream
        return self.buf.data_ptr(), 2 * self.buf.numel(), self.buf


class _Exporter:
    """per-iteration text exports on one background thread (src/gene2vec.py:89
    generateMatrix + the _w2v.txt the target function reads); a failure is
    raised at the next submit or at close()"""

    def __init__(self, txt, w2v, w2v_binary):
        from concurrent.futures import ThreadPoolExecutor
        self.txt, self.w2v, self.w2v_binary = txt, w2v, w2v_binary
        self.pool = ThreadPoolExecutor(max_workers=1)
        self.pending = None

    def _run(self, name, wv, ph):
        with ph("txt"):
            if self.txt:
                gM.outputTxt(name)
        with ph("w2v"):
            if self.w2v:
                wv.save_word2vec_format(name + "_w2v.txt", binary=False)
                if self.w2v_binary:
                    wv.save_word2vec_format(name + "_w2v.bin", binary=True)

    def submit(self, name, wv, ph):
        if self.pending is not None:
            self.pending.result()
        self.pending = self.pool.submit(self._run, name, wv, ph)

    def close(self):
        try:
            if self.pending is not None:
                self.pending.result()
        finally:
            self.pending = None
            self.pool.shutdown(wait=True)


class _Phases:
    """wall seconds per CLI phase, summed over iterations (``--timing``)"""

    def __init__(self):
        self.t = {}

    @contextlib.contextmanager
    def __call__(self, name):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.t[name] = self.t.get(name, 0.0) + time.perf_counter() - t0


def main(argv=None):
    parser = argparse.ArgumentParser(
        description="Please specify data directory, embedding output directory and data file "
                    "ending pattern")
    parser.add_argument("fileAddress", metavar="N", type=str, nargs="+",
                        help="python -m gene2vec_amd.gene2vec data_directory output_directory txt")
    parser.add_argument("--dim", type=int, default=200)
    parser.add_argument("--workers", type=int, default=32)
    parser.add_argument("--iters", type=int, default=10)
    parser.add_argument("--window", type=int, default=1)
    parser.add_argument("--negative", type=int, default=5)
    parser.add_argument("--sample", type=float, default=1e-3)
    parser.add_argument("--device", type=int, default=0)
    parser.add_argument("--mode", choices=("hogwild", "sequential"), default="hogwild")
    parser.add_argument("--grid", type=int, default=0,
                        help="Hogwild SGNS workgroups (G2V_OPT_GRID); 0 = the library's "
                             "staleness-bounded default with its per-call stability cap")
    parser.add_argument("--shuffle-seed", type=int, default=None,
                        help="seed Python's shuffles (the reference leaves them unseeded)")
    parser.add_argument("--hash", choices=("python", "crc32"), default="python",
                        help="seeded_vector hash (gensim default: Python's randomised hash)")
    parser.add_argument("--native-ingest", action="store_true",
                        help="multi-threaded C++ reader + bit-compatible native shuffles "
                             "(same result as the Python ingest for the same seed)")
    parser.add_argument("--no-txt", action="store_true")
    parser.add_argument("--no-w2v", action="store_true")
    parser.add_argument("--w2v-binary", action="store_true")
    parser.add_argument("--timing", default=None,
                        help="write wall seconds per phase (summed over iterations) as JSON")
    parser.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                        help="data-parallel process group under torchrun (nccl = RCCL over "
                             "xGMI; gloo only to rehearse with ranks sharing a GPU)")
    parser.add_argument("--reload-checkpoints", action="store_true",
                        help="load every iteration's model back from the checkpoint just "
                             "written, as src/gene2vec.py:86 does (the kept in-memory model "
                             "is the same state: tables, vocabulary and RNG round-trip exactly)")
    parser.add_argument("--merge-every-jobs", type=int, default=None,
                        help="data-parallel replica merge cadence (gensim jobs per rank); "
                             "default: the plan's -- once per epoch up to 4 ranks; beyond, "
                             "round(750 M / pairs per rank) merges per epoch from 150 M pairs per "
                             "rank, every 3,584 jobs from 125 M (DESIGN.md 7a)")
    parser.add_argument("--merge-rule", choices=("auto", "touch", "align", "mean"),
                        default="auto",
                        help="data-parallel replica merge rule: auto = touch once per epoch "
                             "up to 4 ranks; beyond, from 150 M pairs per rank touch at "
                             "round(750 M / pairs per rank) merges per epoch, from 125 M every "
                             "--merge-every-jobs jobs, from 80 M at 7 merges per epoch, align at 7 "
                             "merges per epoch below (below 150 M only with "
                             "--dp-min-pairs-per-rank; DESIGN.md 7a/7b); an explicit rule uses "
                             "--merge-every-jobs (default 3,584)")
    parser.add_argument("--merge-transport", choices=("auto", "rccl", "host", "torch"),
                        default="auto",
                        help="data-parallel merge: libg2v over RCCL (nccl) or over the host "
                             "collective (gloo) = auto; torch = torch-owned tables merged by "
                             "torch.distributed")
    parser.add_argument("--dp-min-pairs-per-rank", type=int, default=None,
                        help="under torchrun, shard the pairs when every rank gets at least "
                             "this many (any world size); a smaller corpus trains whole on every "
                             "rank (no merges, rank 0 writes).  Default: shard only where the "
                             "merge plan was measured within 1 %% of one model on the target "
                             "function on both test corpora (DESIGN.md 7a): 2 ranks with 80-200 M "
                             "pairs per rank (touch divisor damped to k^beta), 3 ranks with "
                             "80-100 M, 4 with 80-250 M, 8 with 150-200 M; never at 5-7 ranks (6 ranks: up "
                             "to +1.9 %%); C3's 8 x 125 M reads -1.1..-1.2 %% on one corpus, 8 x "
                             "80 M -4.5 %%.  Setting it is an opt-in to those gaps")
    parser.add_argument("--shuffle", choices=("python", "device"), default=None,
                        help="the pair shuffles (src/gene2vec.py:52,80): 'python' = CPython's "
                             "random.shuffle bit for bit on the host; 'device' = keyed "
                             "permutations of the HBM-resident pairs on the GPU, vocabulary "
                             "scanned in the first one's order (needs --native-ingest and a "
                             "pairs-only corpus; default under torchrun)")
    args = parser.parse_args(argv)
    if args.sample == 0 and args.grid == 0 and args.mode == "hogwild":
        # without downsampling the hot genes' rows take most
        # updates, and at the default grid the Hogwild staleness moves the
        # manuscript target function 4-10 % from the sequential order on
        # structured corpora (the loss and SGNS objective stay within 0.2 %)
        print("warning: --sample 0 (the reference keeps gensim's 1e-3): at the default grid "
              "the target function can drift 4-10 % from gensim's order on structured "
              "corpora; --grid 16 holds it within 0.4 % at ~10x the training time "
              "(DESIGN.md section 8)", file=sys.stderr)
    rank, world = _init_dp(args)
    # data-parallel ranks would each redo a serial Fisher-Yates over the whole
    # corpus per iteration: reshuffle on the device instead unless asked
    shuffle_mode = args.shuffle or ("device" if world > 1 else "python")
    ph = _Phases()
    source_dir, export_dir, ending_pattern = args.fileAddress[:3]

    logging.basicConfig(format="%(asctime)s : %(levelname)s : %(message)s", level=logging.INFO)
    print("start!")
    if world > 1 and args.shuffle_seed is None:
        # every rank must shuffle identically: rank 0 draws the seed
        import torch.distributed as dist
        box = [random.randrange(2 ** 63) if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        args.shuffle_seed = box[0]
    rng = random.Random(args.shuffle_seed) if args.shuffle_seed is not None else random
    corpus = None
    pipe = None
    n_lines = None
    with ph("ingest"):
        if args.native_ingest:
            files = os.listdir(source_dir)
            rng.shuffle(files)
            paths = [os.path.join(source_dir, f) for f in files if f.endswith(ending_pattern)]
            print(datetime.datetime.now())
            print(f"native ingest of {len(paths)} files")
            if shuffle_mode == "python":
                # the shuffles depend only on the pair count and rng: start
                # drawing the first one (src/gene2vec.py:52) from a newline
                # count while the files are tokenised
                n_lines = ingest.count_lines(paths)
                pipe = ingest.ShufflePipeline(n_lines, rng, max(1, args.iters))
            try:
                if world > 1 and shuffle_mode == "device":
                    # each rank tokenises its own range of the files; the ranks
                    # then share the tokens (None: not all pairs -> every rank
                    # reads everything)
                    from . import distributed as Dd
                    corpus = Dd.gather_corpus(paths)
                if corpus is None:
                    corpus = ingest.read_corpus(paths)
            except BaseException:
                if pipe is not None:
                    pipe.close(wait=True)
                raise
            n_pairs = corpus.n_sent
        else:
            gene_pairs = read_gene_pairs(source_dir, ending_pattern, rng)
            n_pairs = len(gene_pairs)
        # every line a pair (the generator's output): fixed-length sentences,
        # no 8-byte offsets per pair to upload; shuffles keep the lengths
        pairs_only = corpus is not None and corpus.pairs_only
    if shuffle_mode == "device" and not pairs_only:
        print("--shuffle device needs --native-ingest and a pairs-only corpus: "
              "using Python's shuffle")
        shuffle_mode = "python"
        if corpus is not None:
            pipe = ingest.ShufflePipeline(corpus.n_sent, rng, max(1, args.iters))
    # data parallelism only for corpora big enough that merged replicas match
    # one model; below, every rank trains the whole corpus
    from . import distributed as Dd
    shard = Dd.dp_default_shard(n_pairs, world, args.dp_min_pairs_per_rank)
    if world > 1 and not shard:
        why = (f"< {world} ranks x {args.dp_min_pairs_per_rank}"
               if args.dp_min_pairs_per_rank is not None else
               f"over {world} ranks is outside the measured data-parallel windows "
               f"{ {w: Dd.DP_DEFAULT_WINDOWS[w] for w in sorted(Dd.DP_DEFAULT_WINDOWS)} } "
               "(pairs per rank; DESIGN.md 7a)")
        print(f"{n_pairs} pairs {why}: every rank trains the whole corpus (no sharding, no "
              "merges); rank 0 writes the outputs")
    drank, dworld = (rank, world) if shard else (0, 1)
    dorder = None
    perm_seed = None
    print(datetime.datetime.now())
    print("shuffle start " + str(n_pairs))
    exporter = _Exporter(not args.no_txt, not args.no_w2v, args.w2v_binary)
    with ph("shuffle"):
        if shuffle_mode == "device":
            # the first shuffle (:52) is a device permutation too: one draw,
            # the same on every rank; the vocabulary scan follows its order
            perm_seed = rng.getrandbits(64)
        elif corpus is not None:
            # this shuffle and the reshuffle before every later iteration (:80)
            # are drawn ahead on host threads while the GPU trains
            if n_lines is not None and corpus.n_sent != n_lines:  # never shuffle the wrong n
                pipe.close(wait=True)
                pipe = ingest.ShufflePipeline(corpus.n_sent, rng, max(1, args.iters))
            perm = pipe.next()
            corpus.permute_(perm)
            pipe.release(perm)
        else:
            rng.shuffle(gene_pairs)
    print(datetime.datetime.now())
    print("shuffle done " + str(n_pairs))

    try:
        dimension = args.dim
        hashfxn = _hashfxn(args.hash)
        os.makedirs(export_dir, exist_ok=True)
        outputs = []
        kw = dict(size=dimension, window=args.window, min_count=1, workers=args.workers, iter=1,
                  sg=1, negative=args.negative, sample=args.sample, hashfxn=hashfxn,
                  device=args.device, mode=args.mode, data_parallel=shard, grid=args.grid)
        import gene2vec_amd.word2vec as W
        from . import distributed as Dd
        W.DP_MERGE_RULE, W.DP_MERGE_EVERY_JOBS = Dd.dp_merge_plan(
            n_pairs / max(1, dworld), args.merge_every_jobs, args.merge_rule,
            jobs_per_rank=-(-(-(-n_pairs // max(1, dworld))) // 5000), world=dworld)
        W.DP_MERGE_BETA = Dd.dp_merge_beta(n_pairs / max(1, dworld), dworld, args.merge_rule)
        if shard:
            print(f"data parallel: {dworld} ranks x {n_pairs // dworld} pairs, {W.DP_MERGE_RULE} "
                  f"merge every {W.DP_MERGE_EVERY_JOBS} jobs"
                  + (f", divisor k^{W.DP_MERGE_BETA:.3f}" if W.DP_MERGE_BETA != 1.0 else ""))
        W.DP_MERGE_TRANSPORT = args.merge_transport
        model = None
        for current_iter in range(1, args.iters + 1):
            name = os.path.join(export_dir, f"gene2vec_dim_{dimension}_iter_{current_iter}")
            if current_iter == 1:
                print(f"gene2vec dimension {dimension} iteration {current_iter} start")
                if corpus is None:
                    with ph("train"):
                        model = Word2Vec(gene_pairs, **kw)
                else:
                    with ph("vocab"):
                        model = Word2Vec(**kw)
                        if shuffle_mode == "device":
                            model._build_from_counts(
                                _device_raw_counts(corpus, perm_seed, args.device))
                        else:
                            model._build_from_counts(corpus.vocab_raw_counts())
                        model.corpus_count = corpus.n_sent
                        model.corpus_total_words = int(len(corpus.tokens))
                        ids = _vocab_ids(model, corpus)
                        tok = ids[corpus.tokens]
                        _adopt_vocab_ids(corpus, ids, tok)
                    with ph("train"):
                        if shuffle_mode == "device":
                            dorder = _DeviceOrder(tok, _vocab_ids(model, corpus), args.device,
                                                  drank, dworld)
                            model.train_ids(None, None, 2, total_examples=model.corpus_count,
                                            epochs=model.iter,
                                            device_tokens=dorder.shard(perm_seed))
                        else:
                            model.train_ids(tok, *_sentences(corpus, pairs_only),
                                            total_examples=model.corpus_count,
                                            epochs=model.iter)
            else:
                print(datetime.datetime.now())
                print("shuffle start " + str(n_pairs))
                with ph("shuffle"):
                    if shuffle_mode == "device":
                        # same draw on every rank (one seed, src/gene2vec.py:80's
                        # random.shuffle is the reference's); applied on the device
                        perm_seed = rng.getrandbits(64)
                    elif corpus is not None:
                        perm = pipe.next()
                        corpus.permute_(perm)
                        pipe.release(perm)
                    else:
                        rng.shuffle(gene_pairs)
                print(datetime.datetime.now())
                print("shuffle done " + str(n_pairs))
                print(f"gene2vec dimension {dimension} iteration {current_iter} start")
                prev = os.path.join(export_dir, f"gene2vec_dim_{dimension}_iter_{current_iter - 1}")
                with ph("load"):
                    # src/gene2vec.py:86 reloads the checkpoint it just saved; the
                    # model kept from the last iteration is that state (save/load
                    # round-trips bit for bit), and its device tables and engine stay
                    # resident.  Data-parallel ranks keep theirs too: the epoch ends
                    # with a merge, after which every replica holds the same bits
                    # (one all-reduce result, the same apply kernel), so the engine,
                    # its RCCL communicator and the merge snapshot carry over.
                    if args.reload_checkpoints or model is None:
                        model = Word2Vec.load(prev, device=args.device)
                        model.data_parallel = shard
                        model.grid = args.grid
                if corpus is None:
                    with ph("train"):
                        model.train(gene_pairs, total_examples=model.corpus_count,
                                    epochs=model.iter)
                else:
                    with ph("vocab"):
                        ids = _vocab_ids(model, corpus)
                        if np.array_equal(ids, np.arange(len(ids), dtype=np.int32)):
                            tok = corpus.tokens  # adopted at iteration 1: ids are the model's
                        else:
                            tok = ids[corpus.tokens]
                        if dorder is not None and not np.array_equal(ids, dorder.ids):
                            # another vocabulary numbering: the resident order is
                            # re-uploaded (the model keeps its vocabulary, so never
                            # in the reference's loop)
                            dorder = _DeviceOrder(tok, ids, args.device, drank, dworld)
                    with ph("train"):
                        if dorder is not None:
                            model.train_ids(None, None, 2, total_examples=model.corpus_count,
                                            epochs=model.iter,
                                            device_tokens=dorder.shard(perm_seed))
                        else:
                            model.train_ids(tok, *_sentences(corpus, pairs_only),
                                            total_examples=model.corpus_count,
                                            epochs=model.iter)
            with ph("save"):
                model._sync_host()
                if rank == 0:  # data parallel: the merged replicas are identical
                    model.save(name)
            if rank == 0:
                # the text exports (generateMatrix.py, save_word2vec_format) read
                # this iteration's checkpoint / tables only: they run on a host
                # thread while the next iteration trains (one at a time, in order)
                # a snapshot: the next iteration rebinds model.wv's arrays
                exporter.submit(name, copy.copy(model.wv), ph)
            if world > 1 and args.reload_checkpoints:
                import torch.distributed as dist
                dist.barrier()  # the next iteration loads rank 0's checkpoint
            print(f"gene2vec dimension {dimension} iteration {current_iter} done")
            outputs.append(name)
            if args.reload_checkpoints:
                model = None  # freed (device tables too) before the reload
        dump = os.environ.get("G2V_DUMP_REPLICA")
        if dump and model is not None:  # test hook: every rank's final tables
            model._sync_host()
            np.savez(f"{dump}_rank{rank}.npz", syn0=model.wv.vectors, syn1neg=model.syn1neg)
    finally:
        if pipe is not None:
            pipe.close(wait=True)
    with ph("export_wait"):
        exporter.close()
    if args.timing and rank == 0:
        with open(args.timing, "w") as f:
            json.dump({k: round(v, 4) for k, v in ph.t.items()}, f)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return outputs


def _init_dp(args):
    """torchrun launch (WORLD_SIZE > 1): one rank per GPU, the pair file
    shared and sharded by Word2Vec.train_ids, replicas merged over RCCL.
    Returns (rank, world)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if args.backend == "gloo":
        local %= max(1, torch.cuda.device_count())
    args.device = local
    torch.cuda.set_device(local)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    # Python's per-process hash() seeds a different init on every rank: harmless,
    # Word2Vec broadcasts rank 0's tables before training
    return rank, world


if __name__ == "__main__":
    main()
