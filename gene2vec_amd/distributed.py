"""Data-parallel SGNS across GPUs: one process per GPU, torch.distributed.

The reference has no distribution (gensim Hogwild threads in one process,
src/gene2vec.py:59).  Pairs are independent SGNS examples, so the corpus is
sharded by contiguous pair ranges; every rank keeps a full replica of
syn0/syn1neg (torch-owned device tensors bound into libg2v) and trains its
shard; every ``avg_every_jobs`` gensim jobs the replicas are averaged with one
all-reduce per table (backend "nccl" = RCCL over xGMI on MI355X; "gloo" on
CPU for tests).  The vocabulary is global: counts are summed and first
occurrences reduced with MIN over global token positions, so every rank
builds the identical index order and cum_table.
"""
from __future__ import annotations

import os

import numpy as np


def world_info():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n, rank, world):
    """contiguous [start, end) of n items for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def rank_seed(seed, rank):
    """model.random seed per rank: rank 0 keeps gensim's seed, others offset."""
    return seed + rank


def global_vocab(counts, first, token_offset, device=None):
    """Combine per-rank id counts / first-occurrence positions.

    counts, first: int64[V] for this rank's shard (first = -1 when absent);
    token_offset: global position of this rank's first token.  Returns numpy
    (counts, first) identical on every rank."""
    import torch
    import torch.distributed as dist
    counts = np.asarray(counts, dtype=np.int64)
    first = np.asarray(first, dtype=np.int64)
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return counts, first
    big = np.iinfo(np.int64).max
    fg = np.where(first >= 0, first + token_offset, big)
    c = torch.from_numpy(counts.copy())
    f = torch.from_numpy(fg)
    if device is not None:
        c, f = c.to(device), f.to(device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    dist.all_reduce(f, op=dist.ReduceOp.MIN)
    c, f = c.cpu().numpy(), f.cpu().numpy()
    return c, np.where(f == big, -1, f)


def average_(tensors, group=None):
    """In-place mean of each tensor over ranks (SUM then scale: works on
    nccl/RCCL and gloo alike)."""
    import torch.distributed as dist
    if not dist.is_initialized():
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    for t in tensors:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.mul_(1.0 / world)


def touch_merge_(tensors, olds, beta=1.0, group=None):
    """Row-wise replica merge: new = old + sum_r(d_r) / k**beta, d_r = replica r's
    change since the last merge, k = number of replicas whose row changed.

    A row only one replica trained keeps that replica's full update (plain
    averaging would divide it by N); a row every replica trained gets the
    mean of their updates (summing would overshoot the hot rows -- measured:
    summed deltas diverge).  ``olds`` hold the tables at the last merge and
    are updated in place."""
    import torch
    import torch.distributed as dist
    single = not dist.is_initialized() or dist.get_world_size(group) == 1
    for t, old in zip(tensors, olds):
        # rows are the last dimension: a [2][V][ld] buffer holding both tables
        # merges with one collective per quantity
        d = t - old
        cnt = (d != 0).any(dim=-1).to(t.dtype)
        if not single:
            dist.all_reduce(d, op=dist.ReduceOp.SUM, group=group)
            dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
        k = torch.clamp(cnt, min=1.0)
        if beta != 1.0:
            k = k ** beta
        d.div_(k.unsqueeze(-1))
        old.add_(d)
        t.copy_(old)


class ReplicaTrainer:
    """Drives one rank: trains job windows on an engine-like object and
    merges the replicas between windows.

    engine: has ``train(job_sent, alpha, seed, mode, timing=...)``.
    tables: the torch tensors bound into the engine (merged in place).
    merge:  "touch" (row-wise, default) or "mean" (plain model averaging).
    """

    def __init__(self, engine, tables, avg_every_jobs, mode=0, merge="touch", beta=1.0):
        self.engine = engine
        self.tables = list(tables)
        self.avg_every_jobs = max(1, int(avg_every_jobs))
        self.mode = mode
        self.merge = merge
        self.beta = beta
        self.olds = [t.clone() for t in self.tables] if merge == "touch" else None
        self.averages = 0

    def train_epoch(self, job_sent, alphas, seeds, timing=False):
        n_jobs = len(job_sent) - 1
        for j0 in range(0, n_jobs, self.avg_every_jobs):
            j1 = min(n_jobs, j0 + self.avg_every_jobs)
            self.engine.train(job_sent[j0:j1 + 1], alphas[j0:j1], seeds[j0:j1], self.mode,
                              timing=timing)
            self.sync_replicas()

    def sync_replicas(self):
        if self.merge == "touch":
            touch_merge_(self.tables, self.olds, self.beta)
        else:
            average_(self.tables)
        self.averages += 1
