"""Multi-GPU schedule: users sharded by row across ranks, item-side updates
SUM-all-reduced once per epoch-chunk.

One process per GPU (torchrun / torch.distributed; backend "nccl" is RCCL on
ROCm, "gloo" for the CPU tests).  Each rank owns a contiguous range of users
balanced by rating count, so pu/bu rows never cross ranks; item tables are
replicated and every rank runs its epoch-chunk from the same chunk-start state.

  mode "log":  each rank folds its delta log into per-item sums S_i; the SUM
               all-reduce of S (and of the <pu^2> partials) gives every rank the
               same S, applied with the count-aware weight w(N_i) of the global
               per-item count -- the identical result of one GPU processing every
               rank's users (mf_log_apply, include/surprise_amd.h).
  other modes: each rank contributes its weighted ``local - snapshot`` item delta
               (mf_item_merge's count-aware rule, n_r = the rank's ratings of the
               item), SUM all-reduced and added to the snapshot.
SVD++'s y_j rows are per-rank shared state, merged across ranks by the
count-weighted mean of the rank deltas.
"""
from __future__ import annotations

import os

import numpy as np


def shard_users(row_ptr, world: int):
    """Contiguous user ranges [b[r], b[r+1]) with ~equal rating counts per rank."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    n_users = len(row_ptr) - 1
    nnz = int(row_ptr[-1])
    bounds = [0]
    for r in range(1, world):
        target = nnz * r // world
        b = int(np.searchsorted(row_ptr, target, side="left"))
        b = min(max(b, bounds[-1]), n_users)
        bounds.append(b)
    bounds.append(n_users)
    return np.asarray(bounds, dtype=np.int64)


def chunk_users(users, row_ptr, n_chunks: int):
    """Split a rank's users into n_chunks epoch-chunks of ~equal rating count:
    users sorted by degree (descending) are dealt round-robin, so every chunk
    gets a similar mix of heavy and light users.  Returns a list of int32 arrays,
    each sorted heaviest-first (the order the waves take them)."""
    users = np.asarray(users, dtype=np.int64)
    deg = np.diff(np.asarray(row_ptr, dtype=np.int64))[users]
    order = users[np.argsort(-deg, kind="stable")]
    return [order[c::n_chunks].astype(np.int32) for c in range(n_chunks)]


def item_counts(users, row_ptr, items, n_items: int):
    """Ratings per item among `users` (a rank's n_r in the count-aware merge)."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    users = np.asarray(users, dtype=np.int64)
    if len(users) == 0:
        return np.zeros(n_items, np.int64)
    starts, ends = row_ptr[users], row_ptr[users + 1]
    lens = ends - starts
    idx = np.repeat(starts - np.cumsum(np.concatenate([[0], lens[:-1]])), lens) + np.arange(lens.sum())
    return np.bincount(np.asarray(items)[idx], minlength=n_items)


class DistContext:
    """Rank/world of the current process and the item-delta all-reduce."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    @classmethod
    def from_env(cls, backend: str | None = None):
        """Join (or reuse) the default process group described by torchrun's env vars;
        returns None for a single-process run."""
        import torch.distributed as dist
        if int(os.environ.get("WORLD_SIZE", "1")) <= 1 and not dist.is_initialized():
            return None
        if not dist.is_initialized():
            dist.init_process_group(backend=backend or "nccl")
        return cls()

    def all_reduce_sum(self, tensor):
        self.dist.all_reduce(tensor, op=self.dist.ReduceOp.SUM, group=self.group)

    def barrier(self):
        self.dist.barrier(group=self.group)


class ItemSync:
    """Epoch-chunk protocol shared by the HIP engine and the CPU test engine.

    Subclasses provide ``run_chunk(c)``, ``_merge_local()`` (single-rank fold, may
    be a no-op), ``_delta_into(buf)``, ``_apply(buf)``, ``_delta_buffer()`` and
    ``_gather_users(ctx)``."""

    n_chunks = 1

    def sync_items(self, ctx: DistContext | None):
        world = 1 if ctx is None else ctx.world
        if world == 1:
            self._merge_local()
            return
        buf = self._delta_buffer()
        self._delta_into(buf)
        ctx.all_reduce_sum(buf)
        self._apply(buf)

    def _prepare(self, ctx):
        """Hook run once before the first epoch (e.g. global per-item counts)."""

    def run_epochs(self, n_epochs: int, ctx: DistContext | None = None, on_epoch=None):
        self._prepare(ctx)
        for epoch in range(n_epochs):
            for c in range(self.n_chunks):
                self.run_chunk(c)
                self.sync_items(ctx)
            if on_epoch is not None:
                on_epoch(epoch)
        if ctx is not None and ctx.world > 1:
            self._gather_users(ctx)
