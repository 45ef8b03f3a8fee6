"""Multi-GPU schedule: users sharded by row across ranks, item-side updates
SUM-all-reduced once per epoch-chunk.

One process per GPU (torchrun / torch.distributed; backend "nccl" is RCCL on
ROCm, "gloo" for the CPU tests and for rehearsing several ranks on one GPU).
Each rank owns a contiguous range of users balanced by rating count and holds
ONLY that range on its device: its rows of the CSR (rank-local row_ptr) and its
pu / bu rows.  Item tables are replicated; every rank runs its epoch-chunk from
the same chunk-start item state.

  mode "log":  each rank folds its delta log into per-item sums S_i; the SUM
               all-reduce of S (and of the <pu^2> partials) gives every rank the
               same S, applied with the count-aware weight w(N_i) of the global
               per-item count -- the identical result of one GPU processing every
               rank's users (mf_log_apply, include/surprise_amd.h).
  other modes: each rank contributes its weighted ``local - snapshot`` item delta
               (mf_item_merge's count-aware rule, n_r = the rank's ratings of the
               item), SUM all-reduced and added to the snapshot.
SVD++'s y_j rows: within a chunk every user's end-of-user update is the affine
map y_j <- A_u y_j + c_u (A_u = (1 - lr_yj reg_yj)^|I_u|), so rank r's chunk
result is y_r = A_r y_s + c_r with A_r the product of its users' A_u.  Ranks own
contiguous user ranges in order, so composing the ranks' maps in rank order is
the single-GPU composition over all users in CSR order:
    y = A y_s + sum_r S_r c_r,   A = prod_r A_r,   S_r = prod_{s > r} A_s,
a SUM all-reduce of S_r (y_r - A_r y_s) (mf_item_affine; A_r, S_r are per-item
constants of the schedule, computed once on the host).
"""
from __future__ import annotations

import os
import zlib

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


def local_csr(csr, lo: int, hi: int):
    """Rows [lo, hi) of a user-major CSR with a rank-local row_ptr (starts at 0)."""
    row_ptr, items, ratings = csr
    row_ptr = np.asarray(row_ptr, np.int64)
    k0, k1 = int(row_ptr[lo]), int(row_ptr[hi])
    return (row_ptr[lo:hi + 1] - k0, np.asarray(items)[k0:k1], np.asarray(ratings)[k0:k1])


def chunk_users(users, row_ptr, n_chunks: int, long_chain: int = 256):
    """Split a rank's users into n_chunks epoch-chunks of ~equal rating count, each sorted
    heaviest-first (the order the waves take them): users sorted by degree (descending) are
    dealt round-robin, so every chunk gets a similar mix of heavy and light users (every
    chunk's critical path is about the heaviest user's chain).  Users whose chain alone outlasts
    a chunk -- more than 1 / long_chain of a chunk's ratings -- all go to chunk 0, where their
    chains run side by side instead of one per chunk, when there are at most n_chunks of them
    (else the dealing is unchanged): the full C5's 9 users of 200k-600k ratings take ~112 ms of
    sequential chain each against ~5 ms for a chunk's other 7.9M ratings.
    long_chain = 0: plain round-robin dealing."""
    users = np.asarray(users, dtype=np.int64)
    deg = np.diff(np.asarray(row_ptr, dtype=np.int64))[users]
    order = np.argsort(-deg, kind="stable")
    srt = users[order]
    n_long = 0
    if n_chunks > 1 and len(users) and long_chain > 0:
        thr = deg.sum() / n_chunks / max(1, long_chain)
        n_long = int((deg[order] > thr).sum())
    if n_long <= 1 or n_long > n_chunks:
        return [srt[c::n_chunks].astype(np.int32) for c in range(n_chunks)]
    rest = srt[n_long:]
    out = [rest[c::n_chunks] for c in range(n_chunks)]
    out[0] = np.concatenate([srt[:n_long], out[0]])
    return [c.astype(np.int32) for c in out]


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


def item_log_decay(users, row_ptr, items, n_items: int, decay: float):
    """log of A_r per item: sum over the ratings (u, j) of `users` of |I_u| log(decay) -- the
    product of the end-of-user y maps' factors A_u = decay^|I_u| that touch item j."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    users = np.asarray(users, dtype=np.int64)
    if len(users) == 0 or decay == 1.0:
        return np.zeros(n_items, np.float64)
    deg = np.diff(row_ptr)
    starts, lens = row_ptr[users], deg[users]
    idx = np.repeat(starts - np.cumsum(np.concatenate([[0], lens[:-1]])), lens) + np.arange(lens.sum())
    w = np.repeat(lens.astype(np.float64), lens) * np.log(decay)
    return np.bincount(np.asarray(items)[idx], weights=w, minlength=n_items)


def csr_fingerprint(csr, n_items: int):
    """(n_users, n_items, nnz, crc32 of the CSR bytes) -- ranks must agree on the trainset."""
    row_ptr, items, ratings = csr
    crc = zlib.crc32(np.ascontiguousarray(row_ptr, np.int64).tobytes())
    crc = zlib.crc32(np.ascontiguousarray(items, np.int32).tobytes(), crc)
    crc = zlib.crc32(np.ascontiguousarray(ratings, np.float64).tobytes(), crc)
    return np.array([len(row_ptr) - 1, n_items, int(row_ptr[-1]), crc], np.int64)


class _Done:
    def wait(self):
        return True


class DistContext:
    """Rank/world of the current process and the collectives of the schedule.  With the gloo
    backend device tensors are staged through host memory (gloo is the CPU / rehearsal
    transport); with nccl (RCCL) they stay on the device."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.host_staged = self.backend == "gloo"

    @classmethod
    def from_env(cls, backend: str | None = None, single_rank_group: bool = False):
        """Join (or reuse) the default process group described by torchrun's env vars and bind
        this process to its GPU (LOCAL_RANK); None for a single-process run, unless
        single_rank_group (a world of one rank: exercises the backend's collectives alone)."""
        import torch
        import torch.distributed as dist
        if (int(os.environ.get("WORLD_SIZE", "1")) <= 1 and not dist.is_initialized()
                and not single_rank_group):
            return None
        if not dist.is_initialized():
            backend = backend or os.environ.get("SURPRISE_AMD_DIST_BACKEND", "nccl")
            local = int(os.environ.get("LOCAL_RANK", "0"))
            if backend == "nccl":
                torch.cuda.set_device(local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                n = torch.cuda.device_count()
                if n:
                    torch.cuda.set_device(local % n)
                dist.init_process_group(backend)
        return cls()

    def _run(self, fn, tensor):
        if self.host_staged and tensor.is_cuda:
            h = tensor.cpu()
            fn(h)
            tensor.copy_(h)
        else:
            fn(tensor)

    def all_reduce_sum(self, tensor):
        self._run(lambda t: self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group),
                  tensor)

    def all_reduce_sum_async(self, tensor):
        """SUM all-reduce enqueued behind the current stream's work; returns a handle whose
        wait() makes the current stream wait for it (RCCL: its own stream runs the collective
        meanwhile).  Host-staged (gloo): done at once, wait() is a no-op."""
        if self.host_staged and tensor.is_cuda:
            self.all_reduce_sum(tensor)
            return _Done()
        return self.dist.all_reduce(tensor, op=self.dist.ReduceOp.SUM, group=self.group,
                                    async_op=True)

    def all_reduce_max(self, tensor):
        self._run(lambda t: self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group),
                  tensor)

    def broadcast(self, tensor, src: int = 0):
        self._run(lambda t: self.dist.broadcast(t, src, group=self.group), tensor)

    def all_gather_rows(self, local, counts):
        """Concatenate every rank's rows (rank order); counts[r] = rows of rank r.  Rows are
        padded to the largest shard for the collective and trimmed after."""
        import torch
        m = max(int(max(counts)), 1)
        dev = "cpu" if self.host_staged else local.device
        pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
        pad[:local.shape[0]].copy_(local)
        outs = [torch.empty_like(pad) for _ in range(self.world)]
        self.dist.all_gather(outs, pad, group=self.group)
        return torch.cat([o[:int(c)] for o, c in zip(outs, counts)])

    def barrier(self):
        self.dist.barrier(group=self.group)

    def check_agreement(self, values, what: str):
        """Raise unless every rank passed the same int64 vector."""
        import torch
        v = torch.as_tensor(np.asarray(values, np.int64))
        dev = "cpu" if self.host_staged else torch.device("cuda", torch.cuda.current_device())
        hi, lo = v.clone().to(dev), (-v).to(dev)
        self.all_reduce_max(hi)
        self.all_reduce_max(lo)
        if not torch.equal(hi.cpu(), (-lo).cpu()):
            raise RuntimeError(f"ranks disagree on {what}: max {hi.tolist()} min {(-lo).tolist()}")


class ItemSync:
    """Epoch-chunk protocol shared by the HIP engine and the CPU test engine.

    Subclasses provide ``run_chunk(c)``, ``_merge_local()`` (single-rank fold, may
    be a no-op), ``_delta_into(buf)``, ``_apply(buf)`` and ``_delta_buffer()``."""

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
