"""Device-side training engine: owns the HBM layout and drives the C ABI.

HBM layout for one rank (T = float32 or float64; rows padded to 64-byte multiples):
  row_ptr int64[U+1], items int32[nnz], ratings T[nnz]     user-major CSR, all_ratings() order
  sched   int32[...] per epoch-chunk                        users heaviest-first (Hogwild) or in
                                                            ur order (deterministic mode)
  pu T[U, ldu], bu T[U]                                     user side, owned by one wave per user
  qb T[R, I, ldq] = [q_i | b_i | 0..]                       item factors + item bias in one row,
                                                            R = item replicas
  yj T[R, I, ldu]                                           SVD++ implicit factors
  qb_s, (yj_s)                                              chunk-start snapshot (R > 1 or world > 1)
  delta T[I*ldq (+ I*ldu)]                                  packed item delta for the all-reduce

Every compute step is a HIP kernel behind include/surprise_amd.h; torch only
allocates device memory and supplies the stream.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .dist import ItemSync, chunk_users, item_counts, replica_queues


def _pad64(n: int, dtype: int) -> int:
    per64 = 16 if dtype == _lib.MF_F32 else 8
    return -(-n // per64) * per64


def default_ld(n_factors: int, dtype: int) -> int:
    """User / implicit row length (elements): n_factors padded to a 64-byte multiple."""
    return _pad64(n_factors, dtype)


def default_ldq(n_factors: int, dtype: int) -> int:
    """Item row length: n_factors + the item bias column, padded to a 64-byte multiple."""
    return _pad64(n_factors + 1, dtype)


class MFEngine(ItemSync):
    """SVD / SVD++ SGD on one GPU (one rank of a multi-GPU job)."""

    def __init__(self, csr, n_items, n_factors, *, algo="svd", hyper=None, biased=True,
                 dtype="float32", mode="replica", n_replicas=8, n_chunks=1, users=None,
                 deterministic=False, user_order=None, n_waves=0, device=None, ld=None,
                 world=1, merge="count"):
        torch = _lib.require_gpu()
        self.torch = torch
        self.algo = algo
        self.dev = torch.device("cuda", torch.cuda.current_device()) if device is None else \
            torch.device(device)
        self.dtype = _lib.MF_F64 if str(dtype) in ("float64", "f64", "double") else _lib.MF_F32
        self.tdt = torch.float64 if self.dtype == _lib.MF_F64 else torch.float32
        if n_factors < 1 or n_factors > _lib.MAX_FACTORS[self.dtype]:
            raise ValueError(f"n_factors must be in [1, {_lib.MAX_FACTORS[self.dtype]}] "
                             f"for {dtype}, got {n_factors}")
        self.K = int(n_factors)
        self.ld = int(ld) if ld else default_ld(self.K, self.dtype)
        self.ldq = default_ldq(self.K, self.dtype)
        row_ptr, items, ratings = csr
        self.n_users = len(row_ptr) - 1
        self.n_items = int(n_items)
        self.biased = bool(biased)
        self.deterministic = bool(deterministic)
        if self.deterministic:
            mode, n_replicas, n_chunks, n_waves = "plain", 1, 1, 1
        self.mode = _lib.MODES[mode] if isinstance(mode, str) else int(mode)
        self.n_replicas = int(n_replicas) if self.mode in _lib.REPLICA_MODES else 1
        self.n_chunks = max(1, int(n_chunks))
        self.n_waves = int(n_waves)
        self.world = int(world)
        self.stream = torch.cuda.current_stream(self.dev)

        # ---- CSR + schedules
        dev = self.dev
        self.row_ptr = torch.from_numpy(np.ascontiguousarray(row_ptr, np.int64)).to(dev)
        self.items = torch.from_numpy(np.ascontiguousarray(items, np.int32)).to(dev)
        self.ratings = torch.from_numpy(np.ascontiguousarray(ratings, np.float64)).to(
            dev, self.tdt)
        self._csr = _lib.MfCsr(self.row_ptr.data_ptr(), self.items.data_ptr(),
                               self.ratings.data_ptr(), self.n_users, self.n_items)
        self.users = np.arange(self.n_users) if users is None else np.asarray(users)
        if self.deterministic:
            order = np.asarray(user_order if user_order is not None else self.users, np.int32)
            chunks = [order]
        else:
            chunks = chunk_users(self.users, row_ptr, self.n_chunks)
        # per chunk: the user schedule (replica mode: R queues back to back, rep_ptr[R+1]) and
        # counts[R, I] = ratings of item i trained in replica r (the count-aware merge's n_r)
        R = self.n_replicas
        self.sched, self.rep_ptr, self.counts, self._totals_local = [], [], [], []
        for c in chunks:
            qs = replica_queues(c, row_ptr, R)
            self.sched.append(torch.from_numpy(np.ascontiguousarray(np.concatenate(qs), np.int32)).to(dev))
            ptr = np.zeros(R + 1, np.int32)
            np.cumsum([len(q) for q in qs], out=ptr[1:])
            self.rep_ptr.append(torch.from_numpy(ptr).to(dev))
            cnt = np.stack([item_counts(q, row_ptr, items, self.n_items) for q in qs])
            self.counts.append(torch.from_numpy(cnt.astype(np.int32)).to(dev))
            self._totals_local.append(cnt.sum(0).astype(np.int32))
        self.totals = None  # set by _prepare(): summed over every rank
        self.heads = torch.zeros(R, dtype=torch.int32, device=dev)
        self.work = torch.zeros(1, dtype=torch.float64, device=dev)
        self.merge_rule = merge
        self.dup_items = int(_has_duplicate_items(row_ptr, items))

        # ---- factor tables
        U, I, ld, ldq, R = self.n_users, self.n_items, self.ld, self.ldq, self.n_replicas
        z = lambda *shape: torch.zeros(*shape, dtype=self.tdt, device=dev)
        self.pu, self.bu = z(U, ld), z(U)
        self.qb = z(R, I, ldq)
        self.yj = z(R, I, ld) if algo == "svdpp" else None
        self.need_snap = R > 1 or self.world > 1
        if self.need_snap:
            self.qb_s = z(I, ldq)
            self.yj_s = z(I, ld) if algo == "svdpp" else None
        self._delta = None
        self._hyper = _lib.MfHyper(**(hyper or {}))
        if not self.biased:
            self._hyper.global_mean = 0.0

    # ------------------------------------------------------------------ state in / out
    def set_factors(self, pu, qi, bu=None, bi=None, yj=None):
        """Upload host fp64 arrays (n, K) into the padded device tables (all replicas)."""
        t = self.torch
        K = self.K

        def put(dst2d, src):
            dst2d.zero_()
            dst2d[:, :K].copy_(t.from_numpy(np.ascontiguousarray(src, np.float64)).to(
                self.dev, self.tdt))

        put(self.pu, pu)
        self.bu.copy_(t.from_numpy(np.zeros(self.n_users) if bu is None else
                                   np.asarray(bu, np.float64)).to(self.dev, self.tdt))
        for r in range(self.n_replicas):
            put(self.qb[r], qi)
            self.qb[r][:, K].copy_(t.from_numpy(np.zeros(self.n_items) if bi is None else
                                                np.asarray(bi, np.float64)).to(self.dev, self.tdt))
            if self.yj is not None:
                put(self.yj[r], yj)
        if self.need_snap:
            self.qb_s.copy_(self.qb[0])
            if self.yj is not None:
                self.yj_s.copy_(self.yj[0])

    def get_factors(self):
        """Host fp64 copies (pu, qi, bu, bi, yj) with the padding columns dropped."""
        self.stream.synchronize()
        K = self.K
        h = lambda x: x.to(self.torch.float64).cpu().numpy()
        out = dict(pu=h(self.pu[:, :K]), qi=h(self.qb[0][:, :K]), bu=h(self.bu),
                   bi=h(self.qb[0][:, K]))
        out["yj"] = h(self.yj[0][:, :K]) if self.yj is not None else None
        return out

    # ------------------------------------------------------------------ kernels
    def _ptr(self, t):
        return ctypes.c_void_p(t.data_ptr())

    def run_chunk(self, c: int):
        s = self.sched[c]
        st = ctypes.c_void_p(self.stream.cuda_stream)
        rep = self.mode in _lib.REPLICA_MODES
        rp = self._ptr(self.rep_ptr[c]) if rep else None
        hd = self._ptr(self.heads) if rep else None
        if self.algo == "svd":
            _lib.call("mf_svd_epoch", ctypes.byref(self._csr), self._ptr(s), s.numel(),
                      self._ptr(self.pu), self._ptr(self.bu), self.ld, self._ptr(self.qb),
                      self.ldq, self.K, int(self.biased), ctypes.byref(self._hyper), self.mode,
                      self.n_replicas, rp, hd, self.n_waves, self.dup_items, self.dtype, st)
        else:
            _lib.call("mf_svdpp_epoch", ctypes.byref(self._csr), self._ptr(s), s.numel(),
                      self._ptr(self.pu), self._ptr(self.bu), self.ld, self._ptr(self.qb),
                      self.ldq, self._ptr(self.yj), self.K, ctypes.byref(self._hyper),
                      self.mode, self.n_replicas, rp, hd, self.n_waves, self.dup_items,
                      self.dtype, st)
        self._chunk = c

    def _prepare(self, ctx):
        """Global per-item rating counts of every chunk (all ranks) for the count-aware merge."""
        self.totals = []
        for t in self._totals_local:
            tt = self.torch.from_numpy(t).to(self.dev)
            if ctx is not None and ctx.world > 1:
                ctx.all_reduce_sum(tt)
            self.totals.append(tt)

    def _merge(self, delta_out, apply):
        st = ctypes.c_void_p(self.stream.cuda_stream)
        c = getattr(self, "_chunk", 0)
        count_aware = self.merge_rule == "count"
        if count_aware and self.totals is None:
            self._prepare(None)
        I = self.n_items
        tabs = [(self.qb, self.qb_s, self.ldq, self.K)]
        if self.yj is not None:
            tabs.append((self.yj, self.yj_s, self.ld, -1))
        off = 0
        for tab, snap, ld, bias_col in tabs:
            # item factors / biases: count-aware; SVD++ implicit factors: count-weighted mean
            # (every user of a group moves all its y_j together, which saturates fast)
            rule = (_lib.MF_MERGE_SUM if not count_aware else
                    _lib.MF_MERGE_COUNT if bias_col >= 0 else _lib.MF_MERGE_MEAN)
            use_counts = rule != _lib.MF_MERGE_SUM
            dptr = None
            if delta_out is not None:
                dptr = ctypes.c_void_p(delta_out.data_ptr() + off * delta_out.element_size())
            _lib.call("mf_item_merge", self._ptr(tab), self._ptr(snap), I, ld, self.K, bias_col,
                      self.n_replicas, rule, self._ptr(self.counts[c]) if use_counts else None,
                      self._ptr(self.totals[c]) if use_counts else None,
                      ctypes.byref(self._hyper), self._ptr(self.pu), self.n_users, self.ld,
                      self._ptr(self.work), dptr, int(apply), self.dtype, st)
            off += I * ld

    def _merge_local(self):
        self._merge(None, True)

    def _delta_buffer(self):
        if self._delta is None:
            n = self.n_items * self.ldq
            if self.yj is not None:
                n += self.n_items * self.ld
            self._delta = self.torch.zeros(n, dtype=self.tdt, device=self.dev)
        return self._delta

    def _delta_into(self, buf):
        self._merge(buf, False)

    def _apply(self, buf):
        st = ctypes.c_void_p(self.stream.cuda_stream)
        I = self.n_items
        tabs = [(self.qb, self.qb_s, self.ldq)]
        if self.yj is not None:
            tabs.append((self.yj, self.yj_s, self.ld))
        off = 0
        for tab, snap, ld in tabs:
            _lib.call("mf_item_apply", self._ptr(tab), self._ptr(snap), I, ld, self.n_replicas,
                      ctypes.c_void_p(buf.data_ptr() + off * buf.element_size()), self.dtype, st)
            off += I * ld

    def _gather_users(self, ctx):
        """After the last epoch: every rank keeps only its own users' rows, then a SUM
        all-reduce assembles the full pu / bu on every rank."""
        mask = self.torch.zeros(self.n_users, dtype=self.tdt, device=self.dev)
        mask[self.torch.from_numpy(np.asarray(self.users, np.int64)).to(self.dev)] = 1
        self.pu.mul_(mask[:, None])
        self.bu.mul_(mask)
        ctx.all_reduce_sum(self.pu)
        ctx.all_reduce_sum(self.bu)

    # ------------------------------------------------------------------ inference
    def user_implicit(self):
        """imp[u] = sum_{j in I_u} yj[j] / sqrt|I_u| on device (SVDpp.estimate :518-520)."""
        imp = self.torch.zeros(self.n_users, self.ld, dtype=self.tdt, device=self.dev)
        _lib.call("mf_svdpp_user_implicit", ctypes.byref(self._csr), self._ptr(self.yj[0]),
                  self.ld, self._ptr(imp), self.K, self.dtype,
                  ctypes.c_void_p(self.stream.cuda_stream))
        return imp

    def predict(self, u, i, global_mean, imp=None):
        """Batched estimate on inner ids (-1 = unknown) -> (est fp64, impossible bool)."""
        t = self.torch
        n = len(u)
        du = t.from_numpy(np.ascontiguousarray(u, np.int32)).to(self.dev)
        di = t.from_numpy(np.ascontiguousarray(i, np.int32)).to(self.dev)
        est = t.zeros(n, dtype=self.tdt, device=self.dev)
        bad = t.zeros(n, dtype=t.int32, device=self.dev)
        _lib.call("mf_predict", n, self._ptr(du), self._ptr(di), self._ptr(self.pu),
                  self._ptr(self.bu), self.ld, self._ptr(self.qb[0]), self.ldq,
                  None if imp is None else self._ptr(imp), self.K, int(self.biased),
                  float(global_mean), self._ptr(est), self._ptr(bad), self.dtype,
                  ctypes.c_void_p(self.stream.cuda_stream))
        self.stream.synchronize()
        return est.to(t.float64).cpu().numpy(), bad.cpu().numpy().astype(bool)


def _has_duplicate_items(row_ptr, items) -> bool:
    """True if some user lists the same item twice (the kernels then forward rows in registers)."""
    row_ptr = np.asarray(row_ptr, np.int64)
    if len(items) == 0:
        return False
    users = np.repeat(np.arange(len(row_ptr) - 1, dtype=np.int64), np.diff(row_ptr))
    key = users * (int(np.max(items)) + 1) + np.asarray(items, np.int64)
    return len(np.unique(key)) != len(key)
