"""Device-side training engine: owns the HBM layout and drives the C ABI.

HBM layout for one rank (T = float32 or float64; rows padded to 64-byte multiples):
  row_ptr int64[U+1], items int32[nnz], ratings T[nnz]     user-major CSR, all_ratings() order
  sched   int32[...] per epoch-chunk                        users heaviest-first, or in ur order
                                                            (deterministic mode)
  pu T[U, ldu], bu T[U]                                     user side, owned by one wave per user
  qb T[I, ldq] = [q_i | b_i | 0..]                          item factors + item bias in one row
  yj T[I, ldu]                                              SVD++ implicit factors
  qlog T[nnz_rank, ldq]                                     "log" mode: item delta per rating
  perm int32[nnz_chunk], piece_beg, item_piece_ptr          "log" mode: per-chunk item grouping
  sums T[pieces, ldq]                                       "log" mode: partial sums per piece
  qb_s, yj_s                                                chunk-start snapshots (world > 1)

Every compute step is a HIP kernel behind include/surprise_amd.h; torch only
allocates device memory, supplies the stream and runs the RCCL all-reduce.
"""
from __future__ import annotations

import ctypes
import os
import weakref

import numpy as np

from . import _lib
from .dist import ItemSync, chunk_users, item_counts


def _new_event():
    """A native HIP event (timing disabled) for the engine's fork / join."""
    ev = ctypes.c_void_p()
    _lib.call("mf_event_create", ctypes.byref(ev))
    return ev


def _free_events(evs):
    lib = _lib.load()
    for ev in evs:
        lib.mf_event_destroy(ev)

PIECE_ROWS = 64  # log rows summed by one wave of mf_log_reduce
SVDPP_WAVES_PER_CU = 4  # SVD++ without helper waves: users in flight per CU
HX_CHAINS_PER_CU = 2  # SVD++ helper-wave launch: user chains per CU (1 / 3 / 4 measured slower)
HX_CHAINS_PER_CU_ONE = 4  # ... with one helper wave per chain (workgroups of two waves)
# helpers=None: one helper wave per chain and HX_CHAINS_PER_CU_ONE chains per CU where an
# epoch-chunk holds at least this many users (C5 per-rank shard, 96k users per chunk: 93.9 ->
# 90.4 ms/epoch); below it three helpers and HX_CHAINS_PER_CU (C3, 6040 users: 4 chains per CU
# put more users on the popular rows at once, 0.577 -> 0.728 ms)
HX_ONE_HELPER_MIN_USERS = 50_000


# SVD++ (atomic q rows, deferred y): at most this many users OF ONE RANK per epoch-chunk.  Every
# user of a chunk reads the chunk-start y_j.  Measured on C5's shard (1.25M users, K=128, E=20,
# held-out RMSE - the sequential oracle): one rank at 1 / 2 / 4 / 16 chunks +2.7e-3 / +2.5e-3 /
# +8.1e-4 / +2.1e-4; the same users over 8 ranks at 2 chunks (78k users per rank and chunk, 625k
# in all: C5@8's geometry) +1.6e-4 (profiles/r4_gloo8_c5.json) -- the staleness that costs
# accuracy is y's within one rank; across ranks the rank-order merge composes it.
# ML-1M's 6040 users pass with 1 chunk.  No cap: one GPU holding all 10M C5 users runs 125 chunks.
SVDPP_USERS_PER_CHUNK = 80_000


def default_chunks(algo: str, mode: str, n_users_total: int, world: int = 1) -> int:
    """Epoch-chunks of the default schedules: 1 for SVD's log (the recency fold holds C4 at 20
    epochs with one); SVD++: one per SVDPP_USERS_PER_CHUNK users of a rank (n_users_total over
    `world` ranks), so C5@8 (10M users) runs 16 chunks and the C5 shard on one GPU 16 too."""
    if algo == "svdpp" and mode == "atomic":
        per_rank = -(-int(n_users_total) // max(1, int(world)))
        return max(1, -(-per_rank // SVDPP_USERS_PER_CHUNK))
    return 1


# SVD++ q log (qlog=None: auto).  The q log reads every item row from the chunk-start table, so
# its staleness grows with how often one chunk rates the same item.  Measured (held-out RMSE - the
# exact oracle at E=20, profiles/r5k_probe.jsonl, r5p_probe.jsonl): ML-1M (C3, one
# rank) at 16 chunks -- 13.5 ratings per item and chunk -- +1.9e-3, at 24 / 32 / 64 / 128 chunks
# (9.0 / 6.7 / 3.4 / 1.7) -2.6e-4 / -2.6e-4 / -2.9e-4 / -1.3e-4; C5 (7.7 per item and chunk)
# within 1e-3 of the sequential oracle on the shard, 0.94543 vs the atomic schedule's 0.94641 on
# the full C5.  At C5 it is the faster schedule (shard 70.5 vs 89.7 ms, full 658 vs 845 ms).
QLOG_MAX_RATINGS_PER_ITEM_CHUNK = 10.0


def auto_qlog(algo: str, mode: int, nnz: int, n_items: int, n_chunks: int, world: int,
              exchange, dup_items: bool, deterministic: bool) -> bool:
    """qlog=None: the q log for SVD++ on ONE rank with several epoch-chunks (the default chunking
    gives more than one from 80k users up) whose mean ratings per item and chunk are at most
    QLOG_MAX_RATINGS_PER_ITEM_CHUNK; the atomic schedule otherwise (ML-1M's one chunk: C3;
    several ranks, whose rank-order merge is pinned for the atomic schedule)."""
    return (algo == "svdpp" and mode == _lib.MF_MODE_ATOMIC and not deterministic
            and int(world) == 1 and not exchange and not dup_items and int(n_chunks) >= 2
            and n_items > 0
            and nnz / (float(n_items) * int(n_chunks)) <= QLOG_MAX_RATINGS_PER_ITEM_CHUNK)


def _pad64(n: int, dtype: int) -> int:
    per64 = 16 if dtype == _lib.MF_F32 else 8
    return -(-n // per64) * per64


def default_ld(n_factors: int, dtype: int) -> int:
    """User / implicit row length (elements): n_factors padded to a 64-byte multiple."""
    return _pad64(n_factors, dtype)


ITEM_ROW_ALIGN = 64  # bytes


def default_ldq(n_factors: int, dtype: int, user_bias_col: bool = False) -> int:
    """Item row length: n_factors + the item-bias column [+ the constant column of the user bias,
    read only by the SVD log's lookahead body: user_bias_col], padded to a 64-byte multiple.
    (Reserving the extra column everywhere would push fp64 K=127 / fp32 K=255 rows past 1 KiB and
    cost SVD++ its helper-wave launch there.)"""
    per = ITEM_ROW_ALIGN // (4 if dtype == _lib.MF_F32 else 8)
    return -(-(n_factors + 1 + int(bool(user_bias_col))) // per) * per


def stable_argsort(keys):
    """np.argsort(keys, kind="stable") for non-negative int keys < 2^32, as LSD radix passes over
    16-bit digits (numpy radix-sorts 16-bit keys: 5x faster than its int32 merge sort at 1M)."""
    keys = np.asarray(keys)
    lo = np.argsort((keys & 0xFFFF).astype(np.uint16), kind="stable")
    if not len(keys) or int(keys.max()) < (1 << 16):
        return lo
    return lo[np.argsort((keys[lo] >> 16).astype(np.uint16), kind="stable")]


def position_users(row_ptr):
    """The user of every CSR position (int32[nnz])."""
    row_ptr = np.asarray(row_ptr, np.int64)
    return np.repeat(np.arange(len(row_ptr) - 1, dtype=np.int32), np.diff(row_ptr))


def log_layout(row_ptr, items, users, n_items, piece_rows=PIECE_ROWS, local=False):
    """Item grouping of one epoch-chunk's delta-log rows (MF_MODE_LOG).

    Returns (perm, piece_beg, item_piece_ptr, counts): perm = CSR positions of the ratings of
    `users`, grouped by item, increasing position within an item (the reference's user order);
    an item's rows are cut into pieces of <= piece_rows; counts[i] = ratings of item i.
    local=True: perm holds chunk-local log rows instead -- the users' ratings numbered in
    ascending user order (chunk_log_rows: the SVD++ q log's per-chunk buffer)."""
    row_ptr = np.asarray(row_ptr, np.int64)
    users = np.sort(np.asarray(users, np.int64))
    starts, ends = row_ptr[users], row_ptr[users + 1]
    lens = ends - starts
    tot = int(lens.sum())
    ks = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(tot)
    it = np.asarray(items)[ks]
    order = stable_argsort(it)
    perm = (order if local else ks[order]).astype(np.int32)
    counts = np.bincount(it, minlength=n_items).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(counts)])
    item_piece_ptr, piece_beg = piece_bounds(offs, counts, piece_rows)
    return perm, piece_beg.astype(np.int32), item_piece_ptr, counts.astype(np.int32)


# The split step's side stream.  HIP deals streams over GPU_MAX_HW_QUEUES hardware queues; a side
# stream that lands on the main stream's queue serialises the two launch groups (the headline
# step ~1.75x slower, about one engine in four when each engine takes a fresh pool stream:
# profiles/r5bm_bimodal.jsonl).  "cached": one side stream per device for the process, made
# when the first engine needs it; "-high": at high priority; "pool": a fresh pool stream per
# engine (the round-4 behaviour).
SIDE_STREAM_POLICY = "cached"
_SIDE_STREAMS = {}


def side_stream(torch, dev, which=0, policy=None):
    policy = policy or SIDE_STREAM_POLICY
    prio = -1 if policy.endswith("high") else 0
    if not policy.startswith("cached"):
        return torch.cuda.Stream(device=dev, priority=prio)
    key = (torch.device(dev).index, which, prio)
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=dev, priority=prio)
    return s


def _vp_int(p):
    """A ctypes.c_void_p (or None) as the int a c_void_p structure field takes."""
    return None if p is None else (p.value if isinstance(p, ctypes.c_void_p) else int(p))


def cold_items(counts, share):
    """The hybrid launch's cold items of one chunk: the least-rated items whose ratings add up to
    at most `share` of the chunk's (bool[n_items]; items the chunk does not rate are not cold)."""
    counts = np.asarray(counts, np.int64)
    order = np.argsort(counts, kind="stable")
    cum = np.cumsum(counts[order])
    cold = np.zeros(len(counts), bool)
    n = int(np.searchsorted(cum, share * max(int(counts.sum()), 1), side="right"))
    cold[order[:n]] = True
    return cold & (counts > 0)


def mix_layout(row_ptr, items, users, n_items, cold, piece_rows=PIECE_ROWS):
    """The hybrid launch's cold log of one chunk (mf_svdpp_epoch_mix): the cold items' ratings
    grouped by item (users in order within an item), so a cold rating at CSR position p is log row
    crow[p] (crow -1: a live item); pieces of <= piece_rows rows, each of one item, for
    mf_log_reduce (perm = the identity), item_piece_ptr for mf_log_apply, and every row's
    position among its item's ratings (the recency weight)."""
    perm, pb, ipp, cnt = log_layout(row_ptr, items, users, n_items, piece_rows)
    pitem = np.repeat(np.arange(n_items, dtype=np.int32), np.diff(ipp))
    keep = cold[pitem]
    lens = np.diff(pb)
    pos_keep = np.repeat(keep, lens)
    rows = perm[pos_keep]
    crow = np.full(int(np.asarray(row_ptr)[-1]), -1, np.int32)
    crow[rows] = np.arange(len(rows), dtype=np.int32)
    rpos = (np.arange(len(perm), dtype=np.int64) - np.repeat(pb[ipp[:-1]], cnt))[pos_keep]
    pitem_c = pitem[keep]
    pb_c = np.concatenate([[0], np.cumsum(lens[keep])]).astype(np.int32)
    ipp_c = np.concatenate([[0], np.cumsum(np.bincount(pitem_c, minlength=n_items))]).astype(
        np.int32)
    return dict(crow=crow, rows=len(rows), pb=pb_c, pitem=pitem_c, ipp=ipp_c,
                rpos=rpos.astype(np.int32), totals=np.where(cold, cnt, 0).astype(np.int32))


def qlog_fold_layout(counts, perm, rpos, users, hot_rows=PIECE_ROWS, piece_rows=PIECE_ROWS):
    """mf_svdpp_qlog_fold's layout of one chunk (include/surprise_amd.h mf_qlog_fold_t) from the
    q log's item-grouped positions: perm (log rows), rpos (each row's position among its item's)
    and users (each row's rater), grouped by item with counts[i] rows.  Items of <= hot_rows rows
    are cold (one wavefront takes their rows in turn); the others hot, cut into pieces of
    <= piece_rows positions that the launch's pre-passes reduce first."""
    assert hot_rows <= 64, "a cold item's rows are taken in one 64-lane vector load"
    counts = np.asarray(counts, np.int64)
    n_items = len(counts)
    hot = counts > hot_rows
    at_hot = np.repeat(hot, counts)
    pre = lambda c: np.concatenate([[0], np.cumsum(c)]).astype(np.int32)
    cold_c, hot_c = np.where(hot, 0, counts), np.where(hot, counts, 0)
    hipp, hpb = piece_bounds(np.concatenate([[0], np.cumsum(hot_c)]), hot_c, piece_rows)
    return dict(perm=np.asarray(perm, np.int32)[~at_hot], rpos=np.asarray(rpos, np.int32)[~at_hot],
                item_row_beg=pre(cold_c), users=np.asarray(users, np.int32)[~at_hot],
                hot_perm=np.asarray(perm, np.int32)[at_hot],
                hot_rpos=np.asarray(rpos, np.int32)[at_hot],
                hot_users=np.asarray(users, np.int32)[at_hot],
                hot_piece_beg=hpb.astype(np.int32),
                hot_piece_item=np.repeat(np.arange(n_items, dtype=np.int32), np.diff(hipp)),
                hot_item_piece_ptr=hipp.astype(np.int32), n_hot_pieces=len(hpb) - 1)


def chunk_log_rows(row_ptr, users):
    """First chunk-local log row of each of `users` (the SVD++ q log: a chunk's ratings numbered
    in ascending user order, as log_layout(local=True)): (sorted users, int64 rows)."""
    row_ptr = np.asarray(row_ptr, np.int64)
    users = np.sort(np.asarray(users, np.int64))
    lens = row_ptr[users + 1] - row_ptr[users]
    return users, np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)


def item_positions(row_ptr, items, users, n_items):
    """Position of each rating of `users` among their ratings of the same item, users in order
    (the order the reference applies them): (ks, pos) with ks the CSR positions, ascending."""
    row_ptr = np.asarray(row_ptr, np.int64)
    users = np.sort(np.asarray(users, np.int64))
    starts, lens = row_ptr[users], row_ptr[users + 1] - row_ptr[users]
    tot = int(lens.sum())
    ks = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(tot)
    it = np.asarray(items)[ks]
    order = stable_argsort(it)
    off = np.concatenate([[0], np.cumsum(np.bincount(it, minlength=n_items))])
    pos = np.empty(tot, np.int32)
    pos[order] = np.arange(tot) - off[it[order]]
    return ks, pos


REPLAY_PIECES_PER_WAVE = 8  # replay_piece_rows(): pieces per replay wave kept at least


REPLAY_MAX_ROWS = 256  # measured at C4 (ms/epoch): 64 35.0, 256 33.3, 1024 35.0


def replay_piece_rows(row_ptr, users, waves=4096):
    """Ratings per piece of the checkpoint replay (a multiple of 64, up to REPLAY_MAX_ROWS): long
    pieces cut mf_log_apply's chain of piece rows on a popular item (C4: the top item's ~1M
    ratings were 16k pieces of 64, summed by one wave: fold 1.47 -> 0.46 ms), as long as every
    replay wave (~waves) still gets REPLAY_PIECES_PER_WAVE pieces of 64-rating sub-pieces."""
    deg = np.diff(np.asarray(row_ptr, np.int64))
    nnz = int(deg[np.asarray(users, np.int64)].sum()) if len(users) else 0
    m = nnz // (PIECE_ROWS * waves * REPLAY_PIECES_PER_WAVE)
    return PIECE_ROWS * int(max(1, min(REPLAY_MAX_ROWS // PIECE_ROWS, m)))


def piece_bounds(offs, counts, piece_rows=PIECE_ROWS):
    """Item i's rows [offs[i], offs[i] + counts[i]) cut into pieces of <= piece_rows:
    (item_piece_ptr int32[n_items+1], piece_beg int64[n_pieces+1], the last = offs[-1])."""
    npc = -(-counts // piece_rows)
    item_piece_ptr = np.concatenate([[0], np.cumsum(npc)]).astype(np.int32)
    piece_item = np.repeat(np.arange(len(counts)), npc)
    local = np.arange(len(piece_item)) - item_piece_ptr[piece_item]
    piece_beg = np.concatenate([offs[piece_item] + piece_rows * local,
                                [offs[-1]]]).astype(np.int64)
    return item_piece_ptr, piece_beg


def split_heavy(users, row_ptr, heavy):
    """[rest, heaviest] of a chunk's users (schedule order kept): the heaviest are the
    int(heavy) users of largest degree (heavy >= 1) or those with >= heavy * the largest degree
    (heavy < 1).  One group only when either would be empty."""
    users = np.asarray(users, np.int32)
    deg = np.diff(np.asarray(row_ptr, np.int64))[users]
    if not len(users) or heavy <= 0:
        return [users]
    if heavy >= 1:
        h = np.zeros(len(users), bool)
        h[np.argsort(-deg, kind="stable")[:int(heavy)]] = True
    else:
        h = deg >= heavy * deg.max()
    if h.all() or not h.any():
        return [users]
    return [users[~h], users[h]]


def split_groups(users, row_ptr, heavy, top=0):
    """The launch groups of a split chunk: [light, heavy] (split_heavy), or with top > 0
    [light, top, rest]: the `top` heaviest of the heavy users (main stream) and the rest of
    them (a third stream), each in schedule order."""
    parts = split_heavy(users, row_ptr, heavy)
    if top and len(parts) == 2:
        rest_top = split_heavy(parts[1], row_ptr, top)
        if len(rest_top) == 2:
            return [parts[0], rest_top[1], rest_top[0]]
    return parts


def chain_schedule(users, row_ptr, n_chains, user_cost=16):
    """The users laid out for n_chains user chains taking entries c, c + n_chains, ... (the
    helper-wave SVD++ launch): longest-processing-time-first, each user (heaviest first) to the
    chain with the least work so far (degree + user_cost per user), padded with -1."""
    import heapq
    users = np.asarray(users, np.int32)
    deg = np.diff(np.asarray(row_ptr, np.int64))[users]
    order = np.argsort(-deg, kind="stable")
    n_chains = max(1, min(int(n_chains), len(users)))
    lists = [[] for _ in range(n_chains)]
    heap = [(0, c) for c in range(n_chains)]
    for x in order:
        load, c = heapq.heappop(heap)
        lists[c].append(users[x])
        heapq.heappush(heap, (load + int(deg[x]) + user_cost, c))
    m = max(len(x) for x in lists) if lists else 0
    out = np.full((m, n_chains), -1, np.int32)
    for c, x in enumerate(lists):
        out[:len(x), c] = x
    return out.ravel()


HOT_MIN_RATINGS = 1000  # hot_items(): rows with fewer ratings never bound the launch
HOT_TRIGGER = 0.005     # ... replicas only if the top item holds >= this share of the ratings,
HOT_SHARE = 0.0015      # ... then for every item holding >= this share
HOT_MAX = 64


def hot_items(items, n_items, n=None):
    """Items whose q rows get a delta replica in the SVD++ helper-wave launch (sorted ids).
    n = None: if the most-rated item holds >= HOT_TRIGGER of the ratings (and >=
    HOT_MIN_RATINGS of them), every item holding >= HOT_SHARE (at most HOT_MAX, most-rated
    first), else none; otherwise the n most-rated items.  Measured (tools/exp_hot_rows.sh): at
    C3 (top item 0.57% of the ratings) 0 / 8 / 32 replicas give 0.608 / 0.575 / 0.567 ms per
    epoch; on the C5 shard (top item 0.46%) replicas of its top items change nothing and the
    replica reads cost 14% (99.9 -> 114 ms), so none there."""
    cnt = np.bincount(np.asarray(items, np.int64), minlength=n_items)[:n_items]
    order = np.argsort(-cnt, kind="stable")
    if n is None:
        tot = max(int(cnt.sum()), 1)
        top = int(cnt.max()) if len(cnt) else 0
        if top < max(HOT_MIN_RATINGS, HOT_TRIGGER * tot):
            return order[:0]
        n = min(HOT_MAX, int((cnt >= HOT_SHARE * tot).sum()))
    n = max(0, min(int(n), int((cnt > 0).sum())))
    return np.sort(order[:n])


def ck_row0(row_ptr):
    """First packed checkpoint row of every user, (row_ptr[u] + u + 1) // 2 (the kernels'
    ck_row0): pair m of user u is row ck_row0[u] + m; the log holds ck_row0[n_users] rows."""
    row_ptr = np.asarray(row_ptr, np.int64)
    return (row_ptr + np.arange(len(row_ptr), dtype=np.int64) + 1) >> 1


def ckpt_positions(row_ptr, perm, interval=2, pos_user=None):
    """mf_log_replay's ck_pos of every log position: 2 * (packed checkpoint row of the rating's
    pair) + (the rating's parity within its user).  pos_user: position_users(row_ptr), if at
    hand."""
    if interval != 2:
        raise ValueError("the checkpoint log stores one row per pair of ratings")
    row_ptr = np.asarray(row_ptr, np.int64)
    k = np.asarray(perm, np.int64)
    u = (position_users(row_ptr) if pos_user is None else pos_user)[k]
    j = k - row_ptr[u]
    return (2 * (ck_row0(row_ptr)[u] + (j >> 1)) + (j & 1)).astype(np.int32)


class Predictor:
    """Batched inference on device tables (pu, bu, qb = [q | b], yj): the estimate of
    SVD / SVDpp / NMF for many (u, i) pairs in one launch (mf_predict) and accuracy.rmse / mae
    as one device reduction (mf_rating_errors).  Needs: torch, dev, stream, dtype, tdt, pu, bu,
    qb, ld, ldq, K, biased (+ yj and _csr for SVD++'s implicit term)."""

    def _ptr(self, t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else None

    def user_implicit(self):
        """imp[u] = sum_{j in I_u} yj[j] / sqrt|I_u| on device (SVDpp.estimate :518-520)."""
        self._fork_bound = False  # (main-stream work after the last fold: MFEngine's fork)
        imp = self.torch.zeros(self.n_users, self.ld, dtype=self.tdt, device=self.dev)
        _lib.call("mf_svdpp_user_implicit", ctypes.byref(self._csr), self._ptr(self.yj),
                  self.ld, self._ptr(imp), self.K, self.dtype,
                  ctypes.c_void_p(self.stream.cuda_stream))
        return imp

    def _predict_dev(self, u, i, global_mean, imp=None):
        self._fork_bound = False
        t = self.torch
        n = len(u)
        du = t.from_numpy(np.ascontiguousarray(u, np.int32)).to(self.dev)
        di = t.from_numpy(np.ascontiguousarray(i, np.int32)).to(self.dev)
        est = t.zeros(n, dtype=self.tdt, device=self.dev)
        bad = t.zeros(n, dtype=t.int32, device=self.dev)
        _lib.call("mf_predict", n, self._ptr(du), self._ptr(di), self._ptr(self.pu),
                  self._ptr(self.bu), self.ld, self._ptr(self.qb), self.ldq,
                  None if imp is None else self._ptr(imp), self.K, int(self.biased),
                  float(global_mean), self._ptr(est), self._ptr(bad), self.dtype,
                  ctypes.c_void_p(self.stream.cuda_stream))
        return est, bad

    def predict(self, u, i, global_mean, imp=None):
        """Batched estimate on inner ids (-1 = unknown) -> (est fp64, impossible bool)."""
        est, bad = self._predict_dev(u, i, global_mean, imp)
        self.stream.synchronize()
        return est.to(self.torch.float64).cpu().numpy(), bad.cpu().numpy().astype(bool)

    def rating_errors(self, u, i, r, global_mean, imp=None, fallback=None, offset=0.0,
                      rating_scale=(1, 5)):
        """(rmse, mae, n) of the estimates against r (test() + accuracy.rmse / mae, finished as
        AlgoBase.predict does) -- estimates and errors never leave the device."""
        t = self.torch
        if len(u) == 0:  # (accuracy.rmse / mae raise on an empty prediction list)
            raise ValueError("Prediction list is empty.")
        est, bad = self._predict_dev(u, i, global_mean, imp)
        dr = t.from_numpy(np.ascontiguousarray(r, np.float64)).to(self.dev)  # (fp64 always)
        out = t.zeros(3, dtype=t.float64, device=self.dev)
        fb = float(global_mean if fallback is None else fallback)
        _lib.call("mf_rating_errors", len(u), self._ptr(est), self._ptr(bad), self._ptr(dr), fb,
                  float(offset), float(rating_scale[0]), float(rating_scale[1]), self._ptr(out),
                  self.dtype, ctypes.c_void_p(self.stream.cuda_stream))
        se, ae, n = out.cpu().tolist()
        return (se / n) ** .5, ae / n, int(n)


class PredictTables(Predictor):
    """Device copies of a fitted model's host arrays for batched inference (a model whose training
    engine is gone: fitted on several ranks, or unpickled on a GPU host)."""

    def __init__(self, pu, qi, bu, bi, *, yj=None, csr=None, biased=True, dtype="float32"):
        torch = _lib.require_gpu()
        self.torch = torch
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.stream = torch.cuda.current_stream(self.dev)
        self.dtype = _lib.MF_F64 if str(dtype) in ("float64", "f64", "double") else _lib.MF_F32
        self.tdt = torch.float64 if self.dtype == _lib.MF_F64 else torch.float32
        pu, qi = np.asarray(pu, np.float64), np.asarray(qi, np.float64)
        self.K = int(qi.shape[1])
        self.ld = default_ld(self.K, self.dtype) if self.K else 16
        self.ldq = default_ldq(self.K, self.dtype)
        self.n_users, self.n_items = len(pu), len(qi)
        self.biased = bool(biased)
        z = lambda *shape: torch.zeros(*shape, dtype=self.tdt, device=self.dev)
        put = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(self.dev, self.tdt)
        self.pu, self.qb = z(self.n_users, self.ld), z(self.n_items, self.ldq)
        self.pu[:, :self.K] = put(pu)
        self.qb[:, :self.K] = put(qi)
        self.qb[:, self.K] = put(bi)
        self.bu = put(bu)
        self.yj = None
        if yj is not None:
            self.yj = z(self.n_items, self.ld)
            self.yj[:, :self.K] = put(yj)
            row_ptr, items, _ = csr
            self.row_ptr = torch.from_numpy(np.ascontiguousarray(row_ptr, np.int64)).to(self.dev)
            self.items = torch.from_numpy(np.ascontiguousarray(items, np.int32)).to(self.dev)
            self._csr = _lib.MfCsr(self.row_ptr.data_ptr(), self.items.data_ptr(), 0,
                                   self.n_users, self.n_items)


class MFEngine(ItemSync, Predictor):
    """SVD / SVD++ SGD on one GPU (one rank of a multi-GPU job)."""

    def __init__(self, csr, n_items, n_factors, *, algo="svd", hyper=None, biased=True,
                 dtype="float32", mode="log", n_chunks=1, deterministic=False,
                 user_order=None, n_waves=0, device=None, ld=None, world=1, merge=None,
                 ckpt=True, heavy=None, err_in_row=True, narrow=None, events="native",
                 join="event",
                 helpers=None, ydefer=True, hx_chains_per_cu=None, hot_rows=None,
                 replay_rows=None, gram=None, xcd_split=None, qlog=None, top=None,
                 exchange=None, long_chain=256, overlap_q=True, fused=True, stagger=None,
                 light_replay_wpc=0, log_nt=None, item_align=None, bias_mirror=True,
                 cold_share=0.0, replay_fold=False):
        """csr: this rank's rows only (rank-local row_ptr from 0; dist.local_csr) -- the whole
        trainset for one GPU.  pu / bu hold exactly those rows; get_factors(ctx) gathers.

        Schedule options (the defaults are the measured-best product paths; each alternative
        is held to the default or to its oracle by a GPU test, DESIGN.md 'Switches'):
          ckpt        SVD log: the checkpoint form (one user row per pair of ratings, rebuilt by
                      mf_log_replay) where rows fit 1 KiB; False: the gradient log
          heavy       split each chunk's heaviest users into their own launch on a second
                      stream (>= 1: that many users; < 1: those with >= heavy * the top degree;
                      0: no split; None: 128 on a full MI355X for small epochs)
          err_in_row  checkpoint log: each pair's errors in its row's padding (else elog)
          narrow      checkpoint log: rows of the K factor columns only, errors in elog
                      (MF_EPOCH_CKPT_NARROW); None = where that makes rows of whole 128-byte
                      lines (K * size % 128 == 0, e.g. fp32 K=128: 512 vs 576 B per row)
          events      "native": the split's fork / join as HIP events bound to the kernels that
                      complete them (mf_launch_event); "torch": torch.cuda.Event record / wait
          join        "event": the main stream waits for the side stream's event; "kernel": the
                      heavy replay's last block waits for the light replay (mf_launch_join)
          helpers     SVD++ atomic mode: one user chain per workgroup whose q atomics helper
                      waves issue (MF_EPOCH_SVDPP_HELPERS): True three helpers, 1 one helper
                      per chain (MF_EPOCH_SVDPP_ONE_HELPER, HX_CHAINS_PER_CU_ONE chains per CU),
                      None by the chunk size (HX_ONE_HELPER_MIN_USERS), False none
          ydefer      SVD++ atomic mode: the users' y updates folded per item after the chunk
                      (mf_svdpp_y_fold) instead of float atomics at each user's end
          hx_chains_per_cu  the helper-wave launch's user chains per CU (HX_CHAINS_PER_CU)
          replay_rows checkpoint log: ratings per replay piece (None: replay_piece_rows())
          hot_rows    the helper-wave launch: items whose q row gets a delta replica
                      (mf_svdpp_epoch's hot rows): None = auto (hot_items()), 0 = none, n = the
                      n most-rated items
          gram        checkpoint log, split chunk: the heavy users by the blocked solve
                      (mf_svd_epoch_gram, where the rows carry their errors); None / False: the
                      lookahead chain (mf_svd_epoch_sq)
          xcd_split   the heavy launch on XCD 0, the rest on XCDs 1-7 (None: without gram)
          top         split chunk: the heaviest `top` of the heavy users keep the main stream
                      (XCD 0) and the rest of the heavy launch runs beside them on a third stream
                      (XCD 1), so that its log replay and a first fold of the light + rest sums
                      overlap the top chains (None: HEAVY_TOP_USERS = off; measured slower)
          qlog        SVD++: the item rows read-only within an epoch-chunk, each rating's q / b
                      gradient logged (mf_svdpp_epoch_qlog) and folded after the chunk with the
                      recency weights, y deferred -- no float atomics (oracle:
                      oracle_svdpp_sgd_stalelog); False: the atomic schedule; None: auto_qlog
                      (one rank, several chunks, <= 10 ratings per item and chunk)
          long_chain  epoch-chunk dealing (dist.chunk_users): users of more than 1 / long_chain
                      of a chunk's ratings all go to chunk 0 (when at most n_chunks of them);
                      0: plain round-robin dealing (the dealing before round 4)
          stagger     checkpoint log, large chunks: the chunk's users in two halves (every
                      other user in schedule order), half A's epoch kernel first on the main
                      stream, then half B's epoch on the side stream beside A's log replay, then
                      B's replay -- the same arithmetic (the fold adds both halves' piece sums);
                      None / False: off (measured slower at C4: the concurrent replay's log
                      stream evicts the epoch kernel's item rows from the MALL)
          light_replay_wpc  split chunk: the light group's log replay at this many waves per
                      CU (0: the library's 16) -- fewer leave the heavy chains' memory path
                      quieter while the replay still ends before them
          log_nt      the checkpoint log's / SVD++ q log's rows stored non-temporal (streamed
                      past L2 / MALL: MF_EPOCH_LOG_NT); None: where the log is >= LOG_NT_MIN_BYTES;
                      "heavy" / "light": only that group's launch of a split chunk
          item_align  item rows padded to a multiple of this many bytes (timing probes; None:
                      ITEM_ROW_ALIGN)
          cold_share  SVD++ helper-wave launch on one rank: the least-rated items holding up to
                      this share of a chunk's ratings keep their rows read-only for the chunk,
                      their gradients logged and folded after it (mf_svdpp_epoch_mix); the
                      others take the float atomics (0: off)
          replay_fold checkpoint log, split chunk on one rank: the chunk's fold (mf_log_apply's
                      arithmetic) inside the two log replays -- the wave that completes an
                      item's last piece applies it (mf_launch_fold) -- instead of a launch of its
                      own after them; False: the separate fold
          bias_mirror checkpoint log with SB rows (fp32 K=128, fp64 K=64 / 128): the item biases
                      read from a mirror array, the item rows on whole 128-B lines; False: from
                      the rows
                      (C4: 27 GB of log evicted the item table from the MALL -- epoch kernel
                      18.0 -> 14.6 ms; ML-1M's 0.3-GB log: +3%, off)
          fused       SVD++ q log on one rank: the chunk's fold in one pass over the items
                      (mf_svdpp_qlog_fold: the q gradients' weighted sums, the q step and the y
                      maps' composition together); False: mf_log_reduce + mf_log_apply +
                      mf_svdpp_y_fold (the several-rank exchange always takes that path)
          overlap_q   SVD++ atomic schedule on several ranks over RCCL: q's part of the
                      exchange all-reduced (async) while the y fold runs (False: one buffer)
          exchange    None: the multi-rank exchange (snapshots, the packed all-reduce buffer,
                      the <p^2> ride) when world > 1; True: also at world 1 with a context --
                      TEST ONLY: the device-resident exchange path under RCCL on one GPU
                      (tests/_rccl_worker.py), which must equal the local fold"""
        torch = _lib.require_gpu()
        self.torch = torch
        self.algo = algo
        self.dev = torch.device("cuda", torch.cuda.current_device()) if device is None else \
            torch.device(device)
        self.dtype = _lib.MF_F64 if str(dtype) in ("float64", "f64", "double") else _lib.MF_F32
        self.tdt = torch.float64 if self.dtype == _lib.MF_F64 else torch.float32
        if n_factors < 0 or n_factors > _lib.MAX_FACTORS[self.dtype]:
            raise ValueError(f"n_factors must be in [0, {_lib.MAX_FACTORS[self.dtype]}] "
                             f"for {dtype}, got {n_factors}")
        self.K = int(n_factors)
        # (n_factors = 0 -- the biases alone, baseline_sgd -- still gets a non-empty user row)
        self.ld = int(ld) if ld else (default_ld(self.K, self.dtype) if self.K else 16)
        row_ptr, items, ratings = csr
        row_ptr = np.asarray(row_ptr, np.int64)
        self.n_users = len(row_ptr) - 1
        self.n_items = int(n_items)
        self.biased = bool(biased)
        self.deterministic = bool(deterministic)
        if self.deterministic:
            mode, n_chunks, n_waves = "plain", 1, 1
        self.mode = _lib.MODES[mode] if isinstance(mode, str) else int(mode)
        # (a user listing an item twice: the kernels forward rows in registers)
        self.dup_items = int(_has_duplicate_items(row_ptr, items, self.n_items, torch, self.dev))
        if qlog is None:
            qlog = auto_qlog(algo, self.mode, int(row_ptr[-1] - row_ptr[0]), self.n_items,
                             max(1, int(n_chunks)), world, exchange, self.dup_items,
                             self.deterministic)
        # SVD++ q log: MF_MODE_LOG's log / fold machinery with the deferred-y lookahead chain
        esz0 = 8 if self.dtype == _lib.MF_F64 else 4
        self.qlog_pp = (algo == "svdpp" and not self.deterministic and bool(qlog)
                        and default_ldq(n_factors, self.dtype) * esz0 <= 1024)
        if self.qlog_pp:
            self.mode = _lib.MF_MODE_LOG
        # (the user-bias column of the SVD log's lookahead body: that schedule's rows only)
        self.ldq = default_ldq(self.K, self.dtype,
                               user_bias_col=algo == "svd" and self.mode == _lib.MF_MODE_LOG)
        if item_align:  # (timing probes: item rows padded to this many bytes)
            per = int(item_align) // esz0
            self.ldq = -(-self.ldq // per) * per
        # item-side merge rule: the log fold weights each logged gradient by its recency
        # (MF_MERGE_RECENCY); SVD++'s snapshot-delta merge of q / b across ranks
        # carries each rank's delta through the later ranks' steps (mf_item_merge's
        # MF_MERGE_RECENCY); other snapshot merges by the count-aware rule
        if merge is None:
            merge = "recency" if (self.mode == _lib.MF_MODE_LOG or algo == "svdpp") else "count"
        self.recency = merge == "recency" and self.mode == _lib.MF_MODE_LOG
        self.n_chunks = max(1, int(n_chunks))
        if events not in ("native", "torch") or join not in ("event", "kernel"):
            raise ValueError("events must be 'native' or 'torch', join 'event' or 'kernel'")
        self.n_waves = int(n_waves)
        # (the q log reads the chunk-start rows whatever the users in flight: the launch default)
        if self.n_waves <= 0 and algo == "svdpp" and not self.deterministic and not self.qlog_pp:
            # SVD++ with shared item rows: at most SVDPP_WAVES_PER_CU users in flight per CU.
            # Users that start later then see the q rows (float atomics) of the users before
            # them, as the reference's sequential order does; with every ML-1M user in flight at
            # once the whole epoch reads the epoch-start q and the held-out RMSE drifts +3e-3 ..
            # +5e-3 from the reference at E=20, vs -7e-5 at 4 per CU, same epoch time
            props = torch.cuda.get_device_properties(torch.cuda.current_device())
            self.n_waves = SVDPP_WAVES_PER_CU * props.multi_processor_count
        self.world = int(world)
        self.multi = self.world > 1 or bool(exchange)  # (the exchange path's tables and rules)
        self.fused = bool(fused)
        self.light_replay_wpc = int(light_replay_wpc)  # (split chunk: the light replay's waves/CU)
        self.overlap_q = bool(overlap_q)
        self._q_work = None
        if merge not in ("count", "recency", "sum"):
            raise ValueError("merge must be 'count', 'recency' or 'sum', got %r" % (merge,))
        self.merge_rule = merge
        self._ctx = None
        self.stream = torch.cuda.current_stream(self.dev)
        esz = 8 if self.dtype == _lib.MF_F64 else 4

        # ---- CSR + schedules
        dev = self.dev
        self.row_ptr = torch.from_numpy(np.ascontiguousarray(row_ptr)).to(dev)
        # (padded: mf_log_replay reads up to mf_ckpt_interval() positions past a rating)
        self.items = torch.from_numpy(np.concatenate([np.asarray(items, np.int32),
                                                      np.zeros(64, np.int32)])).to(dev)
        self.ratings = torch.from_numpy(np.ascontiguousarray(ratings, np.float64)).to(
            dev, self.tdt)
        self._csr = _lib.MfCsr(self.row_ptr.data_ptr(), self.items.data_ptr(),
                               self.ratings.data_ptr(), self.n_users, self.n_items)
        self.users = np.arange(self.n_users)
        if self.deterministic:
            order = np.asarray(user_order if user_order is not None else self.users, np.int32)
            chunks = [order]
        else:
            chunks = chunk_users(self.users, row_ptr, self.n_chunks, long_chain=int(long_chain))
        to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        self._row_ptr_h, self._items_h = row_ptr, np.asarray(items, np.int32)
        self._chunk_users = [np.asarray(c, np.int32) for c in chunks]
        esz_q = self.ldq * esz
        # SVD with rows of <= 1 KiB logs in checkpoint form (a user row per pair of ratings + the
        # errors; mf_log_replay rebuilds the gradients)
        # (the replay undoes one user step, dividing by ap = 1 - lr_pu reg_pu: kept well away
        # from 0, else the gradient log)
        h = dict(hyper or {})
        ap = 1.0 - h.get("lr_pu", 0.0) * h.get("reg_pu", 0.0)
        # (rows of more than 1 KiB: only in narrow form of whole lane groups -- the factor columns
        # alone fill one or two 512-B groups, the biases ride beside them: fp64 K = 128)
        whole_rows = (self.K * esz) % 512 == 0 and self.K * esz <= 1024 and narrow is not False
        self.ckpt = (self.mode == _lib.MF_MODE_LOG and bool(ckpt) and algo == "svd"
                     and (esz_q <= 1024 or whole_rows) and abs(ap) >= 0.5)
        # checkpoint log with MF_EPOCH_ERR_IN_ROW where the row has room: each pair's two errors
        # ride in its checkpoint row's padding (the replay gathers no elog entries)
        e0 = ((self.K + 3) & ~1) if self.dtype == _lib.MF_F32 else self.K + 2
        # ... unless narrow rows (the factor columns only, errors in elog) are whole cache lines
        # where the padded rows are not: the replay reads each row twice (C4: 757 -> ~520 B per
        # read), so a 4-byte error gather per rating costs less than the rows' extra line
        lc = _lib.ckpt_narrow_ld(self.K, self.dtype)
        if narrow is None:
            narrow = lc * esz % 128 == 0 or esz_q > 1024
        self.narrow = self.ckpt and bool(narrow) and 0 < lc < self.ldq
        self.ldc = lc if self.narrow else self.ldq  # the checkpoint rows' stride
        # SB rows (narrow, the factor columns fill whole 512-B lane groups: fp32 K=128, fp64 K=64
        # / 128): the epoch kernel reads each item's bias from a mirror array (mf_log_apply's
        # bias_out keeps it) and the item rows are padded to whole 128-B lines, so a row gather
        # touches only the factor lines -- 4 instead of 5 at fp32 K=128 (C4 epoch kernel -9%,
        # profiles/r5u_probes.txt)
        self.sb_mirror = self.narrow and (self.K * esz) % 512 == 0 and bool(bias_mirror)
        if self.sb_mirror:
            per = 128 // esz
            self.ldq = -(-self.ldq // per) * per
        # (read-only after construction: elog is sized for it)
        self._err_in_row = (self.ckpt and not self.narrow and e0 + 2 <= self.ldq
                            and bool(err_in_row))
        if self.qlog_pp and self.dup_items:
            raise ValueError("qlog: a user lists an item twice (the q log reads each item row "
                             "once per rating from the chunk-start table)")
        # gram=True: the heaviest users by the blocked solve (mf_svd_epoch_gram: one workgroup
        # per user, the block's errors from its item-row Gram matrix) instead of the lookahead
        # body's chain, where the checkpoint rows carry their errors.  Off by default: equal to
        # the oracle to 1e-9, but measured slower (ML-1M fp64, the top user alone: 578 us vs the
        # lookahead chain's 187 us)
        self.gram = (self.ckpt and self._err_in_row and not self.narrow and not self.dup_items
                     and self.K >= 1 and bool(gram))
        # ... and then splits each chunk's users in two launches on two streams: the heaviest
        # users (their sequential chains bound a small epoch) beside the rest, whose log replay
        # then overlaps the heavy users' work
        if heavy is None:
            heavy = self._auto_heavy(row_ptr)
        # xcd_split: the heavy launch keeps to XCD 0 and the rest to the other seven (disjoint
        # L2s: the rest's log replay does not evict the heavy chains' item rows) -- where the
        # device deals workgroups round-robin over 8 XCDs (mf_xcd_layout), else no XCD masks;
        # None: split for the lookahead chains, not for the blocked solve (its heavy users finish
        # early, the rest then use every XCD)
        if xcd_split is None:
            xcd_split = not self.gram
        self.heavy_xcd = 1 if heavy > 0 and xcd_split and _lib.xcd_layout_ok() else 0
        C = _lib.load().mf_ckpt_interval() if self.ckpt else 0
        _pu = []
        pos_user = lambda: _pu[0] if _pu else _pu.append(position_users(row_ptr)) or _pu[0]
        # stagger (large chunks): two halves, B's epoch beside A's replay
        # (off by default: measured slower at C4 -- B's epoch beside A's replay 39.7 vs 29.6 ms
        # per epoch in fp32, 70.3 vs 53.3 in fp64, profiles/r5d_c4_stagger.txt)
        if stagger is None:
            stagger = False
        self.stagger = bool(stagger) and self.ckpt and heavy <= 0
        self.side = side_stream(torch, dev) if self.ckpt and (heavy > 0 or self.stagger) \
            else None
        # the top users of the heavy launch on the main stream, the rest of it on a third stream
        # (its replay and the pre-fold then overlap the top chains)
        if top is None:
            top = self.HEAVY_TOP_USERS
        self.top = (int(top) if self.side is not None and heavy >= 1 and int(top) > 0
                    and int(top) < heavy and not self.gram and join == "event" else 0)
        self.side2 = side_stream(torch, dev, 1) if self.top else None
        # the fork / join between the two streams as native events bound to the kernels that
        # complete them (mf_launch_event: no marker packet in the main stream's queue);
        # events="torch": torch.cuda.Event record / wait_event
        self._nev = None
        if self.side is not None and events == "native":
            self._nev = {k: _new_event() for k in ("fork", "join", "mid")}
            weakref.finalize(self, _free_events, list(self._nev.values()))
        self._fork_bound = False  # the last mf_log_apply on the main stream completes "fork"
        # the join as an event the main stream waits for; join="kernel": inside the two replays
        # instead (mf_launch_join: the heavy replay's last block waits for the light replay's;
        # no barrier packet before the fold) -- measured equal (the write-through stores of the
        # light replay cost what the barrier packet did), so off by default
        # the fold inside the replays (replay_fold): per-item piece counters and the launches'
        # arrival counters, zero between folds
        self.replay_fold = bool(replay_fold) and self.side is not None and join == "event" and \
            events == "native"
        self._fold_cnt = self._fold_words = None
        self._folded = False
        self.replay_folds_run = 0  # (chunks folded inside their replays)
        if self.replay_fold:
            self._fold_cnt = torch.zeros(max(self.n_items, 1), dtype=torch.int32, device=dev)
            self._fold_words = torch.zeros(_lib.MF_FOLD_WORDS, dtype=torch.int32, device=dev)
        self._join_words = None
        if self.side is not None and join == "kernel":
            self._join_words = torch.zeros(1024, dtype=torch.int32, device=dev)
            self._join_epoch = 0
        self.sched = []
        self._totals_local = []
        self.logs = []  # "log" mode: per chunk, the item grouping of the log (log_layout)
        for c in chunks:
            c = np.asarray(c, np.int32)
            if self.mode != _lib.MF_MODE_LOG:
                self.sched.append(to_dev(c))
                self._totals_local.append(
                    item_counts(c, row_ptr, items, self.n_items).astype(np.int32))
                continue
            if self.stagger:  # [B, A]: A (every other user from the first) runs first
                parts = [c[1::2], c[0::2]] if len(c) > 1 else [c]
            else:
                parts = split_groups(c, row_ptr, heavy, self.top) if self.side is not None \
                    else [c]
            # (recency, a split chunk: each rating's position among the chunk's ratings of its
            # item, indexed by CSR position; one group: its perm is already in that order)
            kpos = None
            if self.recency and len(parts) > 1:
                ks, pos = item_positions(row_ptr, items, c, self.n_items)
                kpos = np.zeros(int(row_ptr[-1]), np.int32)
                kpos[ks] = pos
            lgs = []
            for us in parts:
                rows = PIECE_ROWS
                if self.ckpt:
                    rows = replay_piece_rows(row_ptr, us) if replay_rows is None else \
                        max(1, int(replay_rows))
                perm, pb, ipp, cnt = log_layout(row_ptr, items, us, self.n_items, rows,
                                                local=self.qlog_pp)
                lg = dict(sched=to_dev(us), perm=to_dev(perm), pb=to_dev(pb), ipp=to_dev(ipp),
                          n_pieces=len(pb) - 1, cnt=cnt)
                if self.ckpt:
                    lg["ck"] = to_dev(ckpt_positions(row_ptr, perm, C, pos_user()))
                # the item of every piece (mf_log_replay's / mf_log_reduce's piece_item)
                lg["pitem"] = to_dev(np.repeat(np.arange(self.n_items, dtype=np.int32),
                                               np.diff(ipp)))
                if self.recency:
                    rp = kpos[perm] if kpos is not None else \
                        np.arange(len(perm), dtype=np.int64) - np.repeat(pb[ipp[:-1]], cnt)
                    lg["rpos"] = to_dev(rp.astype(np.int32))
                if self.qlog_pp and self.recency:  # (the fused fold's layout: with y's below)
                    lg["_fold_src"] = (cnt, perm, rp)
                lgs.append(lg)
            main = lgs[0]
            main["heavy"] = lgs[1] if len(lgs) > 1 else None
            main["mid"] = lgs[2] if len(lgs) > 2 else None  # (the heavy launch's rest, side2)
            self.sched.append(main["sched"])
            self.logs.append(main)
            self._totals_local.append(sum(lg.pop("cnt") for lg in lgs).astype(np.int32))
        self.counts = [to_dev(t) for t in self._totals_local]  # this rank's n_r per chunk
        # SVD++ in atomic mode: the end-of-user y update deferred to a per-item fold after each
        # chunk (mf_svdpp_y_fold; ydefer=False: float atomics at each user's end)
        self.ydefer = (algo == "svdpp" and (self.mode == _lib.MF_MODE_ATOMIC or self.qlog_pp)
                       and not self.deterministic and (bool(ydefer) or self.qlog_pp))
        # ... with helper waves (rows <= 1 KiB, no repeated items): one user chain per CU whose
        # q atomics the workgroup's other three waves issue (mf_svdpp_epoch flag
        # MF_EPOCH_SVDPP_HELPERS); the chains take users in a longest-first balanced layout
        self.hx = self.ydefer and self.ldq * esz <= 1024 and not self.dup_items and \
            (helpers is None or bool(helpers)) and not self.qlog_pp
        # helper waves per chain: 3 (helpers=True) or 1 (helpers=1: MF_EPOCH_SVDPP_ONE_HELPER);
        # None: by the users per epoch-chunk (HX_ONE_HELPER_MIN_USERS)
        if helpers is None:
            big = max((len(c) for c in self.sched), default=0) >= HX_ONE_HELPER_MIN_USERS
            self.hx_helpers = 1 if big else 3
        else:
            self.hx_helpers = 1 if helpers is not True and int(helpers) == 1 else 3
        self._hx_flags = _lib.MF_EPOCH_SVDPP_HELPERS | (
            _lib.MF_EPOCH_SVDPP_ONE_HELPER if self.hx_helpers == 1 else 0)
        self.hx_sched = []
        # the helper-wave launch's status word (mf_svdpp_epoch): checked in get_factors
        self._hx_status = torch.zeros(1, dtype=torch.int32, device=dev) if self.hx else None
        if self.hx:
            props = torch.cuda.get_device_properties(self.dev)
            cpc = (HX_CHAINS_PER_CU if self.hx_helpers == 3 else HX_CHAINS_PER_CU_ONE) \
                if hx_chains_per_cu is None else int(hx_chains_per_cu)
            self.hx_chains = max(1, cpc) * props.multi_processor_count
            for us in self.sched:
                self.hx_sched.append(to_dev(chain_schedule(us.cpu().numpy(), row_ptr,
                                                           self.hx_chains)))
        # ... and delta replicas of the most-rated items' rows (their serialised float atomics
        # bound the launch otherwise)
        hot = hot_items(items, self.n_items, hot_rows) if self.hx else np.zeros(0, np.int64)
        if len(hot) and 3 * self.n_items * self.ldq * esz >= (1 << 32):
            hot = hot[:0]  # (the replica rows must stay inside 32-bit buffer offsets)
        self.hot_list = to_dev(hot.astype(np.int32)) if len(hot) else None
        self.hot_flag = None
        if len(hot):
            flag = np.zeros(self.n_items, np.uint8)
            flag[hot] = 1
            self.hot_flag = to_dev(flag)
        # the hybrid launch (cold_share: one rank, three helper waves per chain)
        self.mix = []
        if cold_share and self.hx and self.hx_helpers == 3 and not self.multi:
            for c, us in enumerate(self.sched):
                cold = cold_items(self._totals_local[c], float(cold_share))
                if len(hot):
                    cold[hot] = False
                self.mix.append(mix_layout(row_ptr, items, us.cpu().numpy(), self.n_items, cold))
            rows = max(m["rows"] for m in self.mix)
            # (the cold log's and the q table's offsets, replicas included, share the helper
            # ring's 31 bits: beyond them the atomic launch runs)
            if max(rows, 2 * self.n_items) * self.ldq * esz >= (1 << 31) - 4096:
                self.mix = []
            for m in self.mix:
                for k in ("crow", "pb", "pitem", "ipp", "rpos", "totals"):
                    m[k] = to_dev(m[k])
                m["perm"] = torch.arange(max(m["rows"], 1), dtype=torch.int32, device=dev)
                m["n_pieces"] = int(m["pb"].numel()) - 1
        self.ycsc = []
        if self.ydefer:
            for us in self.sched:
                perm, pb, ipp, _ = log_layout(row_ptr, items, us.cpu().numpy(), self.n_items)
                iusr = pos_user()[perm]
                self.ycsc.append(dict(users=to_dev(iusr), pb=to_dev(pb), ipp=to_dev(ipp),
                                      n_pieces=len(pb) - 1, _iusr=iusr,
                                      pitem=to_dev(np.repeat(np.arange(self.n_items,
                                                                       dtype=np.int32),
                                                             np.diff(ipp)))))
            # the fused fold's per-chunk layout (q log, one rank): cold items' rows and raters
            # listed directly, hot items' in pieces (qlog_fold_layout)
            if self.qlog_pp and self.fused and self.recency:
                for c, (lg, y) in enumerate(zip(self.logs, self.ycsc)):
                    cnt, perm_c, rp = lg.pop("_fold_src")
                    iusr_c = y.pop("_iusr")
                    lay = qlog_fold_layout(cnt, perm_c, rp, iusr_c)
                    # (empty arrays padded to one entry: the kernel never reads past a range,
                    # and a null pointer would be refused)
                    lg["fold"] = {k: (to_dev(v if len(v) else np.zeros(1, v.dtype))
                                      if isinstance(v, np.ndarray) else v)
                                  for k, v in lay.items()}
            h = dict(hyper or {})
            decay = 1.0 - h.get("lr_yj", 0.0) * h.get("reg_yj", 0.0)
            # A_u = decay^{|I_u|} (the epoch kernel's per-user factor), fp64 on the host
            self.uA = to_dev(np.power(decay, np.diff(row_ptr).astype(np.float64))).to(self.tdt)
        self.totals = None  # set by _prepare(): summed over every rank
        self._pos0 = []  # (recency, several ranks: per chunk, the item counts of earlier ranks)
        # {sum pu^2, count} of the chunk start, double-buffered: chunk t accumulates into slot
        # t % 2 and its fold clears slot (t + 1) % 2 for the next chunk (no separate fill)
        # (+ MF_SQ_PARTS doubles of scratch: the fixed-range partial sums of user_sq that
        # mf_log_apply / mf_svdpp_qlog_fold / mf_user_sq_reduce add in order from 64k users)
        self._works = torch.zeros(2, 2 + _lib.MF_SQ_PARTS, dtype=torch.float64, device=dev)
        self._wt = 0
        self._work_cleared = True
        self.work = self._works[0]
        # checkpoint log: the epoch kernel keeps user_sq[u] = |p_u|^2 (factor columns) current, and
        # the next chunk's <pu^2> is its fixed-order sum, taken right after this chunk's epoch
        # kernels (mf_user_sq_reduce, off the step's critical path; no mf_sumsq pass)
        # (the SVD++ q log too: its kernel stores |p_u|^2 of the users it trains)
        self.user_sq = (torch.zeros(max(self.n_users, 1), dtype=torch.float64, device=dev)
                        if self.ckpt or self.qlog_pp or self.mix else None)
        self._sq_valid = self._sq_pending = False
        # several ranks, checkpoint log: the next chunk's <p^2> rode in this chunk's exchange
        # buffer (already every rank's sum: no collective of its own at the chunk start)
        self._stat_global = False

        # ---- factor tables
        U, I, ld, ldq = self.n_users, self.n_items, self.ld, self.ldq
        z = lambda *shape: torch.zeros(*shape, dtype=self.tdt, device=dev)
        self.pu, self.bu = z(U, ld), z(U)
        # (hot rows: the replica rows n_items .. 2 n_items - 1 of the same allocation, zero
        # between chunks; self.qb is the model's table, rows 0 .. n_items - 1)
        self._qb_alloc = z(2 * I if self.hot_list is not None else I, ldq)
        self.qb = self._qb_alloc[:I]
        self.ibias = z(max(I, 1)) if self.sb_mirror else None  # (qb[:, K]'s mirror, SB rows)
        # the hybrid launch's cold log and its piece sums
        self.clog = z(max(max(m["rows"] for m in self.mix), 1), ldq) if self.mix else None
        self.csums = z(max(max(m["n_pieces"] for m in self.mix), 1), ldq) if self.mix else None
        self.yj = z(I, ld) if algo == "svdpp" else None
        self.ycbuf = z(U, ld) if self.ydefer else None
        if self.ydefer:
            for y in self.ycsc:
                y.pop("_iusr", None)
            n_pc = max(1, max(y["n_pieces"] for y in self.ycsc))
            self.ypc_c, self.ypc_A = z(n_pc, ld), z(n_pc)
        self.fold_sums = None
        if self.qlog_pp and self.fused and self.recency:  # (the fused fold's hot-piece scratch)
            n_hp = max(1, max(lg["fold"]["n_hot_pieces"] for lg in self.logs))
            self.fold_sums = z(n_hp, ldq)
        # every user row on the device belongs to this rank (a rank-local CSR)
        self.u_lo, self.u_hi = 0, self.n_users
        self.qlog = None
        if self.mode == _lib.MF_MODE_LOG:
            k_lo, k_hi = int(row_ptr[self.u_lo]), int(row_ptr[self.u_hi])
            deg = np.diff(row_ptr)
            if len(deg) and int(deg.max()) * ldq * esz >= (1 << 30):
                raise _lib.SurpriseAMDError("a user's delta-log segment would exceed 1 GiB; "
                                            "use mode='atomic'")
            if self.ckpt:  # one packed row per pair of ratings (ck_row0)
                rows = int(ck_row0(row_ptr)[-1])
                if rows >= (1 << 30):
                    raise _lib.SurpriseAMDError("checkpoint log too large for 32-bit positions")
                self.qlog = z(max(rows, 1), self.ldc)
                self._qlog_base = self.qlog.data_ptr()
            elif self.qlog_pp:  # SVD++ q log: one chunk's rows (urow: each user's first row)
                urow = np.zeros(max(self.n_users, 1), np.int64)
                for us in self._chunk_users:
                    su, r0 = chunk_log_rows(row_ptr, us)
                    urow[su] = r0
                self.urow = to_dev(urow)
                self.qlog = z(max(max(int(t.sum()) for t in self._totals_local), 1), ldq)
                self._qlog_base = self.qlog.data_ptr()
            else:  # the gradient log: the kernels index it by absolute CSR position k
                self.qlog = z(max(k_hi - k_lo, 1), ldq)
                self._qlog_base = self.qlog.data_ptr() - k_lo * ldq * esz
            # per chunk: the main group's piece sums, then the heavy group's
            self.sums = z(max(lg["n_pieces"] + sum(lg[g]["n_pieces"] for g in ("heavy", "mid")
                                                   if lg.get(g))
                              for lg in self.logs), ldq)
            # three groups: the light + rest sums pre-folded per item while the top chains run
            self.sbuf = z(I, ldq) if any(lg.get("mid") for lg in self.logs) else None
            if self.ckpt:  # (errors in the rows: elog is never read or written)
                self.elog = z(64 if self.err_in_row else k_hi - k_lo + 64)
                self._elog_base = self.elog.data_ptr() - (0 if self.err_in_row else k_lo * esz)
        lbytes = self.qlog.numel() * self.qlog.element_size() if self.qlog is not None else 0
        # log_nt "heavy" / "light": only that launch group's log stores (split chunks)
        self._nt_group = log_nt if log_nt in ("heavy", "light") else None
        self.log_nt = (bool(log_nt) if log_nt is not None and self._nt_group is None
                       else lbytes >= self.LOG_NT_MIN_BYTES and self._nt_group is None)
        self.log_nt = self.log_nt and (self.ckpt or self.qlog_pp)
        snap_q = self.multi and self.mode != _lib.MF_MODE_LOG
        self.qb_s = z(I, ldq) if snap_q else None
        self.yj_s = z(I, ld) if (self.multi and self.yj is not None) else None
        self._delta = None
        self._hyper = _lib.MfHyper(**(hyper or {}))
        if not self.biased:
            self._hyper.global_mean = 0.0

    def epoch_launch_ratings(self, c):
        """Ratings each epoch-kernel launch of chunk c trains, in launch order (checkpoint log,
        split chunk: the heavy users' launch, then the light users'; else one launch)."""
        if self.ckpt and self.logs[c]["heavy"] is not None:
            out = [int(self.logs[c]["heavy"]["perm"].numel()), int(self.logs[c]["perm"].numel())]
            if self.logs[c].get("mid") is not None:
                out.append(int(self.logs[c]["mid"]["perm"].numel()))
            return out
        return [int(self._totals_local[c].sum())]

    @property
    def err_in_row(self):
        """Checkpoint log with each pair's errors in its row's padding (MF_EPOCH_ERR_IN_ROW)."""
        return self._err_in_row

    HEAVY_USERS = 128     # users in the heavy launch (measured: 64 0.231, 128 0.224, 256 0.232 ms)
    # `top` default: off.  Measured (profiles/r4m_*, r4n_*, r4o_*): the light users' epoch +
    # replay on the other XCDs take about as long as the top chain, so the pre-fold lands on the
    # critical path -- 0.35 ms/epoch fp64 with top = 16 / 32 / 64 against 0.29 without
    HEAVY_TOP_USERS = 0
    HEAVY_USERS_GRAM = 256  # ... with the blocked solve (one workgroup per user)
    HEAVY_MAX_NNZ = 8_000_000
    LOG_NT_MIN_BYTES = 2 << 30  # (logs at least this large: non-temporal log stores)

    def _auto_heavy(self, row_ptr):
        """The heavy/light XCD split pays where the epoch is bound by its longest user chains:
        small epochs (<= HEAVY_MAX_NNZ ratings per chunk) on a full 8-XCD MI355X (256 CUs); larger
        epochs are bandwidth-bound and would leave the heavy XCD idle."""
        if not self.ckpt or self.deterministic:
            return 0.0
        props = self.torch.cuda.get_device_properties(self.dev)
        nnz = int(row_ptr[-1] - row_ptr[0])
        if (props.multi_processor_count != 256 or nnz > self.n_chunks * self.HEAVY_MAX_NNZ
                or self.n_users < 16 * self.HEAVY_USERS):
            return 0.0
        return float(self.HEAVY_USERS_GRAM if self.gram else self.HEAVY_USERS)

    # ------------------------------------------------------------------ state in / out
    def set_factors(self, pu, qi, bu=None, bi=None, yj=None):
        """Upload host fp64 arrays (n, K) into the padded device tables."""
        self._fork_bound = False  # (the side stream must wait for this work)
        t = self.torch
        K = self.K

        def put(dst2d, src):
            dst2d.zero_()
            dst2d[:, :K].copy_(t.from_numpy(np.ascontiguousarray(src, np.float64)).to(
                self.dev, self.tdt))

        put(self.pu, pu)
        self.bu.copy_(t.from_numpy(np.zeros(self.n_users) if bu is None else
                                   np.asarray(bu, np.float64)).to(self.dev, self.tdt))
        put(self.qb, qi)
        self.qb[:, K].copy_(t.from_numpy(np.zeros(self.n_items) if bi is None else
                                         np.asarray(bi, np.float64)).to(self.dev, self.tdt))
        if self.algo == "svd" and self.is_log:  # (the lookahead body's user-bias column)
            self.qb[:, K + 1] = 1
        if self.ibias is not None:
            self.ibias.copy_(self.qb[:, K])
        if self.yj is not None:
            put(self.yj, yj)
        if self.qb_s is not None:
            self.qb_s.copy_(self.qb)
        if self.yj_s is not None:
            self.yj_s.copy_(self.yj)
        if self._hx_status is not None:  # (a re-seeded model starts with a clean status word)
            self._hx_status.zero_()
            self._hx_seen = None
        self._sq_valid = False

    def run_epochs(self, n_epochs, ctx=None, on_epoch=None):
        """ItemSync.run_epochs + the SVD++ helper-wave status word read at every epoch boundary
        without a sync: each epoch's end copies it to pinned host memory behind an event, and
        the next epoch boundary reads the copy once its event has completed -- a helper that
        timed out (lost q deltas) stops training within about an epoch instead of at
        get_factors."""
        if self._hx_status is None:
            return ItemSync.run_epochs(self, n_epochs, ctx, on_epoch)

        def boundary(epoch):
            self._check_hx_status(block=False)
            if on_epoch is not None:
                on_epoch(epoch)
        return ItemSync.run_epochs(self, n_epochs, ctx, boundary)

    def _check_hx_status(self, block):
        """Raise if a helper wave has reported MF_HX_HELPER_TIMEOUT; block=False reads only a copy
        whose event has completed and starts the next copy."""
        t = self.torch
        seen = getattr(self, "_hx_seen", None)
        if seen is not None and (block or seen[1].query()):
            seen[1].synchronize()
            if int(seen[0][0]) & _lib.MF_HX_HELPER_TIMEOUT:
                raise _lib.SurpriseAMDError(
                    "an SVD++ helper wave timed out waiting for q deltas and stopped: item "
                    "updates were lost (mf_svdpp_epoch status)")
            seen = None
        if seen is None and not block:
            host = t.empty(1, dtype=t.int32, pin_memory=True)
            with t.cuda.stream(self.stream):  # (the copy and its event on the engine's stream)
                host.copy_(self._hx_status, non_blocking=True)
                ev = t.cuda.Event()
                ev.record(self.stream)
            self._hx_seen = (host, ev)

    def get_factors(self, ctx=None):
        """Host fp64 copies (pu, qi, bu, bi, yj) with the padding columns dropped.  With ctx
        (several ranks) pu / bu are every rank's rows gathered in rank order (all ranks)."""
        self._fork_bound = False  # (the side stream must wait for this work)
        self.stream.synchronize()
        if getattr(self, "_join_words", None) is not None and int(self._join_words[608]) != 0:
            raise _lib.SurpriseAMDError("the in-kernel join of the two replays timed out: the "
                                        "item folds since are invalid")
        if getattr(self, "heavy_xcd", 0):  # (the XCD-masked launches' slot check)
            _lib.dispatch_check()
        if getattr(self, "_hx_status", None) is not None and \
                int(self._hx_status[0]) & _lib.MF_HX_HELPER_TIMEOUT:
            raise _lib.SurpriseAMDError("an SVD++ helper wave timed out waiting for q deltas and "
                                        "stopped: item updates were lost (mf_svdpp_epoch status)")
        K = self.K
        h = lambda x: x.to(self.torch.float64).cpu().numpy()
        pu, bu = self.pu[:, :K], self.bu
        if ctx is not None and ctx.world > 1:
            n = self.torch.tensor([self.n_users], dtype=self.torch.int64, device=self.dev)
            counts = ctx.all_gather_rows(n, [1] * ctx.world).cpu().tolist()
            pu = ctx.all_gather_rows(pu.contiguous(), counts)
            bu = ctx.all_gather_rows(bu, counts)
        out = dict(pu=h(pu), qi=h(self.qb[:, :K]), bu=h(bu), bi=h(self.qb[:, K]))
        out["yj"] = h(self.yj[:, :K]) if self.yj is not None else None
        return out

    # ------------------------------------------------------------------ kernels
    def _ptr(self, t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else None

    def _bias_out(self, apply):
        """mf_log_apply's bias_out: the SB epoch's item-bias mirror, where the fold moves b_i."""
        ib = getattr(self, "ibias", None)
        return self._ptr(ib) if apply and self.biased and ib is not None else None

    def _st(self):
        return ctypes.c_void_p(self.stream.cuda_stream)

    @property
    def is_log(self):
        return self.mode == _lib.MF_MODE_LOG

    def _epoch(self, sched, n_sched, n_waves, flags, st, xmask=0):
        qlog = ctypes.c_void_p(self._qlog_base) if self.is_log else None
        elog = ctypes.c_void_p(self._elog_base) if self.ckpt else None
        flags |= _lib.MF_EPOCH_DUP_ITEMS if self.dup_items else 0
        flags |= xmask << _lib.MF_EPOCH_XCD_SHIFT
        if self.algo == "svd":
            _lib.call("mf_svd_epoch", ctypes.byref(self._csr), self._ptr(sched), n_sched,
                      self._ptr(self.pu), self._ptr(self.bu), self.ld, self._ptr(self.qb),
                      self.ldq, self.K, int(self.biased), ctypes.byref(self._hyper), self.mode,
                      qlog, elog, n_waves, flags, self.dtype, st)
        elif self.qlog_pp:
            flags |= _lib.MF_EPOCH_LOG_NT if self.log_nt else 0
            _lib.call("mf_svdpp_epoch_qlog", ctypes.byref(self._csr), self._ptr(sched), n_sched,
                      self._ptr(self.pu), self._ptr(self.bu), self.ld, self._ptr(self.qb),
                      self.ldq, self._ptr(self.yj), self.K, ctypes.byref(self._hyper), qlog,
                      self._ptr(self.urow), self._ptr(self.ycbuf), self._ptr(self.user_sq),
                      n_waves, flags, self.dtype, st)
        elif self.mix and flags & _lib.MF_EPOCH_SVDPP_HELPERS:  # the hybrid launch
            _lib.call("mf_svdpp_epoch_mix", ctypes.byref(self._csr), self._ptr(sched), n_sched,
                      self._ptr(self.pu), self._ptr(self.bu), self.ld, self._ptr(self.qb),
                      self.ldq, self._ptr(self.yj), self.K, ctypes.byref(self._hyper),
                      self._ptr(self.clog), self._ptr(self.mix[self._chunk]["crow"]),
                      self._ptr(self.ycbuf), self._ptr(self.user_sq), n_waves, flags,
                      self._ptr(self._hx_status), self._ptr(self.hot_flag), self.dtype, st)
        else:
            _lib.call("mf_svdpp_epoch", ctypes.byref(self._csr), self._ptr(sched), n_sched,
                      self._ptr(self.pu), self._ptr(self.bu), self.ld, self._ptr(self.qb),
                      self.ldq, self._ptr(self.yj), self.K, ctypes.byref(self._hyper),
                      self.mode, qlog, self._ptr(self.ycbuf) if self.ydefer else None,
                      n_waves, flags, self._ptr(self._hx_status) if self.hx else None,
                      self._ptr(self.hot_flag) if self.hot_flag is not None and
                      flags & _lib.MF_EPOCH_SVDPP_HELPERS else None, self.dtype, st)

    def run_chunk(self, c: int, events=None):
        """Run chunk c: the epoch kernel, preceded in "log" mode by the <pu^2> reduction of the
        merge's count-aware weights (taken at the chunk start, like the oracle) and followed by
        the reduction of the chunk's log into per-piece sums (mf_log_reduce, or mf_log_replay
        for the checkpoint form); the fold into the table happens in sync_items.  A split chunk
        runs its heavy users' epoch + replay on the side stream beside the rest, joined before
        returning.  events: optional dict of torch.cuda.Event: "start" (main stream, before the
        epoch kernels), "end" (after the main epoch kernel), "end_h" (after the heavy one),
        "end_r" (after the log replay / reduce / y fold that follow the epoch kernel);
        checkpoint log, split chunk: "l_start" / "l_end" around the light users' epoch kernel
        on the side stream."""
        torch = self.torch
        s = self.sched[c]
        st = self._st()
        ev = events or {}
        self._chunk = c
        if self.ckpt:
            self._run_chunk_ckpt(c, ev)
            return
        if self.qlog_pp or self.mix:  # <p^2> of the chunk start from user_sq (as the ckpt log)
            self._sq_prologue(st)
        elif self.is_log:
            self.work = self._works[self._wt % 2]
            self._wt += 1
            if not self._work_cleared:  # (the last chunk was not folded through mf_log_apply)
                self.work.zero_()
            self._work_cleared = False
            _lib.call("mf_sumsq", ctypes.c_void_p(self.pu.data_ptr() +
                                                  self.u_lo * self.ld * self.pu.element_size()),
                      self.u_hi - self.u_lo, self.K, self.ld, self._ptr(self.work), self.dtype,
                      st)
            self._global_stat()  # (several ranks: every rank's <p^2>)
        if "start" in ev:
            ev["start"].record(self.stream)
        lg = self.logs[c] if self.is_log else None
        hv = lg["heavy"] if lg is not None else None
        if hv is not None:  # heavy users: their own launch (one wave each) on the side stream
            fork = torch.cuda.Event()
            fork.record(self.stream)
            self.side.wait_event(fork)
            sh = ctypes.c_void_p(self.side.cuda_stream)
            n_h = hv["sched"].numel()
            self._epoch(hv["sched"], n_h, n_h, 0, sh, self.heavy_xcd)
            if "end_h" in ev:
                ev["end_h"].record(self.side)
            self._reduce_log(hv, self.sums.data_ptr() +
                             lg["n_pieces"] * self.ldq * self.sums.element_size(), sh)
            join = torch.cuda.Event()
            join.record(self.side)
        lx = (~self.heavy_xcd & 0xFF) if hv is not None and self.heavy_xcd else 0
        if self.hx:
            hs = self.hx_sched[c]
            self._epoch(hs, hs.numel(), self.hx_chains, self._hx_flags, st)
            if self.hot_list is not None:
                _lib.call("mf_svdpp_hot_fold", self._ptr(self.qb), self.ldq, self.n_items,
                          self._ptr(self.hot_list), self.hot_list.numel(), self.dtype, st)
            if self.mix:
                self._cold_fold(c, st)
        else:
            self._epoch(s, s.numel(), self.n_waves, 0, st, lx)
        if "end" in ev:
            ev["end"].record(self.stream)
        if self._q_early():  # (several ranks: q's part of the exchange overlaps the y fold)
            self._exchange_q_begin()
        if self._fused_fold():  # (q log, one rank: the whole fold in _merge_local)
            if "end_r" in ev:
                ev["end_r"].record(self.stream)
            return
        if self.ydefer:
            y = self.ycsc[c]
            _lib.call("mf_svdpp_y_fold", self._ptr(self.yj), self.ld, self.K,
                      self._ptr(self.ycbuf), self._ptr(self.uA), self._ptr(y["users"]),
                      self._ptr(y["pb"]), y["n_pieces"], self._ptr(y["ipp"]), self.n_items,
                      self._ptr(self.ypc_c), self._ptr(self.ypc_A), self._ptr(y["pitem"]),
                      self.dtype, st)
        if lg is not None:
            self._reduce_log(lg, self.sums.data_ptr(), st, lx)
        if hv is not None:
            self.stream.wait_event(join)
        if "end_r" in ev:
            ev["end_r"].record(self.stream)

    def _cold_fold(self, c, st):
        """The hybrid launch's cold items after chunk c: their logged gradients summed per piece
        with the recency weights (mf_log_reduce over the item-grouped cold log), then each cold
        item's step (mf_log_apply with the cold items' counts: a live item's count is 0, its row
        untouched); the same launch sums user_sq into the next chunk's <p^2>."""
        m = self.mix[c]
        if m["n_pieces"] > 0:
            totals = self._totals()[c]
            rec = _lib.MfRecency(m["rpos"].data_ptr(), None, totals.data_ptr(),
                                 self.work.data_ptr())
            _lib.call("mf_log_reduce", self._ptr(self.clog), self.ldq, self.K + 1,
                      self._ptr(m["perm"]), self._ptr(m["pb"]), m["n_pieces"],
                      self._ptr(self.csums), self._ptr(m["pitem"]), ctypes.byref(self._hyper),
                      ctypes.byref(rec), self.dtype, st)
        _lib.call("mf_log_apply", self._ptr(self.qb), self.n_items, self.ldq, self.K,
                  self._bias_col, self._ptr(self.csums), self._ptr(m["ipp"]), None, None,
                  self._ptr(m["totals"]), ctypes.byref(self._hyper), self._ptr(self.work),
                  _lib.MF_MERGE_RECENCY, None, 1, *self._stat_args(True), None, self.dtype, st)

    def _epoch_sq(self, sched, n_sched, n_waves, st, xmask=0, group=None):
        """The checkpoint-log epoch kernel keeping user_sq current (mf_svd_epoch_sq); group: the
        split chunk's launch group ("heavy" / "light"), for log_nt's per-group form."""
        nt = self.log_nt or (group is not None and group == self._nt_group)
        _lib.call("mf_svd_epoch_sq", ctypes.byref(self._csr), self._ptr(sched), n_sched,
                  self._ptr(self.pu), self._ptr(self.bu), self.ld, self._ptr(self.qb), self.ldq,
                  self.K, int(self.biased), ctypes.byref(self._hyper),
                  ctypes.c_void_p(self._qlog_base), ctypes.c_void_p(self._elog_base),
                  self._ptr(self.user_sq), self._ptr(self.ibias), n_waves,
                  (_lib.MF_EPOCH_DUP_ITEMS if self.dup_items else 0) |
                  (_lib.MF_EPOCH_ERR_IN_ROW if self.err_in_row else 0) |
                  (_lib.MF_EPOCH_CKPT_NARROW if self.narrow else 0) |
                  (_lib.MF_EPOCH_LOG_NT if nt else 0) |
                  (xmask << _lib.MF_EPOCH_XCD_SHIFT), self.dtype, st)

    def _heavy_epoch(self, sched, n_sched, st, xmask=0):
        """The heavy users' epoch launch: the blocked solve (gram) or one lookahead chain per
        user."""
        if not self.gram:
            self._epoch_sq(sched, n_sched, n_sched, st, xmask, group="heavy")
            return
        _lib.call("mf_svd_epoch_gram", ctypes.byref(self._csr), self._ptr(sched), n_sched,
                  self._ptr(self.pu), self._ptr(self.bu), self.ld, self._ptr(self.qb), self.ldq,
                  self.K, int(self.biased), ctypes.byref(self._hyper),
                  ctypes.c_void_p(self._qlog_base), self._ptr(self.user_sq), 0,
                  xmask << _lib.MF_EPOCH_XCD_SHIFT, self.dtype, st)

    def _sq_reduce(self, out, st):
        _lib.call("mf_user_sq_reduce", self._ptr(self.user_sq), self.n_users, self.K,
                  self._ptr(out), st)

    def _run_chunk_ckpt(self, c, ev):
        """run_chunk for the checkpoint log.  <pu^2> of this chunk's start is in work slot t % 2:
        summed from user_sq by the previous chunk's mf_log_apply (or here, at the first chunk
        after set_factors or after a chunk that was not folded); the epoch kernels keep user_sq
        current and this chunk's mf_log_apply sums slot (t + 1) % 2.  A split chunk runs on two
        streams: the heavy users' epoch + replay on the main stream (the longest path, no waits
        inside it), the light users' epoch + replay on the side stream after a fork from the
        main stream; the main stream joins the side stream at the end."""
        torch = self.torch
        st = self._st()
        launched = self._sq_prologue(st)
        fork_bound, self._fork_bound = self._fork_bound and not launched, False
        if "start" in ev:
            ev["start"].record(self.stream)
        lg = self.logs[c]
        hv = lg["heavy"]
        sums_h = self.sums.data_ptr() + lg["n_pieces"] * self.ldq * self.sums.element_size()
        ls, ln, lw = lg["sched"], lg["sched"].numel(), self.n_waves
        if hv is None:
            self._epoch_sq(ls, ln, lw, st)
            if "end" in ev:
                ev["end"].record(self.stream)
            self._reduce_log(lg, self.sums.data_ptr(), st)
        elif self.stagger:
            # main: A's epoch, then A's replay; side (after A's epoch): B's epoch, B's replay --
            # B's epoch kernel runs beside A's replay; main joins side before the fold
            side = self.side
            sh = ctypes.c_void_p(side.cuda_stream)
            self._epoch_sq(hv["sched"], hv["sched"].numel(), lw, st, group="heavy")
            if "end" in ev:
                ev["end"].record(self.stream)
            a_done = torch.cuda.Event()
            a_done.record(self.stream)
            side.wait_event(a_done)
            if "l_start" in ev:
                ev["l_start"].record(side)
            self._epoch_sq(ls, ln, lw, sh, group="light")
            if "l_end" in ev:
                ev["l_end"].record(side)
            self._reduce_log(lg, self.sums.data_ptr(), sh)
            b_done = torch.cuda.Event()
            b_done.record(side)
            self._reduce_log(hv, sums_h, st)
            self.stream.wait_event(b_done)
        elif lg.get("mid") is not None:
            self._run_chunk_three(lg, ev, st, fork_bound)
        else:
            side = self.side
            sh = ctypes.c_void_p(side.cuda_stream)
            lx = (~self.heavy_xcd & 0xFF) if self.heavy_xcd else 0
            if self._nev is None:
                self._ev_record("fork", self.stream)
                self._ev_wait(side, "fork")
            else:  # (bound to the previous chunk's mf_log_apply unless a kernel followed it)
                if not fork_bound:
                    _lib.call("mf_event_record", self._nev["fork"], st)
                _lib.call("mf_stream_wait_event", sh, self._nev["fork"])
            n_h = hv["sched"].numel()  # (the longest path first: the host may lag the GPU)
            self._heavy_epoch(hv["sched"], n_h, st, self.heavy_xcd)
            if "end" in ev:
                ev["end"].record(self.stream)
            if "l_start" in ev:  # (the light epoch kernel's own span, on its stream)
                ev["l_start"].record(side)
            self._epoch_sq(ls, ln, lw, sh, lx, group="light")
            if "l_end" in ev:
                ev["l_end"].record(side)
            jw = self._join_words
            if jw is not None:
                self._join_epoch = (self._join_epoch + 1) & 0xFFFFFFFF
                _lib.call("mf_launch_join", self._ptr(jw), 1, self._join_epoch)
            elif self._nev is not None:
                _lib.call("mf_launch_event", self._nev["join"])  # completed by the light replay
            folds = self._replay_folds(c, lg, hv, sums_h)
            if folds:
                _lib.call("mf_launch_fold", ctypes.byref(folds[0]))
            self._reduce_log(lg, self.sums.data_ptr(), sh, lx, self.light_replay_wpc)
            if jw is None and self._nev is None:
                self._ev_record("join", side)
            # (the heavy replay starts when the longest chain ends: by then the light users'
            # work is (nearly) done, so it may spread over every XCD)
            if jw is not None:  # (it ends once the light replay of this chunk has published)
                _lib.call("mf_launch_join", self._ptr(jw), 2, self._join_epoch)
            if folds:  # (the heavy replay completes "fork": the item table is final after it
                # and after the light replay, which the side stream runs before its next epoch)
                self._bind_fork()
                _lib.call("mf_launch_fold", ctypes.byref(folds[1]))
                self._folded = True
                self.replay_folds_run += 1
            self._reduce_log(hv, sums_h, st)
            if jw is None and self._nev is None:
                self._ev_wait(self.stream, "join")
            elif jw is None:
                _lib.call("mf_stream_wait_event", st, self._nev["join"])
        if "end_r" in ev:
            ev["end_r"].record(self.stream)

    def _run_chunk_three(self, lg, ev, st, fork_bound):
        """A chunk split in three (top): main stream = the top heavy users' epoch (XCD 0), then
        their replay; side2 = the rest of the heavy users' epoch and replay (XCD 1); side = the
        light users' epoch and replay (XCDs 2-7), then -- after side2's replay -- a first fold of
        the light + rest piece sums into sbuf (mf_log_apply, apply=0).  The main stream joins
        the side stream before the chunk's fold, which then adds only the top users' pieces."""
        side, side2 = self.side, self.side2
        sh, sh2 = ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(side2.cuda_stream)
        # XCD 0: the top chains alone; XCD 1: the rest of the heavy users (sharing XCD 0 put
        # two chains on a SIMD: the top launch 239 -> 367 us); XCDs 2-7: the light users
        mx = 0x02 if self.heavy_xcd else 0
        lx = (~(self.heavy_xcd | mx) & 0xFF) if self.heavy_xcd else 0
        hv, md = lg["heavy"], lg["mid"]
        esz = self.sums.element_size()
        sums_l = self.sums.data_ptr()
        sums_h = sums_l + lg["n_pieces"] * self.ldq * esz
        sums_m = sums_h + hv["n_pieces"] * self.ldq * esz
        native = self._nev is not None
        if not native:
            self._ev_record("fork", self.stream)
            self._ev_wait(side, "fork")
            self._ev_wait(side2, "fork")
        else:  # (bound to the previous chunk's mf_log_apply unless a kernel followed it)
            if not fork_bound:
                _lib.call("mf_event_record", self._nev["fork"], st)
            _lib.call("mf_stream_wait_event", sh, self._nev["fork"])
            _lib.call("mf_stream_wait_event", sh2, self._nev["fork"])
        self._epoch_sq(hv["sched"], hv["sched"].numel(), hv["sched"].numel(), st, self.heavy_xcd)
        if "end" in ev:
            ev["end"].record(self.stream)
        if "m_start" in ev:
            ev["m_start"].record(side2)
        self._epoch_sq(md["sched"], md["sched"].numel(), md["sched"].numel(), sh2, mx)
        if "m_end" in ev:
            ev["m_end"].record(side2)
        if native:
            _lib.call("mf_launch_event", self._nev["mid"])  # completed by the rest's replay
        self._reduce_log(md, sums_m, sh2, lx | mx)  # (XCDs 1-7: by then the light epoch is done)
        if not native:
            self._ev_record("mid", side2)
        if "l_start" in ev:
            ev["l_start"].record(side)
        ls = lg["sched"]
        self._epoch_sq(ls, ls.numel(), self.n_waves, sh, lx)
        if "l_end" in ev:
            ev["l_end"].record(side)
        self._reduce_log(lg, sums_l, sh, lx)
        if native:
            _lib.call("mf_stream_wait_event", sh, self._nev["mid"])
            _lib.call("mf_launch_event", self._nev["join"])  # completed by the pre-fold
        else:
            self._ev_wait(side, "mid")
        _lib.call("mf_log_apply", self._ptr(self.qb), self.n_items, self.ldq, self.K,
                  self._bias_col, ctypes.c_void_p(sums_l), self._ptr(lg["ipp"]),
                  ctypes.c_void_p(sums_m), self._ptr(md["ipp"]),
                  self._ptr(self._totals()[self._chunk]), ctypes.byref(self._hyper),
                  self._ptr(self.work), self._log_rule(), self._ptr(self.sbuf), 0, None, None, 0,
                  None, self.dtype, sh)
        if not native:
            self._ev_record("join", side)
        self._reduce_log(hv, sums_h, st)  # (the top users' replay: every XCD)
        if native:
            _lib.call("mf_stream_wait_event", st, self._nev["join"])
        else:
            self._ev_wait(self.stream, "join")

    def _sq_prologue(self, st):
        """The chunk-start <p^2> into work slot t % 2 from user_sq (kept current by the epoch
        kernels): summed by the previous chunk's mf_log_apply, or here at the first chunk after
        set_factors / after a chunk that was not folded.  True if it launched a kernel."""
        cur = self._works[self._wt % 2]
        self._wt += 1
        self.work = cur
        self._work_cleared = True  # (written, never accumulated: nothing to clear)
        launched = True  # (a kernel on the main stream after the last mf_log_apply)
        if not self._sq_valid:
            _lib.call("mf_user_sq", self._ptr(self.pu), self.n_users, self.K, self.ld,
                      self._ptr(self.user_sq), self.dtype, st)
            self._sq_reduce(cur, st)
            self._sq_valid = True
            self._stat_global = False  # (a local partial again: _global_stat sums it)
        elif self._sq_pending:  # (the previous chunk was not folded by mf_log_apply)
            self._sq_reduce(cur, st)
            self._stat_global = False
        else:
            launched = False
        launched = self._global_stat() or launched  # (several ranks: every rank's <p^2>)
        self._sq_pending = True
        return launched

    def _ev_record(self, name, stream):
        """Record the engine's cross-stream event `name` on stream."""
        evs = self.__dict__.setdefault("_events", {})
        evs[name] = self.torch.cuda.Event()
        evs[name].record(stream)

    def _ev_wait(self, stream, name):
        stream.wait_event(self._events[name])

    def _reduce_log(self, lg, sums_ptr, st, xmask=0, wpc=0):
        """Piece sums of one user group's log: mf_log_replay (checkpoint form) or mf_log_reduce.
        xmask: run on those XCDs only (bit x: XCD x; 0: all); wpc: the replay's waves per CU
        (0: the library's default)."""
        rec = self._recency_args(lg)
        if self.ckpt:
            _lib.call("mf_log_replay", ctypes.c_void_p(self._qlog_base),
                      ctypes.c_void_p(self._elog_base), self.ldq, self.K, ctypes.byref(self._csr),
                      self._ptr(self.qb), ctypes.byref(self._hyper), self._ptr(lg["perm"]),
                      self._ptr(lg["ck"]), self._ptr(lg["pb"]), lg["n_pieces"],
                      ctypes.c_void_p(sums_ptr), self._ptr(lg["pitem"]), rec,
                      (xmask << _lib.MF_EPOCH_XCD_SHIFT) | (int(wpc) << _lib.MF_REPLAY_WPC_SHIFT) |
                      (_lib.MF_EPOCH_ERR_IN_ROW if self.err_in_row else 0) |
                      (_lib.MF_EPOCH_CKPT_NARROW if self.narrow else 0), self.dtype, st)
        else:
            _lib.call("mf_log_reduce", ctypes.c_void_p(self._qlog_base), self.ldq, self.K + 1,
                      self._ptr(lg["perm"]), self._ptr(lg["pb"]), lg["n_pieces"],
                      ctypes.c_void_p(sums_ptr), self._ptr(lg["pitem"]),
                      ctypes.byref(self._hyper), rec, self.dtype, st)

    def _recency_args(self, lg):
        """mf_recency_t of one user group's log in the current chunk (None: no recency)."""
        if not self.recency:
            return None
        c = getattr(self, "_chunk", 0)
        totals = self._totals()[c]  # (prepares the per-item counts on first use)
        pos0 = self._pos0[c] if self._pos0 else None
        rec = _lib.MfRecency(lg["rpos"].data_ptr(), pos0.data_ptr() if pos0 is not None else None,
                             totals.data_ptr(), self.work.data_ptr())
        return ctypes.byref(rec)

    def _global_stat(self):
        """Several ranks: the chunk-start <p^2> partial in self.work summed over every rank before
        the chunk's replay / reduce reads it (the recency weights) -- one 2-double all-reduce on
        the main stream; True if it launched one."""
        ctx = self._ctx
        if not self._exchanging(ctx) or not self.is_log:
            return False
        if self._stat_global:  # (summed by the previous chunk's exchange)
            self._stat_global = False
            return False
        ctx.all_reduce_sum(self.work[:2])
        return True

    def _prepare(self, ctx):
        """Global per-item rating counts of every chunk (all ranks) for the count-aware rules;
        with SVD++ on several ranks, the per-item factors of the y_j affine merge (dist.py)."""
        self._ctx = ctx
        self.totals = []
        self._pos0 = []
        self._after = []  # (snapshot merge by recency: per chunk, the item counts of later ranks)
        snap_rec = not self.is_log and self.merge_rule == "recency"
        for t in self._totals_local:
            tt = self.torch.from_numpy(t).to(self.dev)
            if self._exchanging(ctx):
                if self.recency or snap_rec:
                    # this rank's ratings of an item follow the earlier ranks' and precede the
                    # later ranks'
                    every = ctx.all_gather_rows(tt[None].to(self.torch.int64),
                                                [1] * ctx.world).cpu()
                    to32 = lambda x: x.to(self.torch.int32).to(self.dev)
                    if self.recency:
                        self._pos0.append(to32(every[:ctx.rank].sum(0)))
                    else:
                        self._after.append(to32(every[ctx.rank + 1:].sum(0)))
                ctx.all_reduce_sum(tt)
            self.totals.append(tt)
        self._yaff = []
        if self.yj_s is not None and self._exchanging(ctx):
            from .dist import item_log_decay
            torch = self.torch
            h = self._hyper
            decay = 1.0 - h.lr_yj * h.reg_yj
            for us in self._chunk_users:
                la = torch.from_numpy(item_log_decay(us, self._row_ptr_h, self._items_h,
                                                     self.n_items, decay))
                every = ctx.all_gather_rows(la[None].to(self.dev), [1] * ctx.world).cpu()
                suffix = torch.flip(torch.cumsum(torch.flip(every, [0]), 0), [0])  # sum_{s>=r}
                s_r = suffix[ctx.rank + 1] if ctx.rank + 1 < ctx.world else torch.zeros_like(la)
                to = lambda x: torch.exp(x).to(self.dev, self.tdt)
                self._yaff.append(dict(a=to(la), s=to(s_r), a_all=to(suffix[0])))

    def _totals(self):
        """Per-item rating counts of every chunk over all ranks (a single rank: its own)."""
        if self.totals is None:
            self._prepare(None)
        return self.totals

    @property
    def _bias_col(self):
        """Item-row column of b_i for mf_log_apply (-1: unbiased, the column never moves)."""
        return self.K if self.biased else -1

    def _count_rule(self):
        if self.merge_rule == "count" and self.totals is None:
            self._prepare(None)
        return self.merge_rule == "count"

    def _snap_rule(self):
        """mf_item_merge's rule for the snapshot tables (several ranks, not the log)."""
        return {"count": _lib.MF_MERGE_COUNT, "recency": _lib.MF_MERGE_RECENCY,
                "sum": _lib.MF_MERGE_SUM}[self.merge_rule]

    def _log_rule(self):
        """mf_log_apply's merge rule."""
        if self.merge_rule != "sum" and self.totals is None:
            self._prepare(None)
        return {"count": _lib.MF_MERGE_COUNT, "recency": _lib.MF_MERGE_RECENCY,
                "sum": _lib.MF_MERGE_SUM}[self.merge_rule]

    def _log_fold(self, delta_out, apply, stat=None):
        """mf_log_apply of the current chunk (its pieces were reduced in run_chunk); stat: also
        sum the next chunk's <p^2> (default: when it applies)."""
        c = getattr(self, "_chunk", 0)
        lg = self.logs[c]
        hv = lg["heavy"]
        sums2 = (ctypes.c_void_p(self.sums.data_ptr() + lg["n_pieces"] * self.ldq *
                                 self.sums.element_size()) if hv is not None else None)
        if apply:
            self._bind_fork()
        three = lg.get("mid") is not None  # (the light + rest sums already folded into sbuf)
        _lib.call("mf_log_apply", self._ptr(self.qb), self.n_items, self.ldq, self.K,
                  self._bias_col, self._ptr(self.sbuf if three else self.sums),
                  None if three else self._ptr(lg["ipp"]), sums2,
                  self._ptr(hv["ipp"]) if hv is not None else None,
                  self._ptr(self._totals()[c]), ctypes.byref(self._hyper),
                  self._ptr(self.work), self._log_rule(),
                  None if delta_out is None else self._ptr(delta_out), int(apply),
                  *self._stat_args(apply if stat is None else stat),
                  self._bias_out(apply), self.dtype, self._st())

    def _replay_folds(self, c, lg, hv, sums_h):
        """mf_fold_t of the light (role 1) and heavy (role 2) replays of split chunk c when the
        fold runs inside them (replay_fold), else None."""
        if not (self.replay_fold and self.ckpt and self.is_log and self.user_sq is not None
                and self.n_users < _lib.MF_SQ_PARTS_MIN and self.recency
                and not self._exchanging(self._ctx)):
            return None
        stat_next, user_sq, n_users = self._stat_args(True)
        bo = self._bias_out(True)
        out = []
        for role in (1, 2):
            out.append(_lib.MfFold(
                self.qb.data_ptr(), self.ldq, self.K, self._bias_col, self._log_rule(),
                self.sums.data_ptr(), lg["ipp"].data_ptr(), sums_h, hv["ipp"].data_ptr(),
                self._totals()[c].data_ptr(), ctypes.addressof(self._hyper),
                self.work.data_ptr(), _vp_int(stat_next), _vp_int(user_sq), n_users,
                _vp_int(bo), self._fold_cnt.data_ptr(), self._fold_words.data_ptr(), role, 2))
        return out

    def _bind_fork(self):
        """The next mf_log_apply completes the "fork" event the side stream waits for (the item
        table the next chunk's light users read); call right before that launch."""
        if self._nev is not None:
            _lib.call("mf_launch_event", self._nev["fork"])
            self._fork_bound = True

    def _stat_args(self, apply):
        """mf_log_apply's (stat_next, user_sq, n_users): the next chunk's <pu^2> slot -- summed
        from user_sq inside the launch (checkpoint log) or cleared for mf_sumsq."""
        if not apply:
            return None, None, 0
        if self.user_sq is not None:
            self._sq_pending = False
            return self._ptr(self._works[self._wt % 2]), self._ptr(self.user_sq), self.n_users
        return self._next_work(), None, 0

    def _next_work(self):
        """The next chunk's <pu^2> accumulator, cleared by this chunk's mf_log_apply."""
        self._work_cleared = True
        return self._ptr(self._works[self._wt % 2])

    def _snap_tables(self):
        """(table, snapshot, ld, bias_col, rule) of the tables merged by snapshot deltas."""
        self._count_rule()  # (prepares the counts)
        tabs = []
        if self.qb_s is not None:
            tabs.append((self.qb, self.qb_s, self.ldq, self.K, self._snap_rule()))
        if self.yj_s is not None:
            # SVD++ implicit factors: the ranks' end-of-user affine maps composed in rank order
            # (mf_item_affine, dist.py)
            tabs.append((self.yj, self.yj_s, self.ld, -1, "affine"))
        return tabs

    def _fused_fold(self):
        """SVD++ q log on one rank: reduce + apply + y composition in one launch."""
        return self.qlog_pp and self.fused and self.recency and not self._exchanging(self._ctx)

    def _merge_local(self):
        if self._folded:  # (the fold ran inside the chunk's replays: replay_fold)
            self._folded = False
            return
        if self._fused_fold():
            c = getattr(self, "_chunk", 0)
            f = self.logs[c]["fold"]
            p = lambda k: f[k].data_ptr()
            lay = _lib.MfQlogFold(p("perm"), p("rpos"), p("item_row_beg"), p("users"),
                                  p("hot_perm"), p("hot_rpos"),
                                  p("hot_users"), p("hot_piece_beg"), p("hot_piece_item"),
                                  p("hot_item_piece_ptr"), int(f["n_hot_pieces"]),
                                  self.fold_sums.data_ptr(), self.ypc_c.data_ptr(),
                                  self.ypc_A.data_ptr())
            _lib.call("mf_svdpp_qlog_fold", self._ptr(self.qb), self.ldq, self.K,
                      self._ptr(self.yj), self.ld, ctypes.c_void_p(self._qlog_base),
                      ctypes.byref(lay), self._ptr(self._totals()[c]), self._ptr(self.work),
                      ctypes.byref(self._hyper), self._ptr(self.ycbuf), self._ptr(self.uA),
                      self.n_items, *self._stat_args(True), self.dtype, self._st())
            return
        if self.is_log:
            self._log_fold(None, True)

    def sync_items(self, ctx):
        """The chunk's item-side exchange: one rank folds locally; several ranks fill ONE packed
        buffer (the log sums, or q's and y's snapshot deltas side by side), SUM-all-reduce it
        once and apply it: one RCCL collective per chunk (the checkpoint log's next <p^2> rides in
        the buffer; the gradient log, ckpt=False, all-reduces its <p^2> at the chunk start -- a
        second, 16-byte collective).
        self._sync_events (dict of "ar_begin" / "ar_end" torch events, set by bench.py's
        instrumented epochs) brackets the collective on the engine's stream."""
        if not self._exchanging(ctx):
            self._merge_local()
            return
        flat, bufs = self._delta_buffer()
        if self._q_work is not None:  # q's part went out after the epoch kernel: y's part now
            ev = getattr(self, "_sync_events", None)
            if ev:  # (the exchange's time left on the critical path, after the y fold)
                ev["ar_begin"].record(self.stream)
            self._delta_into(bufs, which=(1,))
            ctx.all_reduce_sum(bufs[1])
            with self.torch.cuda.stream(self.stream):
                self._q_work.wait()
            self._q_work = None
            if ev:
                ev["ar_end"].record(self.stream)
            self._apply(bufs)
            return
        self._delta_into(bufs)
        ride = self._stat_rides()
        if ride:  # the next chunk's <p^2> partial (summed by _delta_into) rides in the buffer
            flat[-2:].copy_(self._works[self._wt % 2][:2])
        ev = getattr(self, "_sync_events", None)
        if ev:
            ev["ar_begin"].record(self.stream)
        ctx.all_reduce_sum(flat)
        if ev:
            ev["ar_end"].record(self.stream)
        if ride:
            self._works[self._wt % 2][:2].copy_(flat[-2:])
            self._stat_global = True
        self._apply(bufs)

    def _stat_rides(self):
        """Several ranks, checkpoint log: the next chunk's <p^2> is summed from user_sq by this
        chunk's first mf_log_apply (apply = 0, before the all-reduce) and rides in the exchange
        buffer's last two elements -- one collective per chunk instead of two."""
        return self.user_sq is not None and self.multi

    def _q_early(self):
        """SVD++'s atomic schedule on several ranks over a device transport (RCCL): q's snapshot
        delta is ready when the epoch kernel ends, so its all-reduce (async, RCCL's own stream)
        runs while mf_svdpp_y_fold runs; y's part follows in sync_items.  The same arithmetic
        as the one-buffer exchange (two collectives instead of one); host-staged gloo keeps
        the single buffer."""
        ctx = self._ctx
        return (self.overlap_q and self._exchanging(ctx) and not ctx.host_staged
                and self.qb_s is not None and self.yj_s is not None and self.ydefer)

    def _exchange_q_begin(self):
        flat, bufs = self._delta_buffer()
        self._delta_into(bufs, which=(0,))
        with self.torch.cuda.stream(self.stream):
            self._q_work = self._ctx.all_reduce_sum_async(bufs[0])

    def _exchanging(self, ctx):
        """The chunk's item-side updates go through the packed all-reduce (several ranks, or
        the test-only `exchange=True` at world 1) rather than the local fold."""
        return ctx is not None and (ctx.world > 1 or self.multi)

    def _delta_buffer(self):
        """(flat, views): one device buffer holding [log sums (log mode)] + [one delta per
        snapshot table] -- the chunk's whole exchange is one all-reduce."""
        if self._delta is None:
            sizes = ([self.n_items * self.ldq] if self.is_log else []) + \
                [self.n_items * ld for _, _, ld, _, _ in self._snap_tables()] + \
                ([2] if self._stat_rides() else [])
            flat = self.torch.zeros(sum(sizes), dtype=self.tdt, device=self.dev)
            views, o = [], 0
            for n in sizes:
                views.append(flat[o:o + n])
                o += n
            self._delta = (flat, views)
        return self._delta

    def _delta_into(self, bufs, which=None):
        """Fill the exchange buffer's parts (which: the indices of the snapshot tables to fill,
        None = every part)."""
        c = getattr(self, "_chunk", 0)
        st = self._st()
        x = 0
        if self.is_log:  # (self.work already holds every rank's <p^2>: _global_stat)
            self._log_fold(bufs[0], False, stat=self._stat_rides())
            x = 1
        for ti, (tab, snap, ld, bias_col, rule) in enumerate(self._snap_tables()):
            if which is not None and ti not in which:
                x += 1
                continue
            if rule == "affine":
                ya = self._yaff[c]
                _lib.call("mf_item_affine", self._ptr(tab), self._ptr(snap), self.n_items, ld,
                          self._ptr(ya["a"]), self._ptr(ya["s"]), self._ptr(bufs[x]), 0,
                          self.dtype, st)
                x += 1
                continue
            use_counts = rule != _lib.MF_MERGE_SUM
            # (MF_MERGE_RECENCY: the item's ratings on the later ranks in place of n_r)
            cnt = self._after[c] if rule == _lib.MF_MERGE_RECENCY else self.counts[c]
            _lib.call("mf_item_merge", self._ptr(tab), self._ptr(snap), self.n_items, ld, self.K,
                      bias_col, 1, rule, self._ptr(cnt) if use_counts else None,
                      self._ptr(self.totals[c]) if use_counts else None,
                      ctypes.byref(self._hyper),
                      ctypes.c_void_p(self.pu.data_ptr() +
                                      self.u_lo * self.ld * self.pu.element_size()),
                      max(self.u_hi - self.u_lo, 1), self.ld, self._ptr(self.work),
                      self._ptr(bufs[x]), 0, self.dtype, st)
            x += 1

    def _apply(self, bufs):
        c = getattr(self, "_chunk", 0)
        st = self._st()
        x = 0
        if self.is_log:  # bufs[0]: the all-reduced sums
            if not self._snap_tables():
                self._bind_fork()
            _lib.call("mf_log_apply", self._ptr(self.qb), self.n_items, self.ldq, self.K,
                      self._bias_col, self._ptr(bufs[0]), None, None, None,
                      self._ptr(self._totals()[c]),
                      ctypes.byref(self._hyper), self._ptr(self.work), self._log_rule(), None,
                      1, *self._stat_args(not self._stat_rides()), self._bias_out(True),
                      self.dtype, st)
            x = 1
        for tab, snap, ld, _, rule in self._snap_tables():
            if rule == "affine":
                _lib.call("mf_item_affine", self._ptr(tab), self._ptr(snap), self.n_items, ld,
                          self._ptr(self._yaff[c]["a_all"]), None, self._ptr(bufs[x]), 1,
                          self.dtype, st)
            else:
                _lib.call("mf_item_apply", self._ptr(tab), self._ptr(snap), self.n_items, ld, 1,
                          self._ptr(bufs[x]), self.dtype, st)
            x += 1

def _has_duplicate_items(row_ptr, items, n_items=None, torch=None, dev=None) -> bool:
    """True if some user lists the same item twice (the kernels then forward rows in registers).
    Keys user * n_items + item sorted on the device when torch / dev are given (C5's 1B ratings:
    a host sort would take minutes), else on the host."""
    row_ptr = np.asarray(row_ptr, np.int64)
    if len(items) == 0:
        return False
    if torch is not None and dev is not None:
        n = int(n_items) if n_items else int(np.max(items)) + 1
        lens = torch.from_numpy(np.diff(row_ptr)).to(dev)
        users = torch.repeat_interleave(torch.arange(len(lens), device=dev), lens)
        key = users * n + torch.from_numpy(np.asarray(items, np.int32)).to(dev).to(torch.int64)
        del users
        key = torch.sort(key).values
        return bool((key[1:] == key[:-1]).any().item())
    users = np.repeat(np.arange(len(row_ptr) - 1, dtype=np.int64), np.diff(row_ptr))
    key = users * (int(np.max(items)) + 1) + np.asarray(items, np.int64)
    return len(np.unique(key)) != len(key)


class NMFEngine(Predictor):
    """NMF.sgd on one GPU (matrix_factorization.pyx:646-735): per epoch mf_nmf_user_pass then
    mf_nmf_item_pass, then the user-factor buffers swap.  Layout as MFEngine: pu / pu_next
    T[U, ldu], qb T[I, ldq] = [q_i | b_i | 0..], bu T[U]; per rating est T[nnz] (and the item-bias
    step blog T[nnz] when biased); the item-major view csc_ptr / csc_pos / row_user."""

    def __init__(self, csr, csc, n_items, n_factors, *, hyper, biased=False, dtype="float32",
                 device=None, bias_rule="count"):
        torch = _lib.require_gpu()
        self.torch = torch
        self.dev = torch.device("cuda", torch.cuda.current_device()) if device is None else \
            torch.device(device)
        self.dtype = _lib.MF_F64 if str(dtype) in ("float64", "f64", "double") else _lib.MF_F32
        self.tdt = torch.float64 if self.dtype == _lib.MF_F64 else torch.float32
        if n_factors < 1 or n_factors > _lib.MAX_FACTORS[self.dtype]:
            raise ValueError(f"n_factors must be in [1, {_lib.MAX_FACTORS[self.dtype]}] "
                             f"for {dtype}, got {n_factors}")
        self.K = int(n_factors)
        self.ld = default_ld(self.K, self.dtype)
        self.ldq = default_ldq(self.K, self.dtype)
        self.biased = bool(biased)
        row_ptr, items, ratings = csr
        row_ptr = np.asarray(row_ptr, np.int64)
        self.n_users, self.n_items = len(row_ptr) - 1, int(n_items)
        self.stream = torch.cuda.current_stream(self.dev)
        to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.dev)
        self.row_ptr = to_dev(row_ptr)
        self.items = to_dev(np.asarray(items, np.int32))
        self.ratings = to_dev(np.asarray(ratings, np.float64)).to(self.tdt)
        self._csr = _lib.MfCsr(self.row_ptr.data_ptr(), self.items.data_ptr(),
                               self.ratings.data_ptr(), self.n_users, self.n_items)
        csc_ptr, csc_pos = csc
        self.csc_ptr = to_dev(np.asarray(csc_ptr, np.int64))
        self.csc_pos = to_dev(np.asarray(csc_pos, np.int64))
        self.row_user = to_dev(np.repeat(np.arange(self.n_users, dtype=np.int32),
                                         np.diff(row_ptr)))
        z = lambda *shape: torch.zeros(*shape, dtype=self.tdt, device=self.dev)
        nnz = max(len(items), 1)
        self.pu, self.pu_next = z(self.n_users, self.ld), z(self.n_users, self.ld)
        self.bu, self.qb = z(self.n_users), z(self.n_items, self.ldq)
        self.est = z(nnz)
        self.blog = z(nnz) if self.biased else None
        self._hyper = _lib.MfHyper(**hyper)
        if not self.biased:
            self._hyper.global_mean = 0.0  # mf.pyx:682-683
        self.rule = _lib.MF_MERGE_COUNT if bias_rule == "count" else _lib.MF_MERGE_SUM
        # the item pass in pieces of <= PIECE_ROWS ratings (mf_nmf_item_pass's piece form)
        cnt = np.diff(np.asarray(csc_ptr, np.int64))
        ipp, pb = piece_bounds(np.asarray(csc_ptr, np.int64), cnt)
        self.piece_beg, self.item_piece_ptr = to_dev(pb), to_dev(ipp)
        self.n_pieces = len(pb) - 1
        self.piece_scratch = z(max(self.n_pieces, 1), 2 * self.ldq + 1)
        # ratings / users in CSC order (static): the item pieces read them coalesced
        self.csc_ratings = self.ratings[self.csc_pos].contiguous()
        self.csc_user = self.row_user[self.csc_pos].contiguous()
        # the unbiased user pass in the same piece form over the CSR ranges
        ucnt = np.diff(row_ptr)
        upp, upb = piece_bounds(row_ptr, ucnt)
        self.u_piece_beg, self.user_piece_ptr = to_dev(upb), to_dev(upp)
        self.u_piece_user = to_dev(np.repeat(np.arange(self.n_users, dtype=np.int32),
                                             np.diff(upp)))
        self.u_n_pieces = len(upb) - 1
        self.u_piece_scratch = z(max(self.u_n_pieces, 1), 2 * self.ld)

    def _ptr(self, t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else None

    def set_factors(self, pu, qi):
        K, t = self.K, self.torch
        self.pu.zero_()
        self.pu[:, :K].copy_(t.from_numpy(np.ascontiguousarray(pu, np.float64)).to(self.dev, self.tdt))
        self.qb.zero_()
        self.qb[:, :K].copy_(t.from_numpy(np.ascontiguousarray(qi, np.float64)).to(self.dev, self.tdt))
        self.bu.zero_()

    def epoch(self):
        st = ctypes.c_void_p(self.stream.cuda_stream)
        _lib.call("mf_nmf_user_pass", ctypes.byref(self._csr), self._ptr(self.pu),
                  self._ptr(self.pu_next), self._ptr(self.bu), self.ld, self._ptr(self.qb),
                  self.ldq, self.K, int(self.biased), ctypes.byref(self._hyper),
                  self._ptr(self.est), self._ptr(self.blog), self._ptr(self.u_piece_beg),
                  self.u_n_pieces, self._ptr(self.user_piece_ptr), self._ptr(self.u_piece_user),
                  self._ptr(self.u_piece_scratch), self.dtype, st)
        _lib.call("mf_nmf_item_pass", self._ptr(self.csc_ptr), self._ptr(self.csc_pos),
                  self._ptr(self.row_user), self._ptr(self.ratings), self._ptr(self.est),
                  self._ptr(self.blog), self._ptr(self.pu), self.ld, self._ptr(self.qb),
                  self.ldq, self.n_items, self.K, int(self.biased), ctypes.byref(self._hyper),
                  self.rule, self._ptr(self.piece_beg), self.n_pieces,
                  self._ptr(self.item_piece_ptr), self._ptr(self.piece_scratch),
                  self._ptr(self.csc_ratings), self._ptr(self.csc_user), self.dtype, st)
        self.pu, self.pu_next = self.pu_next, self.pu

    def get_factors(self):
        self.stream.synchronize()
        K = self.K
        h = lambda x: x.to(self.torch.float64).cpu().numpy()
        return dict(pu=h(self.pu[:, :K]), qi=h(self.qb[:, :K]), bu=h(self.bu),
                    bi=h(self.qb[:, K]))


def baseline_als_device(csr, csc, n_items, global_mean, n_epochs, reg_u, reg_i,
                        dtype="float64"):
    """baseline_als (optimize_baselines.pyx:14-54) on the device; returns fp64 (bu, bi)."""
    torch = _lib.require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device())
    dt = _lib.MF_F64 if str(dtype) in ("float64", "f64", "double") else _lib.MF_F32
    tdt = torch.float64 if dt == _lib.MF_F64 else torch.float32
    row_ptr, items, ratings = csr
    row_ptr = np.asarray(row_ptr, np.int64)
    n_users = len(row_ptr) - 1
    to_dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    rp, it = to_dev(row_ptr), to_dev(np.asarray(items, np.int32))
    rt = to_dev(np.asarray(ratings, np.float64)).to(tdt)
    cp, cs = to_dev(np.asarray(csc[0], np.int64)), to_dev(np.asarray(csc[1], np.int64))
    ru = to_dev(np.repeat(np.arange(n_users, dtype=np.int32), np.diff(row_ptr)))
    crt, cru = rt[cs].contiguous(), ru[cs].contiguous()  # CSC-ordered copies (coalesced reads)
    bu = torch.zeros(n_users, dtype=tdt, device=dev)
    bi = torch.zeros(n_items, dtype=tdt, device=dev)
    c = _lib.MfCsr(rp.data_ptr(), it.data_ptr(), rt.data_ptr(), n_users, int(n_items))
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda x: ctypes.c_void_p(x.data_ptr())
    for _ in range(n_epochs):
        _lib.call("mf_baseline_als_epoch", ctypes.byref(c), p(cp), p(cs), p(ru), p(bu), p(bi),
                  float(global_mean), float(reg_u), float(reg_i), p(crt), p(cru), dt, st)
    torch.cuda.current_stream(dev).synchronize()
    return bu.to(torch.float64).cpu().numpy(), bi.to(torch.float64).cpu().numpy()
