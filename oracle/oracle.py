"""ctypes front-end of the parity oracle (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product package ``surprise_amd`` never does:
its training path runs the HIP kernels or raises.

What it wraps (see ``mf_oracle.c`` for the reference file:line of each routine):

* ``svd_sgd``            SVD.sgd        (matrix_factorization.pyx:172-267), fp64, bit-exact
* ``svdpp_sgd``          SVDpp.sgd      (matrix_factorization.pyx:420-504), literal O(|I_u|) form
* ``svdpp_sgd_affine``   per-user reformulation of SVDpp.sgd (the form the GPU kernel uses)
* ``svd_sgd_groups``     G-group SUM-of-deltas schedule (multi-GPU / multi-replica semantics)
* ``svdpp_sgd_groups_merge``  SVD++ G-group schedule with the multi-rank merge rules
* ``svd_predict`` / ``svdpp_predict``  SVD.estimate / SVDpp.estimate on inner ids

Initialisation follows SVD.sgd:206-236 / SVDpp.sgd:450-461: ``get_rng`` then
``rng.normal(init_mean, init_std_dev, (n_users, K))`` for pu, then qi, then yj.

Also holds ``py_svd_sgd``: a pure-Python loop restatement for tiny cases, used
to cross-check the C file itself.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


class OracleHyper(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "lr_bu", "lr_bi", "lr_pu", "lr_qi", "lr_yj",
        "reg_bu", "reg_bi", "reg_pu", "reg_qi", "reg_yj")]


def build(force: bool = False) -> str:
    """Compile liboracle.so with the committed Makefile (gcc is in the image)."""
    src = os.path.join(_HERE, "mf_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE, "-B", "liboracle.so"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def hyper(**kw) -> OracleHyper:
    h = OracleHyper()
    for n, _ in OracleHyper._fields_:
        setattr(h, n, float(kw.get(n, 0.0)))
    return h


def svd_hyper(algo_like) -> OracleHyper:
    """Hyper-parameters resolved exactly like SVD/SVDpp.__init__ (mf.pyx:140-147, 398-407)."""
    return hyper(**{n: getattr(algo_like, n, 0.0) for n, _ in OracleHyper._fields_})


def init_factors(rng, n_users, n_items, K, init_mean=0.0, init_std_dev=0.1, with_yj=False):
    """Draw order of SVD.sgd:233-236 / SVDpp.sgd:455-460 (pu, qi[, yj]); fp64 C order."""
    pu = rng.normal(init_mean, init_std_dev, (n_users, K))
    qi = rng.normal(init_mean, init_std_dev, (n_items, K))
    yj = rng.normal(init_mean, init_std_dev, (n_items, K)) if with_yj else None
    return pu, qi, yj


def _csr_args(row_ptr, items, ratings):
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
    items = np.ascontiguousarray(items, dtype=np.int32)
    ratings = np.ascontiguousarray(ratings, dtype=np.float64)
    return row_ptr, items, ratings


def svd_sgd(row_ptr, items, ratings, n_items, K, n_epochs, biased, global_mean, hp,
            pu, qi, bu=None, bi=None):
    """In-place fp64 SVD SGD (mf.pyx:241-262). Returns (pu, qi, bu, bi)."""
    row_ptr, items, ratings = _csr_args(row_ptr, items, ratings)
    n_users = len(row_ptr) - 1
    pu = np.ascontiguousarray(pu, dtype=np.float64)
    qi = np.ascontiguousarray(qi, dtype=np.float64)
    bu = np.zeros(n_users) if bu is None else np.ascontiguousarray(bu, dtype=np.float64)
    bi = np.zeros(n_items) if bi is None else np.ascontiguousarray(bi, dtype=np.float64)
    lib().oracle_svd_sgd(ctypes.c_int64(n_users), _p(row_ptr), _p(items), _p(ratings),
                         ctypes.c_int32(K), ctypes.c_int32(n_epochs), ctypes.c_int32(int(biased)),
                         ctypes.c_double(global_mean), ctypes.byref(hp),
                         _p(pu), _p(qi), _p(bu), _p(bi))
    return pu, qi, bu, bi


def svdpp_sgd(row_ptr, items, ratings, n_items, K, n_epochs, global_mean, hp, pu, qi, yj,
              bu=None, bi=None, affine=False):
    """In-place fp64 SVD++ SGD (mf.pyx:463-498); affine=True uses the per-user form."""
    row_ptr, items, ratings = _csr_args(row_ptr, items, ratings)
    n_users = len(row_ptr) - 1
    pu = np.ascontiguousarray(pu, dtype=np.float64)
    qi = np.ascontiguousarray(qi, dtype=np.float64)
    yj = np.ascontiguousarray(yj, dtype=np.float64)
    bu = np.zeros(n_users) if bu is None else np.ascontiguousarray(bu, dtype=np.float64)
    bi = np.zeros(n_items) if bi is None else np.ascontiguousarray(bi, dtype=np.float64)
    fn = lib().oracle_svdpp_sgd_affine if affine else lib().oracle_svdpp_sgd
    fn(ctypes.c_int64(n_users), _p(row_ptr), _p(items), _p(ratings), ctypes.c_int32(K),
       ctypes.c_int32(n_epochs), ctypes.c_double(global_mean), ctypes.byref(hp),
       _p(pu), _p(qi), _p(yj), _p(bu), _p(bi))
    return pu, qi, yj, bu, bi


def svdpp_sgd_hotstale(row_ptr, items, ratings, n_items, K, n_epochs, global_mean, hp, pu, qi,
                       yj, hot, bu=None, bi=None):
    """SVD++ in the GPU helper-wave schedule's form: y deferred per epoch, q live except the
    items with hot[i] != 0 (epoch-start snapshot, steps folded with the count-aware weight)."""
    row_ptr, items, ratings = _csr_args(row_ptr, items, ratings)
    n_users = len(row_ptr) - 1
    pu = np.ascontiguousarray(pu, dtype=np.float64)
    qi = np.ascontiguousarray(qi, dtype=np.float64)
    yj = np.ascontiguousarray(yj, dtype=np.float64)
    bu = np.zeros(n_users) if bu is None else np.ascontiguousarray(bu, dtype=np.float64)
    bi = np.zeros(n_items) if bi is None else np.ascontiguousarray(bi, dtype=np.float64)
    hot = np.ascontiguousarray(hot, dtype=np.int32)
    lib().oracle_svdpp_sgd_hotstale(ctypes.c_int64(n_users), ctypes.c_int64(n_items), _p(row_ptr),
                                    _p(items), _p(ratings), ctypes.c_int32(K),
                                    ctypes.c_int32(n_epochs), ctypes.c_double(global_mean),
                                    ctypes.byref(hp), _p(hot), _p(pu), _p(qi), _p(yj), _p(bu),
                                    _p(bi))
    return pu, qi, yj, bu, bi


def svdpp_sgd_stalelog(row_ptr, items, ratings, n_items, K, n_epochs, global_mean, hp, pu, qi,
                       yj, stale, chunk_of_user=None, n_chunks=1, merge=3, bu=None, bi=None):
    """SVD++ with y deferred per epoch-chunk, q / b live except the items with stale[i] != 0,
    whose steps are logged against the chunk-start row and folded after the chunk (merge 3:
    recency weights, 2: count-aware).  Returns (pu, qi, yj, bu, bi)."""
    row_ptr, items, ratings = _csr_args(row_ptr, items, ratings)
    n_users = len(row_ptr) - 1
    pu = np.ascontiguousarray(pu, dtype=np.float64)
    qi = np.ascontiguousarray(qi, dtype=np.float64)
    yj = np.ascontiguousarray(yj, dtype=np.float64)
    bu = np.zeros(n_users) if bu is None else np.ascontiguousarray(bu, dtype=np.float64)
    bi = np.zeros(n_items) if bi is None else np.ascontiguousarray(bi, dtype=np.float64)
    stale = np.ascontiguousarray(stale, dtype=np.int32)
    c = (np.zeros(n_users, np.int32) if chunk_of_user is None
         else np.ascontiguousarray(chunk_of_user, dtype=np.int32))
    lib().oracle_svdpp_sgd_stalelog(
        ctypes.c_int64(n_users), ctypes.c_int64(n_items), _p(row_ptr), _p(items), _p(ratings),
        ctypes.c_int32(K), ctypes.c_int32(n_epochs), ctypes.c_double(global_mean),
        ctypes.byref(hp), _p(c), ctypes.c_int32(n_chunks), _p(stale), ctypes.c_int32(merge),
        _p(pu), _p(qi), _p(yj), _p(bu), _p(bi))
    return pu, qi, yj, bu, bi


def svd_sgd_groups(row_ptr, items, ratings, n_items, K, n_epochs, biased, global_mean, hp,
                   pu, qi, group_of_user, n_groups, chunk_of_user=None, n_chunks=1,
                   bu=None, bi=None):
    """G-group SUM-of-deltas schedule; returns (pu, qi, bu, bi)."""
    row_ptr, items, ratings = _csr_args(row_ptr, items, ratings)
    n_users = len(row_ptr) - 1
    pu = np.ascontiguousarray(pu, dtype=np.float64)
    qi = np.ascontiguousarray(qi, dtype=np.float64)
    bu = np.zeros(n_users) if bu is None else np.ascontiguousarray(bu, dtype=np.float64)
    bi = np.zeros(n_items) if bi is None else np.ascontiguousarray(bi, dtype=np.float64)
    g = np.ascontiguousarray(group_of_user, dtype=np.int32)
    c = (np.zeros(n_users, np.int32) if chunk_of_user is None
         else np.ascontiguousarray(chunk_of_user, dtype=np.int32))
    lib().oracle_svd_sgd_groups(ctypes.c_int64(n_users), ctypes.c_int64(n_items), _p(row_ptr),
                                _p(items), _p(ratings), ctypes.c_int32(K),
                                ctypes.c_int32(n_epochs), ctypes.c_int32(int(biased)),
                                ctypes.c_double(global_mean), ctypes.byref(hp), _p(g),
                                ctypes.c_int32(n_groups), _p(c), ctypes.c_int32(n_chunks),
                                _p(pu), _p(qi), _p(bu), _p(bi))
    return pu, qi, bu, bi


def svdpp_sgd_groups_merge(row_ptr, items, ratings, n_items, K, n_epochs, global_mean, hp,
                           pu, qi, yj, group_of_user, n_groups, chunk_of_user=None, n_chunks=1,
                           merge=2, merge_y=4, bu=None, bi=None, bias_fold=False):
    """SVD++ G-group schedule (multi-rank semantics): q/b merged by `merge` (0 SUM, 1 MEAN,
    2 count-aware, 3 rank-order composition), y by `merge_y` (4: the GPU's affine composition in
    group order, users reading the chunk-start y); bias_fold: item biases read at the chunk start
    and their steps folded per item with recency weights after the chunk.
    Returns (pu, qi, yj, bu, bi)."""
    row_ptr, items, ratings = _csr_args(row_ptr, items, ratings)
    n_users = len(row_ptr) - 1
    pu = np.ascontiguousarray(pu, dtype=np.float64)
    qi = np.ascontiguousarray(qi, dtype=np.float64)
    yj = np.ascontiguousarray(yj, dtype=np.float64)
    bu = np.zeros(n_users) if bu is None else np.ascontiguousarray(bu, dtype=np.float64)
    bi = np.zeros(n_items) if bi is None else np.ascontiguousarray(bi, dtype=np.float64)
    g = np.ascontiguousarray(group_of_user, dtype=np.int32)
    c = (np.zeros(n_users, np.int32) if chunk_of_user is None
         else np.ascontiguousarray(chunk_of_user, dtype=np.int32))
    lib().oracle_svdpp_sgd_groups_merge_b(
        ctypes.c_int64(n_users), ctypes.c_int64(n_items), _p(row_ptr), _p(items), _p(ratings),
        ctypes.c_int32(K), ctypes.c_int32(n_epochs), ctypes.c_double(global_mean),
        ctypes.byref(hp), _p(g), ctypes.c_int32(n_groups), _p(c), ctypes.c_int32(n_chunks),
        ctypes.c_int32(merge), ctypes.c_int32(merge_y), ctypes.c_int32(int(bias_fold)), _p(pu),
        _p(qi), _p(yj), _p(bu), _p(bi))
    return pu, qi, yj, bu, bi


def svd_sgd_deltalog(row_ptr, items, ratings, n_items, K, n_epochs, biased, global_mean, hp,
                     pu, qi, chunk_of_user=None, n_chunks=1, merge=2, bu=None, bi=None):
    """Delta-log schedule (the GPU's MF_MODE_LOG): every user against the chunk-start item
    snapshot, item deltas merged per item with the count-aware weight (merge=2) or summed (0)."""
    row_ptr, items, ratings = _csr_args(row_ptr, items, ratings)
    n_users = len(row_ptr) - 1
    pu = np.ascontiguousarray(pu, dtype=np.float64)
    qi = np.ascontiguousarray(qi, dtype=np.float64)
    bu = np.zeros(n_users) if bu is None else np.ascontiguousarray(bu, dtype=np.float64)
    bi = np.zeros(n_items) if bi is None else np.ascontiguousarray(bi, dtype=np.float64)
    c = (np.zeros(n_users, np.int32) if chunk_of_user is None
         else np.ascontiguousarray(chunk_of_user, dtype=np.int32))
    lib().oracle_svd_sgd_deltalog(ctypes.c_int64(n_users), ctypes.c_int64(n_items), _p(row_ptr),
                                  _p(items), _p(ratings), ctypes.c_int32(K),
                                  ctypes.c_int32(n_epochs), ctypes.c_int32(int(biased)),
                                  ctypes.c_double(global_mean), ctypes.byref(hp), _p(c),
                                  ctypes.c_int32(n_chunks), ctypes.c_int32(merge),
                                  _p(pu), _p(qi), _p(bu), _p(bi))
    return pu, qi, bu, bi


def svdpp_sgd_deltalog(row_ptr, items, ratings, n_items, K, n_epochs, global_mean, hp, pu, qi,
                       yj, chunk_of_user=None, n_chunks=1, merge=2, merge_y=0, bu=None, bi=None):
    """SVD++ delta-log schedule: q/b as svd_sgd_deltalog, y_j shared and updated at the end of
    each user (merge_y=0, the GPU's semantics) or logged and merged by their mean (1)."""
    row_ptr, items, ratings = _csr_args(row_ptr, items, ratings)
    n_users = len(row_ptr) - 1
    pu = np.ascontiguousarray(pu, dtype=np.float64)
    qi = np.ascontiguousarray(qi, dtype=np.float64)
    yj = np.ascontiguousarray(yj, dtype=np.float64)
    bu = np.zeros(n_users) if bu is None else np.ascontiguousarray(bu, dtype=np.float64)
    bi = np.zeros(n_items) if bi is None else np.ascontiguousarray(bi, dtype=np.float64)
    c = (np.zeros(n_users, np.int32) if chunk_of_user is None
         else np.ascontiguousarray(chunk_of_user, dtype=np.int32))
    lib().oracle_svdpp_sgd_deltalog(ctypes.c_int64(n_users), ctypes.c_int64(n_items), _p(row_ptr),
                                    _p(items), _p(ratings), ctypes.c_int32(K),
                                    ctypes.c_int32(n_epochs), ctypes.c_double(global_mean),
                                    ctypes.byref(hp), _p(c), ctypes.c_int32(n_chunks),
                                    ctypes.c_int32(merge), ctypes.c_int32(merge_y),
                                    _p(pu), _p(qi), _p(yj), _p(bu), _p(bi))
    return pu, qi, yj, bu, bi


def nmf_sgd(row_ptr, items, ratings, n_items, K, n_epochs, biased, global_mean, pu, qi,
            reg_pu=.06, reg_qi=.06, reg_bu=.02, reg_bi=.02, lr_bu=.005, lr_bi=.005,
            bu=None, bi=None, bias_log=False):
    """In-place fp64 NMF.sgd (mf.pyx:646-735); bias_log=True: the GPU's snapshot + count-aware
    schedule for the item biases. Returns (pu, qi, bu, bi)."""
    row_ptr, items, ratings = _csr_args(row_ptr, items, ratings)
    n_users = len(row_ptr) - 1
    pu = np.ascontiguousarray(pu, dtype=np.float64)
    qi = np.ascontiguousarray(qi, dtype=np.float64)
    bu = np.zeros(n_users) if bu is None else np.ascontiguousarray(bu, dtype=np.float64)
    bi = np.zeros(n_items) if bi is None else np.ascontiguousarray(bi, dtype=np.float64)
    cnt = np.bincount(items, minlength=n_items).astype(np.int64)
    lib().oracle_nmf_sgd(ctypes.c_int64(n_users), ctypes.c_int64(n_items), _p(row_ptr), _p(items),
                         _p(ratings), _p(cnt), ctypes.c_int32(K), ctypes.c_int32(n_epochs),
                         ctypes.c_int32(int(biased)), ctypes.c_double(global_mean),
                         *[ctypes.c_double(x) for x in (reg_pu, reg_qi, reg_bu, reg_bi, lr_bu,
                                                        lr_bi)],
                         ctypes.c_int32(int(bias_log)), _p(pu), _p(qi), _p(bu), _p(bi))
    return pu, qi, bu, bi


def baseline_als(row_ptr, items, ratings, n_items, csc_ptr, csc_pos, global_mean, n_epochs=10,
                 reg_u=15, reg_i=10):
    """fp64 baseline_als (optimize_baselines.pyx:14-54); csc_ptr / csc_pos = Trainset.csc().
    Returns (bu, bi)."""
    row_ptr, items, ratings = _csr_args(row_ptr, items, ratings)
    n_users = len(row_ptr) - 1
    row_user = np.repeat(np.arange(n_users, dtype=np.int32), np.diff(row_ptr))
    csc_ptr = np.ascontiguousarray(csc_ptr, np.int64)
    csc_pos = np.ascontiguousarray(csc_pos, np.int64)
    bu, bi = np.zeros(n_users), np.zeros(n_items)
    lib().oracle_baseline_als(ctypes.c_int64(n_users), ctypes.c_int64(n_items), _p(row_ptr),
                              _p(items), _p(ratings), _p(csc_ptr), _p(csc_pos), _p(row_user),
                              ctypes.c_double(global_mean), ctypes.c_int32(n_epochs),
                              ctypes.c_double(reg_u), ctypes.c_double(reg_i), _p(bu), _p(bi))
    return bu, bi


def svd_predict(u, i, K, biased, global_mean, pu, qi, bu, bi):
    """SVD.estimate on inner ids (-1 = unknown). Returns (est, impossible)."""
    u = np.ascontiguousarray(u, dtype=np.int32)
    i = np.ascontiguousarray(i, dtype=np.int32)
    est = np.zeros(len(u))
    imp = np.zeros(len(u), np.int32)
    lib().oracle_svd_predict(ctypes.c_int64(len(u)), _p(u), _p(i), ctypes.c_int32(K),
                             ctypes.c_int32(int(biased)), ctypes.c_double(global_mean),
                             _p(np.ascontiguousarray(pu, np.float64)),
                             _p(np.ascontiguousarray(qi, np.float64)),
                             _p(np.ascontiguousarray(bu, np.float64)),
                             _p(np.ascontiguousarray(bi, np.float64)), _p(est), _p(imp))
    return est, imp.astype(bool)


def svdpp_predict(u, i, row_ptr, items, K, global_mean, pu, qi, yj, bu, bi):
    u = np.ascontiguousarray(u, dtype=np.int32)
    i = np.ascontiguousarray(i, dtype=np.int32)
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
    items = np.ascontiguousarray(items, dtype=np.int32)
    est = np.zeros(len(u))
    lib().oracle_svdpp_predict(ctypes.c_int64(len(u)), _p(u), _p(i), _p(row_ptr), _p(items),
                               ctypes.c_int32(K), ctypes.c_double(global_mean),
                               _p(np.ascontiguousarray(pu, np.float64)),
                               _p(np.ascontiguousarray(qi, np.float64)),
                               _p(np.ascontiguousarray(yj, np.float64)),
                               _p(np.ascontiguousarray(bu, np.float64)),
                               _p(np.ascontiguousarray(bi, np.float64)), _p(est))
    return est


def finish_estimates(est, impossible, global_mean, offset, rating_scale, clip=True):
    """AlgoBase.predict post-processing (algo_base.py:156-169): impossible ->
    default_prediction() = global_mean, subtract offset, clip."""
    est = np.where(impossible, global_mean, est) - offset
    if clip:  # Python's min(hi, est) / max(lo, est) keep the bound when est is NaN: fmin/fmax
        lo, hi = rating_scale
        est = np.fmax(lo, np.fmin(hi, est))
    return est


def rmse(r_true, est):
    """accuracy.rmse (accuracy.py:47-49): sqrt(np.mean of squared errors)."""
    d = np.asarray(r_true, np.float64) - np.asarray(est, np.float64)
    return float(np.sqrt(np.mean(d * d)))


def mae(r_true, est):
    d = np.asarray(r_true, np.float64) - np.asarray(est, np.float64)
    return float(np.mean(np.abs(d)))


def py_svd_sgd(row_ptr, items, ratings, K, n_epochs, biased, global_mean, hp, pu, qi, bu, bi):
    """Pure-Python loop restatement of mf.pyx:241-262 (tiny cases only)."""
    g = global_mean if biased else 0.0
    for _ in range(n_epochs):
        for u in range(len(row_ptr) - 1):
            for k in range(row_ptr[u], row_ptr[u + 1]):
                i, r = int(items[k]), float(ratings[k])
                dot = 0.0
                for f in range(K):
                    dot += qi[i, f] * pu[u, f]
                err = r - (g + bu[u] + bi[i] + dot)
                if biased:
                    bu[u] += hp.lr_bu * (err - hp.reg_bu * bu[u])
                    bi[i] += hp.lr_bi * (err - hp.reg_bi * bi[i])
                for f in range(K):
                    puf, qif = pu[u, f], qi[i, f]
                    pu[u, f] += hp.lr_pu * (err * qif - hp.reg_pu * puf)
                    qi[i, f] += hp.lr_qi * (err * puf - hp.reg_qi * qif)
    return pu, qi, bu, bi


def time_svdpp_epochs(row_ptr, items, ratings, n_items, K, n_epochs, seed=0, affine=False):
    """Wall-clock of the C restatement of SVDpp.sgd (1 thread) for the SVD++ cpu_baseline leg:
    the reference's per-rating loop (u_impl re-summed over I_u and every y_j of I_u stepped, per
    rating: O(|I_u| K), mf.pyx:463-498), or (affine) the per-user affine form, O(K) per rating."""
    import time
    rng = np.random.RandomState(seed)
    n_users = len(row_ptr) - 1
    pu, qi, yj = init_factors(rng, n_users, n_items, K, with_yj=True)
    hp = hyper(lr_bu=.007, lr_bi=.007, lr_pu=.007, lr_qi=.007, lr_yj=.007,
               reg_bu=.02, reg_bi=.02, reg_pu=.02, reg_qi=.02, reg_yj=.02)
    gm = float(np.mean(ratings))
    t0 = time.perf_counter()
    svdpp_sgd(row_ptr, items, ratings, n_items, K, n_epochs, gm, hp, pu, qi, yj, affine=affine)
    return time.perf_counter() - t0


def time_svd_epochs(row_ptr, items, ratings, n_items, K, n_epochs, seed=0):
    """Wall-clock of the C restatement (1 thread) for the cpu_baseline leg."""
    import time
    rng = np.random.RandomState(seed)
    pu, qi, _ = init_factors(rng, len(row_ptr) - 1, n_items, K)
    hp = hyper(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005,
               reg_bu=.02, reg_bi=.02, reg_pu=.02, reg_qi=.02)
    gm = float(np.mean(ratings))
    t0 = time.perf_counter()
    svd_sgd(row_ptr, items, ratings, n_items, K, n_epochs, True, gm, hp, pu, qi)
    return time.perf_counter() - t0
