"""SVD and SVD++ behind Surprise's AlgoBase plugin API, trained by HIP kernels.

Mirrors surprise/prediction_algorithms/matrix_factorization.pyx:
  SVD    __init__ :129-151, fit :153-170, sgd :172-267, estimate :269-299
  SVDpp  __init__ :389-411, fit :413-418, sgd :420-504, estimate :506-522

Same constructor arguments, defaults and learning-rate / regularisation
fall-backs; same initialisation draws (get_rng, then rng.normal for pu, qi[, yj]
in that order, fp64); same attributes after fit (``pu``, ``qi``, ``bu``, ``bi``
[, ``yj``] as fp64 numpy).  ``sgd`` runs the epochs on the GPU through
libsurprise_amd.so and raises if the library or the GPU is missing -- there is
no CPU fallback.  Extra, keyword-only device options:

  dtype              "float64" (the reference's arithmetic, mf.pyx's double arrays) or
                     "float32" (about 1.7x the fp64 rate at ML-1M, held within 1e-3 of the
                     fp64 reference's held-out RMSE by the parity tests); None (default):
                     float64 up to 256 factors (the fp64 row limit of the device kernels),
                     float32 above it (up to 512)
  mode               item-side schedule: "log" (default; item rows read from the chunk-start
                     snapshot, per-rating item deltas logged and folded in once per
                     epoch-chunk -- race-free, bit-reproducible), "atomic" (shared rows,
                     float atomics), "plain" (shared rows, plain stores) or "auto" ("log" for
                     SVD, "atomic" for SVD++)
  chunks_per_epoch   epoch-chunks (item merges / all-reduces per epoch); "auto" (default): 1
                     for SVD, one per 80,000 users of a rank for SVD++ (engine.default_chunks)
  deterministic      True: one wavefront, users in Trainset order -- the reference's exact
                     sequence (bit-for-bit the reference's factors in fp64); False: the parallel
                     schedule; None (SVD default, "auto"): the exact sequence for small fits --
                     at most EXACT_MAX_UPDATES rating-updates (n_ratings x n_epochs) and
                     EXACT_MAX_WORK updates x factors, with mode, chunks_per_epoch and n_waves
                     left at their defaults and not distributed -- the parallel schedule
                     otherwise (SVDpp: False)
  n_waves            wavefronts per launch (0 = fill the GPU)
  distributed        opt-in: shard users over the torch.distributed ranks of the job (one
                     process per GPU, torchrun env); every rank must fit the same trainset

The fork's per-fit side effects in SVD.fit (:158-169: a print and an unused
``movie_to_mean`` dict) do not change results and are not reproduced.
"""
from __future__ import annotations

import gc
import operator

import numpy as np

from . import _lib
from .algo_base import AlgoBase
from .predictions import Prediction, PredictionImpossible
from .trainset import Trainset
from .utils import get_rng


# deterministic=None: the reference's exact order where it costs little.  u1 (80k ratings) SVD
# K=100 E=20 fp64: 45 ms exact vs 4.5 ms parallel on one MI355X, and the exact order lands on the
# reference's RMSE to the last digit where the parallel schedule is +5.5e-2 off on the diverging
# unbiased case (profiles/r5k_probe.jsonl)
EXACT_MAX_UPDATES = 2_000_000
EXACT_MAX_WORK = 200_000_000


class _MFBase(AlgoBase):
    _algo = "svd"

    def _device_options(self, dtype, mode, chunks_per_epoch, deterministic, n_waves,
                        distributed):
        if mode not in ("auto",) + tuple(_lib.MODES):
            raise ValueError(f"mode must be 'auto' or one of {sorted(_lib.MODES)}, got {mode!r}")
        self._dtype_auto = dtype is None
        self.dtype = dtype if dtype is not None else self._auto_dtype()
        self.mode = mode
        self.chunks_per_epoch = chunks_per_epoch
        self.deterministic = deterministic
        self.n_waves = n_waves
        self.distributed = distributed
        self._engine = None
        self._imp = None

    def _auto_dtype(self):
        """dtype=None: fp64 where the device rows allow it (<= 256 factors), else fp32.  Resolved
        again at fit time, so a model whose n_factors changed after construction follows it.
        (fp64 rows of more than 126 factors (SVD; 127 SVD++) exceed 1 KiB: those models train on
        the slower paths -- the gradient log instead of the checkpoint log, SVD++ without the
        helper-wave launch -- DESIGN.md 2.)"""
        return "float64" if getattr(self, "n_factors", 0) <= _lib.MAX_FACTORS[_lib.MF_F64] \
            else "float32"

    def _resolve_deterministic(self, n_ratings):
        """deterministic=None ("auto", SVD's default): the exact sequential order for a small fit
        (EXACT_MAX_UPDATES, EXACT_MAX_WORK) with every schedule option at its default."""
        if self.deterministic is not None:
            return bool(self.deterministic)
        updates = int(n_ratings) * int(self.n_epochs)
        return (self._algo == "svd" and self.mode == "auto" and self.chunks_per_epoch == "auto"
                and not self.n_waves and not self.distributed
                and not getattr(self, "_engine_options", None)
                and updates <= EXACT_MAX_UPDATES
                and updates * max(int(self.n_factors), 1) <= EXACT_MAX_WORK)

    def __getstate__(self):
        state = self.__dict__.copy()
        state["_engine"] = None  # device handles never pickle (dump.py, joblib workers)
        state["_imp"] = None
        return state

    def _resolve_mode(self):
        """auto: "log" for SVD; "atomic" for SVD++, whose shared y_j rows make the one-chunk
        log schedule drift (+1.5e-3 to +2.7e-3 RMSE on ML-1M)."""
        if self.mode != "auto":
            return self.mode
        return "log" if self._algo == "svd" else "atomic"

    def _hyper(self, global_mean):
        return dict(lr_bu=self.lr_bu, lr_bi=self.lr_bi, lr_pu=self.lr_pu, lr_qi=self.lr_qi,
                    lr_yj=getattr(self, "lr_yj", 0.0), reg_bu=self.reg_bu, reg_bi=self.reg_bi,
                    reg_pu=self.reg_pu, reg_qi=self.reg_qi, reg_yj=getattr(self, "reg_yj", 0.0),
                    global_mean=float(global_mean))

    def fit_arrays(self, row_ptr, items, ratings, n_items, rating_scale=(1, 5), offset=0):
        """Array-native fit on a user-major CSR (no reference counterpart): for
        trainsets too large for Python dicts."""
        ts = Trainset.from_csr(row_ptr, items, ratings, n_items, rating_scale, offset)
        return self.fit(ts)

    def _init_factors(self, n_users, n_items, with_yj, ctx):
        """pu, qi[, yj] drawn as SVD.sgd / SVDpp.sgd draw them (mf.pyx:227-231, :454-461): one
        rng, pu then qi then yj, fp64.  On several ranks every rank must start from the same
        factors: with an int seed each rank draws the identical stream itself; otherwise
        (random_state None or a RandomState, whose stream differs per process) rank 0 draws
        and broadcasts."""
        K = self.n_factors

        def draw():
            rng = get_rng(self.random_state)
            pu = rng.normal(self.init_mean, self.init_std_dev, (n_users, K))
            qi = rng.normal(self.init_mean, self.init_std_dev, (n_items, K))
            yj = rng.normal(self.init_mean, self.init_std_dev, (n_items, K)) if with_yj else None
            return pu, qi, yj

        if ctx is None or ctx.world == 1 or isinstance(self.random_state, (int, np.integer)):
            return draw()
        import torch
        if ctx.rank == 0:
            arrs = draw()
        else:
            arrs = (np.empty((n_users, K)), np.empty((n_items, K)),
                    np.empty((n_items, K)) if with_yj else None)
        out = []
        for a in arrs:
            if a is None:
                out.append(None)
                continue
            t = torch.from_numpy(np.ascontiguousarray(a))
            if not ctx.host_staged:
                t = t.cuda()
            ctx.broadcast(t, 0)
            out.append(t.cpu().numpy())
        return tuple(out)

    def _run_sgd(self, trainset, with_yj):
        from .engine import MFEngine
        from .dist import DistContext, csr_fingerprint, local_csr, shard_users

        _lib.require_gpu()
        if getattr(self, "_dtype_auto", False):
            self.dtype = self._auto_dtype()
        if isinstance(trainset, Trainset):
            csr = trainset.csr()
            user_order = trainset.sched_order()
        else:  # a reference surprise.Trainset (duck-typed: ur dict-of-lists)
            csr = Trainset(trainset.ur, None, trainset.n_users, trainset.n_items,
                           trainset.n_ratings, trainset.rating_scale, trainset.offset, {}, {}).csr()
            user_order = np.fromiter(trainset.ur.keys(), np.int32, len(trainset.ur))
        global_mean = self.trainset.global_mean
        n_users, n_items = trainset.n_users, trainset.n_items

        det = self._resolve_deterministic(csr[0][-1] - csr[0][0])
        self.exact_order_ = det  # (what the fit ran: the reference's sequence or the parallel one)
        ctx = DistContext.from_env() if (self.distributed and not det) else None
        if ctx is not None and ctx.world > 1:
            # every rank must hold the same trainset: it shards it by user range below
            ctx.check_agreement(csr_fingerprint(csr, n_items), "the trainset (users, items, "
                                "ratings, CSR crc32)")
        pu, qi, yj = self._init_factors(n_users, n_items, with_yj, ctx)
        lo, hi = 0, n_users
        world = 1 if ctx is None else ctx.world
        if world > 1:
            b = shard_users(csr[0], world)
            lo, hi = int(b[ctx.rank]), int(b[ctx.rank + 1])
            csr = local_csr(csr, lo, hi)
        chunks = self.chunks_per_epoch
        if chunks == "auto":
            from .engine import default_chunks
            chunks = default_chunks(self._algo, self._resolve_mode(), n_users, world)
        eng = MFEngine(csr, n_items, self.n_factors, algo=self._algo,
                       hyper=self._hyper(global_mean), biased=getattr(self, "biased", True),
                       dtype=self.dtype, mode=self._resolve_mode(),
                       n_chunks=chunks, deterministic=det,
                       user_order=user_order, n_waves=self.n_waves, world=world,
                       **getattr(self, "_engine_options", {}))
        eng.set_factors(pu[lo:hi], qi, yj=yj)
        del pu
        verbose = self.verbose

        def on_epoch(e):
            if verbose:
                print("Processing epoch {}".format(e))

        eng.run_epochs(self.n_epochs, ctx, on_epoch=on_epoch if verbose else None)
        f = eng.get_factors(ctx)
        # inference (test()) needs every user's row on the device: a sharded engine is dropped
        # and test() falls back to the batched path's host arrays via a fresh single-GPU view
        self._engine = eng if world == 1 else None
        self._imp = None
        self.bu, self.bi, self.pu, self.qi = f["bu"], f["bi"], f["pu"], f["qi"]
        if with_yj:
            self.yj = f["yj"]

    # ------------------------------------------------------------------ batched test()
    def _device_model(self):
        """The device tables inference runs on: the training engine, or (model fitted on several
        ranks / unpickled on a GPU host) device copies of the fitted arrays.  None without a
        GPU: then test() is the reference's per-prediction estimate()."""
        if self._engine is not None:
            return self._engine
        if getattr(self, "pu", None) is None:
            return None
        try:
            _lib.require_gpu()
        except _lib.SurpriseAMDError:
            return None
        from .engine import PredictTables
        ts = _as_trainset(self.trainset)
        self._engine = PredictTables(self.pu, self.qi, self.bu, self.bi,
                                     yj=getattr(self, "yj", None) if self._algo == "svdpp" else None,
                                     csr=ts.csr() if self._algo == "svdpp" else None,
                                     biased=getattr(self, "biased", True), dtype=self.dtype)
        self._imp = None
        return self._engine

    def _columns(self, testset):
        """(raw uids, raw iids, r_ui_trans) columns of a testset: a list of triples (ids as
        lists), or column-native -- a RatingColumns or a structured array with uid / iid /
        rating fields (ids as arrays, no Python objects per rating)."""
        from .dataset import RatingColumns
        if isinstance(testset, RatingColumns):
            return testset.uid, testset.iid, np.asarray(testset.rating, np.float64)
        if isinstance(testset, np.ndarray) and testset.dtype.names:
            return (testset["uid"], testset["iid"], np.asarray(testset["rating"], np.float64))
        if isinstance(testset, np.ndarray):
            testset = testset.tolist()
        rows = testset if isinstance(testset, list) else list(testset)
        if not rows:
            return [], [], np.zeros(0)
        g = operator.itemgetter
        return (list(map(g(0), rows)), list(map(g(1), rows)),
                np.fromiter(map(g(2), rows), np.float64, len(rows)))

    def _inner_columns(self, ruids, riids):
        """Vectorised raw -> inner id mapping (-1 = unknown, the 'UKN__' case of
        algo_base.py:137-144)."""
        ts = _as_trainset(self.trainset)
        return (_map_ids(ruids, ts._raw2inner_id_users), _map_ids(riids, ts._raw2inner_id_items))

    def test(self, testset, verbose=False):
        """AlgoBase.test (algo_base.py:191-218): the ids are mapped with one vectorised lookup
        and all estimates come from one batched HIP launch; the returned Predictions are the
        reference's (same est, offset, clip, was_impossible details).  Without a GPU (an
        unpickled model on a CPU host) it is the reference's per-prediction estimate()."""
        eng = None if verbose else self._device_model()
        if eng is None:
            return AlgoBase.test(self, testset, verbose)
        ruids, riids, r = self._columns(testset)
        if not len(r):
            return []
        u, i = self._inner_columns(ruids, riids)
        est, impossible = self._predict_inner(u, i)
        ts = self.trainset
        est = np.where(impossible, self.default_prediction(), est) - ts.offset
        lo, hi = ts.rating_scale
        est = np.fmax(lo, np.fmin(hi, est))  # algo_base.py:166-169 (NaN -> upper bound)
        reason = "User and item are unkown."
        if isinstance(ruids, np.ndarray):  # (column-native testset: Python scalars, as listed)
            ruids, riids = ruids.tolist(), riids.tolist()
        # (Prediction is a namedtuple: tuple.__new__ is its _make without the length check; a
        # fresh details dict per prediction, as the reference builds them)
        # (the cyclic GC stays off while 2 x len(testset) containers are created: its passes
        # over every live object would otherwise grow with the caller's heap)
        new, P = tuple.__new__, Prediction
        was = gc.isenabled()
        gc.disable()
        try:
            return [new(P, (a, b, c, e, {"was_impossible": True, "reason": reason} if x
                            else {"was_impossible": False}))
                    for a, b, c, e, x in zip(ruids, riids, (r - ts.offset).tolist(),
                                             est.tolist(), impossible.tolist())]
        finally:
            if was:
                gc.enable()

    def test_metrics(self, testset):
        """(rmse, mae) of the model on a testset -- accuracy.rmse(algo.test(testset)) and
        accuracy.mae(...) without building Prediction objects: ids mapped in one vectorised
        lookup, estimates and the error reduction on the device (mf_predict +
        mf_rating_errors).  No reference counterpart; equal to the reference pipeline's values
        (tests/test_gpu_parity.py)."""
        eng = self._device_model()
        if eng is None:
            from . import accuracy
            preds = AlgoBase.test(self, testset)
            return accuracy.rmse(preds, verbose=False), accuracy.mae(preds, verbose=False)
        ruids, riids, r = self._columns(testset)
        u, i = self._inner_columns(ruids, riids)
        ts = self.trainset
        gm, imp = self._predict_args()
        rmse, mae, _ = eng.rating_errors(u, i, r, gm, imp=imp, fallback=self.default_prediction(),
                                         offset=ts.offset, rating_scale=ts.rating_scale)
        return rmse, mae

    def _predict_args(self):
        return (self.trainset.global_mean if getattr(self, "biased", True) else 0.0), None

    def _predict_inner(self, u, i):
        gm, imp = self._predict_args()
        return self._device_model().predict(u, i, gm, imp=imp)


def _map_ids(raw, mapping):
    """raw ids -> inner ids through a Trainset's raw2inner map, vectorised (-1 if absent)."""
    from .trainset import _IdentityIds
    if isinstance(mapping, _IdentityIds):
        a = np.asarray(raw)
        if a.dtype.kind in "iu":
            out = a.astype(np.int64)
            return np.where((out >= 0) & (out < mapping.n), out, -1).astype(np.int32)
        return np.array([mapping[x] if x in mapping else -1 for x in raw], np.int32)
    import pandas as pd
    m = pd.Series(mapping, dtype="int64") if len(mapping) else pd.Series([], dtype="int64")
    idx = m.index.get_indexer(pd.Index(raw if isinstance(raw, np.ndarray) else list(raw)))
    out = np.full(len(idx), -1, np.int32)
    hit = idx >= 0
    out[hit] = m.to_numpy()[idx[hit]]
    return out


class SVD(_MFBase):
    """Biased MF / PMF trained by parallel SGD on the GPU (matrix_factorization.pyx:19-299)."""

    _algo = "svd"

    def __init__(self, n_factors=100, n_epochs=20, biased=True, init_mean=0, init_std_dev=.1,
                 lr_all=.005, reg_all=.02, lr_bu=None, lr_bi=None, lr_pu=None, lr_qi=None,
                 reg_bu=None, reg_bi=None, reg_pu=None, reg_qi=None, random_state=None,
                 verbose=False, *, dtype=None, mode="auto",
                 chunks_per_epoch="auto", deterministic=None, n_waves=0, distributed=False):
        self.n_factors = n_factors
        self.n_epochs = n_epochs
        self.biased = biased
        self.init_mean = init_mean
        self.init_std_dev = init_std_dev
        self.lr_bu = lr_bu if lr_bu is not None else lr_all
        self.lr_bi = lr_bi if lr_bi is not None else lr_all
        self.lr_pu = lr_pu if lr_pu is not None else lr_all
        self.lr_qi = lr_qi if lr_qi is not None else lr_all
        self.reg_bu = reg_bu if reg_bu is not None else reg_all
        self.reg_bi = reg_bi if reg_bi is not None else reg_all
        self.reg_pu = reg_pu if reg_pu is not None else reg_all
        self.reg_qi = reg_qi if reg_qi is not None else reg_all
        self.random_state = random_state
        self.verbose = verbose
        self._device_options(dtype, mode, chunks_per_epoch, deterministic, n_waves, distributed)
        AlgoBase.__init__(self)

    def fit(self, trainset):
        AlgoBase.fit(self, trainset)
        self.sgd(trainset)
        return self

    def sgd(self, trainset):
        """mf.pyx:172-267 on the device: init on the host (bit-identical draws), epochs in HIP."""
        self._run_sgd(trainset, with_yj=False)

    def estimate(self, u, i):
        """mf.pyx:269-299 (host numpy fp64, per call)."""
        known_user = self.trainset.knows_user(u)
        known_item = self.trainset.knows_item(i)
        if self.biased:
            est = self.trainset.global_mean
            if known_user:
                est += self.bu[u]
            if known_item:
                est += self.bi[i]
            if known_user and known_item:
                est += np.dot(self.qi[i], self.pu[u])
        else:
            if known_user and known_item:
                est = np.dot(self.qi[i], self.pu[u])
            else:
                raise PredictionImpossible("User and item are unkown.")
        return est

class SVDpp(_MFBase):
    """SVD++ trained on the GPU in the exact per-user affine form (mf.pyx:302-522)."""

    _algo = "svdpp"

    def __init__(self, n_factors=20, n_epochs=20, init_mean=0, init_std_dev=.1, lr_all=.007,
                 reg_all=.02, lr_bu=None, lr_bi=None, lr_pu=None, lr_qi=None, lr_yj=None,
                 reg_bu=None, reg_bi=None, reg_pu=None, reg_qi=None, reg_yj=None,
                 random_state=None, verbose=False, *, dtype=None, mode="auto",
                 chunks_per_epoch="auto", deterministic=False, n_waves=0,
                 distributed=False):
        self.n_factors = n_factors
        self.n_epochs = n_epochs
        self.init_mean = init_mean
        self.init_std_dev = init_std_dev
        self.lr_bu = lr_bu if lr_bu is not None else lr_all
        self.lr_bi = lr_bi if lr_bi is not None else lr_all
        self.lr_pu = lr_pu if lr_pu is not None else lr_all
        self.lr_qi = lr_qi if lr_qi is not None else lr_all
        self.lr_yj = lr_yj if lr_yj is not None else lr_all
        self.reg_bu = reg_bu if reg_bu is not None else reg_all
        self.reg_bi = reg_bi if reg_bi is not None else reg_all
        self.reg_pu = reg_pu if reg_pu is not None else reg_all
        self.reg_qi = reg_qi if reg_qi is not None else reg_all
        self.reg_yj = reg_yj if reg_yj is not None else reg_all
        self.random_state = random_state
        self.verbose = verbose
        self._device_options(dtype, mode, chunks_per_epoch, deterministic, n_waves, distributed)
        AlgoBase.__init__(self)

    def fit(self, trainset):
        AlgoBase.fit(self, trainset)
        self.sgd(trainset)
        return self

    def sgd(self, trainset):
        """mf.pyx:420-504 on the device (per-user affine form, exact without duplicate items)."""
        self._run_sgd(trainset, with_yj=True)

    def estimate(self, u, i):
        """mf.pyx:506-522 (host numpy fp64, per call)."""
        est = self.trainset.global_mean
        if self.trainset.knows_user(u):
            est += self.bu[u]
        if self.trainset.knows_item(i):
            est += self.bi[i]
        if self.trainset.knows_user(u) and self.trainset.knows_item(i):
            Iu = len(self.trainset.ur[u])
            u_impl_feedback = (sum(self.yj[j] for (j, _) in self.trainset.ur[u]) / np.sqrt(Iu))
            est += np.dot(self.qi[i], self.pu[u] + u_impl_feedback)
        return est

    def _predict_args(self):
        if self._imp is None:
            self._imp = self._device_model().user_implicit()
        return self.trainset.global_mean, self._imp


def _as_trainset(trainset):
    """Our Trainset for a reference (dict-of-lists) surprise.Trainset, duck-typed."""
    if isinstance(trainset, Trainset):
        return trainset
    return Trainset(trainset.ur, trainset.ir, trainset.n_users, trainset.n_items,
                    trainset.n_ratings, trainset.rating_scale, trainset.offset, {}, {})


class NMF(_MFBase):
    """Non-negative MF trained on the GPU (matrix_factorization.pyx:525-759).

    Same constructor arguments and defaults as the reference (:628-644), same
    ``rng.uniform`` initialisation draws (pu then qi, :673-677), same attributes.  An
    epoch is two race-free HIP passes (include/surprise_amd.h, mf_nmf_user_pass /
    mf_nmf_item_pass): unbiased, this is the reference's arithmetic up to summation
    order; biased, the item biases follow the delta-log schedule (epoch-start snapshot,
    count-aware merge).  Keyword-only device option: ``dtype``."""

    _algo = "nmf"

    def __init__(self, n_factors=15, n_epochs=50, biased=False, reg_pu=.06, reg_qi=.06,
                 reg_bu=.02, reg_bi=.02, lr_bu=.005, lr_bi=.005, init_low=0, init_high=1,
                 random_state=None, verbose=False, *, dtype=None):
        self.n_factors = n_factors
        self.n_epochs = n_epochs
        self.biased = biased
        self.reg_pu = reg_pu
        self.reg_qi = reg_qi
        self.lr_bu = lr_bu
        self.lr_bi = lr_bi
        self.reg_bu = reg_bu
        self.reg_bi = reg_bi
        self.init_low = init_low
        self.init_high = init_high
        self.random_state = random_state
        self.verbose = verbose
        if self.init_low < 0:
            raise ValueError('init_low should be greater than zero')
        self._device_options(dtype, "auto", 1, False, 0, False)
        AlgoBase.__init__(self)

    def fit(self, trainset):
        AlgoBase.fit(self, trainset)
        self.sgd(trainset)
        return self

    def sgd(self, trainset):
        """mf.pyx:646-735 on the device."""
        from .engine import NMFEngine

        _lib.require_gpu()
        if getattr(self, "_dtype_auto", False):
            self.dtype = self._auto_dtype()
        ts = _as_trainset(trainset)
        rng = get_rng(self.random_state)
        n_users, n_items, K = trainset.n_users, trainset.n_items, self.n_factors
        pu = rng.uniform(self.init_low, self.init_high, size=(n_users, K))
        qi = rng.uniform(self.init_low, self.init_high, size=(n_items, K))
        hyper = dict(lr_bu=self.lr_bu, lr_bi=self.lr_bi, reg_bu=self.reg_bu, reg_bi=self.reg_bi,
                     reg_pu=self.reg_pu, reg_qi=self.reg_qi,
                     global_mean=float(self.trainset.global_mean))
        eng = NMFEngine(ts.csr(), ts.csc(), n_items, K, hyper=hyper, biased=self.biased,
                        dtype=self.dtype)
        eng.set_factors(pu, qi)
        for e in range(self.n_epochs):
            if self.verbose:
                print("Processing epoch {}".format(e))
            eng.epoch()
        f = eng.get_factors()
        self._engine = eng
        self.bu, self.bi, self.pu, self.qi = f["bu"], f["bi"], f["pu"], f["qi"]

    def estimate(self, u, i):
        """mf.pyx:737-759 (host numpy fp64, per call)."""
        return SVD.estimate(self, u, i)


