"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference goldens.

Tolerances:
  * deterministic mode (one wavefront, reference order), fp64 on the device: factors within
    1e-9 of the reference's bit-exact arrays (only the dot-product summation order and FMA
    contraction differ);
  * deterministic fp32: factors within 1e-4, test RMSE within 1e-5;
  * the default "log" schedule (race-free, bit-reproducible) against ITS oracle
    (oracle_svd_sgd_deltalog, itself pinned to the reference goldens): fp64 factors within
    1e-9 -- the kernel computes exactly the schedule the oracle defines;
  * every parallel schedule ("log" = auto, "atomic"): held-out RMSE within 1e-3 of the
    reference on the same seed -- the bar BASELINE.json's north_star sets.  The exception is
    svd_k100_e20_unbiased (reference RMSE 2.28: the unbiased K=100 model diverges on u1, and
    the log schedule moves it by +5.5e-2 -- its CPU oracle alone does the same);
    there the log kernel is held to its oracle, the delta is recorded with an explicit bound
    and the deterministic mode meets the reference.
"""
import os
import pickle

import numpy as np
import pytest

import oracle as orc
from conftest import GOLDEN
from test_oracle_golden import (_oracle_test_rmse, run_oracle, run_oracle_log,
                                run_oracle_stalelog)

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-3


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from surprise_amd import _lib
    _lib.load()
    return torch


def _rmse(preds):
    from surprise_amd import accuracy
    return accuracy.rmse(preds, verbose=False)


def test_library_is_the_in_tree_hip_build(torch):
    from surprise_amd import _lib
    lib = _lib.load()
    assert lib._name == _lib.LIB_PATH
    assert lib.mf_version() >= 200


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_wave_sum_selftest(torch, dtype):
    import ctypes
    from surprise_amd import _lib
    tdt = getattr(torch, dtype)
    x = torch.randn(37 * 64, dtype=tdt, device="cuda")
    out = torch.zeros(37, dtype=tdt, device="cuda")
    _lib.call("mf_selftest_wave_sum", ctypes.c_void_p(x.data_ptr()),
              ctypes.c_void_p(out.data_ptr()), 37, 0 if dtype == "float32" else 1, None)
    torch.cuda.synchronize()
    ref = x.view(37, 64).double().sum(1)
    tol = 1e-4 if dtype == "float32" else 1e-12
    assert torch.allclose(out.double(), ref, atol=tol)


# ------------------------------------------------------- BASELINE configs[0] at its own size

@pytest.fixture(scope="module")
def synth_ml100k(golden, tmp_path_factory):
    """BASELINE configs[0]'s data: the ML-100k-shape synthetic ratings written to a file and read
    back through Reader / Dataset / KFold(5, random_state=0) -- the path make_golden.py ran the
    reference on (tests/golden/make_golden.py: synth_ml100k); the fold's CSR equals the
    reference's (sha)."""
    from surprise_amd import Dataset, Reader, synthetic
    from surprise_amd.model_selection import KFold
    from test_oracle_golden import _sha
    g = golden[0]["synth_ml100k"]
    u, i, r = synthetic.shape("ml-100k")
    path = tmp_path_factory.mktemp("ml100k") / "synth.tsv"
    with open(path, "w") as fh:
        for a, b, c in zip(u.tolist(), i.tolist(), r.tolist()):
            fh.write("%d\t%d\t%d\n" % (a, b, int(c)))
    data = Dataset.load_from_file(str(path), Reader(line_format="user item rating", sep="\t"))
    ts, test = next(KFold(5, random_state=0).split(data))
    assert (ts.n_users, ts.n_items, ts.n_ratings, len(test)) == \
        (g["n_users"], g["n_items"], g["n_ratings"], g["n_test"])
    assert _sha(*ts.csr()) == g["sha_csr"]
    return g, data, ts, test


def test_configs0_ml100k_svd_k20_e5_deterministic_fp64_equals_reference(torch, synth_ml100k):
    """BASELINE configs[0] (SVD n_factors=20 n_epochs=5, ML-100k shape, KFold(5, rs=0) fold 0)
    on the GPU at its own size, the reference's order (one wave) in fp64: factors within 1e-9
    of the oracle's, which are the reference's bit-for-bit (sha pinned in
    test_oracle_golden.test_synthetic_fold_matches_reference), and the held-out RMSE within
    1e-9 of the reference's own (golden.json synth_ml100k.svd_k20_e5)."""
    from surprise_amd import SVD
    g, _, ts, test = synth_ml100k
    params = dict(n_factors=20, n_epochs=5, random_state=0)
    row_ptr, items, ratings = ts.csr()
    _, f = run_oracle("SVD", params, row_ptr, items, ratings, ts.n_items, ts.global_mean)
    algo = SVD(**params, dtype="float64", deterministic=True).fit(ts)
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), f[k], rtol=0, atol=1e-9, err_msg=k)
    assert abs(_rmse(algo.test(test)) - g["svd_k20_e5"]["rmse"]) < 1e-9


@pytest.mark.parametrize("dtype", ["float64", "float32"])
def test_configs0_ml100k_parallel_schedule_within_1e3(torch, synth_ml100k, dtype):
    """configs[0] on the parallel schedule (the checkpoint log): held-out RMSE within 1e-3 of the
    reference's (mf.pyx:241-262 run by make_golden.py)."""
    from surprise_amd import SVD
    g, _, ts, test = synth_ml100k
    from surprise_amd import _lib
    algo = SVD(n_factors=20, n_epochs=5, random_state=0, dtype=dtype, deterministic=False).fit(ts)
    assert algo._engine.mode == _lib.MF_MODE_LOG and not algo.exact_order_
    got = _rmse(algo.test(test))
    assert abs(got - g["svd_k20_e5"]["rmse"]) < RMSE_TOL, (got, g["svd_k20_e5"]["rmse"])


@pytest.mark.parametrize("dtype", ["float64", "float32"])
def test_configs0_ml100k_default_is_the_exact_order(torch, synth_ml100k, dtype):
    """SVD's default (deterministic=None) at configs[0]'s size (80k ratings x 5 epochs, within
    EXACT_MAX_UPDATES): the reference's exact sequence -- in fp64 the reference's held-out RMSE to
    1e-9, in fp32 within 1e-4 of it."""
    from surprise_amd import SVD
    g, _, ts, test = synth_ml100k
    algo = SVD(n_factors=20, n_epochs=5, random_state=0, dtype=dtype).fit(ts)
    assert algo.exact_order_ and algo._engine.deterministic
    got = _rmse(algo.test(test))
    tol = 1e-9 if dtype == "float64" else 1e-4
    assert abs(got - g["svd_k20_e5"]["rmse"]) < tol, (got, g["svd_k20_e5"]["rmse"])


def test_configs0_ml100k_cross_validate_through_the_mirror(torch, synth_ml100k):
    """configs[0] driven the reference's way: cross_validate(SVD(...), data, cv=KFold(5, rs=0))
    (validation.py:29-142, split.py:86-122).  Fold 0 is the golden's fold: within 1e-3 of the
    reference's RMSE; every fold trains (RMSE below the fold's global-mean predictor)."""
    from surprise_amd import SVD
    from surprise_amd.model_selection import KFold, cross_validate
    g, data, _, _ = synth_ml100k
    res = cross_validate(SVD(n_factors=20, n_epochs=5, random_state=0), data,
                         measures=["rmse", "mae"], cv=KFold(5, random_state=0))
    assert len(res["test_rmse"]) == 5 and len(res["fit_time"]) == 5
    assert abs(res["test_rmse"][0] - g["svd_k20_e5"]["rmse"]) < RMSE_TOL, res["test_rmse"]
    for k, (tr, te) in enumerate(KFold(5, random_state=0).split(data)):
        r = np.array([x[2] for x in te])
        base = float(np.sqrt(np.mean((r - tr.global_mean) ** 2)))
        assert res["test_rmse"][k] < base, (k, res["test_rmse"][k], base)
        assert 0 < res["test_mae"][k] < res["test_rmse"][k]


# ----------------------------------------------------------------------------- u1 fixture

@pytest.mark.parametrize("name", ["svd_k20_e5", "svd_k10_e3_hyper", "svd_k5_e2_unbiased"])
def test_svd_deterministic_fp64_matches_reference_arrays(torch, golden, u1, name):
    from surprise_amd import SVD
    meta, arr = golden
    case = meta["cases"][name]
    ts, test = u1
    algo = SVD(**case["params"], dtype="float64", deterministic=True).fit(ts)
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), arr[name + "_" + k], rtol=0, atol=1e-9)
    assert abs(_rmse(algo.test(test)) - case["rmse"]) < 1e-9


def test_svd_deterministic_fp32_matches_reference(torch, golden, u1):
    from surprise_amd import SVD
    meta, arr = golden
    case = meta["cases"]["svd_k20_e5"]
    ts, test = u1
    algo = SVD(**case["params"], deterministic=True).fit(ts)
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), arr["svd_k20_e5_" + k], rtol=0, atol=1e-4)
    assert abs(_rmse(algo.test(test)) - case["rmse"]) < 1e-5


@pytest.mark.parametrize("name", ["svd_k20_e5", "svd_k5_e2_unbiased", "svd_k10_e3_hyper"])
@pytest.mark.parametrize("chunks", [1, 3])
@pytest.mark.parametrize("merge", ["count", "recency"])
def test_log_mode_fp64_matches_deltalog_oracle(torch, golden, u1, name, chunks, merge):
    """The log schedule's fold -- count-aware weight or recency weights (replay-side) -- in fp64
    against oracle_svd_sgd_deltalog (merge 2 / 3) on the same chunking, to 1e-9."""
    from surprise_amd import SVD
    from surprise_amd.dist import chunk_users
    meta, _ = golden
    case = meta["cases"][name]
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    cou = np.zeros(ts.n_users, np.int32)
    for c, us in enumerate(chunk_users(np.arange(ts.n_users), row_ptr, chunks)):
        cou[us] = c
    P, f = run_oracle_log("SVD", case["params"], row_ptr, items, ratings, ts.n_items,
                          ts.global_mean, cou, chunks, merge=2 if merge == "count" else 3)
    algo = SVD(**case["params"], dtype="float64", chunks_per_epoch=chunks)
    algo._engine_options = {"merge": merge}
    algo.fit(ts)
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), f[k], rtol=0, atol=1e-9, err_msg=k)
    ref = _oracle_test_rmse(P, f, "SVD", ts, list(test))[1]
    assert abs(_rmse(algo.test(test)) - ref) < 1e-9


@pytest.mark.parametrize("name", ["svd_k100_e20", "svd_k100_e20_unbiased"])
def test_log_mode_long_runs_track_deltalog_oracle(torch, golden, u1, name):
    """20 epochs: fp64 within 1e-6 RMSE of the schedule's oracle, fp32 within 1e-4."""
    from surprise_amd import SVD
    meta, _ = golden
    case = meta["cases"][name]
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    P, f = run_oracle_log("SVD", case["params"], row_ptr, items, ratings, ts.n_items,
                          ts.global_mean, merge=3)
    ref = _oracle_test_rmse(P, f, "SVD", ts, list(test))[1]
    got64 = _rmse(SVD(**case["params"], dtype="float64", deterministic=False).fit(ts).test(test))
    got32 = _rmse(SVD(**case["params"], dtype="float32", deterministic=False).fit(ts).test(test))
    assert abs(got64 - ref) < 1e-6, (got64, ref)
    assert abs(got32 - ref) < 1e-4, (got32, ref)


def test_unbiased_k100_u1_default_meets_reference_parallel_delta_recorded(torch, golden, u1):
    """svd_k100_e20_unbiased (mf.pyx:238-239, 253-255: no biases, mu = 0): the reference's
    held-out RMSE is 2.2754 -- the model diverges on u1 (the global mean alone scores 1.137).
    SVD's default at this size (80k ratings x 20 epochs <= EXACT_MAX_UPDATES) is the exact
    order: the reference's RMSE to 1e-9 in fp64.  The parallel schedule (deterministic=False)
    ends +5.5e-2 from it and does NOT meet the 1e-3 bar on this diverging model:
    its CPU restatement (oracle_svd_sgd_deltalog, merge=3) ends at the same +5.51e-2 and only
    approaches the reference as the chunks approach one user each (+3.8e-3 at 128 chunks), so
    the schedule, not the kernel, moves it.  That delta is bounded so a change is visible."""
    from surprise_amd import SVD
    meta, _ = golden
    case = meta["cases"]["svd_k100_e20_unbiased"]
    ts, test = u1
    algo = SVD(**case["params"], dtype="float64").fit(ts)
    assert algo.exact_order_
    assert abs(_rmse(algo.test(test)) - case["rmse"]) < 1e-9
    delta = _rmse(SVD(**case["params"], dtype="float64", deterministic=False).fit(ts)
                  .test(test)) - case["rmse"]
    assert 0.050 < delta < 0.060, delta


def test_log_mode_is_bit_reproducible(torch, u1):
    from surprise_amd import SVD
    ts, _ = u1
    a = SVD(n_factors=100, n_epochs=5, random_state=0, deterministic=False).fit(ts)
    b = SVD(n_factors=100, n_epochs=5, random_state=0, deterministic=False).fit(ts)
    assert not a.exact_order_ and a._engine.mode == __import__("surprise_amd")._lib.MF_MODE_LOG
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k))


@pytest.mark.parametrize("name", ["svd_k20_e5", "svd_k100_e20", "svd_k128_e20",
                                  "svd_k10_e3_hyper"])
@pytest.mark.parametrize("mode", ["auto", "atomic"])
def test_svd_parallel_rmse_within_1e3(torch, golden, u1, name, mode):
    from surprise_amd import SVD
    meta, arr = golden
    case = meta["cases"][name]
    ts, test = u1
    algo = SVD(**case["params"], mode=mode, deterministic=False).fit(ts)
    preds = algo.test(test)
    assert abs(_rmse(preds) - case["rmse"]) < RMSE_TOL
    assert sum(p.details["was_impossible"] for p in preds) == case["impossible"]


@pytest.mark.parametrize("name", ["svdpp_k10_e3", "svdpp_k8_e2_hyper"])
def test_svdpp_deterministic_fp64_matches_reference_arrays(torch, golden, u1, name):
    from surprise_amd import SVDpp
    meta, arr = golden
    case = meta["cases"][name]
    ts, test = u1
    algo = SVDpp(**case["params"], dtype="float64", deterministic=True).fit(ts)
    for k in ("pu", "qi", "yj", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), arr[name + "_" + k], rtol=0, atol=1e-9)
    assert abs(_rmse(algo.test(test)) - case["rmse"]) < 1e-9


@pytest.mark.parametrize("name", ["svdpp_k20_e20", "svdpp_k100_e20", "svdpp_k10_e3"])
@pytest.mark.parametrize("mode", ["auto", "atomic"])
def test_svdpp_parallel_rmse_within_1e3(torch, golden, u1, name, mode):
    from surprise_amd import SVDpp
    meta, _ = golden
    case = meta["cases"][name]
    ts, test = u1
    algo = SVDpp(**case["params"], mode=mode).fit(ts)
    assert abs(_rmse(algo.test(test)) - case["rmse"]) < RMSE_TOL


@pytest.mark.parametrize("opt", [{"helpers": False}, {"ydefer": False},
                                 {"hx_chains_per_cu": 1}, {"helpers": 1}])
def test_svdpp_atomic_alternatives_rmse_within_1e3(torch, golden, u1, opt):
    """SVD++'s non-default atomic-mode paths (MFEngine helpers=False: the chain wave issues its
    own q atomics; ydefer=False: y_j updated by float atomics at each user's end;
    hx_chains_per_cu=1: one helper-wave chain per CU; helpers=1: one helper wave per chain,
    4 chains per CU -- MF_EPOCH_SVDPP_ONE_HELPER) within 1e-3 of the reference's held-out RMSE,
    like the default."""
    from surprise_amd import SVDpp
    meta, _ = golden
    case = meta["cases"]["svdpp_k20_e20"]
    ts, test = u1
    algo = SVDpp(**case["params"], mode="atomic")
    algo._engine_options = opt
    algo.fit(ts)
    eng = algo._engine
    want = {"helpers": (False, True), "ydefer": (False, False), "hx_chains_per_cu": (True, True)}
    if opt.get("helpers") == 1:
        want["helpers"] = (True, True)
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        assert eng.hx_helpers == 1 and eng.hx_chains == 4 * cus
    assert (eng.hx, eng.ydefer) == want[next(iter(opt))]
    assert abs(_rmse(algo.test(test)) - case["rmse"]) < RMSE_TOL


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_svdpp_hot_row_replicas_rmse_within_1e3(torch, golden, u1, dtype):
    """Delta replicas of the 32 most-rated items' q rows (MFEngine hot_rows: half the chains'
    atomics on a hot row go to its replica, every read sums both, mf_svdpp_hot_fold after each
    chunk) hold the reference's RMSE like the default, and leave the replica rows zero."""
    from surprise_amd import SVDpp
    meta, _ = golden
    case = meta["cases"]["svdpp_k20_e20"]
    ts, test = u1
    algo = SVDpp(**case["params"], mode="atomic", dtype=dtype)
    algo._engine_options = {"hot_rows": 32}
    algo.fit(ts)
    eng = algo._engine
    assert eng.hx and eng.hot_list is not None and eng.hot_list.numel() == 32
    assert eng._qb_alloc.shape[0] == 2 * eng.n_items
    assert float(eng._qb_alloc[eng.n_items:].abs().max()) == 0.0
    assert abs(_rmse(algo.test(test)) - case["rmse"]) < RMSE_TOL


def test_batched_test_equals_per_call_estimate(torch, u1):
    """The HIP predict kernel (batched test()) agrees with the reference-style estimate()."""
    from surprise_amd import SVD, SVDpp
    from surprise_amd.algo_base import AlgoBase
    ts, test = u1
    for algo in (SVD(n_factors=30, n_epochs=3, random_state=0),
                 SVD(n_factors=30, n_epochs=3, biased=False, random_state=0),
                 SVDpp(n_factors=12, n_epochs=2, random_state=0)):
        algo.fit(ts)
        fast = algo.test(test)
        slow = AlgoBase.test(algo, test)
        np.testing.assert_allclose([p.est for p in fast], [p.est for p in slow], atol=1e-5)
        assert [p.details for p in fast] == [p.details for p in slow]
        assert [p[:3] for p in fast] == [p[:3] for p in slow]


@pytest.mark.parametrize("name", ["svd_k20_e5", "svd_k20_e5_unbiased", "svd_k10_e3_hyper"])
@pytest.mark.parametrize("dtype", ["float64", "float32"])
def test_blocked_solve_heavy_users_match_deltalog_oracle(torch, golden, u1, name, dtype):
    """The heavy users' blocked solve (mf_svd_epoch_gram: 16-rating blocks, the errors from the
    block's item-row Gram matrix) forced on u1's 64 heaviest users beside the lookahead chains of
    the rest -- partial blocks, odd rating counts, the unbiased layout and separate lr / reg per
    parameter included -- against oracle_svd_sgd_deltalog(merge=3): fp64 to 1e-9, fp32 to 1e-4;
    and equal to the same split without the blocked solve (gram=False) within rounding."""
    from surprise_amd import SVD
    meta, _ = golden
    if name == "svd_k20_e5_unbiased":  # (fp64 K=5 rows have no room for the error columns)
        params = dict(meta["cases"]["svd_k20_e5"]["params"], biased=False)
    else:
        params = meta["cases"][name]["params"]
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    P, f = run_oracle_log("SVD", params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                          merge=3)
    fits = {}
    for gram in (True, False):
        algo = SVD(**params, dtype=dtype)
        algo._engine_options = {"heavy": 64, "gram": gram}
        algo.fit(ts)
        eng = algo._engine
        assert eng.logs[0]["heavy"] is not None and eng.gram == gram
        fits[gram] = algo
    tol = 1e-9 if dtype == "float64" else 1e-4
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(getattr(fits[True], k), f[k], rtol=0, atol=tol, err_msg=k)
        np.testing.assert_allclose(getattr(fits[True], k), getattr(fits[False], k), rtol=0,
                                   atol=tol, err_msg=k)


def test_unknown_user_and_item_match_reference(torch, golden):
    """test_algorithms.py:28-57 with the reference's estimates as known answers."""
    from surprise_amd import SVD, SVDpp, Dataset, Reader
    meta, _ = golden
    reader = Reader(line_format="user item rating", sep=" ", skip_lines=3, rating_scale=(1, 5))
    data = Dataset.load_from_file(os.path.join(GOLDEN, "custom_dataset"), reader)
    ts = data.build_full_trainset()
    for key, rows in meta["unknown"].items():
        kw = dict(random_state=0, dtype="float64", deterministic=True)
        if key == "SVD_unbiased":
            kw["biased"] = False
        algo = (SVDpp if key.startswith("SVDpp") else SVD)(**kw).fit(ts)
        for uid, iid, est, details in rows:
            p = algo.predict(uid, iid, None)
            assert abs(p.est - est) < 1e-9, (key, uid, iid)
            assert p.details == details
        # batched path gives the same
        preds = algo.test([(r[0], r[1], 3.0) for r in rows])
        assert [p.details for p in preds] == [r[3] for r in rows]
        np.testing.assert_allclose([p.est for p in preds], [r[2] for r in rows], atol=1e-9)


def test_sensitivity_sweep_cross_validate(torch, golden):
    """test_SVD.py:25-108 through cross_validate + PredefinedKFold: every parameter changes
    the RMSE, and non-divergent settings match the reference's values."""
    from surprise_amd import SVD, SVDpp, Dataset, Reader
    from surprise_amd.model_selection import PredefinedKFold, cross_validate
    meta, _ = golden
    data = Dataset.load_from_folds([(os.path.join(GOLDEN, "u1_ml100k_train"),
                                     os.path.join(GOLDEN, "u1_ml100k_test"))], Reader("ml-100k"))
    pkf = PredefinedKFold()
    got = {}
    for key, rec in meta["sensitivity"].items():
        klass = SVDpp if key.startswith("SVDpp") else SVD
        res = cross_validate(klass(**rec["params"]), data, ["rmse"], pkf)
        got[key] = float(res["test_rmse"][0])
        params = rec["params"]
        divergent = any(v == 5 for k, v in params.items() if k.startswith(("lr", "reg")))
        if not divergent:
            assert abs(got[key] - rec["test_rmse"]) < RMSE_TOL, key
    assert got["SVD_default"] not in [v for k, v in got.items() if k.startswith("SVD_")
                                      and k != "SVD_default"]
    assert got["SVDpp_default"] != got["SVDpp_n_factors"]


def test_pickle_round_trip(torch, u1, tmp_path):
    """test_dump.py: dumped predictions and the dumped algorithm's predictions are equal."""
    from surprise_amd import SVD, dump
    ts, test = u1
    algo = SVD(n_factors=10, n_epochs=2, random_state=0).fit(ts)
    preds = algo.test(test)
    f = str(tmp_path / "dump")
    dump.dump(f, preds, algo)
    preds2, algo2 = dump.load(f)
    assert algo2._engine is None
    assert preds == preds2
    preds3 = algo2.test(test)  # device tables rebuilt from the unpickled arrays
    assert algo2._engine is not None
    np.testing.assert_allclose([p.est for p in preds3], [p.est for p in preds], atol=1e-5)
    s = pickle.dumps(SVD(n_factors=3))  # unfitted: __init__ touches no GPU state
    assert pickle.loads(s).n_factors == 3


# ----------------------------------------------------------------------------- synthetic shapes

def _synthetic_fold(name):
    from surprise_amd import Dataset, synthetic
    from surprise_amd.model_selection import KFold
    u, i, r = synthetic.shape(name)
    return next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))


@pytest.fixture(scope="module")
def ml1m():
    return _synthetic_fold("ml-1m")


def _oracle_rmse(algo, params, ts, test, **kw):
    row_ptr, items, ratings = ts.csr()
    P, f = run_oracle(algo, params, row_ptr, items, ratings, ts.n_items, ts.global_mean, **kw)
    tlist = list(test)
    return _oracle_test_rmse(P, f, algo, ts, tlist)[1]


@pytest.mark.slow
@pytest.mark.parametrize("mode", ["auto", "atomic"])
def test_c2_ml1m_svd_k100_e20_rmse_within_1e3(torch, ml1m, mode):
    """BASELINE configs[1]: SVD n_factors=100 n_epochs=20 on the ML-1M shape, KFold(5, rs=0)
    fold 0; the fp64 sequential oracle is the reference Cython restated bit-exactly."""
    from surprise_amd import SVD
    ts, test = ml1m
    params = dict(n_factors=100, n_epochs=20, random_state=0)
    ref = _oracle_rmse("SVD", params, ts, test)
    got = _rmse(SVD(**params, mode=mode).fit(ts).test(test))
    assert abs(got - ref) < RMSE_TOL, (got, ref)


@pytest.mark.slow
@pytest.mark.parametrize("top", [None, 16])
def test_headline_configuration_fp64_matches_deltalog_oracle(torch, ml1m, top):
    """The bench headline's own kernel configuration at factor level: SVD K=100 in fp64 on the
    ML-1M-shape fold through the default path, which at this size splits every epoch into the
    128 heaviest users' launch on XCD 0 beside the other users' launch on XCDs 1-7 (top=None,
    the default) -- or with the engine option top=16 the 16 heaviest on XCD 0 and the other
    112 on XCD 1 on a third stream, the light + rest sums pre-folded and the top users' added by
    the last mf_log_apply -- each group with its own checkpoint replay (the split u1 is too
    small to take).  pu, qi, bu, bi after 3 epochs equal
    oracle_svd_sgd_deltalog(merge=3) -- the schedule restated on the CPU, pinned to the
    reference by the u1 goldens -- to 1e-9."""
    from surprise_amd import SVD
    ts, test = ml1m
    params = dict(n_factors=100, n_epochs=3, random_state=0)
    algo = SVD(**params, dtype="float64", deterministic=False)
    if top is not None:
        algo._engine_options = {"top": top}
    algo.fit(ts)
    eng = algo._engine
    assert eng.ckpt and eng.logs[0]["heavy"] is not None, "the heavy/light split is off"
    if top:
        assert eng.logs[0]["heavy"]["sched"].numel() == top
        assert eng.logs[0]["mid"]["sched"].numel() == eng.HEAVY_USERS - top
    else:
        assert eng.logs[0]["heavy"]["sched"].numel() == eng.HEAVY_USERS
        assert eng.logs[0].get("mid") is None
    from surprise_amd import _lib
    if _lib.xcd_layout_ok():  # (the XCD masks need the 8-XCD round-robin dispatch)
        assert eng.heavy_xcd == 1, "the XCD-masked launches are off"
    else:  # (report what the device showed: a partitioned or non-round-robin dispatch)
        import ctypes
        ids = torch.zeros(64, dtype=torch.int32, device="cuda")
        _lib.call("mf_selftest_xcc", ctypes.c_void_p(ids.data_ptr()), 64, None)
        torch.cuda.synchronize()
        import warnings
        warnings.warn("XCD layout check failed; XCC_ID of blocks 0..63: %s" % ids.tolist())
        assert eng.heavy_xcd == 0
    row_ptr, items, ratings = ts.csr()
    P, f = run_oracle_log("SVD", params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                          merge=3)
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), f[k], rtol=0, atol=1e-9, err_msg=k)
    ref = _oracle_test_rmse(P, f, "SVD", ts, list(test))[1]
    assert abs(_rmse(algo.test(test)) - ref) < 1e-9


_C3_REF = {}


@pytest.mark.slow
@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_c3_ml1m_svdpp_k100_rmse_within_1e3(torch, ml1m, dtype):
    """BASELINE configs[2]: SVD++ n_factors=100 on the ML-1M shape at the reference's default 20
    epochs (mf.pyx:389-411), in the product's fp32 and in the reference's fp64 arithmetic; the
    oracle is the exact per-user affine form of SVDpp.sgd in fp64 (pinned bit-for-bit to the
    literal form on u1, tests/test_oracle_golden.py)."""
    from surprise_amd import SVDpp
    ts, test = ml1m
    params = dict(n_factors=100, n_epochs=20, random_state=0)
    if "ref" not in _C3_REF:
        _C3_REF["ref"] = _oracle_rmse("SVDpp", params, ts, test, affine=True)
    ref = _C3_REF["ref"]
    got = _rmse(SVDpp(**params, dtype=dtype).fit(ts).test(test))
    assert abs(got - ref) < RMSE_TOL, (got, ref)


@pytest.mark.parametrize("K,dtype", [(128, "float32"), (64, "float64")])
def test_svdpp_item_bias_beside_lane_groups_rmse(torch, u1, K, dtype):
    """The helper-wave launch with the item bias carried beside the lane groups (the factor
    columns fill whole 512-byte groups: fp32 K=128, fp64 K=64 -- C5's layout) within 1e-3
    of the exact per-user oracle's held-out RMSE, and hot-row replicas (which keep the bias in
    the row) within 1e-3 of it too."""
    from surprise_amd import SVDpp
    ts, test = u1
    params = dict(n_factors=K, n_epochs=10, random_state=0)
    ref = _oracle_rmse("SVDpp", params, ts, test, affine=True)
    for opt in ({}, {"hot_rows": 16}):
        algo = SVDpp(**params, mode="atomic", dtype=dtype)
        algo._engine_options = opt
        algo.fit(ts)
        assert algo._engine.hx
        got = _rmse(algo.test(test))
        assert abs(got - ref) < RMSE_TOL, (opt, got, ref)


@pytest.mark.parametrize("K,chunks", [(10, 1), (10, 3), (64, 2)])
@pytest.mark.parametrize("fused", [True, False])
def test_svdpp_qlog_fp64_matches_stalelog_oracle(torch, u1, K, chunks, fused):
    """SVD++ with the q log (mf_svdpp_epoch_qlog: item rows read-only within a chunk, gradient
    rows folded with recency weights, y deferred) in fp64 against oracle_svdpp_sgd_stalelog with
    every item stale, same chunking, to 1e-9 -- K=64 is the layout with the item bias beside the
    lane group (fp64 K * 8 = 512 B).  fused: the one-pass fold (mf_svdpp_qlog_fold); else
    mf_log_reduce + mf_log_apply + mf_svdpp_y_fold."""
    from surprise_amd import SVDpp
    from surprise_amd.dist import chunk_users
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    params = dict(n_factors=K, n_epochs=3, random_state=0)
    cou = np.zeros(ts.n_users, np.int32)
    for c, us in enumerate(chunk_users(np.arange(ts.n_users), row_ptr, chunks)):
        cou[us] = c
    P, f = run_oracle_stalelog(params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                               cou, chunks)
    algo = SVDpp(**params, dtype="float64", chunks_per_epoch=chunks)
    algo._engine_options = {"qlog": True, "fused": fused, "log_nt": fused}  # (nt with fused)
    algo.fit(ts)
    assert algo._engine.qlog_pp and not algo._engine.hx
    assert algo._engine._fused_fold() == fused
    for k in ("pu", "qi", "yj", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), f[k], rtol=0, atol=1e-9, err_msg=k)
    ref = _oracle_test_rmse(P, f, "SVDpp", ts, list(test))[1]
    assert abs(_rmse(algo.test(test)) - ref) < 1e-9


def test_svdpp_qlog_fp32_k128_tracks_stalelog_oracle(torch, u1):
    """The q log at C5's layout (fp32 K=128: one lane group, the item bias beside it) over 4
    chunks: held-out RMSE within 1e-4 of its fp64 oracle, and within 1e-3 of the exact
    per-user reference form."""
    from surprise_amd import SVDpp
    from surprise_amd.dist import chunk_users
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    params = dict(n_factors=128, n_epochs=10, random_state=0)
    cou = np.zeros(ts.n_users, np.int32)
    for c, us in enumerate(chunk_users(np.arange(ts.n_users), row_ptr, 4)):
        cou[us] = c
    P, f = run_oracle_stalelog(params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                               cou, 4)
    ref = _oracle_test_rmse(P, f, "SVDpp", ts, list(test))[1]
    algo = SVDpp(**params, chunks_per_epoch=4, dtype="float32")
    algo._engine_options = {"qlog": True}
    got = _rmse(algo.fit(ts).test(test))
    assert algo._engine.qlog_pp
    assert abs(got - ref) < 1e-4, (got, ref)
    exact = _oracle_rmse("SVDpp", params, ts, test, affine=True)
    assert abs(got - exact) < RMSE_TOL, (got, exact)


@pytest.mark.parametrize("K", [1, 3, 17, 64, 65, 100, 128, 200, 256, 300, 512])
def test_factor_counts_deterministic_fp32(torch, u1, K):
    """Every lane layout (V = 1, 2, 4, 8 elements per lane, padded and unpadded ld)."""
    from surprise_amd import SVD
    ts, test = u1
    params = dict(n_factors=K, n_epochs=2, random_state=0)
    row_ptr, items, ratings = ts.csr()
    P, f = run_oracle("SVD", params, row_ptr, items, ratings, ts.n_items, ts.global_mean)
    algo = SVD(**params, deterministic=True, dtype="float32").fit(ts)
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), f[k], rtol=0, atol=2e-4)


def test_duplicate_items_forwarding_fp64(torch):
    """A user rating the same item twice: the second rating must see the first's update."""
    from surprise_amd import SVD, Trainset
    rng = np.random.RandomState(1)
    n_users, n_items = 40, 12
    rows = [rng.randint(0, n_items, size=rng.randint(1, 30)) for _ in range(n_users)]
    row_ptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    items = np.concatenate(rows).astype(np.int32)
    ratings = rng.randint(1, 6, size=len(items)).astype(np.float64)
    ts = Trainset.from_csr(row_ptr, items, ratings, n_items)
    params = dict(n_factors=16, n_epochs=3, random_state=0)
    P, f = run_oracle("SVD", params, row_ptr, items, ratings, n_items, ts.global_mean)
    algo = SVD(**params, dtype="float64", deterministic=True).fit(ts)
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), f[k], rtol=0, atol=1e-9)


def test_zero_epochs_and_single_rating_users(torch):
    from surprise_amd import SVD, Trainset
    row_ptr = np.array([0, 1, 2, 3, 5], np.int64)
    items = np.array([0, 1, 0, 2, 1], np.int32)
    ratings = np.array([5, 3, 1, 4, 2], np.float64)
    ts = Trainset.from_csr(row_ptr, items, ratings, 3)
    a0 = SVD(n_factors=4, n_epochs=0, random_state=0).fit(ts)
    rng = np.random.RandomState(0)
    np.testing.assert_allclose(a0.pu, rng.normal(0, .1, (4, 4)), atol=1e-7)
    params = dict(n_factors=4, n_epochs=7, random_state=0)
    P, f = run_oracle("SVD", params, row_ptr, items, ratings, 3, ts.global_mean)
    a = SVD(**params, dtype="float64", deterministic=True).fit(ts)
    np.testing.assert_allclose(a.pu, f["pu"], atol=1e-9)


@pytest.mark.parametrize("K,dtype,chunks", [(20, "float64", 1), (20, "float64", 3),
                                            (100, "float64", 2), (100, "float32", 1),
                                            (126, "float32", 2)])
def test_checkpoint_log_matches_gradient_log(torch, u1, K, dtype, chunks):
    """The checkpoint log (one user row per pair of ratings, errors in the rows' padding -- or in
    elog where the row has no room, K=126 fp32 --, mf_log_replay rebuilding the gradients by
    undoing one step, <pu^2> from user_sq) against the gradient log (a whole gradient row per
    rating, mf_log_reduce, mf_sumsq): the same epochs from the same state.  Same arithmetic up
    to the summation of the statistic and one rounding per rating: fp64 within 1e-10, fp32
    within 1e-5."""
    from surprise_amd import _lib
    from surprise_amd.engine import MFEngine
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    rng = np.random.RandomState(0)
    pu0, qi0 = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    out = []
    for ck in (True, False):
        eng = MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype=dtype,
                       mode="log", n_chunks=chunks, ckpt=ck)
        assert eng.ckpt == ck
        assert eng.err_in_row == (ck and K != 126)
        eng.set_factors(pu0, qi0)
        eng.run_epochs(4)
        out.append(eng.get_factors())
    tol = 1e-10 if dtype == "float64" else 1e-5
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(out[0][k], out[1][k], rtol=0, atol=tol, err_msg=k)
    assert _lib.load().mf_ckpt_interval() >= 2


def test_heavy_user_split_matches_single_launch(torch, u1):
    """The two-stream split (the heaviest users' epoch kernel + replay on their own stream, the
    default for small epochs on a full MI355X; here forced with heavy=0.25) computes the same
    schedule as one launch: per item the two groups' piece sums are added in a fixed order
    (mf_log_apply's sums2)."""
    from surprise_amd.engine import MFEngine
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    K = 20
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    rng = np.random.RandomState(1)
    pu0, qi0 = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    out = []
    for heavy in (0.0, 0.25):
        eng = MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype="float64",
                       mode="log", heavy=heavy)
        assert (eng.logs[0]["heavy"] is not None) == (heavy > 0)
        eng.set_factors(pu0, qi0)
        eng.run_epochs(3)
        out.append(eng.get_factors())
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(out[0][k], out[1][k], rtol=0, atol=1e-10, err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("which,K,dtype,chunks", [("ml1m", 100, "float64", 1),
                                                  ("ml1m", 100, "float32", 2),
                                                  ("u1", 128, "float32", 1),
                                                  ("u1", 128, "float64", 2)])
def test_replay_fold_equals_separate_fold(torch, request, which, K, dtype, chunks):
    """The split chunk's fold inside its two log replays (engine option replay_fold,
    mf_launch_fold: the wave that completes an item's last piece applies the item, the last
    block of both replays sums the next chunk's <p^2>) against the separate mf_log_apply launch:
    the same arithmetic in the same order (apply_item), so the fits are bit-identical -- with a
    batched predict between epochs, several chunks (the <p^2> slots), fp32 K=128's item-bias
    mirror and fp64 K=128's narrow rows."""
    from surprise_amd.engine import MFEngine
    ts, _ = request.getfixturevalue(which)
    row_ptr, items, ratings = ts.csr()
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    heavy = 0.25 if which == "u1" else None
    rng = np.random.RandomState(5)
    pu0, qi0 = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    uu = np.arange(ts.n_users, dtype=np.int32) % ts.n_users
    ii = np.arange(ts.n_users, dtype=np.int32) % ts.n_items
    out = []
    for rf in (True, False):
        eng = MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype=dtype,
                       mode="log", n_chunks=chunks, heavy=heavy, replay_fold=rf)
        assert eng.ckpt and eng.logs[0]["heavy"] is not None
        eng.set_factors(pu0, qi0)
        ests = [None]
        eng.run_epochs(2)
        ests[0] = eng.predict(uu, ii, ts.global_mean)[0]
        eng.run_epochs(2)
        f = eng.get_factors()
        f["est"] = ests[0]
        assert eng.replay_folds_run == (4 * chunks if rf else 0), eng.replay_folds_run
        assert int(eng._fold_cnt.abs().sum()) == 0 if rf else True  # (counters back to 0)
        out.append(f)
    for k in ("pu", "qi", "bu", "bi", "est"):
        np.testing.assert_array_equal(out[0][k], out[1][k], err_msg=k)


@pytest.mark.parametrize("which,chunks", [("u1", 1), ("u1", 3), ("ml1m", 1)])
@pytest.mark.parametrize("top", [0, 16])
def test_native_fork_and_kernel_join_equal_torch_events(torch, request, monkeypatch, which,
                                                          chunks, top):
    """The split chunk's fork as a native event bound to the previous chunk's mf_log_apply
    (mf_launch_event) and its join inside the two replays (mf_launch_join: the heavy replay's
    last block waits for the light replay's) against torch.cuda.Event record / wait_event: the
    same kernels on the same data, so the fits are bit-identical -- with main-stream work (a
    batched predict) between epochs, after which the fork must be recorded again.  top=16
    (ML-1M: the heavy launch split in two on two streams, the light + rest sums pre-folded):
    native events against torch events, both with the event join."""
    from surprise_amd.engine import MFEngine
    ts, _ = request.getfixturevalue(which)
    row_ptr, items, ratings = ts.csr()
    K = 100
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    heavy = 0.25 if which == "u1" else None  # (ML-1M: the default split, 128 heaviest users)
    rng = np.random.RandomState(3)
    pu0, qi0 = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    uu = np.arange(ts.n_users, dtype=np.int32) % ts.n_users
    ii = np.arange(ts.n_users, dtype=np.int32) % ts.n_items
    out = []
    for native in ("1", "0"):
        kjoin = native == "1" and top == 0
        eng = MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype="float32",
                       mode="log", n_chunks=chunks, heavy=heavy,
                       events="native" if native == "1" else "torch",
                       join="kernel" if kjoin else "event", top=top)
        assert eng.logs[0]["heavy"] is not None and (eng._nev is not None) == (native == "1")
        assert (eng._join_words is not None) == kjoin
        if top and which == "ml1m":
            assert eng.logs[0]["mid"] is not None
        eng.set_factors(pu0, qi0)
        ests = []
        eng.run_epochs(2)
        ests.append(eng.predict(uu, ii, ts.global_mean)[0])
        eng.run_epochs(2)
        f = eng.get_factors()
        f["est"] = np.concatenate(ests)
        out.append(f)
    for k in ("pu", "qi", "bu", "bi", "est"):
        np.testing.assert_array_equal(out[0][k], out[1][k], err_msg=k)


@pytest.mark.parametrize("K,dtype,heavy", [(100, "float32", 0.25), (20, "float64", 0.0),
                                            (60, "float64", 0.25)])
def test_errors_in_checkpoint_rows_equal_elog(torch, u1, monkeypatch, K, dtype, heavy):
    """MF_EPOCH_ERR_IN_ROW (each pair's errors stored in its checkpoint row's padding, read back
    by the replay from the loaded row) against the errors in elog (err_in_row=False):
    the same values reach the same operations, so the fits are bit-identical (split and unsplit
    chunks)."""
    from surprise_amd.engine import MFEngine
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    rng = np.random.RandomState(2)
    pu0, qi0 = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    out = []
    for in_row in (True, False):
        eng = MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype=dtype,
                       mode="log", heavy=heavy, err_in_row=in_row)
        assert eng.ckpt and eng.err_in_row == in_row
        eng.set_factors(pu0, qi0)
        eng.run_epochs(3)
        out.append(eng.get_factors())
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_array_equal(out[0][k], out[1][k], err_msg=k)


@pytest.mark.parametrize("K,dtype,heavy,auto", [(128, "float32", 0.0, True),
                                                 (64, "float32", 0.25, True),
                                                 (48, "float64", 0.0, True),
                                                 (64, "float64", 0.25, True),
                                                 (21, "float32", 0.25, False),
                                                 (20, "float64", 0.0, False)])
def test_narrow_checkpoint_rows_match_padded_rows(torch, u1, K, dtype, heavy, auto):
    """MF_EPOCH_CKPT_NARROW (checkpoint rows of the K factor columns only, errors in elog, the
    bias column's gradient summed from the errors) against the padded rows: the same gradients,
    the bias column summed in another order (fp64 within 1e-12, fp32 within 1e-5); auto: the
    engine picks narrow rows by itself (rows of whole 128-byte lines).  fp32 K=128 and fp64
    K=64 fill whole lane groups: the epoch kernel then also carries both biases beside the
    groups (one lane group instead of two, the SB form of epoch_body_la)."""
    from surprise_amd.engine import MFEngine
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    rng = np.random.RandomState(4)
    pu0, qi0 = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    out = []
    for narrow in (None if auto else True, False):
        eng = MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype=dtype,
                       mode="log", heavy=heavy, narrow=narrow)
        assert eng.ckpt and eng.narrow == (narrow is not False)
        assert eng.qlog.shape[1] == (eng.ldc if eng.narrow else eng.ldq)
        eng.set_factors(pu0, qi0)
        eng.run_epochs(3)
        out.append(eng.get_factors())
    tol = 1e-12 if dtype == "float64" else 1e-5
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(out[0][k], out[1][k], rtol=0, atol=tol, err_msg=k)


@pytest.mark.parametrize("K,heavy", [(20, 0.0), (100, 16), (128, 0.0)])
def test_nontemporal_log_stores_match_deltalog_oracle(torch, u1, K, heavy):
    """log_nt (MF_EPOCH_LOG_NT, the default for logs of >= 2 GiB -- C4): the checkpoint rows
    stored non-temporal change a cache policy, not a value: fp64 factors equal
    oracle_svd_sgd_deltalog (merge=3) to 1e-9 (K=20 padded rows with errors, K=100 with the
    heavy split, K=128 the narrow rows)."""
    from surprise_amd.engine import MFEngine
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    rng = np.random.RandomState(10)
    pu0, qi0 = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    eng = MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype="float64",
                   mode="log", heavy=heavy, log_nt=True)
    assert eng.ckpt and eng.log_nt
    eng.set_factors(pu0, qi0)
    eng.run_epochs(3)
    got = eng.get_factors()
    hp = orc.hyper(**{k: v for k, v in hyper.items() if k != "global_mean"})
    pu, qi, bu, bi = orc.svd_sgd_deltalog(row_ptr, items, ratings, ts.n_items, K, 3, True,
                                          ts.global_mean, hp, pu0.copy(), qi0.copy(), merge=3)
    for k, ref in (("pu", pu), ("qi", qi), ("bu", bu), ("bi", bi)):
        np.testing.assert_allclose(got[k], ref, rtol=0, atol=1e-9, err_msg=k)


@pytest.mark.parametrize("K", [20, 128])
def test_staggered_halves_match_deltalog_oracle(torch, u1, K):
    """stagger (large chunks' default): the chunk's users in two halves, half B's epoch kernel
    beside half A's log replay -- the fold adds both halves' piece sums, so fp64 factors equal
    oracle_svd_sgd_deltalog (merge=3) to 1e-9 (K=128: the narrow rows of C4 at fp64)."""
    from surprise_amd.engine import MFEngine
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    rng = np.random.RandomState(9)
    pu0, qi0 = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    eng = MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype="float64",
                   mode="log", heavy=0, stagger=True)
    assert eng.stagger and eng.logs[0]["heavy"] is not None
    eng.set_factors(pu0, qi0)
    eng.run_epochs(3)
    got = eng.get_factors()
    hp = orc.hyper(**{k: v for k, v in hyper.items() if k != "global_mean"})
    pu, qi, bu, bi = orc.svd_sgd_deltalog(row_ptr, items, ratings, ts.n_items, K, 3, True,
                                          ts.global_mean, hp, pu0.copy(), qi0.copy(), merge=3)
    for k, ref in (("pu", pu), ("qi", qi), ("bu", bu), ("bi", bi)):
        np.testing.assert_allclose(got[k], ref, rtol=0, atol=1e-9, err_msg=k)


@pytest.mark.parametrize("K,heavy,mirror", [(128, 0.0, True), (128, 16, True),
                                             (128, 0.0, False), (64, 16, True), (64, 0.0, False)])
def test_fp64_k128_checkpoint_rows_match_deltalog_oracle(torch, golden, u1, K, heavy, mirror):
    """fp64 K=128 (the C4 factor count at the reference's precision, mf.pyx:206-239): item rows
    of 1088 B, so the checkpoint log runs in narrow form -- rows of the 128 factor columns (two
    whole lane groups), both biases beside the groups in the epoch kernel, the replay's third
    lane group holding the bias column alone.  K=64 is the one-group form (512-B rows).  mirror:
    the epoch kernel reads the item biases from the mirror mf_log_apply keeps (bias_out) and the
    item rows lie on whole 128-B lines (the default); else from the rows.  Factors equal
    oracle_svd_sgd_deltalog (merge=3) to 1e-9, with and without the heavy users' split, over 2
    chunks (the mirror crosses the chunk boundary)."""
    from surprise_amd.dist import chunk_users
    from surprise_amd.engine import MFEngine
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    rng = np.random.RandomState(8)
    pu0, qi0 = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    bi0 = rng.normal(0, .1, ts.n_items)  # (a non-zero start, so a stale mirror would show)
    eng = MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype="float64",
                   mode="log", heavy=heavy, n_chunks=2, bias_mirror=mirror)
    assert eng.ckpt and eng.narrow and eng.ldc == K and eng.sb_mirror == mirror
    assert (eng.ldq * 8) % 128 == 0 if mirror else True
    if K == 128:
        assert eng.ldq * 8 > 1024
    eng.set_factors(pu0, qi0, bi=bi0)
    eng.run_epochs(3)
    got = eng.get_factors()
    hp = orc.hyper(**{k: v for k, v in hyper.items() if k != "global_mean"})
    cou = np.zeros(ts.n_users, np.int32)
    for c, us in enumerate(chunk_users(np.arange(ts.n_users), row_ptr, 2)):
        cou[us] = c
    pu, qi, bu, bi = orc.svd_sgd_deltalog(row_ptr, items, ratings, ts.n_items, K, 3, True,
                                          ts.global_mean, hp, pu0.copy(), qi0.copy(), cou, 2,
                                          merge=3, bi=bi0.copy())
    for k, ref in (("pu", pu), ("qi", qi), ("bu", bu), ("bi", bi)):
        np.testing.assert_allclose(got[k], ref, rtol=0, atol=1e-9, err_msg=k)
    if mirror:  # (the mirror holds the table's biases after the last fold)
        np.testing.assert_array_equal(eng.ibias.cpu().numpy(), eng.qb[:, K].cpu().numpy())


@pytest.mark.parametrize("rows,dtype,narrow,heavy", [(256, "float64", False, 0.0),
                                                     (1024, "float32", True, 0.0),
                                                     (128, "float32", False, 0.25)])
def test_long_replay_pieces_match_64_rating_pieces(torch, ml1m, monkeypatch, rows, dtype, narrow,
                                                    heavy):
    """mf_log_replay over pieces longer than 64 ratings (taken 64 at a time; engine
    replay_piece_rows, long at C4's size) against the default 64-rating pieces on the ML-1M
    shape: the same gradients summed in another grouping (fp64 within 1e-11, fp32 within
    1e-5)."""
    import surprise_amd.engine as E
    ts, _ = ml1m
    row_ptr, items, ratings = ts.csr()
    K = 32
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    rng = np.random.RandomState(5)
    pu0, qi0 = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    out = []
    for r in (rows, 64):
        monkeypatch.setattr(E, "replay_piece_rows", lambda row_ptr, users, r=r: r)
        eng = E.MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype=dtype,
                         mode="log", heavy=heavy, narrow=narrow, n_chunks=2)
        assert eng.ckpt and eng.narrow == narrow
        groups = [g for lg in eng.logs for g in (lg, lg["heavy"]) if g is not None]
        longest = max(int(np.diff(g["pb"].cpu().numpy()).max()) for g in groups)
        assert (longest > 64) == (r > 64)
        eng.set_factors(pu0, qi0)
        eng.run_epochs(2)
        out.append(eng.get_factors())
    tol = 1e-11 if dtype == "float64" else 1e-5
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(out[0][k], out[1][k], rtol=0, atol=tol, err_msg=k)


def test_user_sq_statistic_equals_sumsq(torch, u1):
    """<pu^2> for the next chunk, summed from the epoch kernel's per-user |p_u|^2 inside
    mf_log_apply, equals mf_sumsq over the updated pu (fp64, up to summation order)."""
    import ctypes
    from surprise_amd import _lib
    from surprise_amd.engine import MFEngine
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    K = 40
    hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
                 reg_pu=.02, reg_qi=.02, global_mean=float(ts.global_mean))
    rng = np.random.RandomState(3)
    eng = MFEngine((row_ptr, items, ratings), ts.n_items, K, hyper=hyper, dtype="float64",
                   mode="log", n_chunks=2, heavy=0.25)
    eng.set_factors(rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K)))
    for c in (0, 1, 0):
        eng.run_chunk(c)
        eng.sync_items(None)
        nxt = eng._works[eng._wt % 2].cpu().numpy()
        ref = torch.zeros(2, dtype=torch.float64, device="cuda")
        _lib.call("mf_sumsq", ctypes.c_void_p(eng.pu.data_ptr()), eng.n_users, K, eng.ld,
                  ctypes.c_void_p(ref.data_ptr()), _lib.MF_F64,
                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        ref = ref.cpu().numpy()
        assert nxt[1] == ref[1] == ts.n_users * K
        assert abs(nxt[0] - ref[0]) <= 1e-12 * ref[0], (nxt, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [20, 100, 130])
@pytest.mark.parametrize("fused", [False, True])
def test_svdpp_y_fold_equals_sequential_composition(torch, K, fused):
    """mf_svdpp_y_fold (per-piece composition, then each item's pieces in order) equals applying
    y_j <- A_u y_j + c_u for the item's users one after the other (fp64), on a CSR with items
    of 0, 1, 64, 65 and ~300 users (several pieces) and K across the lane layouts; fused (with
    piece_item): single-piece items applied by their piece's wave."""
    import ctypes
    from surprise_amd import _lib
    from surprise_amd.engine import log_layout, position_users
    rng = np.random.RandomState(5)
    n_users, n_items = 400, 9
    pop = np.array([0, 1, 64, 65, 300, 20, 399, 7, 2], np.float64)  # users per item, roughly
    rows = [np.flatnonzero(rng.rand(n_items) < pop / n_users) for _ in range(n_users)]
    row_ptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    items = np.concatenate(rows).astype(np.int32)
    perm, pb, ipp, cnt = log_layout(row_ptr, items, np.arange(n_users), n_items)
    assert cnt[0] == 0 and cnt.max() > 64
    iusr = position_users(row_ptr)[perm]
    ld = K + (-K % 16)
    y0 = rng.normal(0, .1, (n_items, ld))
    c = rng.normal(0, .01, (n_users, ld))
    A = rng.uniform(.5, 1., n_users)
    want = y0.copy()
    for x in range(len(perm)):  # CSR order within every item
        u, j = iusr[x], items[perm[x]]
        want[j, :K] = A[u] * want[j, :K] + c[u, :K]
    dev = "cuda"
    t = lambda a, dt=torch.float64: torch.tensor(a, dtype=dt, device=dev)
    y, cb, Ab = t(y0), t(c), t(A)
    i32 = lambda a: t(np.asarray(a, np.int32), torch.int32)
    users, pbd, ippd = i32(iusr), i32(pb), i32(ipp)
    n_pc = len(pb) - 1
    sc, sa = torch.zeros(n_pc, ld, dtype=torch.float64, device=dev), torch.zeros(n_pc, dtype=torch.float64, device=dev)
    p = lambda z: ctypes.c_void_p(z.data_ptr())
    pitem = i32(np.repeat(np.arange(n_items, dtype=np.int32), np.diff(ipp)))
    _lib.call("mf_svdpp_y_fold", p(y), ld, K, p(cb), p(Ab), p(users), p(pbd), n_pc, p(ippd),
              n_items, p(sc), p(sa), p(pitem) if fused else None, _lib.MF_F64, None)
    torch.cuda.synchronize()
    got = y.cpu().numpy()
    np.testing.assert_allclose(got[:, :K], want[:, :K], rtol=0, atol=1e-12)
    np.testing.assert_array_equal(got[:, K:], y0[:, K:])  # padding columns untouched


def test_test_metrics_equal_reference_pipeline(torch, u1):
    """test_metrics(): ids mapped vectorised, estimates + error reduction on the device (no
    Prediction objects) -- equal to accuracy.rmse / mae over the reference-style per-call
    predictions (AlgoBase.test -> estimate), unknown ids included."""
    from surprise_amd import NMF, SVD, SVDpp, accuracy
    from surprise_amd.algo_base import AlgoBase
    ts, test = u1
    test = list(test) + [("no-such-user", "1", 4.0), ("1", "no-such-item", 2.0)]
    for algo in (SVD(n_factors=30, n_epochs=3, random_state=0, dtype="float64"),
                 SVD(n_factors=30, n_epochs=3, biased=False, random_state=0, dtype="float64"),
                 SVDpp(n_factors=12, n_epochs=2, random_state=0, dtype="float64"),
                 NMF(n_factors=8, n_epochs=3, random_state=0, dtype="float64")):
        algo.fit(ts)
        slow = AlgoBase.test(algo, test)
        rmse, mae = algo.test_metrics(test)
        assert abs(rmse - accuracy.rmse(slow, verbose=False)) < 1e-12
        assert abs(mae - accuracy.mae(slow, verbose=False)) < 1e-12
        fast = algo.test(test)
        assert [p.details for p in fast] == [p.details for p in slow]
        np.testing.assert_allclose([p.est for p in fast], [p.est for p in slow], atol=1e-12)
        # the column-native testset (RatingColumns: id arrays, no tuple per rating): the same
        from surprise_amd.dataset import RatingColumns
        ru, ri, rr = zip(*test)
        cols = RatingColumns(np.array(ru, dtype=object), np.array(ri, dtype=object), rr)
        np.testing.assert_allclose(algo.test_metrics(cols), (rmse, mae), rtol=0, atol=1e-12)
        assert [p.est for p in algo.test(cols)] == [p.est for p in fast]


def _many_users_csr(n_users=70_000, n_items=400, seed=3):
    """A trainset past MF_SQ_PARTS_MIN users (the <p^2> statistic summed in fixed-range parts):
    4-11 ratings per user over a few hundred items."""
    from surprise_amd import Trainset
    rng = np.random.RandomState(seed)
    rows = [np.sort(rng.choice(n_items, rng.randint(4, 12), replace=False)) for _ in range(n_users)]
    row_ptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    items = np.concatenate(rows).astype(np.int32)
    ratings = rng.randint(1, 6, len(items)).astype(np.float64)
    return Trainset.from_csr(row_ptr, items, ratings, n_items), (row_ptr, items, ratings)


def test_user_sq_sum_in_fixed_parts_above_64k_rows(torch):
    """mf_user_sq_reduce from MF_SQ_PARTS_MIN rows: MF_SQ_PARTS fixed-range partial sums (their
    own launch) added in order -- the sum to 1e-12 relative, the count exact, bit-identical on a
    second call; below the threshold the one-workgroup sum."""
    import ctypes
    from surprise_amd import _lib
    for n in (1000, 65_535, 65_536, 300_001):
        x = torch.rand(n, dtype=torch.float64, device="cuda")
        outs = []
        for _ in range(2):
            out = torch.full((2 + _lib.MF_SQ_PARTS,), -1.0, dtype=torch.float64, device="cuda")
            _lib.call("mf_user_sq_reduce", ctypes.c_void_p(x.data_ptr()), n, 7,
                      ctypes.c_void_p(out.data_ptr()), None)
            torch.cuda.synchronize()
            outs.append(out.cpu().numpy())
        ref = float(x.sum())
        assert abs(outs[0][0] - ref) <= 1e-12 * ref, (n, outs[0][0], ref)
        assert outs[0][1] == n * 7
        assert outs[0][0] == outs[1][0]
        if n >= 65_536:  # (the parts: each fixed range's own sum)
            xs = x.cpu().numpy()
            b = np.arange(_lib.MF_SQ_PARTS + 1) * n // _lib.MF_SQ_PARTS
            np.testing.assert_allclose(outs[0][2:], [xs[b[i]:b[i + 1]].sum()
                                                     for i in range(_lib.MF_SQ_PARTS)], rtol=1e-12)
        else:
            assert (outs[0][2:] == -1.0).all()  # (scratch untouched below the threshold)


def test_log_and_qlog_past_64k_users_match_their_oracles(torch):
    """The fold's next-chunk <p^2> summed in parts (70k users): SVD's checkpoint log (2 chunks)
    and SVD++'s q log with the fused fold (3 chunks) in fp64 equal oracle_svd_sgd_deltalog(merge=3)
    / oracle_svdpp_sgd_stalelog on the same chunking to 1e-9."""
    from surprise_amd import SVD, SVDpp
    from surprise_amd.dist import chunk_users
    ts, (row_ptr, items, ratings) = _many_users_csr()
    assert ts.n_users >= 65_536
    for algo_cls, chunks in ((SVD, 2), (SVDpp, 3)):
        params = dict(n_factors=8, n_epochs=2, random_state=0)
        cou = np.zeros(ts.n_users, np.int32)
        for c, us in enumerate(chunk_users(np.arange(ts.n_users), row_ptr, chunks)):
            cou[us] = c
        if algo_cls is SVD:
            _, f = run_oracle_log("SVD", params, row_ptr, items, ratings, ts.n_items,
                                  ts.global_mean, cou, chunks, merge=3)
            algo = SVD(**params, dtype="float64", deterministic=False, chunks_per_epoch=chunks)
            keys = ("pu", "qi", "bu", "bi")
        else:
            _, f = run_oracle_stalelog(params, row_ptr, items, ratings, ts.n_items,
                                       ts.global_mean, cou, chunks)
            algo = SVDpp(**params, dtype="float64", chunks_per_epoch=chunks)
            algo._engine_options = {"qlog": True}
            keys = ("pu", "qi", "yj", "bu", "bi")
        algo.fit(ts)
        if algo_cls is SVDpp:
            assert algo._engine.qlog_pp and algo._engine._fused_fold()
        else:
            assert algo._engine.ckpt
        for k in keys:
            np.testing.assert_allclose(getattr(algo, k), f[k], rtol=0, atol=1e-9,
                                       err_msg="%s %s" % (algo_cls.__name__, k))


@pytest.mark.parametrize("lr_yj,reg_yj", [(None, None), (.004, None), (None, .05)])
def test_svdpp_shared_step_chain_and_general_chain_match_stalelog_oracle(torch, u1, lr_yj, reg_yj):
    """SVD++'s chain carries s = p + m alone where p and m take the same step (lr_pu = lr_yj and
    reg_pu = reg_yj: the defaults), p_n and m_n recovered from a^n (p_0 - m_0) at the user's end;
    with other values it carries p and m apart.  Both on the q log in fp64 against
    oracle_svdpp_sgd_stalelog at 1e-9 (K=64: the item bias beside the lane group)."""
    from surprise_amd import SVDpp
    from surprise_amd.dist import chunk_users
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    params = dict(n_factors=64, n_epochs=3, random_state=0)
    if lr_yj is not None:
        params["lr_yj"] = lr_yj
    if reg_yj is not None:
        params["reg_yj"] = reg_yj
    cou = np.zeros(ts.n_users, np.int32)
    for c, us in enumerate(chunk_users(np.arange(ts.n_users), row_ptr, 2)):
        cou[us] = c
    P, f = run_oracle_stalelog(params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                               cou, 2)
    algo = SVDpp(**params, dtype="float64", chunks_per_epoch=2)
    algo._engine_options = {"qlog": True}
    algo.fit(ts)
    assert algo._engine.qlog_pp
    for k in ("pu", "qi", "yj", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), f[k], rtol=0, atol=1e-9, err_msg=k)


@pytest.mark.parametrize("K", [10, 64])
def test_svdpp_hybrid_launch_all_cold_matches_stalelog_oracle(torch, u1, K):
    """The hybrid helper-wave launch (mf_svdpp_epoch_mix) with every item cold (cold_share 1, no
    hot replicas): no float atomic is left, every gradient goes to the item-grouped cold log and
    the cold fold (mf_log_reduce + mf_log_apply) -- oracle_svdpp_sgd_stalelog with every item
    stale, to 1e-9 in fp64, over 2 chunks."""
    from surprise_amd import SVDpp
    from surprise_amd.dist import chunk_users
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    params = dict(n_factors=K, n_epochs=3, random_state=0)
    cou = np.zeros(ts.n_users, np.int32)
    for c, us in enumerate(chunk_users(np.arange(ts.n_users), row_ptr, 2)):
        cou[us] = c
    P, f = run_oracle_stalelog(params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                               cou, 2)
    algo = SVDpp(**params, dtype="float64", chunks_per_epoch=2, mode="atomic")
    algo._engine_options = {"cold_share": 1.0, "hot_rows": 0, "helpers": True, "qlog": False}
    algo.fit(ts)
    eng = algo._engine
    assert eng.hx and eng.mix and eng.hot_list is None
    assert all(int((m["crow"] >= 0).sum()) == int(m["totals"].sum()) for m in eng.mix)
    for k in ("pu", "qi", "yj", "bu", "bi"):
        np.testing.assert_allclose(getattr(algo, k), f[k], rtol=0, atol=1e-9, err_msg=k)


@pytest.mark.parametrize("name", ["svdpp_k20_e20", "svdpp_k100_e20"])
@pytest.mark.parametrize("dtype", ["float64", "float32"])
def test_svdpp_hybrid_launch_rmse_within_1e3(torch, golden, u1, name, dtype):
    """The hybrid launch with the least-rated items holding half the ratings cold (their rows
    read-only per chunk, gradients logged and folded) and the rest on the helper waves' float
    atomics, hot replicas included: held-out RMSE within 1e-3 of the reference's."""
    from surprise_amd import SVDpp
    meta, _ = golden
    case = meta["cases"][name]
    ts, test = u1
    algo = SVDpp(**case["params"], dtype=dtype, mode="atomic")
    algo._engine_options = {"cold_share": 0.5, "qlog": False}
    algo.fit(ts)
    eng = algo._engine
    assert eng.hx and eng.mix
    cold = int((eng.mix[0]["crow"] >= 0).sum())
    assert 0.3 * ts.n_ratings < cold <= 0.5 * ts.n_ratings, cold
    assert abs(_rmse(algo.test(test)) - case["rmse"]) < RMSE_TOL


def test_split_engines_share_one_side_stream(torch, u1):
    """The split step's side stream is one per device for the process (engine.side_stream,
    SIDE_STREAM_POLICY "cached"): a fresh pool stream per engine landed on the main stream's
    hardware queue in about one engine of four and serialised the two launch groups
    (profiles/r5bm_bimodal.jsonl)."""
    from surprise_amd import engine as E
    ts, _ = u1
    csr = ts.csr()
    engs = [E.MFEngine(csr, ts.n_items, 16, dtype="float32", mode="log", heavy=0.25)
            for _ in range(3)]
    assert all(e.side is not None for e in engs)
    assert len({e.side.cuda_stream for e in engs}) == 1
    assert engs[0].side.cuda_stream != torch.cuda.current_stream().cuda_stream
