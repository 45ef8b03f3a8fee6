"""Pins the parity oracle (oracle/mf_oracle.c) against outputs of the reference itself.

The golden values in tests/golden/ were produced by running nickmvincent/Surprise's
compiled Cython (tests/golden/make_golden.py).  SVD is checked bit-for-bit (sha256 of
the fp64 factor arrays); SVD++ too for the literal form, and the per-user affine form
(the GPU kernel's formulation) to 1e-10.
"""
import os

import numpy as np
import pytest

import oracle as orc
from conftest import GOLDEN
from surprise_amd.utils import get_rng


def _sha(*arrays):
    import hashlib
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()


class _Params:
    """Hyper-parameter resolution of SVD/SVDpp.__init__ (mf.pyx:140-147, 398-407)."""

    def __init__(self, algo, p):
        svdpp = algo == "SVDpp"
        self.n_factors = p.get("n_factors", 20 if svdpp else 100)
        self.n_epochs = p.get("n_epochs", 20)
        self.biased = p.get("biased", True)
        self.init_mean = p.get("init_mean", 0)
        self.init_std_dev = p.get("init_std_dev", .1)
        lr_all = p.get("lr_all", .007 if svdpp else .005)
        reg_all = p.get("reg_all", .02)
        for n in ("bu", "bi", "pu", "qi", "yj"):
            lr, reg = p.get("lr_" + n), p.get("reg_" + n)
            setattr(self, "lr_" + n, lr if lr is not None else lr_all)
            setattr(self, "reg_" + n, reg if reg is not None else reg_all)
        self.random_state = p.get("random_state")


def run_oracle(algo, params, row_ptr, items, ratings, n_items, global_mean, affine=False):
    P = _Params(algo, params)
    rng = get_rng(P.random_state)
    n_users = len(row_ptr) - 1
    pu, qi, yj = orc.init_factors(rng, n_users, n_items, P.n_factors, P.init_mean,
                                  P.init_std_dev, with_yj=(algo == "SVDpp"))
    hp = orc.svd_hyper(P)
    if algo == "SVD":
        pu, qi, bu, bi = orc.svd_sgd(row_ptr, items, ratings, n_items, P.n_factors, P.n_epochs,
                                     P.biased, global_mean, hp, pu, qi)
        return P, dict(pu=pu, qi=qi, bu=bu, bi=bi)
    pu, qi, yj, bu, bi = orc.svdpp_sgd(row_ptr, items, ratings, n_items, P.n_factors,
                                       P.n_epochs, global_mean, hp, pu, qi, yj, affine=affine)
    return P, dict(pu=pu, qi=qi, yj=yj, bu=bu, bi=bi)


def test_oracle_build_flags():
    # the bit-exactness below relies on no FMA contraction
    assert "-ffp-contract=off" in open(os.path.join(os.path.dirname(orc.__file__), "Makefile")).read()


def test_u1_trainset_matches_reference(golden, u1):
    meta, arr = golden
    ts, test = u1
    g = meta["u1"]
    assert (ts.n_users, ts.n_items, ts.n_ratings, len(test)) == \
        (g["n_users"], g["n_items"], g["n_ratings"], g["n_test"])
    assert ts.global_mean == g["global_mean"]  # np.mean in all_ratings order: exact
    row_ptr, items, ratings = ts.csr()
    np.testing.assert_array_equal(row_ptr, arr["u1_row_ptr"])
    np.testing.assert_array_equal(items, arr["u1_items"])
    np.testing.assert_array_equal(ratings, arr["u1_ratings"])
    for raw, inner in g["raw2inner_users_first"]:
        assert ts.to_inner_uid(raw) == inner
    for raw, inner in g["raw2inner_items_first"]:
        assert ts.to_inner_iid(raw) == inner


def _test_inner(ts, test):
    u = np.array([ts._raw2inner_id_users.get(r, -1) for (r, _, _) in test], np.int32)
    i = np.array([ts._raw2inner_id_items.get(r, -1) for (_, r, _) in test], np.int32)
    return u, i


def _oracle_test_rmse(P, f, algo, ts, test):
    u, i = _test_inner(ts, test)
    row_ptr, items, _ = ts.csr()
    if algo == "SVD":
        est, imp = orc.svd_predict(u, i, P.n_factors, P.biased, ts.global_mean, f["pu"], f["qi"],
                                   f["bu"], f["bi"])
    else:
        est = orc.svdpp_predict(u, i, row_ptr, items, P.n_factors, ts.global_mean, f["pu"],
                                f["qi"], f["yj"], f["bu"], f["bi"])
        imp = np.zeros(len(u), bool)
    est = orc.finish_estimates(est, imp, ts.global_mean, ts.offset, ts.rating_scale)
    r = np.array([x[2] for x in test]) - ts.offset
    return est, orc.rmse(r, est), orc.mae(r, est)


@pytest.mark.parametrize("name", ["svd_k20_e5", "svd_k100_e20", "svd_k100_e20_unbiased",
                                  "svd_k128_e20", "svd_k10_e3_hyper", "svd_k5_e2_unbiased"])
def test_svd_oracle_bit_exact(golden, u1, name):
    meta, arr = golden
    case = meta["cases"][name]
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    P, f = run_oracle("SVD", case["params"], row_ptr, items, ratings, ts.n_items, ts.global_mean)
    assert _sha(f["pu"], f["qi"]) == case["sha_pu_qi"]
    assert _sha(f["bu"], f["bi"]) == case["sha_bu_bi"]
    if name + "_pu" in arr:
        np.testing.assert_array_equal(f["pu"], arr[name + "_pu"])
        np.testing.assert_array_equal(f["qi"], arr[name + "_qi"])
    est, rmse, mae = _oracle_test_rmse(P, f, "SVD", ts, test)
    # np.dot in the reference's estimate may sum in another order than the oracle's loop
    np.testing.assert_allclose(est, arr[name + "_est"], rtol=0, atol=1e-12)
    assert abs(rmse - case["rmse"]) < 1e-12 and abs(mae - case["mae"]) < 1e-12


@pytest.mark.parametrize("name", ["svdpp_k20_e20", "svdpp_k100_e20", "svdpp_k10_e3",
                                  "svdpp_k8_e2_hyper"])
def test_svdpp_oracle_bit_exact(golden, u1, name):
    meta, arr = golden
    case = meta["cases"][name]
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    P, f = run_oracle("SVDpp", case["params"], row_ptr, items, ratings, ts.n_items,
                      ts.global_mean)
    assert _sha(f["pu"], f["qi"]) == case["sha_pu_qi"]
    assert _sha(f["yj"]) == case["sha_yj"]
    assert _sha(f["bu"], f["bi"]) == case["sha_bu_bi"]
    est, rmse, _ = _oracle_test_rmse(P, f, "SVDpp", ts, test)
    np.testing.assert_allclose(est, arr[name + "_est"], rtol=0, atol=1e-12)
    assert abs(rmse - case["rmse"]) < 1e-12


@pytest.mark.parametrize("name", ["svdpp_k20_e20", "svdpp_k10_e3", "svdpp_k8_e2_hyper"])
def test_svdpp_affine_form_matches_reference(golden, u1, name):
    """The per-user reformulation the GPU kernel implements."""
    meta, arr = golden
    case = meta["cases"][name]
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    P, f = run_oracle("SVDpp", case["params"], row_ptr, items, ratings, ts.n_items,
                      ts.global_mean, affine=True)
    if name + "_pu" in arr:
        for k in ("pu", "qi", "yj", "bu", "bi"):
            np.testing.assert_allclose(f[k], arr[name + "_" + k], rtol=0, atol=1e-10)
    _, rmse, _ = _oracle_test_rmse(P, f, "SVDpp", ts, test)
    assert abs(rmse - case["rmse"]) < 1e-10


def test_python_restatement_matches_c(u1):
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    rng = np.random.RandomState(5)
    pu, qi, _ = orc.init_factors(rng, ts.n_users, ts.n_items, 4)
    hp = orc.hyper(lr_bu=.005, lr_bi=.004, lr_pu=.006, lr_qi=.005, reg_bu=.02, reg_bi=.03,
                   reg_pu=.02, reg_qi=.01)
    a = orc.svd_sgd(row_ptr, items, ratings, ts.n_items, 4, 1, True, ts.global_mean, hp,
                    pu.copy(), qi.copy())
    b = orc.py_svd_sgd(row_ptr, items, ratings, 4, 1, True, ts.global_mean, hp, pu.copy(),
                       qi.copy(), np.zeros(ts.n_users), np.zeros(ts.n_items))
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_sensitivity_sweep_known_answers(golden, u1):
    """test_SVD.py:25-108 turned into known answers: every hyper-parameter changes the
    cross-validated RMSE, and the oracle reproduces each value."""
    meta, _ = golden
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    seen = set()
    for key, rec in meta["sensitivity"].items():
        algo = key.split("_")[0]
        P, f = run_oracle(algo, rec["params"], row_ptr, items, ratings, ts.n_items,
                          ts.global_mean)
        _, rmse, _ = _oracle_test_rmse(P, f, algo, ts, test)
        assert abs(rmse - rec["test_rmse"]) < 1e-12, key
        seen.add(round(rec["test_rmse"], 12))
    assert len(seen) == len(meta["sensitivity"])  # all distinct, as test_SVD.py asserts


def test_groups_schedule_g1_equals_sequential(u1):
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    rng = np.random.RandomState(0)
    pu, qi, _ = orc.init_factors(rng, ts.n_users, ts.n_items, 8)
    hp = orc.hyper(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005,
                   reg_bu=.02, reg_bi=.02, reg_pu=.02, reg_qi=.02)
    a = orc.svd_sgd(row_ptr, items, ratings, ts.n_items, 8, 3, True, ts.global_mean, hp,
                    pu.copy(), qi.copy())
    b = orc.svd_sgd_groups(row_ptr, items, ratings, ts.n_items, 8, 3, True, ts.global_mean, hp,
                           pu.copy(), qi.copy(), np.zeros(ts.n_users), 1)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=0, atol=1e-15)


def test_synthetic_fold_matches_reference(golden, tmp_path):
    """The repo's generator -> a ratings file -> this repo's Reader/Dataset/KFold gives the
    same trainset (sha of the CSR) as the reference's; the oracle then reproduces the
    reference's SVD / SVD++ factors bit-for-bit."""
    from surprise_amd import Dataset, Reader, synthetic
    from surprise_amd.model_selection import KFold
    meta, _ = golden
    g = meta["synth_ml100k"]
    u, i, r = synthetic.shape("ml-100k")
    path = tmp_path / "synth.tsv"
    with open(path, "w") as fh:
        for a, b, c in zip(u.tolist(), i.tolist(), r.tolist()):
            fh.write("%d\t%d\t%d\n" % (a, b, int(c)))
    data = Dataset.load_from_file(str(path), Reader(line_format="user item rating", sep="\t"))
    ts, test = next(KFold(5, random_state=0).split(data))
    assert (ts.n_users, ts.n_items, ts.n_ratings, len(test)) == \
        (g["n_users"], g["n_items"], g["n_ratings"], g["n_test"])
    assert ts.global_mean == g["global_mean"]
    row_ptr, items, ratings = ts.csr()
    assert _sha(row_ptr, items, ratings) == g["sha_csr"]
    P, f = run_oracle("SVD", dict(n_factors=20, n_epochs=5, random_state=0), row_ptr, items,
                      ratings, ts.n_items, ts.global_mean)
    assert _sha(f["pu"], f["qi"]) == g["svd_k20_e5"]["sha_pu_qi"]
    _, rmse, _ = _oracle_test_rmse(P, f, "SVD", ts, test)
    assert abs(rmse - g["svd_k20_e5"]["rmse"]) < 1e-12
    P, f = run_oracle("SVDpp", dict(n_factors=10, n_epochs=2, random_state=0), row_ptr, items,
                      ratings, ts.n_items, ts.global_mean)
    assert _sha(f["pu"], f["qi"], f["yj"]) == g["svdpp_k10_e2"]["sha_pu_qi_yj"]


# ----------------------------------------------------------------------------- delta-log schedule

def run_oracle_log(algo, params, row_ptr, items, ratings, n_items, global_mean, chunk_of_user=None,
                   n_chunks=1, merge=2):
    """The GPU's default schedule (MF_MODE_LOG) restated: oracle_*_sgd_deltalog."""
    P = _Params(algo, params)
    rng = get_rng(P.random_state)
    n_users = len(row_ptr) - 1
    pu, qi, yj = orc.init_factors(rng, n_users, n_items, P.n_factors, P.init_mean,
                                  P.init_std_dev, with_yj=(algo == "SVDpp"))
    hp = orc.svd_hyper(P)
    if algo == "SVD":
        pu, qi, bu, bi = orc.svd_sgd_deltalog(row_ptr, items, ratings, n_items, P.n_factors,
                                              P.n_epochs, P.biased, global_mean, hp, pu, qi,
                                              chunk_of_user, n_chunks, merge)
        return P, dict(pu=pu, qi=qi, bu=bu, bi=bi)
    pu, qi, yj, bu, bi = orc.svdpp_sgd_deltalog(row_ptr, items, ratings, n_items, P.n_factors,
                                                P.n_epochs, global_mean, hp, pu, qi, yj,
                                                chunk_of_user, n_chunks, merge)
    return P, dict(pu=pu, qi=qi, yj=yj, bu=bu, bi=bi)


@pytest.mark.parametrize("name", ["svd_k20_e5", "svd_k5_e2_unbiased", "svd_k10_e3_hyper"])
@pytest.mark.parametrize("merge", [2, 3])
def test_deltalog_one_user_per_chunk_is_the_reference(golden, u1, name, merge):
    """Pins the delta-log oracle to the reference: one user per chunk = SVD.sgd bit-for-bit,
    with the count-aware (2) and the recency-weighted (3) fold alike."""
    meta, _ = golden
    case = meta["cases"][name]
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    P, f = run_oracle_log("SVD", case["params"], row_ptr, items, ratings, ts.n_items,
                          ts.global_mean, np.arange(ts.n_users), ts.n_users, merge=merge)
    assert _sha(f["pu"], f["qi"]) == case["sha_pu_qi"]
    assert _sha(f["bu"], f["bi"]) == case["sha_bu_bi"]


def test_deltalog_svdpp_one_user_per_chunk_is_the_affine_form(u1):
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    params = dict(n_factors=6, n_epochs=2, random_state=0)
    _, a = run_oracle("SVDpp", params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                      affine=True)
    _, b = run_oracle_log("SVDpp", params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                          np.arange(ts.n_users), ts.n_users)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.parametrize("name", ["svd_k20_e5", "svd_k100_e20", "svd_k10_e3_hyper"])
@pytest.mark.parametrize("merge", [2, 3])
def test_deltalog_one_chunk_within_1e3_of_reference(golden, u1, name, merge):
    """The schedule itself (all users of the epoch against one snapshot, count-aware or
    recency-weighted fold) stays within the north-star tolerance of the sequential reference."""
    meta, _ = golden
    case = meta["cases"][name]
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    P, f = run_oracle_log("SVD", case["params"], row_ptr, items, ratings, ts.n_items,
                          ts.global_mean, merge=merge)
    assert abs(_oracle_test_rmse(P, f, "SVD", ts, list(test))[1] - case["rmse"]) < 1e-3


# ----------------------------------------------------------------------------- NMF, baselines

@pytest.fixture(scope="module")
def golden_ext():
    import json
    with open(os.path.join(GOLDEN, "golden_ext.json")) as f:
        meta = json.load(f)
    return meta, dict(np.load(os.path.join(GOLDEN, "golden_ext_arrays.npz")))


def run_oracle_nmf(params, ts):
    """NMF.__init__ defaults (mf.pyx:628-644) + NMF.sgd via the oracle."""
    p = dict(n_factors=15, n_epochs=50, biased=False, reg_pu=.06, reg_qi=.06, reg_bu=.02,
             reg_bi=.02, lr_bu=.005, lr_bi=.005, init_low=0, init_high=1, random_state=None)
    p.update(params)
    rng = get_rng(p["random_state"])
    pu = rng.uniform(p["init_low"], p["init_high"], size=(ts.n_users, p["n_factors"]))
    qi = rng.uniform(p["init_low"], p["init_high"], size=(ts.n_items, p["n_factors"]))
    row_ptr, items, ratings = ts.csr()
    pu, qi, bu, bi = orc.nmf_sgd(row_ptr, items, ratings, ts.n_items, p["n_factors"],
                                 p["n_epochs"], p["biased"], ts.global_mean, pu, qi,
                                 *[p[k] for k in ("reg_pu", "reg_qi", "reg_bu", "reg_bi", "lr_bu",
                                                  "lr_bi")])
    return p, dict(pu=pu, qi=qi, bu=bu, bi=bi)


def run_oracle_bsl(bsl_options, ts):
    """BaselineOnly.fit -> compute_baselines (algo_base.py:220-254) via the oracle."""
    row_ptr, items, ratings = ts.csr()
    method = bsl_options.get("method", "als")
    if method == "als":
        ptr, pos = ts.csc()
        return orc.baseline_als(row_ptr, items, ratings, ts.n_items, ptr, pos, ts.global_mean,
                                bsl_options.get("n_epochs", 10), bsl_options.get("reg_u", 15),
                                bsl_options.get("reg_i", 10))
    lr, reg = bsl_options.get("learning_rate", .005), bsl_options.get("reg", .02)
    hp = orc.hyper(lr_bu=lr, lr_bi=lr, reg_bu=reg, reg_bi=reg)
    _, _, bu, bi = orc.svd_sgd(row_ptr, items, ratings, ts.n_items, 0,
                               bsl_options.get("n_epochs", 20), True, ts.global_mean, hp,
                               np.zeros((ts.n_users, 0)), np.zeros((ts.n_items, 0)))
    return bu, bi


@pytest.mark.parametrize("name", ["nmf_default", "nmf_k5_e3", "nmf_k8_e5_hyper",
                                  "nmf_biased_k10_e10", "nmf_biased_k4_e3"])
def test_nmf_oracle_bit_exact(golden_ext, u1, name):
    meta, _ = golden_ext
    case = meta["cases"][name]
    ts, test = u1
    p, f = run_oracle_nmf(case["params"], ts)
    assert _sha(f["pu"], f["qi"]) == case["sha_pu_qi"]
    assert _sha(f["bu"], f["bi"]) == case["sha_bu_bi"]


@pytest.mark.parametrize("name", ["bsl_als_default", "bsl_als_e3_reg", "bsl_sgd_default",
                                  "bsl_sgd_hyper"])
def test_baseline_oracle(golden_ext, u1, name):
    """baseline_sgd is bit-exact (SVD with no factors); baseline_als sums ir[i] in the reference's
    list order, bit-exact as well."""
    meta, arr = golden_ext
    case = meta["cases"][name]
    ts, _ = u1
    bu, bi = run_oracle_bsl(case["params"]["bsl_options"], ts)
    assert _sha(bu, bi) == case["sha_bu_bi"]


# ----------------------------------------------------------------------------- multi-rank rules

def _groups_of(row_ptr, world):
    from surprise_amd.dist import shard_users
    b = shard_users(row_ptr, world)
    return (np.searchsorted(b, np.arange(len(row_ptr) - 1), side="right") - 1).astype(np.int32)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("name", ["svdpp_k20_e20", "svdpp_k100_e20"])
@pytest.mark.parametrize("merge", [2, 3])
def test_svdpp_multirank_rule_within_1e3_of_reference(golden, u1, world, name, merge):
    """The SVD++ multi-rank schedule of the GPU path (dist.py): users sharded by contiguous
    rating-balanced ranges, q/b by the rank-order composition (merge=3, the product's rule) or
    the count-aware merge (2, round 3's), y_j by the affine composition of the ranks'
    end-of-user maps in rank order (merge_y=4) -- within the north-star 1e-3 of the
    reference's RMSE (golden) at 2, 4 and 8 ranks."""
    meta, _ = golden
    case = meta["cases"][name]
    ts, test = u1
    row_ptr, items, ratings = ts.csr()
    P = _Params("SVDpp", case["params"])
    pu, qi, yj = orc.init_factors(get_rng(P.random_state), ts.n_users, ts.n_items, P.n_factors,
                                  P.init_mean, P.init_std_dev, with_yj=True)
    pu, qi, yj, bu, bi = orc.svdpp_sgd_groups_merge(
        row_ptr, items, ratings, ts.n_items, P.n_factors, P.n_epochs, ts.global_mean,
        orc.svd_hyper(P), pu, qi, yj, _groups_of(row_ptr, world), world, merge=merge,
        merge_y=4)
    f = dict(pu=pu, qi=qi, yj=yj, bu=bu, bi=bi)
    rmse = _oracle_test_rmse(P, f, "SVDpp", ts, list(test))[1]
    assert abs(rmse - case["rmse"]) < 1e-3, (world, rmse, case["rmse"])


def test_svdpp_rank_order_q_merge_composes_the_ranks_steps(u1):
    """merge=3 restated: each group's chunk alone (the oracle with only that group's users
    active) moves q / b from the chunk start x_s to x_g; the merged row is
    x_s + sum_g (1 - eta)^{N_>g} (x_g - x_s), N_>g = the item's ratings in later groups,
    eta = lr_qi (<pu^2> + reg_qi) for q (<pu^2> over every user at the chunk start) and
    lr_bi (1 + reg_bi) for b."""
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    K, n_items, G = 6, ts.n_items, 3
    rng = np.random.RandomState(5)
    pu, qi, yj = orc.init_factors(rng, ts.n_users, n_items, K, with_yj=True)
    hp = orc.hyper(lr_bu=.007, lr_bi=.007, lr_pu=.007, lr_qi=.007, lr_yj=.007, reg_bu=.02,
                   reg_bi=.02, reg_pu=.02, reg_qi=.02, reg_yj=.02)
    g_of = _groups_of(row_ptr, G)
    got = orc.svdpp_sgd_groups_merge(row_ptr, items, ratings, n_items, K, 1, ts.global_mean, hp,
                                     pu.copy(), qi.copy(), yj.copy(), g_of, G, merge=3,
                                     merge_y=4)
    user_of = np.repeat(np.arange(ts.n_users), np.diff(row_ptr))
    eta_q = .007 * ((pu ** 2).mean() + .02)
    eta_b = .007 * (1 + .02)
    want_q, want_b = qi.copy(), np.zeros(n_items)
    for g in range(G):
        alone = np.where(g_of == g, 0, -1).astype(np.int32)  # (other users: no chunk)
        x = orc.svdpp_sgd_groups_merge(row_ptr, items, ratings, n_items, K, 1, ts.global_mean,
                                       hp, pu.copy(), qi.copy(), yj.copy(),
                                       np.zeros(ts.n_users, np.int32), 1, alone, 1, merge=0,
                                       merge_y=4)
        later = np.bincount(items[g_of[user_of] > g], minlength=n_items)
        want_q += (1 - eta_q) ** later[:, None] * (x[1] - qi)
        want_b += (1 - eta_b) ** later * x[4]
    np.testing.assert_allclose(got[1], want_q, rtol=0, atol=1e-12)
    np.testing.assert_allclose(got[4], want_b, rtol=0, atol=1e-12)


def test_svdpp_affine_rule_one_group_composes_in_user_order(u1):
    """merge_y=4 with ONE group: every user reads the chunk-start y and the maps compose in user
    order -- equal to the composition done by hand from the per-user maps (a second, pure-numpy
    restatement of the same rule on a small K)."""
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    K, n_items = 4, ts.n_items
    rng = np.random.RandomState(3)
    pu, qi, yj = orc.init_factors(rng, ts.n_users, n_items, K, with_yj=True)
    hp = orc.hyper(lr_bu=.007, lr_bi=.007, lr_pu=.007, lr_qi=.007, lr_yj=.007, reg_bu=.02,
                   reg_bi=.02, reg_pu=.02, reg_qi=.02, reg_yj=.02)
    g = np.zeros(ts.n_users, np.int32)
    a = orc.svdpp_sgd_groups_merge(row_ptr, items, ratings, n_items, K, 1, ts.global_mean, hp,
                                   pu.copy(), qi.copy(), yj.copy(), g, 1, merge=0, merge_y=4)
    # numpy restatement: users in order, imp from y0, maps onto a running y
    P, Q, Y0, Y = pu.copy(), qi.copy(), yj.copy(), yj.copy()
    bu, bi = np.zeros(ts.n_users), np.zeros(n_items)
    decay = 1 - .007 * .02
    for u in range(ts.n_users):
        s, e = row_ptr[u], row_ptr[u + 1]
        if e == s:
            continue
        js = items[s:e]
        sq = np.sqrt(e - s)
        imp = (Y0[js] / sq).sum(0)
        c = np.zeros(K)
        for k in range(s, e):
            i = items[k]
            err = ratings[k] - (ts.global_mean + bu[u] + bi[i] + Q[i] @ (P[u] + imp))
            bu[u] += .007 * (err - .02 * bu[u])
            bi[i] += .007 * (err - .02 * bi[i])
            pf, qf = P[u].copy(), Q[i].copy()
            P[u] += .007 * (err * qf - .02 * pf)
            Q[i] += .007 * (err * (pf + imp) - .02 * qf)
            c = decay * c + .007 * (err * qf / sq)
            imp = decay * imp + .007 * err * qf
        Y[js] = decay ** (e - s) * Y[js] + c
    np.testing.assert_allclose(a[2], Y, rtol=0, atol=1e-11)
    np.testing.assert_allclose(a[1], Q, rtol=0, atol=1e-11)


def test_svdpp_cpu_baseline_leg_on_a_user_prefix(u1, monkeypatch):
    """bench.py's SVD++ cpu_baseline: the reference-order restatement on a user prefix, scaled
    to the whole fold by sum n_u^2; one process per core of the (here: 2-core) share."""
    import sys
    sys.path.insert(0, os.path.dirname(GOLDEN.rstrip("/").rsplit("/", 1)[0]))
    import bench
    monkeypatch.setattr(bench, "BOX_CPU_SHARE", 2)
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    n = int(row_ptr[-1])
    cb = bench.cpu_baseline_svdpp((row_ptr, items, ratings), ts.n_items, 10, n, target_s=0.2)
    assert cb["kind"] == "port" and cb["cores"] == min(2, len(os.sched_getaffinity(0)))
    assert cb["value"] > 0 and cb["single_core"]["value"] > 0
    assert cb["affine_form_single_core"]["value"] > cb["single_core"]["value"]
    assert "mf.pyx:463-498" in cb["sample"]


def run_oracle_stalelog(params, row_ptr, items, ratings, n_items, global_mean,
                        chunk_of_user=None, n_chunks=1, stale=None, merge=3):
    """SVD++ with the q log (the GPU's qlog option): oracle_svdpp_sgd_stalelog, every item
    stale unless `stale` says otherwise."""
    P = _Params("SVDpp", params)
    rng = get_rng(P.random_state)
    n_users = len(row_ptr) - 1
    pu, qi, yj = orc.init_factors(rng, n_users, n_items, P.n_factors, P.init_mean,
                                  P.init_std_dev, with_yj=True)
    hp = orc.svd_hyper(P)
    st = np.ones(n_items, np.int32) if stale is None else stale
    pu, qi, yj, bu, bi = orc.svdpp_sgd_stalelog(row_ptr, items, ratings, n_items, P.n_factors,
                                                P.n_epochs, global_mean, hp, pu, qi, yj, st,
                                                chunk_of_user, n_chunks, merge)
    return P, dict(pu=pu, qi=qi, yj=yj, bu=bu, bi=bi)


@pytest.mark.parametrize("merge", [2, 3])
def test_stalelog_svdpp_one_user_per_chunk_is_the_affine_form(u1, merge):
    """Pins the q-log oracle (oracle_svdpp_sgd_stalelog) to the reference's per-user form: with
    one user per chunk every stale row is read once (no repeated items) and folded with weight
    1, so it is oracle_svdpp_sgd_affine (itself pinned to the reference arrays) bit-for-bit; and
    with nothing stale it is the atomic schedule's deferred-y form at any chunking."""
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    params = dict(n_factors=6, n_epochs=2, random_state=0)
    _, a = run_oracle("SVDpp", params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                      affine=True)
    _, b = run_oracle_stalelog(params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                               np.arange(ts.n_users, dtype=np.int32), ts.n_users, merge=merge)
    for k in a:
        np.testing.assert_allclose(b[k], a[k], rtol=0, atol=1e-13, err_msg=k)
    # nothing stale, one chunk: the helper-wave schedule's oracle (hotstale with no hot item)
    P = _Params("SVDpp", params)
    pu, qi, yj = orc.init_factors(get_rng(0), ts.n_users, ts.n_items, 6, P.init_mean,
                                  P.init_std_dev, with_yj=True)
    c = orc.svdpp_sgd_hotstale(row_ptr, items, ratings, ts.n_items, 6, 2, ts.global_mean,
                               orc.svd_hyper(P), pu, qi, yj, np.zeros(ts.n_items, np.int32))
    _, d = run_oracle_stalelog(params, row_ptr, items, ratings, ts.n_items, ts.global_mean,
                               stale=np.zeros(ts.n_items, np.int32), merge=merge)
    for k, x in zip(("pu", "qi", "yj", "bu", "bi"), c):
        np.testing.assert_array_equal(d[k], x, err_msg=k)
