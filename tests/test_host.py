"""Host-side mirror of the reference's plugin API and data model (no GPU needed)."""
import os
import pickle
import warnings

import numpy as np
import pytest

from conftest import GOLDEN
from surprise_amd import (SVD, SVDpp, AlgoBase, Dataset, Prediction, PredictionImpossible,
                          Reader, Trainset, accuracy, synthetic)
from surprise_amd.model_selection import KFold, PredefinedKFold, get_cv
from surprise_amd.utils import get_rng


def test_reader_offset_and_parse():
    r = Reader(line_format="user item rating", sep=",", rating_scale=(-10, 10))
    assert r.offset == 11
    assert r.parse_line("a, b, -3") == ("a", "b", 8.0, None)
    assert Reader("ml-100k").sep == "\t" and Reader("ml-1m").sep == "::"
    with pytest.raises(ValueError):
        Reader("nope")
    with pytest.raises(ValueError):
        Reader(line_format="user item stars")


def test_get_rng_semantics():
    assert get_rng(None) is np.random.mtrand._rand
    a, b = get_rng(3), get_rng(3)
    assert a.normal() == b.normal()
    rs = np.random.RandomState(1)
    assert get_rng(rs) is rs
    with pytest.raises(ValueError):
        get_rng("x")


def test_trainset_all_ratings_order_and_dicts(u1):
    ts, _ = u1
    row_ptr, items, ratings = ts.csr()
    trip = list(ts.all_ratings())
    assert len(trip) == ts.n_ratings
    us = np.array([t[0] for t in trip])
    assert np.all(np.diff(us) >= 0)  # user-major, inner-id order
    np.testing.assert_array_equal([t[1] for t in trip], items)
    # ur built lazily from the CSR agrees with all_ratings; ir holds every rating once
    assert sum(len(v) for v in ts.ur.values()) == ts.n_ratings
    assert sum(len(v) for v in ts.ir.values()) == ts.n_ratings
    assert ts.knows_user(0) and not ts.knows_user(ts.n_users) and not ts.knows_user("UKN__1")
    assert ts.knows_item(0) and not ts.knows_item("UKN__x")
    raw = ts.to_raw_uid(5)
    assert ts.to_inner_uid(raw) == 5
    with pytest.raises(ValueError):
        ts.to_inner_uid("no-such-user")
    assert len(ts.build_testset()) == ts.n_ratings


def test_trainset_ir_raw_order_matches_reference_construct(u1):
    """ir lists keep raw insertion order (dataset.py:236-237)."""
    ts, _ = u1
    rows = [l.split("\t") for l in open(os.path.join(GOLDEN, "u1_ml100k_train"))]
    first_item = rows[0][1]
    iid = ts.to_inner_iid(first_item)
    expected = [(ts.to_inner_uid(r[0]), float(r[2])) for r in rows if r[1] == first_item]
    assert ts.ir[iid] == expected


def test_dict_built_trainset_csr_roundtrip(u1):
    ts, _ = u1
    ts2 = Trainset(ts.ur, None, ts.n_users, ts.n_items, ts.n_ratings, ts.rating_scale, ts.offset,
                   {}, {})
    for a, b in zip(ts.csr(), ts2.csr()):
        np.testing.assert_array_equal(a, b)
    assert ts2.global_mean == ts.global_mean


def test_kfold_partitions_and_determinism():
    u, i, r = synthetic.shape("tiny")
    data = Dataset.load_from_arrays(u, i, r)
    folds = list(KFold(4, random_state=2).split(data))
    assert sum(len(te) for _, te in folds) == len(r)
    assert all(tr.n_ratings + len(te) == len(r) for tr, te in folds)
    folds2 = list(KFold(4, random_state=2).split(data))
    for (a, ta), (b, tb) in zip(folds, folds2):
        for x, y in zip(a.csr(), b.csr()):
            np.testing.assert_array_equal(x, y)
    with pytest.raises(ValueError):
        next(KFold(1).split(data))
    assert isinstance(get_cv(None), KFold) and get_cv(3).n_splits == 3


def test_load_from_df_structured_array():
    import pandas as pd
    df = pd.DataFrame({"u": [1, 2, 2, 3], "i": [10, 10, 20, 30], "r": [4, 3, 5, 1]})
    data = Dataset.load_from_df(df, Reader(rating_scale=(1, 5)))
    ts = data.build_full_trainset()
    assert (ts.n_users, ts.n_items, ts.n_ratings) == (3, 3, 4)
    assert ts.to_inner_uid(2) == 1 and ts.global_mean == np.mean([4, 3, 5, 1])


def test_load_builtin_never_downloads(monkeypatch, tmp_path):
    monkeypatch.setenv("SURPRISE_DATA_FOLDER", str(tmp_path))
    import importlib
    import surprise_amd.reader as rd
    importlib.reload(rd)
    import surprise_amd.dataset as ds
    importlib.reload(ds)
    with pytest.raises(ValueError):
        ds.Dataset.load_builtin("ml-1m")
    importlib.reload(rd)
    importlib.reload(ds)


def test_accuracy_known_answers():
    """test_accuracy.py:17-69 of the reference."""
    preds = [Prediction(0, 0, 0, 0, None), Prediction(1, 1, 1, 1, None)]
    assert accuracy.rmse(preds, verbose=False) == 0
    preds = [Prediction(0, 0, 0, 0, None), Prediction(0, 0, 0, 2, None)]
    assert accuracy.rmse(preds, verbose=False) == np.sqrt((0 + 4) / 2)
    preds = [Prediction(0, 0, 2, 1, None), Prediction(0, 0, 3, 4, None)]
    assert accuracy.rmse(preds, verbose=False) == np.sqrt((1 + 1) / 2)
    preds = [Prediction(0, 0, 0, 0, None), Prediction(1, 1, 1, 1, None)]
    assert accuracy.mae(preds, verbose=False) == 0
    preds = [Prediction(0, 0, 0, 0, None), Prediction(0, 0, 0, 2, None)]
    assert accuracy.mae(preds, verbose=False) == abs(0 - 2) / 2
    preds = [Prediction(0, 0, 2, 1, None), Prediction(0, 0, 3, 4, None)]
    assert accuracy.mae(preds, verbose=False) == (abs(2 - 1) + abs(3 - 4)) / 2
    with pytest.raises(ValueError):
        accuracy.rmse([], verbose=False)


def test_constructor_kwargs_and_fallbacks():
    a = SVD()
    assert (a.n_factors, a.n_epochs, a.biased, a.init_mean, a.init_std_dev) == (100, 20, True, 0, .1)
    assert a.lr_bu == a.lr_qi == .005 and a.reg_pu == .02
    a = SVD(lr_all=.1, reg_all=.3, lr_bi=.2, reg_qi=.4)
    assert (a.lr_bu, a.lr_bi, a.reg_pu, a.reg_qi) == (.1, .2, .3, .4)
    p = SVDpp()
    assert (p.n_factors, p.lr_yj, p.reg_yj) == (20, .007, .02)
    p = SVDpp(lr_yj=.5, reg_yj=.6)
    assert (p.lr_yj, p.reg_yj) == (.5, .6)
    # exactly the reference's parameter names are accepted (test_SVD.py passes them by name)
    SVD(n_factors=1, n_epochs=1, biased=False, init_mean=0, init_std_dev=.1, lr_all=5, reg_all=5,
        lr_bu=5, lr_bi=5, lr_pu=5, lr_qi=5, reg_bu=5, reg_bi=5, reg_pu=5, reg_qi=5,
        random_state=1, verbose=False)


def test_unfitted_algo_pickles_without_gpu():
    a = pickle.loads(pickle.dumps(SVD(n_factors=7)))
    assert a.n_factors == 7 and a._engine is None


def test_estimate_and_predict_semantics_host(golden):
    """AlgoBase.predict / SVD.estimate on host factors: unknown ids, offset, clip and the
    PredictionImpossible fallback (algo_base.py:101-176), checked against the reference's
    values for custom_dataset (factors trained by the oracle, fp64)."""
    import oracle as orc
    meta, _ = golden
    reader = Reader(line_format="user item rating", sep=" ", skip_lines=3, rating_scale=(1, 5))
    ts = Dataset.load_from_file(os.path.join(GOLDEN, "custom_dataset"), reader).build_full_trainset()
    for key, rows in meta["unknown"].items():
        svdpp = key.startswith("SVDpp")
        biased = key != "SVD_unbiased"
        algo = (SVDpp if svdpp else SVD)(random_state=0, **({} if svdpp else dict(biased=biased)))
        AlgoBase.fit(algo, ts)
        rng = get_rng(0)
        pu, qi, yj = orc.init_factors(rng, ts.n_users, ts.n_items, algo.n_factors,
                                      with_yj=svdpp)
        rp, it, rt = ts.csr()
        hp = orc.svd_hyper(algo)
        if svdpp:
            algo.pu, algo.qi, algo.yj, algo.bu, algo.bi = orc.svdpp_sgd(
                rp, it, rt, ts.n_items, algo.n_factors, algo.n_epochs, ts.global_mean, hp, pu,
                qi, yj)
        else:
            algo.pu, algo.qi, algo.bu, algo.bi = orc.svd_sgd(
                rp, it, rt, ts.n_items, algo.n_factors, algo.n_epochs, biased, ts.global_mean,
                hp, pu, qi)
        for uid, iid, est, details in rows:
            p = algo.predict(uid, iid, None)
            assert abs(p.est - est) < 1e-12, (key, uid, iid)
            assert p.details == details


def test_train_is_deprecated_alias():
    class Old(AlgoBase):
        def train(self, trainset):
            AlgoBase.train(self, trainset)
    with pytest.warns(UserWarning):
        Old()


def test_predictions_str():
    s = str(Prediction("u", "i", 3.0, 2.5, {"was_impossible": False}))
    assert "r_ui = 3.00" in s and "est = 2.50" in s
    assert issubclass(PredictionImpossible, Exception)


def test_synthetic_shapes_are_planted():
    u, i, r = synthetic.shape("ml-100k")
    assert len(r) == 100_000 and u.max() == 942 and i.max() <= 1681
    assert np.bincount(u).min() >= 20
    key = u.astype(np.int64) * 1682 + i
    assert len(np.unique(key)) == len(key)
    assert set(np.unique(r)) <= {1, 2, 3, 4, 5}
    u2, i2, r2 = synthetic.shape("ml-100k")
    np.testing.assert_array_equal(r, r2)


def test_fit_without_gpu_fails_loudly(u1):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from surprise_amd._lib import SurpriseAMDError
    ts, _ = u1
    with pytest.raises(SurpriseAMDError):
        SVD(n_factors=2, n_epochs=1).fit(ts)


def test_nmf_and_baseline_argument_errors():
    """test_NMF.py (init_low < 0) and test_bsl_options.py (unknown method): raised before any
    device work."""
    import pytest
    from surprise_amd import NMF, BaselineOnly, Trainset
    with pytest.raises(ValueError):
        NMF(n_factors=1, n_epochs=1, init_low=-1, random_state=1)
    ts = Trainset.from_csr(np.array([0, 1], np.int64), np.array([0], np.int32),
                           np.array([3.0]), 1)
    algo = BaselineOnly(bsl_options={"method": "wrong_name"})
    with pytest.raises(ValueError, match="Invalid method wrong_name"):
        algo.fit(ts)


def test_layout_helpers_match_their_definitions():
    """engine.stable_argsort = np.argsort(kind="stable") (16-bit radix passes, keys past 2^16
    included); position_users = the searchsorted definition; log_layout groups by item in
    increasing CSR position."""
    from surprise_amd.engine import log_layout, position_users, stable_argsort
    rng = np.random.RandomState(3)
    for hi in (1, 7, 3706, 65536, 70000, 1 << 20):
        keys = rng.randint(0, hi, size=5000).astype(np.int32)
        np.testing.assert_array_equal(stable_argsort(keys), np.argsort(keys, kind="stable"))
    assert len(stable_argsort(np.zeros(0, np.int32))) == 0
    deg = rng.randint(0, 9, size=50)
    row_ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    k = np.arange(row_ptr[-1])
    np.testing.assert_array_equal(position_users(row_ptr),
                                  np.searchsorted(row_ptr, k, side="right") - 1)
    items = rng.randint(0, 70000, size=row_ptr[-1]).astype(np.int32)
    perm, _, _, counts = log_layout(row_ptr, items, np.arange(50), 70000)
    np.testing.assert_array_equal(perm, np.argsort(items, kind="stable"))
    np.testing.assert_array_equal(counts, np.bincount(items, minlength=70000))


def test_piece_bounds_partition_every_range():
    """engine.piece_bounds (the NMF / log piece form): each range [offs[i], offs[i]+counts[i])
    is cut into consecutive pieces of 1..piece_rows rows, owner i's pieces are
    [ptr[i], ptr[i+1]) in order, empty ranges have none, and the last bound is offs[-1]."""
    from surprise_amd.engine import piece_bounds
    rng = np.random.RandomState(5)
    for rows in (1, 7, 64):
        counts = rng.choice([0, 1, 63, 64, 65, 200, 1805], size=40)
        offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        ptr, beg = piece_bounds(offs, counts, rows)
        assert ptr[0] == 0 and ptr[-1] == len(beg) - 1 and beg[-1] == offs[-1]
        sizes = np.diff(beg)
        assert sizes.min() >= 1 and sizes.max() <= rows
        for i, n in enumerate(counts):
            b = beg[ptr[i]:ptr[i + 1] + 1]
            assert ptr[i + 1] - ptr[i] == -(-n // rows)
            if n:
                assert b[0] == offs[i] and b[-1] == offs[i + 1]


# ------------------------------------------------------------------ log layouts (host side)

def _random_csr(seed=0, n_users=200, n_items=50):
    rng = np.random.RandomState(seed)
    deg = rng.randint(1, 30, n_users)
    row_ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    items = np.concatenate([rng.choice(n_items, d, replace=False) for d in deg]).astype(np.int32)
    return rng, row_ptr, items


def test_packed_checkpoint_rows_are_one_per_pair_and_in_bounds():
    """ckpt_positions / ck_row0 (the kernels' packed log): every pair of a user's ratings has its
    own row, both ratings of a pair share it, and the rows fit in ck_row0[n_users]."""
    from surprise_amd.engine import ck_row0, ckpt_positions, log_layout
    _, row_ptr, items = _random_csr()
    perm, _, _, _ = log_layout(row_ptr, items, np.arange(len(row_ptr) - 1), 50)
    ck = ckpt_positions(row_ptr, perm)
    row, odd = ck >> 1, ck & 1
    u = np.searchsorted(row_ptr, perm, side="right") - 1
    j = perm - row_ptr[u]
    assert np.array_equal(odd, j & 1)
    assert np.array_equal(row, ck_row0(row_ptr)[u] + j // 2)
    assert row.max() < ck_row0(row_ptr)[-1]
    pairs = {}
    for r, uu, jj in zip(row, u, j // 2):
        assert pairs.setdefault(int(r), (int(uu), int(jj))) == (int(uu), int(jj))


def test_recency_positions_follow_user_order_within_items():
    """The recency fold's positions: a rating's rank among the chunk's ratings of its item in
    user order, the same from a chunk's single-group perm and from the general form."""
    from surprise_amd.engine import item_positions, log_layout
    rng, row_ptr, items = _random_csr(1)
    users = rng.choice(len(row_ptr) - 1, 120, replace=False)
    perm, pb, ipp, cnt = log_layout(row_ptr, items, users, 50)
    rp = np.arange(len(perm)) - np.repeat(pb[ipp[:-1]], cnt)
    ks, pos = item_positions(row_ptr, items, users, 50)
    kpos = np.zeros(int(row_ptr[-1]), np.int32)
    kpos[ks] = pos
    assert np.array_equal(rp, kpos[perm])
    for i in range(50):  # positions 0..N_i-1 in increasing CSR position
        sel = items[perm] == i
        assert np.array_equal(rp[sel], np.arange(sel.sum()))
        assert np.all(np.diff(perm[sel]) > 0)


def test_hot_items_policy():
    """engine.hot_items: the items whose SVD++ q rows get a delta replica."""
    from surprise_amd.engine import hot_items, HOT_MAX
    items = np.concatenate([np.full(2000, 7), np.full(700, 3), np.full(300, 5),
                            np.arange(10000).repeat(30)])               # 303,000 ratings
    np.testing.assert_array_equal(hot_items(items, 10000), [3, 7])    # top 0.67%: >= 0.15%
    np.testing.assert_array_equal(hot_items(items, 10000, 3), [3, 5, 7])  # the 3 most rated
    assert len(hot_items(items, 10000, 0)) == 0
    assert len(hot_items(np.arange(50).repeat(20), 50)) == 0          # top item < 1000 ratings
    flat = np.concatenate([np.full(1600, 0), np.arange(1, 1000).repeat(300)])  # top 0.53%
    assert len(hot_items(flat, 1000)) == 1
    assert len(hot_items(np.arange(300).repeat(1000)[::-1], 300)) == 0  # top 0.33%: none
    many = np.concatenate([np.full(3000, 1), np.arange(2, 200).repeat(1000)])
    assert len(hot_items(many, 200)) == HOT_MAX


def test_replay_piece_rows_policy():
    """engine.replay_piece_rows: 64 at ML-1M size, REPLAY_MAX_ROWS at C4's."""
    from surprise_amd.engine import replay_piece_rows, REPLAY_MAX_ROWS
    assert replay_piece_rows(np.array([0, 800_000]), np.array([0])) == 64
    assert replay_piece_rows(np.array([0, 99_000_000]), np.array([0])) == REPLAY_MAX_ROWS
    assert replay_piece_rows(np.array([0, 10]), np.array([], np.int64)) == 64


def test_testset_columns_list_and_column_native():
    """_MFBase._columns: a list of triples and the column-native forms give the same columns."""
    from surprise_amd import SVD
    from surprise_amd.dataset import RatingColumns
    rows = [(1, 10, 4.0), (2, 20, 3.5), (7, 10, 1.0)]
    a = SVD()
    ru, ri, r = a._columns(rows)
    assert ru == [1, 2, 7] and ri == [10, 20, 10] and r.tolist() == [4.0, 3.5, 1.0]
    cu, ci, cr = a._columns(RatingColumns([1, 2, 7], [10, 20, 10], [4.0, 3.5, 1.0]))
    assert cu.tolist() == ru and ci.tolist() == ri and cr.tolist() == r.tolist()
    st = np.array(rows, dtype=[("uid", "i8"), ("iid", "i8"), ("rating", "f8")])
    su, si, sr = a._columns(st)
    assert su.tolist() == ru and si.tolist() == ri and sr.tolist() == r.tolist()
    assert a._columns([])[2].shape == (0,)


# ------------------------------------------------------------------ fcp / ShuffleSplit /
# train_test_split / print_summary (the reference's tests: test_accuracy.py:49-69,
# test_split.py:94-229, validation.py:772-811)

def _pred(true_r, est, u0=None):
    return u0, None, true_r, est, None


def test_fcp_known_answers():
    """test_accuracy.py:49-69."""
    preds = [_pred(0, 0, "u1"), _pred(1, 1, "u1"), _pred(2, 2, "u2"), _pred(100, 100, "u2")]
    assert accuracy.fcp(preds, verbose=False) == 1
    with pytest.raises(ValueError):
        accuracy.fcp([_pred(0, 0, "u1"), _pred(0, 0, "u1")], verbose=False)
    with pytest.raises(ValueError):
        accuracy.fcp([_pred(0, 0, "u1")], verbose=False)
    preds = [_pred(1, 0, "u1"), _pred(0, 1, "u1"), _pred(2, 0, "u2"), _pred(0, 2, "u2")]
    assert accuracy.fcp(preds, verbose=False) == 0
    with pytest.raises(ValueError):
        accuracy.fcp([])
    # the reference's means run over the users with at least one pair of each kind
    preds = [_pred(1, 1, "a"), _pred(2, 2, "a"), _pred(3, 3, "a"),
             _pred(1, 2, "b"), _pred(2, 1, "b")]
    assert accuracy.fcp(preds, verbose=False) == 3 / (3 + 1)


def test_cross_validate_fcp_measure_resolves(u1):
    """fit_and_score resolves measures by name (validation.py:754-756): 'fcp' is one of them."""
    from surprise_amd.model_selection import fit_and_score

    class ByItem(AlgoBase):
        def fit(self, trainset):
            AlgoBase.fit(self, trainset)
            return self

        def estimate(self, u, i):
            return 1.0 + (i % 5 if isinstance(i, int) else 0)

    ts, test = u1
    m = fit_and_score(ByItem(), ts, list(test), ["rmse", "fcp"])[0]
    assert set(m) == {"rmse", "fcp"} and 0 < m["fcp"] < 1


def _custom_data():
    return Dataset.load_from_file(os.path.join(GOLDEN, "custom_dataset"),
                                  Reader(line_format="user item rating", sep=" ", skip_lines=3,
                                         rating_scale=(1, 5)))


def test_shuffle_split_like_reference():
    """test_split.py:94-178 on the reference's custom_dataset (5 ratings)."""
    from surprise_amd.model_selection import ShuffleSplit
    data = _custom_data()
    with pytest.raises(ValueError):
        ShuffleSplit(n_splits=0)
    for kw in (dict(test_size=10), dict(train_size=10), dict(test_size=3, train_size=3)):
        with pytest.raises(ValueError):
            next(ShuffleSplit(**kw).split(data))
    for kw in (dict(test_size=3, train_size=0), dict(test_size=0, train_size=3)):
        with pytest.raises(ValueError):
            ShuffleSplit(**kw)
    next(ShuffleSplit(test_size=1, train_size=1).split(data))
    for kw, n_test, n_train in ((dict(test_size=1), 1, 4), (dict(test_size=.2), 1, 4),
                                (dict(test_size=2, train_size=2), 2, 2),
                                (dict(test_size=None, train_size=2), 3, 2),
                                (dict(test_size=None, train_size=.2), 4, 1), ({}, 1, 4)):
        splits = list(ShuffleSplit(**kw).split(data))
        assert all(len(te) == n_test and tr.n_ratings == n_train for tr, te in splits), kw
    assert len(list(ShuffleSplit().split(data))) == 5
    ss = ShuffleSplit(random_state=None)
    assert [te for _, te in ss.split(data)] != [te for _, te in ss.split(data)]
    for ss in (ShuffleSplit(random_state=1), ShuffleSplit(random_state=1, shuffle=False)):
        assert [te for _, te in ss.split(data)] == [te for _, te in ss.split(data)]
    # index logic: the permutation's first train_size ratings train, the next test_size test
    tr, te = next(ShuffleSplit(n_splits=1, test_size=2, train_size=2, random_state=7)
                  .split(data))
    perm = np.random.RandomState(7).permutation(5)
    assert te == [data.raw_ratings[i][:3] for i in perm[2:4]]
    assert sorted(r for _, _, r in tr.all_ratings()) == sorted(
        data.raw_ratings[i][2] + tr.offset for i in perm[:2])


def test_train_test_split_like_reference():
    """test_split.py:181-229."""
    from surprise_amd.model_selection import train_test_split
    data = _custom_data()
    for kw, n_test, n_train in ((dict(test_size=2, train_size=None), 2, 3),
                                (dict(test_size=.2, train_size=None), 1, 4),
                                (dict(test_size=2, train_size=3), 2, 3),
                                (dict(test_size=None, train_size=2), 3, 2),
                                (dict(test_size=None, train_size=.2), 4, 1)):
        tr, te = train_test_split(data, **kw)
        assert len(te) == n_test and tr.n_ratings == n_train, kw
    # random_state=None: the global numpy RNG moves on between calls (a single 1-rating testset
    # repeats with probability 1/5, so compare a few draws)
    draws = [train_test_split(data, random_state=None)[1] for _ in range(8)]
    assert any(d != draws[0] for d in draws[1:])
    assert train_test_split(data, random_state=1)[1] == train_test_split(data, random_state=1)[1]
    assert train_test_split(data, random_state=1, shuffle=None)[1] == \
        train_test_split(data, random_state=1, shuffle=None)[1]


def test_print_summary_table(capsys):
    from surprise_amd.model_selection import print_summary
    print_summary(SVD(), ["rmse", "mae"], {"rmse": np.array([1.0, 0.5]),
                                           "mae": np.array([0.8, 0.6])},
                  {}, (1.0, 3.0), (0.25, 0.75), 2)
    out = capsys.readouterr().out.splitlines()
    assert out[0] == "Evaluating RMSE, MAE of algorithm SVD on 2 split(s)."
    assert out[1] == ""
    assert out[2].split() == ["Fold", "1", "Fold", "2", "Mean", "Std"]
    assert out[3].split() == ["RMSE", "(testset)", "1.0000", "0.5000", "0.7500", "0.2500"]
    assert out[4].split() == ["MAE", "(testset)", "0.8000", "0.6000", "0.7000", "0.1000"]
    assert out[5].split() == ["Fit", "time", "1.00", "3.00", "2.00", "1.00"]
    assert out[6].split() == ["Test", "time", "0.25", "0.75", "0.50", "0.25"]
    assert out[3].index("1.0000") == 18  # '{:<18}' label column, '{:<8}' per value


def test_roofline_executed_bytes_and_span_bounds():
    """bench.roofline_of on a made-up split step: the dominant kernel's rate uses the concurrent
    launches' wall span, every launch and the step report frac <= 1 for plausible timings, and
    SURVEY 8(d)'s figure rides as a rate without a frac."""
    import bench
    lay = {"s": 8, "K": 100, "ldq": 104, "ld": 104, "algo": "svd", "ckpt": True, "narrow": False,
           "err_in_row": True, "ldc": 104, "hx": False, "n_items": 3706, "n_chunks": 1,
           "launches": {"heavy": {"ratings": 121840, "users": 128, "pieces": 3000},
                        "light": {"ratings": 678327, "users": 5912, "pieces": 14000}}}
    per_r = 4 + 8 + 102 * 8 + 104 * 8 / 2
    assert bench.executed_bytes(lay, 1, 0) == per_r
    ph = {"epoch_kernel": {"span_ms_per_step": 0.246, "ratings_per_step": 800167,
                           "launches": {"heavy": {"per_step": 1, "avg_us": 246.0,
                                                  "ratings": 121840},
                                        "light": {"per_step": 1, "avg_us": 131.0,
                                                  "ratings": 678327}}}}
    rl = bench.roofline_of("svd", 100, "f64", 800167, 0.294, "ml-1m", ph, lay,
                           {"top_user_ratings": 1805, "alone_us": 199.0})
    dk = rl["dominant_kernel"]
    assert abs(rl["achieved"] - dk["executed_bytes_per_step"] / 0.246e-3 / 1e9) < 1e-6
    assert 0 < rl["frac"] <= 1 and rl["step"]["frac"] <= 1
    assert all(0 < v["frac"] <= 1 for v in dk["launches"].values())
    assert "frac" not in rl["survey_8d"]
    assert abs(rl["chain_latency"]["frac"] - 199 / 246) < 1e-12


def test_bench_line_stays_small_and_keeps_the_contract():
    """round 4's 21.9 KB stdout line went unparsed by the driver.  The line
    built from a canned full result (round 4's final-tree bench dictionary, every leg present)
    stays under bench.LINE_LIMIT (< 12 KB, the largest line a driver parsed) and keeps the
    contract's fields, the roofline's dominant kernel per launch, cpu_baseline and rmse."""
    import json
    import bench
    full = json.load(open(os.path.join(os.path.dirname(bench.__file__), "profiles",
                                       "r4u_bench.json")))
    assert len(json.dumps(full)) > 20000
    line = bench.compact_line(full, "gpurun_out/bench_detail_ml-1m_n1.json")
    text = json.dumps(line)
    assert len(text) <= bench.LINE_LIMIT < 12000, len(text)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line, k
    assert abs(line["value"] / full["value"] - 1) < 1e-4
    rl = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rl, k
    assert set(rl["dominant_kernel"]["launches"]) == {"heavy", "light"}
    assert "frac" in rl["step"] and "frac" in rl["chain_latency"]
    cb = line["cpu_baseline"]
    assert {"value", "unit", "cores", "kind", "sample"} <= set(cb)
    assert "value" in cb["single_core"] and "cython_equivalent_single_core" in cb
    assert line["rmse"]["delta"] == full["rmse"]["delta"]  # (full precision)
    for leg in ("f32_leg", "svdpp_c3", "c4", "predict"):
        assert leg in line, leg
    assert line["detail"].endswith(".json")
    # a pathological result still keeps the headline under the limit
    fat = dict(full, data="x" * 4000)
    assert len(json.dumps(bench.compact_line(fat))) <= bench.LINE_LIMIT + 4000


def test_default_chunks_counts_users_per_rank():
    """SVD++'s epoch-chunks follow the users of ONE rank (engine.SVDPP_USERS_PER_CHUNK): C5@8
    (10M users, 8 ranks) and the C5 shard on one GPU both run 16 chunks of <= 80k users per rank,
    the geometries the scale tests pin; one GPU with all of C5 runs 125; SVD's log runs 1."""
    from surprise_amd.engine import SVDPP_USERS_PER_CHUNK, default_chunks
    assert default_chunks("svdpp", "atomic", 10_000_000, 8) == 16
    assert default_chunks("svdpp", "atomic", 1_250_000) == 16
    assert default_chunks("svdpp", "atomic", 1_250_000, 8) == 2
    assert default_chunks("svdpp", "atomic", 10_000_000) == 125
    assert default_chunks("svdpp", "atomic", 6040) == 1
    assert default_chunks("svd", "log", 10_000_000) == 1
    for users, world in ((10_000_000, 8), (1_250_000, 1), (999_999, 3)):
        c = default_chunks("svdpp", "atomic", users, world)
        assert -(-users // world) <= c * SVDPP_USERS_PER_CHUNK


def test_default_ldq_reserves_the_user_bias_column_only_for_the_svd_log():
    """column K+1 (the SVD log lookahead body's constant user-bias column) only where
    that body reads it -- rows stay within 1 KiB at fp64 K=126 / fp32 K=254 for the SVD log and
    at fp64 K=127 / fp32 K=255 elsewhere (SVD++ keeps its helper-wave launch); fp64 K=63
    without the column keeps one lane group (64 * 8 = 512 B)."""
    from surprise_amd import _lib
    from surprise_amd.engine import default_ldq
    F32, F64 = _lib.MF_F32, _lib.MF_F64
    assert default_ldq(127, F64) * 8 == 1024 and default_ldq(255, F32) * 4 == 1024
    assert default_ldq(126, F64, user_bias_col=True) * 8 == 1024
    assert default_ldq(254, F32, user_bias_col=True) * 4 == 1024
    assert default_ldq(127, F64, user_bias_col=True) * 8 > 1024  # (K + 2 columns do not fit)
    assert default_ldq(63, F64) * 8 == 512
    for K in (1, 10, 100, 128):
        for dt, s in ((F32, 4), (F64, 8)):
            for col in (False, True):
                ldq = default_ldq(K, dt, user_bias_col=col)
                assert ldq >= K + 1 + int(col) and (ldq * s) % 64 == 0


def test_split_groups_light_top_rest():
    """A split chunk's launch groups (engine `heavy`, `top`): [light, heavy], or [light, top,
    rest] -- a partition of the chunk, schedule order kept inside each group, the top users the
    heaviest of the heavy ones."""
    from surprise_amd.engine import split_groups
    rng = np.random.RandomState(3)
    deg = rng.randint(1, 2000, size=3000)
    row_ptr = np.concatenate([[0], np.cumsum(deg)])
    users = np.argsort(-deg, kind="stable").astype(np.int32)  # heaviest-first, as chunks are
    two = split_groups(users, row_ptr, 128)
    three = split_groups(users, row_ptr, 128, top=16)
    assert [len(p) for p in two] == [3000 - 128, 128]
    assert [len(p) for p in three] == [3000 - 128, 16, 112]
    np.testing.assert_array_equal(np.sort(np.concatenate(three)), np.arange(3000))
    np.testing.assert_array_equal(np.sort(np.concatenate(three[1:])), np.sort(two[1]))
    assert deg[three[1]].min() >= deg[three[2]].max()
    for p in three:  # (schedule order kept: heaviest first)
        assert np.all(np.diff(deg[p]) <= 0)
    assert len(split_groups(users, row_ptr, 128, top=200)) == 2  # (top >= heavy: no third)


def test_default_dtype_is_fp64_up_to_the_fp64_row_limit():
    """The drop-in classes compute in the reference's fp64 by default; above the fp64 kernels'
    256-factor rows they fall back to fp32 (up to 512) instead of refusing the model."""
    from surprise_amd import NMF, SVD, SVDpp
    assert SVD().dtype == "float64" and SVDpp().dtype == "float64" and NMF().dtype == "float64"
    assert SVD(n_factors=256).dtype == "float64"
    assert SVD(n_factors=300).dtype == "float32"
    assert SVD(n_factors=10, dtype="float32").dtype == "float32"
    # the default follows n_factors set after construction (resolved again at fit)
    a = SVD(n_factors=10)
    a.n_factors = 300
    assert a._dtype_auto and a._auto_dtype() == "float32"
    b = SVD(n_factors=10, dtype="float64")
    b.n_factors = 300
    assert not b._dtype_auto  # (an explicit dtype stays: fit then refuses 300 fp64 factors)


def test_default_schedule_is_the_exact_order_for_small_svd_fits():
    """SVD(deterministic=None), the default: the reference's exact sequence when the fit is small
    (n_ratings x n_epochs <= EXACT_MAX_UPDATES and x n_factors <= EXACT_MAX_WORK) and every
    schedule option is at its default; the parallel schedule otherwise.  SVDpp: parallel."""
    from surprise_amd import SVD, SVDpp
    from surprise_amd.matrix_factorization import EXACT_MAX_UPDATES, EXACT_MAX_WORK
    u1 = 80_000
    assert SVD(n_factors=100, n_epochs=20)._resolve_deterministic(u1)      # 1.6M updates
    assert SVD(n_factors=20, n_epochs=5)._resolve_deterministic(u1)        # configs[0]
    assert not SVD(n_factors=100, n_epochs=20)._resolve_deterministic(1_000_209)  # ML-1M
    assert not SVD(n_factors=100, n_epochs=21)._resolve_deterministic(100_000)  # 2.1M updates
    assert not SVD(n_factors=200, n_epochs=20)._resolve_deterministic(u1)  # 3.2e8 > EXACT_MAX_WORK
    assert EXACT_MAX_UPDATES * 100 == EXACT_MAX_WORK
    for kw in (dict(mode="log"), dict(chunks_per_epoch=2), dict(n_waves=64),
               dict(distributed=True), dict(deterministic=False)):
        assert not SVD(n_factors=20, n_epochs=5, **kw)._resolve_deterministic(u1), kw
    assert SVD(n_factors=20, n_epochs=5, deterministic=True)._resolve_deterministic(10 ** 9)
    opt = SVD(n_factors=20, n_epochs=5)
    opt._engine_options = {"heavy": 16}  # (an engine option asks for the parallel schedule)
    assert not opt._resolve_deterministic(u1)
    assert not SVDpp(n_factors=20, n_epochs=5)._resolve_deterministic(u1)


def test_qlog_fold_layout_partitions_cold_and_hot_items():
    """mf_svdpp_qlog_fold's layout (engine.qlog_fold_layout): every item-grouped position is
    either a cold item's (listed directly, item_row_beg / item_user_beg ranges) or a hot item's
    (more than hot_rows rows: pieces of <= 64 positions, each piece of one item, in order)."""
    from surprise_amd.engine import qlog_fold_layout
    rng = np.random.RandomState(5)
    counts = rng.choice([0, 1, 3, 64, 65, 200, 700], size=40)
    tot = int(counts.sum())
    perm = rng.permutation(tot).astype(np.int32)
    rpos = np.concatenate([np.arange(c) for c in counts]).astype(np.int32)
    users = rng.randint(0, 1000, tot).astype(np.int32)
    lay = qlog_fold_layout(counts, perm, rpos, users, hot_rows=64)
    hot = counts > 64
    assert lay["item_row_beg"][-1] + len(lay["hot_perm"]) == tot
    np.testing.assert_array_equal(np.diff(lay["item_row_beg"]), np.where(hot, 0, counts))
    np.testing.assert_array_equal(np.diff(lay["hot_item_piece_ptr"]), np.where(hot, -(-counts // 64), 0))
    pb = lay["hot_piece_beg"]
    assert pb[0] == 0 and pb[-1] == len(lay["hot_perm"]) and np.all(np.diff(pb) <= 64)
    assert lay["n_hot_pieces"] == len(pb) - 1 == len(lay["hot_piece_item"])
    offs = np.concatenate([[0], np.cumsum(counts)])
    for i in range(len(counts)):
        rows = perm[offs[i]:offs[i + 1]]
        if hot[i]:
            p0, p1 = lay["hot_item_piece_ptr"][i], lay["hot_item_piece_ptr"][i + 1]
            assert np.all(lay["hot_piece_item"][p0:p1] == i)
            np.testing.assert_array_equal(lay["hot_perm"][pb[p0]:pb[p1]], rows)
            np.testing.assert_array_equal(lay["hot_rpos"][pb[p0]:pb[p1]], np.arange(counts[i]))
        else:
            b0, b1 = lay["item_row_beg"][i], lay["item_row_beg"][i + 1]
            np.testing.assert_array_equal(lay["perm"][b0:b1], rows)
            np.testing.assert_array_equal(lay["users"][b0:b1], users[offs[i]:offs[i + 1]])


def test_auto_qlog_rule():
    """engine.auto_qlog (qlog=None): the SVD++ q log on ONE rank with several chunks of at most
    QLOG_MAX_RATINGS_PER_ITEM_CHUNK ratings per item -- C5 (full: 125 chunks, shard: 16), ML-1M at
    24+ chunks -- and the float-atomic schedule for ML-1M's default single chunk (C3), 16 chunks
    (13.5 per item: +1.9e-3 measured), several ranks, the exchange path, duplicate items, SVD."""
    from surprise_amd import _lib
    from surprise_amd.engine import auto_qlog, default_chunks
    A = _lib.MF_MODE_ATOMIC
    ml1m = (800_167, 3706)
    c5 = (989_997_254, 1_000_000)
    c5_shard = (123_000_000, 1_000_000)
    assert default_chunks("svdpp", "atomic", 10_000_000) == 125
    assert auto_qlog("svdpp", A, *c5, 125, 1, None, False, False)
    assert auto_qlog("svdpp", A, *c5_shard, 16, 1, None, False, False)
    assert not auto_qlog("svdpp", A, *ml1m, 1, 1, None, False, False)  # C3
    assert not auto_qlog("svdpp", A, *ml1m, 16, 1, None, False, False)
    assert auto_qlog("svdpp", A, *ml1m, 24, 1, None, False, False)
    assert not auto_qlog("svdpp", A, *c5_shard, 16, 8, None, False, False)  # several ranks
    assert not auto_qlog("svdpp", A, *c5_shard, 16, 1, True, False, False)  # exchange (test)
    assert not auto_qlog("svdpp", A, *c5_shard, 16, 1, None, True, False)   # duplicate items
    assert not auto_qlog("svdpp", A, *c5_shard, 16, 1, None, False, True)   # deterministic
    assert not auto_qlog("svd", _lib.MF_MODE_LOG, *c5_shard, 16, 1, None, False, False)
    assert not auto_qlog("svdpp", _lib.MF_MODE_PLAIN, *c5_shard, 16, 1, None, False, False)
