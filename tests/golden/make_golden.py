"""Generates the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the CPU container only (the reference is not on the GPU box):
    oracle/build_ref.sh            # out-of-tree Cython build of /root/reference in /tmp
    PYTHONPATH=/tmp/surprise_ref_build python tests/golden/make_golden.py

Inputs are the reference's own test data files (tests/u1_ml100k_train / _test,
tests/custom_dataset; copied here verbatim as data fixtures) and this repo's
seeded synthetic generator (surprise_amd.synthetic, regenerated at test time).
Outputs are values only: RMSE/MAE, per-prediction estimates, sha256 of factor
arrays, full factor arrays for the small cases, and a CPU timing calibration.
No reference source is copied.
"""
import contextlib
import hashlib
import io
import json
import os
import shutil
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_TESTS = "/root/reference/tests"
sys.path.insert(1, REPO)

import surprise  # noqa: E402  (the reference, via PYTHONPATH)
from surprise import SVD, SVDpp, Dataset, Reader, accuracy  # noqa: E402
from surprise.model_selection import PredefinedKFold, KFold, cross_validate  # noqa: E402

assert "surprise_ref_build" in surprise.__file__, surprise.__file__


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()


def quiet_fit(algo, ts):
    with contextlib.redirect_stdout(io.StringIO()):
        algo.fit(ts)
    return algo


def trainset_csr(ts):
    row_ptr = [0]
    items, ratings = [], []
    for u, lst in ts.ur.items():
        assert u == len(row_ptr) - 1
        for i, r in lst:
            items.append(i)
            ratings.append(r)
        row_ptr.append(len(items))
    return np.array(row_ptr, np.int64), np.array(items, np.int32), np.array(ratings, np.float64)


def main():
    # ---- data fixtures (the reference's own test data files)
    for f in ("u1_ml100k_train", "u1_ml100k_test", "custom_dataset"):
        shutil.copyfile(os.path.join(REF_TESTS, f), os.path.join(HERE, f))

    out = {"generator": "tests/golden/make_golden.py", "reference": surprise.__file__}
    arrays = {}

    # ---- u1 fixture: trainset semantics + SVD / SVD++ known answers
    data = Dataset.load_from_folds([(os.path.join(HERE, "u1_ml100k_train"),
                                     os.path.join(HERE, "u1_ml100k_test"))], Reader("ml-100k"))
    ts, test = next(PredefinedKFold().split(data))
    row_ptr, items, ratings = trainset_csr(ts)
    arrays["u1_row_ptr"], arrays["u1_items"], arrays["u1_ratings"] = row_ptr, items, ratings
    out["u1"] = dict(n_users=ts.n_users, n_items=ts.n_items, n_ratings=ts.n_ratings,
                     global_mean=float(ts.global_mean), n_test=len(test),
                     raw2inner_users_first=[[k, v] for k, v in list(ts._raw2inner_id_users.items())[:10]],
                     raw2inner_items_first=[[k, v] for k, v in list(ts._raw2inner_id_items.items())[:10]])
    cases = [
        ("svd_k20_e5", "SVD", dict(n_factors=20, n_epochs=5, random_state=0), True),
        ("svd_k100_e20", "SVD", dict(n_factors=100, n_epochs=20, random_state=0), False),
        ("svd_k100_e20_unbiased", "SVD", dict(n_factors=100, n_epochs=20, biased=False,
                                              random_state=0), False),
        ("svd_k128_e20", "SVD", dict(n_factors=128, n_epochs=20, random_state=0), False),
        ("svd_k10_e3_hyper", "SVD", dict(n_factors=10, n_epochs=3, init_mean=.05, init_std_dev=.2,
                                         lr_all=.007, reg_all=.03, lr_bu=.01, lr_bi=.002,
                                         lr_pu=.004, lr_qi=.006, reg_bu=.05, reg_bi=.01,
                                         reg_pu=.015, reg_qi=.025, random_state=7), True),
        ("svd_k5_e2_unbiased", "SVD", dict(n_factors=5, n_epochs=2, biased=False,
                                           random_state=3), True),
        ("svdpp_k20_e20", "SVDpp", dict(n_factors=20, n_epochs=20, random_state=0), False),
        ("svdpp_k100_e20", "SVDpp", dict(n_factors=100, n_epochs=20, random_state=0), False),
        ("svdpp_k10_e3", "SVDpp", dict(n_factors=10, n_epochs=3, random_state=0), True),
        ("svdpp_k8_e2_hyper", "SVDpp", dict(n_factors=8, n_epochs=2, lr_yj=.01, reg_yj=.05,
                                            lr_pu=.003, reg_qi=.04, random_state=11), True),
    ]
    out["cases"] = {}
    for name, klass, kw, full in cases:
        algo = {"SVD": SVD, "SVDpp": SVDpp}[klass](**kw)
        t0 = time.perf_counter()
        quiet_fit(algo, ts)
        dt = time.perf_counter() - t0
        preds = algo.test(test)
        est = np.array([p.est for p in preds])
        rec = dict(algo=klass, params=kw, rmse=float(accuracy.rmse(preds, verbose=False)),
                   mae=float(accuracy.mae(preds, verbose=False)), fit_seconds=dt,
                   sha_pu_qi=sha(algo.pu, algo.qi), sha_bu_bi=sha(algo.bu, algo.bi),
                   impossible=int(sum(p.details["was_impossible"] for p in preds)))
        if klass == "SVDpp":
            rec["sha_yj"] = sha(algo.yj)
        arrays[name + "_est"] = est
        if full:
            arrays[name + "_pu"], arrays[name + "_qi"] = algo.pu, algo.qi
            arrays[name + "_bu"], arrays[name + "_bi"] = algo.bu, algo.bi
            if klass == "SVDpp":
                arrays[name + "_yj"] = algo.yj
        out["cases"][name] = rec
        print(name, rec["rmse"], rec["sha_pu_qi"][:16], "%.2fs" % dt)
    arrays["u1_test_r"] = np.array([r for (_, _, r) in test], np.float64)
    out["u1_test_ids"] = [[u, i] for (u, i, _) in test[:5]]

    # ---- test_SVD.py sensitivity sweep as known answers (cross_validate + PredefinedKFold)
    pkf = PredefinedKFold()
    sweep = {}
    base = dict(n_factors=1, n_epochs=1, random_state=1)
    variants = [("default", {}), ("n_factors", dict(n_factors=2)), ("n_epochs", dict(n_epochs=2)),
                ("biased", dict(biased=False)), ("lr_all", dict(lr_all=5)),
                ("reg_all", dict(reg_all=5)), ("lr_bu", dict(lr_bu=5)), ("lr_bi", dict(lr_bi=5)),
                ("lr_pu", dict(lr_pu=5)), ("lr_qi", dict(lr_qi=5)), ("reg_bu", dict(reg_bu=5)),
                ("reg_bi", dict(reg_bi=5)), ("reg_pu", dict(reg_pu=5)), ("reg_qi", dict(reg_qi=5))]
    for vname, extra in variants:
        kw = dict(base, **extra)
        with contextlib.redirect_stdout(io.StringIO()):
            res = cross_validate(SVD(**kw), data, ["rmse"], pkf, n_jobs=1)
        sweep["SVD_" + vname] = dict(params=kw, test_rmse=float(res["test_rmse"][0]))
    for vname, extra in [("default", {}), ("n_factors", dict(n_factors=2))]:
        kw = dict(base, **extra)
        res = cross_validate(SVDpp(**kw), data, ["rmse"], pkf, n_jobs=1)
        sweep["SVDpp_" + vname] = dict(params=kw, test_rmse=float(res["test_rmse"][0]))
    out["sensitivity"] = sweep

    # ---- unknown user / item (test_algorithms.py:28-57) on custom_dataset
    reader = Reader(line_format="user item rating", sep=" ", skip_lines=3, rating_scale=(1, 5))
    cdata = Dataset.load_from_file(os.path.join(HERE, "custom_dataset"), reader)
    cts = cdata.build_full_trainset()
    unk = {}
    for klass in (SVD, SVDpp):
        for biased in ((True, False) if klass is SVD else (True,)):
            kw = dict(random_state=0)
            if klass is SVD:
                kw["biased"] = biased
            algo = quiet_fit(klass(**kw), cts)
            key = klass.__name__ + ("" if biased else "_unbiased")
            unk[key] = [[q[0], q[1], algo.predict(q[0], q[1], None).est,
                         algo.predict(q[0], q[1], None).details]
                        for q in (("user0", "unknown_item"), ("unkown_user", "item0"),
                                  ("unkown_user", "unknown_item"), ("user0", "item0"))]
    out["unknown"] = unk

    # ---- synthetic ml-100k shape through the reference's file reader + KFold(5, rs=0)
    from surprise_amd import synthetic
    u, i, r = synthetic.shape("ml-100k")
    path = "/tmp/surprise_golden_synth_ml100k.tsv"
    with open(path, "w") as f:
        for a, b, c in zip(u.tolist(), i.tolist(), r.tolist()):
            f.write("%d\t%d\t%d\n" % (a, b, int(c)))
    sdata = Dataset.load_from_file(path, Reader(line_format="user item rating", sep="\t"))
    sts, stest = next(KFold(5, random_state=0).split(sdata))
    srow, sitems, sratings = trainset_csr(sts)
    algo = quiet_fit(SVD(n_factors=20, n_epochs=5, random_state=0), sts)
    preds = algo.test(stest)
    out["synth_ml100k"] = dict(n_users=sts.n_users, n_items=sts.n_items, n_ratings=sts.n_ratings,
                               global_mean=float(sts.global_mean), n_test=len(stest),
                               sha_csr=sha(srow, sitems, sratings),
                               svd_k20_e5=dict(rmse=float(accuracy.rmse(preds, verbose=False)),
                                               sha_pu_qi=sha(algo.pu, algo.qi)))
    algo = quiet_fit(SVDpp(n_factors=10, n_epochs=2, random_state=0), sts)
    preds = algo.test(stest)
    out["synth_ml100k"]["svdpp_k10_e2"] = dict(rmse=float(accuracy.rmse(preds, verbose=False)),
                                               sha_pu_qi_yj=sha(algo.pu, algo.qi, algo.yj))
    print("synth", out["synth_ml100k"])

    # ---- CPU calibration: reference Cython sgd vs the oracle restatement, same data, 1 thread
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc
    u, i, r = synthetic.shape("ml-1m")
    from surprise_amd.dataset import Dataset as MyDataset
    from surprise_amd.model_selection import KFold as MyKFold
    mts, _ = next(MyKFold(5, random_state=0).split(MyDataset.load_from_arrays(u, i, r)))
    rp, it, rt = mts.csr()
    ref_ts = surprise.Trainset(mts.ur, mts.ir, mts.n_users, mts.n_items, mts.n_ratings, (1, 5), 0,
                               {}, {})
    algo = SVD(n_factors=100, n_epochs=1, random_state=0)
    algo.trainset = ref_ts
    t0 = time.perf_counter()
    algo.sgd(ref_ts)
    t_ref = time.perf_counter() - t0
    t_orc = min(orc.time_svd_epochs(rp, it, rt, mts.n_items, 100, 1) for _ in range(3))
    out["calibration"] = dict(workload="SVD K=100, 1 epoch, synthetic ml-1m KFold(5,rs=0) fold 0",
                              n_ratings=int(mts.n_ratings), reference_seconds=t_ref,
                              oracle_seconds=t_orc,
                              reference_updates_per_s=mts.n_ratings / t_ref,
                              oracle_updates_per_s=mts.n_ratings / t_orc,
                              oracle_over_reference=t_ref / t_orc,
                              host=open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0]
                              .strip(" :\t"))
    print("calibration", out["calibration"])

    np.savez_compressed(os.path.join(HERE, "golden_arrays.npz"), **arrays)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, default=lambda o: o.item() if hasattr(o, "item") else str(o))


if __name__ == "__main__":
    main()
