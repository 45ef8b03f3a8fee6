"""NMF and baseline-ALS epochs on the ML-1M shape: epoch time,
rating-updates/s, and the held-out RMSE next to the fp64 oracle (the reference loop restated).

    python tools/bench_ext.py [--epochs 50] [--factors 15]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--epochs", type=int, default=50)
    p.add_argument("--factors", type=int, default=15)
    p.add_argument("--shape", default="ml-1m")
    a = p.parse_args()
    import torch
    import oracle as orc
    from surprise_amd import Dataset, synthetic
    from surprise_amd.engine import NMFEngine, baseline_als_device
    from surprise_amd.model_selection import KFold

    u, i, r = synthetic.shape(a.shape)
    ts, test = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
    csr, csc = ts.csr(), ts.csc()
    n = int(ts.n_ratings)
    uu = np.array([ts._raw2inner_id_users.get(x, -1) for x in test.uid.tolist()], np.int32)
    ii = np.array([ts._raw2inner_id_items.get(x, -1) for x in test.iid.tolist()], np.int32)
    out = {"shape": a.shape, "train_ratings": n}

    K, E = a.factors, a.epochs
    rng = np.random.RandomState(0)
    pu0 = rng.uniform(0, 1, (ts.n_users, K))
    qi0 = rng.uniform(0, 1, (ts.n_items, K))
    hyper = dict(reg_pu=.06, reg_qi=.06, reg_bu=.02, reg_bi=.02, lr_bu=.005, lr_bi=.005,
                 global_mean=float(ts.global_mean))
    eng = NMFEngine(csr, csc, ts.n_items, K, hyper=hyper)
    eng.set_factors(pu0, qi0)
    eng.epoch()  # warm-up (not counted; restart from the same factors below)
    eng.set_factors(pu0, qi0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(E):
        eng.epoch()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / E
    est, imp = eng.predict(uu, ii, 0.0)
    est = orc.finish_estimates(est, imp, ts.global_mean, 0, (1, 5))
    rmse_gpu = orc.rmse(test.rating, est)
    t = time.perf_counter()
    pu, qi, bu, bi = orc.nmf_sgd(*csr, ts.n_items, K, E, False, ts.global_mean, pu0, qi0)
    cpu_dt = (time.perf_counter() - t) / E
    e2, imp2 = orc.svd_predict(uu, ii, K, False, ts.global_mean, pu, qi, bu, bi)
    e2 = orc.finish_estimates(e2, imp2, ts.global_mean, 0, (1, 5))
    out["nmf"] = {"n_factors": K, "epochs": E, "dtype": "f32", "epoch_ms": dt * 1e3,
                  "updates_per_s": n / dt, "rmse_gpu": rmse_gpu,
                  "rmse_oracle_fp64": orc.rmse(test.rating, e2),
                  "oracle_epoch_ms_1_thread": cpu_dt * 1e3}

    torch.cuda.synchronize()
    t = time.perf_counter()
    bu, bi = baseline_als_device(csr, csc, ts.n_items, ts.global_mean, 10, 15, 10)
    dt = (time.perf_counter() - t) / 10
    bu2, bi2 = orc.baseline_als(*csr, ts.n_items, *csc, ts.global_mean, 10, 15, 10)
    out["baseline_als"] = {"epochs": 10, "dtype": "f64", "epoch_ms_incl_h2d": dt * 1e3,
                           "max_abs_diff_vs_oracle": float(max(np.abs(bu - bu2).max(),
                                                               np.abs(bi - bi2).max()))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
