"""Scale check on one GPU: BASELINE configs[3]'s shape (SVD K=128, 2M users x 200k items x 100M
ratings; the 4-GPU config run whole on one MI355X) through the array-native path.

Prints one JSON line: epoch time and rating-updates/s of the default "log" schedule, and the
held-out RMSE (1% of the ratings, seed 0) of the GPU fit next to the fp64 sequential oracle
(the reference loop restated, oracle/) trained on the same CSR with the same initial factors.

    python tools/scale_run.py --shape c4 --factors 128 --epochs 5
    python tools/scale_run.py --algo svdpp --shape c5-shard --factors 128 --epochs 3 --no-oracle
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


def log(msg):
    print("[scale_run %7.1fs] %s" % (time.perf_counter() - T0, msg), flush=True)


T0 = time.perf_counter()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shape", default="c4")
    p.add_argument("--factors", type=int, default=128)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--holdout", type=float, default=0.01)
    p.add_argument("--mode", default="auto")
    p.add_argument("--no-oracle", action="store_true")
    p.add_argument("--algo", default="svd", choices=["svd", "svdpp"])
    a = p.parse_args()
    import torch
    from surprise_amd import synthetic
    from surprise_amd.engine import MFEngine

    U, I, N = synthetic.SHAPES[a.shape]
    uid, iid, r = synthetic.shape(a.shape)
    log("generated %d ratings" % len(r))
    rng = np.random.RandomState(0)
    test = rng.random_sample(len(r)) < a.holdout
    tu, ti, tr = uid[~test], iid[~test], r[~test]
    order = np.argsort(tu, kind="stable")  # user-major, file order within a user
    items = np.ascontiguousarray(ti[order])
    ratings = np.ascontiguousarray(tr[order])
    row_ptr = np.zeros(U + 1, np.int64)
    np.cumsum(np.bincount(tu, minlength=U), out=row_ptr[1:])
    del order, tu, ti, tr
    gm = float(ratings.mean())
    K, E = a.factors, a.epochs
    log("train CSR: %d ratings, held out %d" % (len(ratings), int(test.sum())))
    init = np.random.RandomState(0)
    pu0 = init.normal(0, .1, (U, K))
    qi0 = init.normal(0, .1, (I, K))
    pp = a.algo == "svdpp"
    yj0 = init.normal(0, .1, (I, K)) if pp else None
    lr, reg = (.007, .02) if pp else (.005, .02)  # SVDpp / SVD defaults (mf.pyx:398-407, :140-147)
    hyper = dict(lr_bu=lr, lr_bi=lr, lr_pu=lr, lr_qi=lr, lr_yj=lr, reg_bu=reg, reg_bi=reg,
                 reg_pu=reg, reg_qi=reg, reg_yj=reg, global_mean=gm)
    mode = ("atomic" if pp else "log") if a.mode == "auto" else a.mode
    eng = MFEngine((row_ptr, items, ratings), I, K, hyper=hyper, mode=mode, algo=a.algo)
    eng.set_factors(pu0, qi0, yj=yj0)
    torch.cuda.synchronize()
    log("engine ready")
    times = []
    for e in range(E):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for c in range(eng.n_chunks):
            eng.run_chunk(c)
            eng.sync_items(None)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
        log("epoch %d: %.2f ms" % (e, times[-1] * 1e3))
    tu_, ti_ = uid[test], iid[test]
    est, _ = eng.predict(tu_, ti_, gm, imp=eng.user_implicit() if pp else None)
    est = np.clip(est, 1, 5)
    rmse_gpu = float(np.sqrt(np.mean((r[test] - est) ** 2)))
    # a reference point that needs no oracle: the RMSE of the global mean on the held-out set
    out = {"shape": a.shape, "algo": a.algo, "n_users": U, "n_items": I,
           "train_ratings": int(len(ratings)), "n_factors": K, "epochs": E, "mode": mode,
           "rmse_global_mean": float(np.sqrt(np.mean((r[test] - gm) ** 2))),
           "epoch_ms": [t * 1e3 for t in times],
           "updates_per_s": len(ratings) / float(np.median(times)),
           "rmse_gpu": rmse_gpu}
    del eng
    if not a.no_oracle and not pp:
        import oracle as orc
        hp = orc.hyper(**{k: v for k, v in hyper.items() if k != "global_mean"})
        t = time.perf_counter()
        pu, qi, bu, bi = orc.svd_sgd(row_ptr, items, ratings, I, K, E, True, gm, hp, pu0, qi0)
        out["oracle_seconds"] = time.perf_counter() - t
        e_, imp = orc.svd_predict(tu_, ti_, K, True, gm, pu, qi, bu, bi)
        e_ = orc.finish_estimates(e_, imp, gm, 0, (1, 5))
        out["rmse_oracle_fp64"] = orc.rmse(r[test], e_)
        out["delta"] = rmse_gpu - out["rmse_oracle_fp64"]
        log("oracle done")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
