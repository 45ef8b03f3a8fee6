"""Experiment: held-out RMSE delta vs the fp64 sequential oracle and epoch time, per item-side
schedule (mode) and concurrency (n_waves).  Used to pick the product defaults."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402
from surprise_amd import SVD, SVDpp, Dataset, Reader, accuracy, synthetic  # noqa: E402
from surprise_amd.model_selection import KFold, PredefinedKFold  # noqa: E402
from test_oracle_golden import _oracle_test_rmse, run_oracle  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")


def u1():
    data = Dataset.load_from_folds([(os.path.join(G, "u1_ml100k_train"),
                                     os.path.join(G, "u1_ml100k_test"))], Reader("ml-100k"))
    return next(PredefinedKFold().split(data))


def synth(name):
    u, i, r = synthetic.shape(name)
    return next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))


def oracle_rmse(algo, params, ts, test, affine=False):
    rp, it, rt = ts.csr()
    P, f = run_oracle(algo, params, rp, it, rt, ts.n_items, ts.global_mean, affine=affine)
    return _oracle_test_rmse(P, f, algo, ts, list(test))[1]


def xcc_histogram(n_blocks=4096):
    import ctypes
    from surprise_amd import _lib
    out = torch.zeros(n_blocks, dtype=torch.int32, device="cuda")
    _lib.call("mf_selftest_xcc", ctypes.c_void_p(out.data_ptr()), n_blocks, None)
    torch.cuda.synchronize()
    ids = out.cpu().numpy()
    print("xcc ids of blocks 0..15:", ids[:16].tolist(), "histogram:",
          np.bincount(ids, minlength=8).tolist(), flush=True)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    xcc_histogram()
    rows = []
    sets = []
    if which in ("all", "u1"):
        sets.append(("u1", u1(), [("SVD", dict(n_factors=20, n_epochs=5, random_state=0)),
                                  ("SVD", dict(n_factors=100, n_epochs=20, random_state=0)),
                                  ("SVD", dict(n_factors=100, n_epochs=20, biased=False,
                                               random_state=0)),
                                  ("SVDpp", dict(n_factors=20, n_epochs=20, random_state=0))]))
    if which in ("all", "ml1m"):
        sets.append(("ml-1m", synth("ml-1m"), [("SVD", dict(n_factors=100, n_epochs=20,
                                                            random_state=0)),
                                               ("SVDpp", dict(n_factors=100, n_epochs=5,
                                                              random_state=0))]))
    for dname, (ts, test), cases in sets:
        for algo, params in cases:
            ref = oracle_rmse(algo, params, ts, test, affine=(algo == "SVDpp"))
            for mode, nw, ch in (("log", 0, 1), ("log", 0, 4), ("atomic", 0, 1),
                                 ("plain", 0, 1)):
                    if nw and nw > ts.n_users:
                        continue
                    klass = SVD if algo == "SVD" else SVDpp
                    m = klass(**params, mode=mode, n_waves=nw, chunks_per_epoch=ch)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    m.fit(ts)
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                    got = accuracy.rmse(m.test(test), verbose=False)
                    rec = dict(data=dname, algo=algo, params=params, mode=mode, n_waves=nw, chunks=ch,
                               rmse=got, ref=ref, delta=got - ref, fit_s=dt)
                    rows.append(rec)
                    print(json.dumps(rec), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "exp_modes_%s.json" % which), "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
