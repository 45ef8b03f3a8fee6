"""Round-5 probe (GPU box): one SVD++ user chain alone -- ns per rating of the q-log epoch kernel
and of the helper-wave (atomic) launch, K=128 fp32 (C5's layout) and K=100 fp64, over a 1M-item
table; the SVD checkpoint kernel's chain beside it.  One JSON line per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402


def main():
    import torch
    from surprise_amd.engine import MFEngine
    out = open(sys.argv[1], "w") if len(sys.argv) > 1 else None
    n, n_items = 200_000, 1_000_000
    rng = np.random.RandomState(0)
    items = rng.choice(n_items, n, replace=False).astype(np.int32)
    ratings = rng.randint(1, 6, n).astype(np.float64)
    row_ptr = np.array([0, n], np.int64)
    hyper = dict(lr_bu=.007, lr_bi=.007, lr_pu=.007, lr_qi=.007, lr_yj=.007, reg_bu=.02,
                 reg_bi=.02, reg_pu=.02, reg_qi=.02, reg_yj=.02, global_mean=3.0)
    cases = [("svdpp", 128, "float32", dict(qlog=True)), ("svdpp", 128, "float32", dict(qlog=False)),
             ("svdpp", 100, "float64", dict(qlog=True)), ("svdpp", 100, "float64", dict(qlog=False)),
             ("svd", 128, "float32", dict(mode="log")), ("svd", 100, "float64", dict(mode="log"))]
    for algo, K, dt, kw in cases:
        eng = MFEngine((row_ptr, items, ratings), n_items, K, algo=algo, hyper=hyper, dtype=dt,
                       **kw)
        eng.set_factors(rng.normal(0, .1, (1, K)), rng.normal(0, .1, (n_items, K)),
                        yj=rng.normal(0, .1, (n_items, K)) if algo == "svdpp" else None)
        eng.run_epochs(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run_epochs(3)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 3 * 1e3
        r = dict(algo=algo, K=K, dtype=dt, opts={k: str(v) for k, v in kw.items()},
                 qlog=bool(getattr(eng, "qlog_pp", False)), hx=bool(getattr(eng, "hx", False)),
                 ratings=n, ms_per_epoch=ms, ns_per_rating=ms * 1e6 / n)
        print(json.dumps(r), flush=True)
        if out:
            out.write(json.dumps(r) + "\n")
            out.flush()
        del eng


if __name__ == "__main__":
    main()
