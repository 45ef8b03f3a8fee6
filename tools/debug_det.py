"""Debug: deterministic kernel vs oracle, one user per launch, tiny data (prints first divergence)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as orc  # noqa: E402
import torch  # noqa: E402
from surprise_amd.engine import MFEngine  # noqa: E402

row_ptr = np.array([0, 1, 2, 3, 5], np.int64)
items = np.array([0, 1, 0, 2, 1], np.int32)
ratings = np.array([5, 3, 1, 4, 2], np.float64)
K = 4
rng = np.random.RandomState(0)
pu0 = rng.normal(0, .1, (4, K))
qi0 = rng.normal(0, .1, (3, K))
gm = float(ratings.mean())
hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02, reg_pu=.02,
             reg_qi=.02, global_mean=gm)
hp = orc.hyper(**{k: v for k, v in hyper.items() if k != "global_mean"})
for dtype in ("float64", "float32"):
    eng = MFEngine((row_ptr, items, ratings), 3, K, hyper=hyper, dtype=dtype, deterministic=True)
    eng.set_factors(pu0, qi0)
    pu, qi, bu, bi = pu0.copy(), qi0.copy(), np.zeros(4), np.zeros(3)
    for u in range(4):
        # oracle: just user u
        rp = np.zeros(5, np.int64)
        rp[u + 1:] = row_ptr[u + 1] - row_ptr[u]
        sl = slice(row_ptr[u], row_ptr[u + 1])
        orc.svd_sgd(rp, items[sl], ratings[sl], 3, K, 1, True, gm, hp, pu, qi, bu, bi)
        eng.sched = [torch.tensor([u], dtype=torch.int32, device="cuda")]
        eng.run_chunk(0)
        f = eng.get_factors()
        d = {k: float(np.abs(f[k] - v).max()) for k, v in dict(pu=pu, qi=qi, bu=bu, bi=bi).items()}
        print(dtype, "after user", u, "items", items[sl], {k: "%.2e" % v for k, v in d.items()})
        if max(d.values()) > 1e-6:
            print(" gpu pu", f["pu"][u], "\n orc pu", pu[u])
            print(" gpu qi", f["qi"], "\n orc qi", qi)
            print(" gpu bu/bi", f["bu"], f["bi"], "\n orc", bu, bi)
            break
