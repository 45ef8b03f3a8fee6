"""Probe: host enqueue time of one SVD epoch step (run_chunk + sync_items) vs its GPU time, ML-1M
shape, K=100 -- is the step launch-bound on the host?"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from surprise_amd import Dataset, synthetic  # noqa: E402
from surprise_amd.engine import MFEngine  # noqa: E402
from surprise_amd.model_selection import KFold  # noqa: E402

u, i, r = synthetic.shape("ml-1m")
ts, _ = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
rp, it, rt = ts.csr()
hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02, reg_pu=.02,
             reg_qi=.02, global_mean=float(ts.global_mean))
for heavy in (0, 128):
    eng = MFEngine((rp, it, rt), ts.n_items, 100, hyper=hyper, mode="log", heavy=heavy)
    rng = np.random.RandomState(0)
    eng.set_factors(rng.normal(0, .1, (ts.n_users, 100)), rng.normal(0, .1, (ts.n_items, 100)))
    eng._prepare(None)
    for _ in range(5):
        eng.run_chunk(0)
        eng.sync_items(None)
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        eng.run_chunk(0)
        eng.sync_items(None)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("heavy %3d: host enqueue %.1f us/step, wall %.1f us/step" %
          (heavy, (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6), flush=True)
