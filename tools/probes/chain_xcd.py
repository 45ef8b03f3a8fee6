"""Probe (GPU box): the product SVD step (heavy split) with the heavy launch's XCD mask varied --
XCD 0 (default), XCDs 0-1, 0-3, or no masks at all -- step time and the heavy launch's span."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from surprise_amd import Dataset, synthetic  # noqa: E402
from surprise_amd.engine import MFEngine  # noqa: E402
from surprise_amd.model_selection import KFold  # noqa: E402

u, i, r = synthetic.shape("ml-1m")
ts, _ = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
rp, it, rt = ts.csr()
K = 100
for dt in ("float64", "float32"):
    rng = np.random.RandomState(0)
    eng = MFEngine((rp, it, rt), ts.n_items, K, hyper=bench.hyper_for("svd", float(ts.global_mean)),
                   dtype=dt)
    eng.set_factors(rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K)))
    eng._prepare(None)
    for mask in (0x01, 0x03, 0x0F, 0x00):
        eng.heavy_xcd = mask
        sec, ph = bench.run_steps(eng, None, 40, 5, torch)
        e = ph["epoch_launches"]["ms_and_ratings"]
        print("%-8s heavy XCD mask %#04x: %.4f ms/step, heavy / light epoch %s" %
              (dt, mask, sec / 40 * 1e3, e), flush=True)
