"""Probe (GPU box): what makes the heavy launch of the product SVD step (128 users on XCD 0) take
~245 us beside the light users when its 128 chains alone take ~190: the product step, then the
same with the light group's epoch kernel or its replay left out (timing only)."""
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
for dt in ("float64", "float32"):
    rng = np.random.RandomState(0)
    eng = MFEngine((rp, it, rt), ts.n_items, 100, hyper=bench.hyper_for("svd", float(ts.global_mean)),
                   dtype=dt)
    eng.set_factors(rng.normal(0, .1, (ts.n_users, 100)), rng.normal(0, .1, (ts.n_items, 100)))
    eng._prepare(None)
    ep, rl = eng._epoch_sq, eng._reduce_log
    light = (~eng.heavy_xcd) & 0xFF
    cases = {
        "product": (ep, rl),
        "no light epoch": (lambda s_, n, w, st, x=0: None if x == light else ep(s_, n, w, st, x), rl),
        "no light replay": (ep, lambda lg, p, st, x=0: None if x == light else rl(lg, p, st, x)),
        "neither": (lambda s_, n, w, st, x=0: None if x == light else ep(s_, n, w, st, x),
                    lambda lg, p, st, x=0: None if x == light else rl(lg, p, st, x)),
    }
    for name, (e, r_) in cases.items():
        eng._epoch_sq, eng._reduce_log = e, r_
        sec, ph = bench.run_steps(eng, None, 40, 5, torch)
        print("%-8s %-16s %.4f ms/step, heavy / light epoch %s, main-stream replay %.4f" % (
            dt, name, sec / 40 * 1e3, ph["epoch_launches"]["ms_and_ratings"], ph["replay_ms"]),
            flush=True)
    del eng
