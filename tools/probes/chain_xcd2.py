"""Probe (GPU box): the product SVD step with the heavy and light launches' XCD masks set apart
(they may overlap): the light epoch + replay keep their XCDs while the heavy chains spread."""
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
    ep, rl = eng._epoch_sq, eng._reduce_log
    for hm, lm in ((0x01, 0xFE), (0x03, 0xFE), (0x03, 0xFC), (0x0F, 0xFE), (0x01, 0xFF)):
        eng.heavy_xcd = hm
        auto = ~hm & 0xFF
        eng._epoch_sq = lambda s, n, w, st, x=0, _lm=lm, _a=auto: ep(s, n, w, st, _lm if x == _a else x)
        eng._reduce_log = lambda lg, p, st, x=0, _lm=lm, _a=auto: rl(lg, p, st, _lm if x == _a else x)
        sec, ph = bench.run_steps(eng, None, 40, 5, torch)
        e = ph["epoch_launches"]["ms_and_ratings"]
        print("%-8s heavy XCDs %#04x light XCDs %#04x: %.4f ms/step, heavy / light epoch %s" %
              (dt, hm, lm, sec / 40 * 1e3, e), flush=True)
