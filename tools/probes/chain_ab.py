"""Probe (GPU box): the top user's chain in two engines -- (a) a CSR of that user alone, (b) the
full ML-1M-shape CSR with a schedule of only that user -- timed with events around the epoch
kernel (median of 20), fp64 and fp32.  Same user, same items, same kernel."""
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
deg = np.diff(rp)
top = int(np.argmax(deg))
K = 100


def timed(eng, reps=20):
    out = []
    for _ in range(reps + 3):
        ev = {k: torch.cuda.Event(enable_timing=True) for k in ("start", "end")}
        eng.run_chunk(0, events=ev)
        eng.sync_items(None)
        torch.cuda.synchronize()
        out.append(ev["start"].elapsed_time(ev["end"]) * 1e3)
    return float(np.median(out[3:]))


order = np.argsort(-deg, kind="stable")
for dt in ("float64", "float32"):
    rng = np.random.RandomState(0)
    pu, qi = rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K))
    hyper = bench.hyper_for("svd", float(ts.global_mean))
    b = MFEngine((rp, it, rt), ts.n_items, K, hyper=hyper, dtype=dt, heavy=0)
    b.set_factors(pu, qi)
    b._prepare(None)
    full = b.logs[0]["sched"]
    for k in (1, 8, 32, 128, 512):
        b.logs[0]["sched"] = torch.tensor(np.sort(order[:k]), dtype=torch.int32, device="cuda")
        t = timed(b)
        print("%-8s one launch, the top %4d users only: epoch kernel %.1f us (%.1f ns/rating of "
              "the top chain)" % (dt, k, t, t * 1e3 / deg[top]), flush=True)
    ep = b._epoch_sq
    for k, m in ((128, 0x01), (128, 0x03), (32, 0x01), (1, 0x01)):
        b.logs[0]["sched"] = torch.tensor(np.sort(order[:k]), dtype=torch.int32, device="cuda")
        b._epoch_sq = lambda s_, n, w, st, x=0, _m=m: ep(s_, n, n, st, _m)  # one wave per user
        t = timed(b)
        print("%-8s one launch, the top %4d users only, on XCD mask %#04x: epoch kernel %.1f us"
              % (dt, k, m, t), flush=True)
    b._epoch_sq = ep
    b.logs[0]["sched"] = full
    t = timed(b)
    print("%-8s one launch, every user: epoch kernel %.1f us" % (dt, t), flush=True)
    c = MFEngine((rp, it, rt), ts.n_items, K, hyper=hyper, dtype=dt)  # the product (heavy split)
    c.set_factors(pu, qi)
    c._prepare(None)
    t = timed(c)
    print("%-8s product split: heavy launch (128 users, XCD 0) beside the light one: %.1f us"
          % (dt, t), flush=True)
