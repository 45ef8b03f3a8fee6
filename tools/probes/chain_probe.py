"""Probe: epoch-kernel time for subsets of the ML-1M-shape schedule (is the epoch bound by the
heaviest users' dependent chains or by throughput?).  Prints one line per subset."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from surprise_amd import Dataset, synthetic  # noqa: E402
from surprise_amd.engine import MFEngine  # noqa: E402
from surprise_amd.model_selection import KFold  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "log"
algo = os.environ.get("PROBE_ALGO", "svd")
K = int(sys.argv[2]) if len(sys.argv) > 2 else 100
u, i, r = synthetic.shape("ml-1m")
ts, _ = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
rp, it, rt = ts.csr()
hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02, reg_pu=.02,
             reg_qi=.02, global_mean=float(ts.global_mean))
eng = MFEngine((rp, it, rt), ts.n_items, K, hyper=hyper, mode=mode, algo=algo, heavy=0,
               dtype=os.environ.get("PROBE_DTYPE", "float32"))
rng = np.random.RandomState(0)
eng.set_factors(rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K)),
                yj=rng.normal(0, .1, (ts.n_items, K)) if algo == "svdpp" else None)
full = eng.sched[0].clone()
W0 = eng.n_waves  # the engine's default wave count (SVD++: capped per CU)
deg = np.diff(rp)
order = full.cpu().numpy()


def t_sched(s, n_waves=None, reps=10):
    eng.sched[0] = torch.from_numpy(np.ascontiguousarray(s, np.int32)).cuda()
    eng.n_waves = W0 if n_waves is None else n_waves
    ts_ = []
    for _ in range(reps + 2):
        ev = {k: torch.cuda.Event(enable_timing=True) for k in ("start", "end")}
        eng.run_chunk(0, events=ev)
        eng.sync_items(None)
        torch.cuda.synchronize()
        ts_.append(ev["start"].elapsed_time(ev["end"]))
    return float(np.median(ts_[2:])) * 1e3


print("algo", algo, "mode", mode, "K", K, "max deg", deg.max(), "ratings", deg.sum())
cases = [("full", order, None), ("top1", order[:1], None), ("top16", order[:16], None),
         ("top256", order[:256], None), ("top1024", order[:1024], None),
         ("drop-top64", order[64:], None), ("drop-top256", order[256:], None),
         ("drop-top1024", order[1024:], None),
         ("full-2048waves", order, 2048), ("full-8192waves", order, 8192)]
if len(sys.argv) > 3 and sys.argv[3] == "waves":
    cases = [("full-%dwaves" % w, order, w) for w in (2048, 4096, 6040, 8192, 12288, 16384)]
if len(sys.argv) > 3 and sys.argv[3] == "chain":
    cases = [("full", order, None), ("top1", order[:1], None), ("top8", order[:8], None),
             ("top128", order[:128], None), ("top128-512waves", order[:128], 512)]
if len(sys.argv) > 3 and sys.argv[3] == "fast":
    cases = [c for c in cases if c[0] in ("full", "top1", "drop-top64")]
for name, s, nw in cases:
    us = t_sched(s, nw)
    n = int(deg[s].sum())
    print("%-16s users %5d ratings %7d max %4d  %8.1f us  %.1f ns/rating(max chain)  %.2f Gupd/s"
          % (name, len(s), n, deg[s].max(), us, us * 1e3 / deg[s].max(), n / us / 1e3), flush=True)
