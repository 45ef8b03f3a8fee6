"""Round-5 probe (GPU box): the headline step's join between the light replay (side stream) and
the fold (main stream), and (replay_rows) shorter replay pieces: the heavy replay is bound by its
longest piece's chain of row gathers.  The product step waits on a HIP event (engine join="event", events
"native"); the alternatives are the in-kernel join (join="kernel": the heavy replay's last block
waits for the light replay), torch events, and the fold inside the replays (replay_fold: no
fold launch, no join before it).  ML-1M fold 0, SVD K=100, fp64 and fp32, 60 timed
steps x 3 repeats each (bench.run_steps)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from surprise_amd import Dataset, synthetic  # noqa: E402
from surprise_amd.engine import MFEngine  # noqa: E402
from surprise_amd.model_selection import KFold  # noqa: E402

out = open(sys.argv[1], "w")
u, i, r = synthetic.shape("ml-1m")
ts, _ = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
rp, it, rt = ts.csr()
for dt in ("float64", "float32"):
    for name, kw in (("event (product)", {}), ("kernel join", {"join": "kernel"}),
                     ("torch events", {"events": "torch"}),
                     ("fold in the replays", {"replay_fold": True}),
                     ("replay pieces of 32", {"replay_rows": 32}),
                     ("replay pieces of 16", {"replay_rows": 16})):
        rng = np.random.RandomState(0)
        eng = MFEngine((rp, it, rt), ts.n_items, 100,
                       hyper=bench.hyper_for("svd", float(ts.global_mean)), dtype=dt, **kw)
        eng.set_factors(rng.normal(0, .1, (ts.n_users, 100)), rng.normal(0, .1, (ts.n_items, 100)))
        eng._prepare(None)
        ms = []
        for rep in range(3):
            sec, ph = bench.run_steps(eng, None, 60, 5, torch)
            ms.append(round(sec / 60 * 1e3, 4))
        rec = dict(dtype=dt, join=name, ms_per_step=ms)
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")
        del eng
