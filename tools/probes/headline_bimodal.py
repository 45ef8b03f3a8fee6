"""Round-5 probe (GPU box): the headline engine in fp32 sometimes runs a whole instance at ~0.29
ms per step instead of ~0.166 (profiles/r5pr_join.jsonl, r5rf_replay_fold.jsonl).  Builds 10
engines in a row, each after a dummy allocation of a different size (the caching allocator then
places the engine's buffers elsewhere), and records ms per step with the device addresses of the
engine's main buffers (mod 2 MiB / 256 MiB) and its launch decisions.  argv[2]: the engine's
side-stream policy (engine.SIDE_STREAM_POLICY), run in a fresh process per policy."""
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

import surprise_amd.engine as E  # noqa: E402
if len(sys.argv) > 2:
    E.SIDE_STREAM_POLICY = sys.argv[2]
out = open(sys.argv[1], "a")
u, i, r = synthetic.shape("ml-1m")
ts, _ = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
rp, it, rt = ts.csr()
pads = []
for n in range(10):
    pads.append(torch.empty((n * 37 + 1) * 1 << 20, dtype=torch.uint8, device="cuda"))
    dt = "float32" if n % 5 else "float64"
    rng = np.random.RandomState(0)
    eng = MFEngine((rp, it, rt), ts.n_items, 100,
                   hyper=bench.hyper_for("svd", float(ts.global_mean)), dtype=dt)
    eng.set_factors(rng.normal(0, .1, (ts.n_users, 100)), rng.normal(0, .1, (ts.n_items, 100)))
    eng._prepare(None)
    ms = []
    for rep in range(2):
        sec, ph = bench.run_steps(eng, None, 40, 5, torch)
        ms.append(round(sec / 40 * 1e3, 4))
    addr = {k: getattr(eng, k).data_ptr() for k in ("qb", "pu", "sums", "user_sq")
            if getattr(eng, k, None) is not None}
    addr["qlog"] = int(eng._qlog_base)
    addr["elog"] = int(eng._elog_base)
    rec = dict(policy=E.SIDE_STREAM_POLICY, n=n, dtype=dt, ms_per_step=ms, heavy_xcd=int(eng.heavy_xcd),
               epoch_launches=ph.get("epoch_launches", {}).get("ms_and_ratings"),
               replay_ms=ph.get("replay_ms"),
               mod2m={k: v % (2 << 20) for k, v in addr.items()},
               mod256m={k: v % (256 << 20) for k, v in addr.items()})
    print(json.dumps(rec), flush=True)
    out.write(json.dumps(rec) + "\n")
    del eng
