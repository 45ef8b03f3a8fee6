"""Probe (GPU box): the per-rating latency of ONE user's chain, alone on the GPU.  Builds a CSR
holding only the k heaviest users of the ML-1M-shape fold 0 (all 3706 items), runs whole epochs
(epoch kernel + replay / y fold + item fold) and prints us/epoch and ns per rating of the longest
chain, for SVD (log) and SVD++ (atomic, helper waves) in fp32 and fp64.
usage: python tools/chain_alone.py [k ...]"""
import os
import sys
import time

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
order = np.argsort(-deg, kind="stable")
K = 100
for k in [int(x) for x in sys.argv[1:]] or [1]:
    users = np.sort(order[:k])
    lens = deg[users]
    rp_k = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    it_k = np.concatenate([it[rp[x]:rp[x + 1]] for x in users]).astype(np.int32)
    rt_k = np.concatenate([rt[rp[x]:rp[x + 1]] for x in users])
    variants = [("svd", "log", {}), ("svdpp", "atomic", {})]
    if os.environ.get("CHAIN_PP_VARIANTS"):
        variants = [("svdpp", "atomic", {}), ("svdpp", "atomic", {"helpers": False}),
                    ("svdpp", "atomic", {"hot_rows": 0}),
                    ("svdpp", "atomic", {"helpers": False, "hot_rows": 0})]
    for algo, mode, kw in variants:
        for dt in ("float32",) if kw else ("float32", "float64"):
            rng = np.random.RandomState(0)
            eng = MFEngine((rp_k, it_k, rt_k), ts.n_items, K, algo=algo, mode=mode, dtype=dt,
                           hyper=bench.hyper_for(algo, float(ts.global_mean)), **kw)
            eng.set_factors(rng.normal(0, .1, (k, K)), rng.normal(0, .1, (ts.n_items, K)),
                            yj=rng.normal(0, .1, (ts.n_items, K)) if algo == "svdpp" else None)
            eng._prepare(None)
            steps = 30
            sec, _ = bench.run_steps(eng, None, steps, 3, torch, instrument=False)
            us = sec / steps * 1e6
            print(kw, "%-6s %-8s users %4d  max chain %4d  %8.1f us/epoch  %6.1f ns/rating"
                  % (algo, dt, k, lens.max(), us, us * 1e3 / lens.max()), flush=True)
