"""Probe (GPU box): is the SVD++ helper-wave epoch bound by the serialised float atomics on the
most popular items' q rows?  Times the C3 epoch (ML-1M shape, K=100) on the original CSR and on
copies whose top-N items are split into R clone items (each rating of a split item goes to clone
x % R), which divides the atomics per q-row line by R and changes nothing else about the work.
Timing only (the clones change the model).
usage: python tools/svdpp_hot_probe.py [--shape c5 --users N --factors K] [RxN ...]"""
import os
import sys
import json
from types import SimpleNamespace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    import torch
    from surprise_amd.engine import MFEngine
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="ml-1m")
    ap.add_argument("--users", type=int, default=0)
    ap.add_argument("--factors", type=int, default=100)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("specs", nargs="*")
    a = ap.parse_args()
    csr, _, I, n_glob, _ = bench.workload(SimpleNamespace(shape=a.shape, users=a.users), 0, 1)
    row_ptr, items, ratings = csr
    gm = float(ratings.mean())
    cnt = np.bincount(items, minlength=I)
    order = np.argsort(-cnt, kind="stable")
    out = []
    from surprise_amd.engine import default_chunks
    for spec in (a.specs or ["1x0", "4x64", "4x256", "8x64"]):
        R, N = (int(x) for x in spec.split("x"))
        it = np.asarray(items, np.int32).copy()
        n_items = I
        if R > 1 and N > 0:
            clone0 = np.full(I, -1, np.int64)
            clone0[order[:N]] = I + np.arange(N) * (R - 1)  # clones 1..R-1 of item order[j]
            hit = clone0[it] >= 0
            r = np.arange(len(it)) % R
            sel = hit & (r > 0)
            it[sel] = (clone0[it[sel]] + r[sel] - 1).astype(np.int32)
            n_items = I + N * (R - 1)
        K = a.factors
        rng = np.random.RandomState(0)
        pu = rng.normal(0, .1, (len(row_ptr) - 1, K))
        qi = rng.normal(0, .1, (n_items, K))
        yj = rng.normal(0, .1, (n_items, K))
        eng = MFEngine((row_ptr, it, ratings), n_items, K, algo="svdpp",
                       hyper=bench.hyper_for("svdpp", gm), mode="atomic", dtype="float32",
                       n_chunks=default_chunks("svdpp", "atomic", n_glob))
        eng.set_factors(pu, qi, yj=yj)
        eng._prepare(None)
        elapsed, phases = bench.run_steps(eng, None, a.steps, 2, torch, instrument=False)
        top = np.sort(np.bincount(it, minlength=n_items))[::-1][:3].tolist()
        out.append(dict(shape=a.shape, users=len(row_ptr) - 1, R=R, N=N,
                        ms_per_epoch=elapsed / a.steps * 1e3, top_item_counts=top))
        print(json.dumps(out[-1]), flush=True)
        del eng
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
