"""Round-5 probe (GPU box): is C3 (ML-1M fold, SVD++ K=100 fp32, one chunk, the helper-wave
launch) bound by its heaviest user's chain?  One epoch of the whole fold vs the same engine on the
heaviest user alone (same hyper-parameters, same launch kind), and vs the 8 / 64 heaviest."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402


def main():
    import torch
    from surprise_amd.engine import MFEngine
    from test_gpu_parity import _synthetic_fold
    out = open(sys.argv[1], "w")
    ts, _ = _synthetic_fold("ml-1m")
    row_ptr, items, ratings = ts.csr()
    deg = np.diff(row_ptr)
    order = np.argsort(-deg, kind="stable")
    hyper = dict(lr_bu=.007, lr_bi=.007, lr_pu=.007, lr_qi=.007, lr_yj=.007, reg_bu=.02,
                 reg_bi=.02, reg_pu=.02, reg_qi=.02, reg_yj=.02, global_mean=float(ts.global_mean))
    K = 100
    rng = np.random.RandomState(0)
    for dt in ("float32", "float64"):
        for top in (0, 1, 8, 64):
            if top:
                us = np.sort(order[:top])
                rp = np.concatenate([[0], np.cumsum(deg[us])]).astype(np.int64)
                it = np.concatenate([items[row_ptr[u]:row_ptr[u + 1]] for u in us])
                rt = np.concatenate([ratings[row_ptr[u]:row_ptr[u + 1]] for u in us])
                csr = (rp, it, rt)
            else:
                csr = (row_ptr, items, ratings)
            n_u = len(csr[0]) - 1
            eng = MFEngine(csr, ts.n_items, K, algo="svdpp", hyper=hyper, dtype=dt, mode="atomic")
            eng.set_factors(rng.normal(0, .1, (n_u, K)), rng.normal(0, .1, (ts.n_items, K)),
                            yj=rng.normal(0, .1, (ts.n_items, K)))
            eng.run_epochs(2)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run_epochs(10)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 10 * 1e3
            r = dict(dtype=dt, top_users=top or "all", users=n_u, ratings=int(csr[0][-1]),
                     max_degree=int(np.diff(csr[0]).max()), hx=bool(eng.hx),
                     helpers=int(getattr(eng, "hx_helpers", 0)), ms_per_epoch=ms)
            print(json.dumps(r), flush=True)
            out.write(json.dumps(r) + "\n")
            del eng


if __name__ == "__main__":
    main()
