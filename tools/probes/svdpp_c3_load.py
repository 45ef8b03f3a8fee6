"""Round-5 probe (GPU box): what stretches C3's chains under full load?  C3 (ML-1M fold, SVD++
K=100 fp32, one chunk, the helper-wave launch) runs at ~0.57 ms per epoch while its heaviest user
alone takes ~0.32 ms, though LPT dealing (engine.chain_schedule) gives no chain much more work
than that user.  Sweeps, one engine each, fp32:
  * load: the heaviest 1 / 512 / 1536 / 3000 users and all 6040 (the longest chain stays ~1.8k
    ratings; more chains run beside it);
  * atomics: no hot-row replicas; the hybrid launch (cold share 0.5, half the ratings' atomics
    gone);
  * launch shape: 4 chains per CU; one helper per chain.
Each line: ms per epoch, the longest chain's ratings (chain_schedule's dealing) and ns per
rating of that chain."""
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
    cases = [("all", None, {}), ("top1", 1, {}), ("top512", 512, {}), ("top1536", 1536, {}),
             ("top3000", 3000, {}), ("all_no_replicas", None, {"hot_rows": 0}),
             ("all_cold0.5", None, {"cold_share": 0.5, "qlog": False}),
             ("top1_cold0.5", 1, {"cold_share": 0.5, "qlog": False}),
             ("all_4chains_per_cu", None, {"hx_chains_per_cu": 4}),
             ("all_one_helper", None, {"helpers": 1})]
    for name, top, kw in cases:
        if top:
            us = np.sort(order[:top])
            rp = np.concatenate([[0], np.cumsum(deg[us])]).astype(np.int64)
            it = np.concatenate([items[row_ptr[u]:row_ptr[u + 1]] for u in us])
            rt = np.concatenate([ratings[row_ptr[u]:row_ptr[u + 1]] for u in us])
            csr = (rp, it, rt)
        else:
            csr = (row_ptr, items, ratings)
        n_u = len(csr[0]) - 1
        try:
            eng = MFEngine(csr, ts.n_items, K, algo="svdpp", hyper=hyper, dtype="float32",
                           mode="atomic", **kw)
        except Exception as e:  # (a shape the engine refuses: recorded, not fatal)
            r = dict(case=name, error=repr(e)[:200])
            print(json.dumps(r), flush=True)
            out.write(json.dumps(r) + "\n")
            continue
        eng.set_factors(rng.normal(0, .1, (n_u, K)), rng.normal(0, .1, (ts.n_items, K)),
                        yj=rng.normal(0, .1, (ts.n_items, K)))
        eng.run_epochs(2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run_epochs(10)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 10 * 1e3
        longest = None
        if getattr(eng, "hx_sched", None):
            s = eng.hx_sched[0].cpu().numpy()
            n_ch = int(getattr(eng, "hx_chains", 0) or 0)
            if n_ch > 0 and len(s) % n_ch == 0:
                lay = s.reshape(-1, n_ch)
                d = np.diff(np.asarray(csr[0], np.int64))
                longest = int(max(d[lay[:, c][lay[:, c] >= 0]].sum() for c in range(n_ch)))
        r = dict(case=name, users=n_u, ratings=int(csr[0][-1]), hx=bool(eng.hx),
                 helpers=int(getattr(eng, "hx_helpers", 0)), chains=int(getattr(eng, "hx_chains", 0) or 0),
                 mix=bool(getattr(eng, "mix", None)), ms_per_epoch=round(ms, 4),
                 longest_chain_ratings=longest,
                 ns_per_rating_longest=round(ms * 1e6 / longest, 1) if longest else None)
        print(json.dumps(r), flush=True)
        out.write(json.dumps(r) + "\n")
        del eng


if __name__ == "__main__":
    main()
