"""CPU experiment (oracle/ only): SVD++ with a q / b LOG for cold items (rows read at the
epoch-chunk start, steps folded per item after the chunk; oracle_svdpp_sgd_stalelog) and live
float-atomic-style updates for the rest, against the reference loop (seq) and against the GPU's
current rule (live: nothing stale), held-out RMSE per epoch.
  ml-1m: BASELINE configs[2] (C3: SVD++ K=100, the bench's ML-1M-shape fold, 1 chunk)
  proxy: tools/c5_merge_proxy.py's C5-shard miniature (K=128, --chunks C epoch-chunks)
cases: seq | live | tT_mM (items with fewer than T training ratings stale, fold merge M; T=0:
every item stale)
usage: python tools/svdpp_stalelog_probe.py ml-1m|proxy CASE [--chunks C] [--epochs E]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import bench
    import oracle as orc
    from make_scale_golden import group_schedule
    p = argparse.ArgumentParser()
    p.add_argument("data")
    p.add_argument("case")
    p.add_argument("--chunks", type=int, default=1)
    p.add_argument("--epochs", type=int, default=20)
    a = p.parse_args()
    if a.data == "ml-1m":
        args = argparse.Namespace(shape="ml-1m", users=0)
        csr, test, n_items, _, _ = bench.workload(args, 0, 1)
        K = 100
        pu, qi, yj = bench.init_tables("ml-1m", 0, len(csr[0]) - 1, n_items, K, True)
    else:
        from c5_merge_proxy import data
        csr, test, n_items = data(8)
        K = 128
        pu, qi, yj = bench.init_tables("c5", 0, len(csr[0]) - 1, n_items, K, True, 0)
    row_ptr, items, ratings = csr
    gm = float(ratings.mean())
    hp = orc.hyper(**{k: v for k, v in bench.hyper_for("svdpp", gm).items()
                      if k != "global_mean"})
    tu, ti, tr = (np.asarray(x) for x in test)
    tu, ti = tu.astype(np.int32), ti.astype(np.int32)
    _, c_of = group_schedule(row_ptr, 1, a.chunks)
    cnt = np.bincount(items, minlength=n_items)
    if a.case in ("seq", "live"):
        stale = np.zeros(n_items, np.int32)
        merge = 3
    else:
        t, m = a.case.split("_")
        T, merge = int(t[1:]), int(m[1:])
        stale = (np.ones(n_items) if T == 0 else cnt < T).astype(np.int32)
    share = float(cnt[stale != 0].sum()) / len(items)
    bu, bi = np.zeros(len(row_ptr) - 1), np.zeros(n_items)
    for e in range(a.epochs):
        t0 = time.time()
        if a.case == "seq":
            pu, qi, yj, bu, bi = orc.svdpp_sgd(row_ptr, items, ratings, n_items, K, 1, gm,
                                               hp, pu, qi, yj, bu, bi, affine=True)
        else:
            pu, qi, yj, bu, bi = orc.svdpp_sgd_stalelog(
                row_ptr, items, ratings, n_items, K, 1, gm, hp, pu, qi, yj, stale, c_of,
                a.chunks, merge=merge, bu=bu, bi=bi)
        est = orc.svdpp_predict(tu, ti, row_ptr, items, K, gm, pu, qi, yj, bu, bi)
        r = orc.rmse(tr, orc.finish_estimates(est, np.zeros(len(tu), bool), gm, 0, (1, 5)))
        print("%s %s c%d (stale share %.3f) epoch %d: %.10f (%.1fs)" % (
            a.data, a.case, a.chunks, share, e + 1, r, time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
