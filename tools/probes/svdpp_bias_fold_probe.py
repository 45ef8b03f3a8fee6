"""CPU experiment (oracle/ only): SVD++ with the item bias stale within an epoch-chunk and folded
per item with recency weights afterwards (oracle_svdpp_sgd_groups_merge(bias_fold=True)) against
the reference loop and against the GPU's current rule (bias steps live), held-out RMSE per epoch.
  ml-1m: BASELINE configs[2] (C3: SVD++ K=100, the bench's ML-1M-shape fold, 1 chunk)
  proxy: tools/c5_merge_proxy.py's C5-shard miniature (K=128), G ranks x C chunks
usage: python tools/svdpp_bias_fold_probe.py ml-1m|proxy [--groups G] [--chunks C]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import bench
    import oracle as orc
    from make_scale_golden import group_schedule
    p = argparse.ArgumentParser()
    p.add_argument("data")
    p.add_argument("--groups", type=int, default=1)
    p.add_argument("--chunks", type=int, default=1)
    p.add_argument("--epochs", type=int, default=20)
    p.add_argument("--case", default="all")
    a = p.parse_args()
    if a.data == "ml-1m":
        args = argparse.Namespace(shape="ml-1m", users=0)
        csr, test, n_items, _, _ = bench.workload(args, 0, 1)
        K = 100
        pu0, qi0, yj0 = bench.init_tables("ml-1m", 0, len(csr[0]) - 1, n_items, K, True)
    else:
        from c5_merge_proxy import data
        csr, test, n_items = data(8)
        K = 128
        pu0, qi0, yj0 = bench.init_tables("c5", 0, len(csr[0]) - 1, n_items, K, True, 0)
    row_ptr, items, ratings = csr
    gm = float(ratings.mean())
    hp = orc.hyper(**{k: v for k, v in bench.hyper_for("svdpp", gm).items()
                      if k != "global_mean"})
    tu, ti, tr = (np.asarray(x) for x in test)
    tu, ti = tu.astype(np.int32), ti.astype(np.int32)
    g_of, c_of = group_schedule(row_ptr, a.groups, a.chunks)
    cases = ["seq", "live", "fold"] if a.case == "all" else [a.case]
    for case in cases:
        pu, qi, yj = pu0.copy(), qi0.copy(), yj0.copy()
        bu, bi = np.zeros(len(row_ptr) - 1), np.zeros(n_items)
        for e in range(a.epochs):
            t0 = time.time()
            if case == "seq":
                pu, qi, yj, bu, bi = orc.svdpp_sgd(row_ptr, items, ratings, n_items, K, 1, gm,
                                                   hp, pu, qi, yj, bu, bi, affine=True)
            else:
                pu, qi, yj, bu, bi = orc.svdpp_sgd_groups_merge(
                    row_ptr, items, ratings, n_items, K, 1, gm, hp, pu, qi, yj, g_of, a.groups,
                    c_of, a.chunks, merge=3, merge_y=4, bu=bu, bi=bi, bias_fold=case == "fold")
            est = orc.svdpp_predict(tu, ti, row_ptr, items, K, gm, pu, qi, yj, bu, bi)
            r = orc.rmse(tr, orc.finish_estimates(est, np.zeros(len(tu), bool), gm, 0, (1, 5)))
            print("%s %s g%d c%d epoch %d: %.10f (%.1fs)" % (a.data, case, a.groups, a.chunks,
                                                          e + 1, r, time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
