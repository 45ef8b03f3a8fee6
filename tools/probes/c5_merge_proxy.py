"""CPU experiment (oracle/ only, build container): which multi-rank SVD++ item merge holds the
sequential reference on a miniature of the C5 shard.

The miniature keeps the C5 shard's per-item and per-user rating counts (125 ratings per item per
epoch, 100 per user, Zipf items, lognormal users) at 1/8 of its users and items: 156,250 users x
125,000 items x 15.6M ratings, SVD++ K=128, bench.py's generator / initial factors / hyper-
parameters.  Each case prints its held-out RMSE after every epoch:
  seq           oracle_svdpp_sgd_affine: the reference loop (exact per-user form)
  gG_cC_mM      oracle_svdpp_sgd_groups_merge: G ranks (dist.shard_users) x C epoch-chunks
                (dist.chunk_users inside a rank), q / b merged by rule M (0 SUM, 2 count-aware,
                3 affine composition in rank order), y composed in rank order (merge_y 4)
usage: python tools/c5_merge_proxy.py CASE [CASE ...] [--epochs 20] [--scale 8]
"""
import argparse
import json
import os
import sys
import time
from multiprocessing import Process

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def data(scale):
    from surprise_amd import synthetic
    U, I = 1_250_000 // scale, 1_000_000 // scale
    N = U * 100
    truth = synthetic.sharded_truth(U, I, N)
    csr, test = synthetic.sharded_rows(truth, 0, U, threads=2)
    return csr, test, I


def run(case, epochs, scale, out_dir):
    import bench
    import oracle as orc
    from make_scale_golden import group_schedule
    csr, test, n_items = data(scale)
    row_ptr, items, ratings = csr
    gm = float(ratings.mean())
    K = 128
    pu, qi, yj = bench.init_tables("c5", 0, len(row_ptr) - 1, n_items, K, True, 0)
    hp = orc.hyper(**{k: v for k, v in bench.hyper_for("svdpp", gm).items()
                      if k != "global_mean"})
    tu, ti, tr = (np.asarray(x) for x in test)
    tu, ti = tu.astype(np.int32), ti.astype(np.int32)
    bu, bi = np.zeros(len(row_ptr) - 1), np.zeros(n_items)
    if case != "seq":
        g, c, m = (int(x[1:]) for x in case.split("_"))
        g_of, c_of = group_schedule(row_ptr, g, c)
    curve = []
    for e in range(epochs):
        t0 = time.time()
        if case == "seq":
            pu, qi, yj, bu, bi = orc.svdpp_sgd(row_ptr, items, ratings, n_items, K, 1, gm, hp,
                                               pu, qi, yj, bu, bi, affine=True)
        else:
            pu, qi, yj, bu, bi = orc.svdpp_sgd_groups_merge(
                row_ptr, items, ratings, n_items, K, 1, gm, hp, pu, qi, yj, g_of, g, c_of, c,
                merge=m, merge_y=4, bu=bu, bi=bi)
        est = orc.svdpp_predict(tu, ti, row_ptr, items, K, gm, pu, qi, yj, bu, bi)
        curve.append(orc.rmse(tr, orc.finish_estimates(est, np.zeros(len(tu), bool), gm, 0,
                                                       (1, 5))))
        print("%s epoch %d: %.10f (%.0fs)" % (case, e + 1, curve[-1], time.time() - t0),
              flush=True)
    with open(os.path.join(out_dir, "%s.json" % case), "w") as f:
        json.dump({"case": case, "scale": scale, "rmse_by_epoch": curve}, f)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("cases", nargs="+")
    p.add_argument("--epochs", type=int, default=20)
    p.add_argument("--scale", type=int, default=8)
    p.add_argument("--out", default="/tmp/c5_merge_proxy")
    a = p.parse_args()
    os.makedirs(a.out, exist_ok=True)
    procs = [Process(target=run, args=(c, a.epochs, a.scale, a.out)) for c in a.cases]
    for x in procs:
        x.start()
    for x in procs:
        x.join()


if __name__ == "__main__":
    main()
