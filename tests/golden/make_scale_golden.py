"""Generate tests/golden/scale_golden.json: held-out RMSE of the fp64 sequential oracle on
bench.py's own C4 / C5-shard workloads (TEST INFRASTRUCTURE; run in the build container, never
on the GPU box).

  c4        BASELINE configs[3]'s shape (2M users x 200k items x 100M ratings, 1% held out),
            SVD K=128, the reference loop restated (oracle_svd_sgd <- mf.pyx:241-262)
  c5shard   the first 1.25M users of configs[4]'s shape (every item: 1M; one of 8 ranks' share),
            SVD++ K=128 in the exact per-user form (oracle_svdpp_sgd_affine <- mf.pyx:463-498)
  c5_u60000 the first 60k users of configs[4]'s shape, the same oracle: the miniature on which the
            long-chain dealing of dist.chunk_users fires at 8 epoch-chunks
  c5at8_cN_mM  the same 1.25M users in C5@8's multi-rank schedule: split 8 ways by
            dist.shard_users (bench.py --gpus 8), each rank's users dealt into N epoch-chunks by
            dist.chunk_users, the ranks' q / b deltas merged by rule M (3: carried through the
            later ranks' steps -- the GPU's MF_MERGE_RECENCY; 2: round 3's count-aware rule) and
            their y maps composed in rank order (oracle_svdpp_sgd_groups_merge(merge=M,
            merge_y=4)).  N = 2 puts 625k users (78k per rank) in a chunk: C5@8's chunk at 16
            chunks per epoch over 10M users

Same CSR, held-out triples, initial factors (init_tables), global mean and hyper-parameters as
`bench.py --shape c4` / `--shape c5 --users 1250000` (imported from bench.py, not re-stated).
The held-out RMSE is recorded after every epoch up to --epochs, so a GPU test can hold any
E <= epochs to the reference's value; estimates are clipped to [1, 5] like bench.rmse_leg.

usage: python tests/golden/make_scale_golden.py {c4|c5shard|c5_u60000|c5at8_cN_mM} [--epochs 20]
(each case merges its entry into scale_golden.json; c4 ~25 min, c5shard ~1 h on one core)
"""
import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bench  # noqa: E402
import oracle as orc  # noqa: E402

OUT = os.path.join(HERE, "scale_golden.json")
CASES = {"c4": dict(shape="c4", users=0, algo="svd", K=128),
         "c5shard": dict(shape="c5", users=1_250_000, algo="svdpp", K=128),
         # the C5 miniature on which dist.chunk_users' long-chain dealing fires: the first 60k
         # users at 8 epoch-chunks put 8 users of > 1/256 of a chunk's ratings into chunk 0
         # (bench.py --shape c5 --users 60000 --chunks 8), as the full C5's 9 long users at 125
         "c5_u60000": dict(shape="c5", users=60_000, algo="svdpp", K=128)}
for _n in (2, 4, 8):
    for _m in (2, 3):  # the q / b merge: 2 count-aware (round 3), 3 rank-order composition
        CASES["c5at8_c%d_m%d" % (_n, _m)] = dict(shape="c5", users=1_250_000, algo="svdpp",
                                                 K=128, groups=8, chunks=_n, merge=_m)


def group_schedule(row_ptr, groups, chunks):
    """(group_of_user, chunk_of_user) of bench.py --gpus `groups` --chunks `chunks`: contiguous
    user ranges of equal rating count (dist.shard_users), each rank's users dealt into its
    epoch-chunks by dist.chunk_users on rank-local ids (MFEngine's chunking)."""
    from surprise_amd.dist import chunk_users, shard_users
    n = len(row_ptr) - 1
    b = shard_users(row_ptr, groups)
    g_of = np.zeros(n, np.int32)
    c_of = np.zeros(n, np.int32)
    for g in range(groups):
        lo, hi = int(b[g]), int(b[g + 1])
        g_of[lo:hi] = g
        loc = np.asarray(row_ptr[lo:hi + 1], np.int64) - int(row_ptr[lo])
        for c, us in enumerate(chunk_users(np.arange(hi - lo), loc, chunks)):
            c_of[lo + np.asarray(us, np.int64)] = c
    return g_of, c_of


def main():
    p = argparse.ArgumentParser()
    p.add_argument("case", choices=sorted(CASES))
    p.add_argument("--epochs", type=int, default=20)
    a = p.parse_args()
    c = CASES[a.case]
    args = SimpleNamespace(shape=c["shape"], users=c["users"])
    t0 = time.time()
    csr, test, n_items, n_users, desc = bench.workload(args, 0, 1)
    row_ptr, items, ratings = csr
    gm = float(ratings.sum()) / len(ratings)
    K, svdpp = c["K"], c["algo"] == "svdpp"
    pu, qi, yj = bench.init_tables(c["shape"], 0, len(row_ptr) - 1, n_items, K, svdpp, 0)
    h = bench.hyper_for(c["algo"], gm)
    hp = orc.hyper(**{k: v for k, v in h.items() if k != "global_mean"})
    tu, ti, tr = (np.asarray(x) for x in test)
    tu, ti = tu.astype(np.int32), ti.astype(np.int32)
    print("%s: %s (%.0fs)" % (a.case, desc, time.time() - t0), flush=True)
    bu, bi = np.zeros(len(row_ptr) - 1), np.zeros(n_items)
    curve, secs = [], []
    groups = c.get("groups")
    if groups:
        g_of, c_of = group_schedule(row_ptr, groups, c["chunks"])
    for e in range(a.epochs):
        t1 = time.time()
        if groups:
            pu, qi, yj, bu, bi = orc.svdpp_sgd_groups_merge(
                row_ptr, items, ratings, n_items, K, 1, gm, hp, pu, qi, yj, g_of, groups, c_of,
                c["chunks"], merge=c["merge"], merge_y=4, bu=bu, bi=bi)
            est = orc.svdpp_predict(tu, ti, row_ptr, items, K, gm, pu, qi, yj, bu, bi)
            imp = np.zeros(len(tu), bool)
        elif svdpp:
            pu, qi, yj, bu, bi = orc.svdpp_sgd(row_ptr, items, ratings, n_items, K, 1, gm, hp,
                                               pu, qi, yj, bu, bi, affine=True)
            est = orc.svdpp_predict(tu, ti, row_ptr, items, K, gm, pu, qi, yj, bu, bi)
            imp = np.zeros(len(tu), bool)
        else:
            pu, qi, bu, bi = orc.svd_sgd(row_ptr, items, ratings, n_items, K, 1, True, gm, hp,
                                         pu, qi, bu, bi)
            est, imp = orc.svd_predict(tu, ti, K, True, gm, pu, qi, bu, bi)
        secs.append(time.time() - t1)
        curve.append(orc.rmse(tr, orc.finish_estimates(est, imp, gm, 0, (1, 5))))
        print("  epoch %d: held-out RMSE %.10f (%.0fs)" % (e + 1, curve[-1], secs[-1]), flush=True)
    entry = {
        "workload": desc, "algo": c["algo"], "n_factors": K, "shape": c["shape"],
        "users": c["users"] or None, "train_ratings": int(len(ratings)),
        "held_out": int(len(tr)), "n_items": int(n_items), "global_mean": gm,
        "data_fingerprint": bench.data_fingerprint(csr, (tu, ti, tr)),
        "rmse_by_epoch": curve,
        "global_mean_rmse": orc.rmse(tr, np.full(len(tr), gm)),
        "oracle": (("oracle_svdpp_sgd_groups_merge(merge=%d, merge_y=4): %d ranks x %d epoch-"
                    "chunks, per-user affine form inside a rank" % (c.get("merge"), groups,
                                                                   c["chunks"]))
                   if groups else "oracle_svdpp_sgd_affine (mf.pyx:463-498)" if svdpp
                   else "oracle_svd_sgd (mf.pyx:241-262)") + ", fp64, one host thread",
        "oracle_seconds_per_epoch": float(np.mean(secs)),
        "generator": "tests/golden/make_scale_golden.py %s --epochs %d" % (a.case, a.epochs),
    }
    import fcntl
    with open(OUT + ".lock", "w") as lk:  # (the cases may run concurrently)
        fcntl.flock(lk, fcntl.LOCK_EX)
        data = json.load(open(OUT)) if os.path.exists(OUT) else {}
        data[a.case] = entry
        with open(OUT, "w") as f:
            json.dump(data, f, indent=1)
    print("wrote %s[%s]" % (OUT, a.case))


if __name__ == "__main__":
    main()
