"""One process of bench.py's all-core CPU baseline (TEST / MEASUREMENT INFRASTRUCTURE ONLY).

Pins itself to one host core (in-process, os.sched_setaffinity: no re-exec), loads the training
CSR bench.py wrote as .npy files, runs `epochs` epochs of the fp64 C restatement of SVD.sgd
(mf_oracle.c: oracle_svd_sgd <- matrix_factorization.pyx:241-262) and prints one JSON line with
its compute-only wall time.  Never touches a GPU.

    python oracle/cpu_worker.py DIR CORE EPOCHS K [svd|svdpp]

svdpp: the restatement of SVDpp.sgd in the reference's per-rating form (oracle_svdpp_sgd <-
matrix_factorization.pyx:463-498) over the CSR in DIR (bench.py writes a user-prefix sample).
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    d, core, epochs, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    algo = sys.argv[5] if len(sys.argv) > 5 else "svd"
    os.sched_setaffinity(0, {core})
    import oracle as orc
    row_ptr = np.load(os.path.join(d, "row_ptr.npy"))
    items = np.load(os.path.join(d, "items.npy"))
    ratings = np.load(os.path.join(d, "ratings.npy"))
    n_items = int(np.load(os.path.join(d, "n_items.npy")))
    timer = orc.time_svdpp_epochs if algo == "svdpp" else orc.time_svd_epochs
    t = timer(row_ptr, items, ratings, n_items, K, epochs, seed=core)
    print(json.dumps({"core": core, "epochs": epochs, "seconds": t,
                      "updates": int(row_ptr[-1]) * epochs}), flush=True)


if __name__ == "__main__":
    main()
