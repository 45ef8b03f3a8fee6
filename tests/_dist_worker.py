"""Child process of tests/test_gpu_dist.py: one rank of a multi-rank fit on the box's single GPU
(gloo carries the collectives; every rank's kernels run on cuda:0).  The fit goes through the
product path: SVD/SVDpp(distributed=True).fit(trainset) under torchrun-style env vars."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dataset(name):
    """(trainset, testset list) -- u1: the reference's fixture; pop2: the union of two ML-1M-shape
    synthetic user populations over one item set (bench.py's 2-GPU weak-scaling data)."""
    from surprise_amd import Dataset, Reader
    from surprise_amd.model_selection import KFold, PredefinedKFold
    if name == "u1":
        g = os.path.join(ROOT, "tests", "golden")
        data = Dataset.load_from_folds([(os.path.join(g, "u1_ml100k_train"),
                                         os.path.join(g, "u1_ml100k_test"))], Reader("ml-100k"))
        ts, test = next(PredefinedKFold().split(data))
        return ts, list(test)
    from surprise_amd import synthetic
    U, I, N = synthetic.SHAPES["ml-1m"]
    parts = [synthetic.population(p, U, I, N) for p in range(2)]
    u = np.concatenate([parts[0][0], parts[1][0] + U])
    i = np.concatenate([parts[0][1], parts[1][1]])
    r = np.concatenate([parts[0][2], parts[1][2]])
    ts, test = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
    return ts, list(test)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rank", type=int)
    p.add_argument("--world", type=int)
    p.add_argument("--port", type=int)
    p.add_argument("--out")
    p.add_argument("--algo", default="SVD")
    p.add_argument("--mode", default="auto")
    p.add_argument("--data", default="u1")
    p.add_argument("--factors", type=int, default=20)
    p.add_argument("--epochs", type=int, default=5)
    p.add_argument("--dtype", default="float64")
    p.add_argument("--seed", default="0")
    a = p.parse_args()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port), RANK=str(a.rank),
                      LOCAL_RANK=str(a.rank), WORLD_SIZE=str(a.world),
                      HSA_ENABLE_IPC_MODE_LEGACY="0", SURPRISE_AMD_DIST_BACKEND="gloo")
    from surprise_amd import SVD, SVDpp, accuracy
    from surprise_amd.dist import DistContext
    ts, test = dataset(a.data)
    klass = SVD if a.algo == "SVD" else SVDpp
    seed = None if a.seed == "none" else int(a.seed)
    algo = klass(n_factors=a.factors, n_epochs=a.epochs, random_state=seed, dtype=a.dtype,
                 mode=a.mode, distributed=True).fit(ts)
    rmse = accuracy.rmse(algo.test(test), verbose=False)
    out = dict(pu=algo.pu, qi=algo.qi, bu=algo.bu, bi=algo.bi, rmse=rmse)
    if a.algo != "SVD":
        out["yj"] = algo.yj
    np.savez(a.out.replace(".npz", "_r%d.npz" % a.rank), **out)
    ctx = DistContext.from_env()
    ctx.barrier()
    ctx.dist.destroy_process_group()


if __name__ == "__main__":
    main()
