"""Child process of tests/test_gpu_dist.py: one rank of a 2-rank fit on the box's single GPU
(gloo carries the all-reduces; the kernels run on cuda:0 in every rank)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rank", type=int)
    p.add_argument("--world", type=int)
    p.add_argument("--port", type=int)
    p.add_argument("--out")
    p.add_argument("--algo", default="SVD")
    p.add_argument("--mode", default="auto")
    a = p.parse_args()
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port), RANK=str(a.rank),
                      WORLD_SIZE=str(a.world), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    torch.cuda.set_device(0)
    from surprise_amd import SVD, SVDpp, Dataset, Reader, accuracy
    from surprise_amd.model_selection import PredefinedKFold
    g = os.path.join(ROOT, "tests", "golden")
    data = Dataset.load_from_folds([(os.path.join(g, "u1_ml100k_train"),
                                     os.path.join(g, "u1_ml100k_test"))], Reader("ml-100k"))
    ts, test = next(PredefinedKFold().split(data))
    klass = SVD if a.algo == "SVD" else SVDpp
    algo = klass(n_factors=20, n_epochs=5, random_state=0, dtype="float64", mode=a.mode).fit(ts)
    rmse = accuracy.rmse(algo.test(test), verbose=False)
    if a.rank == 0:
        np.savez(a.out, pu=algo.pu, qi=algo.qi, bu=algo.bu, bi=algo.bi, rmse=rmse)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
