"""Child process of tests/test_gpu_dist.py::test_rccl_single_rank_collectives: a world-size-1
RCCL (backend "nccl") process group joined through DistContext.from_env -- the path the driver's
8-GPU run takes -- and every collective the engine uses, on device tensors."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_path = sys.argv[1]
    import torch
    from surprise_amd.dist import DistContext
    ctx = DistContext.from_env("nccl", single_rank_group=True)
    dev = torch.device("cuda", torch.cuda.current_device())
    res = {"backend": ctx.backend, "world": ctx.world, "rank": ctx.rank,
           "host_staged": ctx.host_staged}
    # all_reduce_sum on the engine's exchange dtypes (fp32 / fp64 flat buffers)
    for dt in (torch.float32, torch.float64):
        x = torch.arange(1 << 20, dtype=dt, device=dev) * 0.5
        ref = x.clone()
        ctx.all_reduce_sum(x)
        torch.cuda.synchronize()
        res["sum_%s" % str(dt).split(".")[1]] = bool(torch.equal(x, ref)) and x.is_cuda
    y = torch.tensor([3, -7, 11], dtype=torch.int64, device=dev)
    ctx.all_reduce_max(y)
    res["max"] = y.cpu().tolist()
    z = torch.full((5,), 2.5, dtype=torch.float64, device=dev)
    ctx.broadcast(z, 0)
    res["broadcast"] = z.cpu().tolist()
    rows = torch.arange(12, dtype=torch.float32, device=dev).view(3, 4)
    g = ctx.all_gather_rows(rows, [3])
    res["gather_equal"] = bool(torch.equal(g, rows)) and g.is_cuda
    ctx.check_agreement([1, 2, 3], "a test vector")
    res["agreement"] = True
    # the engine's fused exchange on one rank: MFEngine.sync_items with this context (world 1:
    # the local fold) after a chunk, through the same device stream RCCL orders against
    import numpy as np
    from surprise_amd.engine import MFEngine
    rng = np.random.RandomState(0)
    n_users, n_items, K = 50, 30, 8
    deg = rng.randint(3, 12, n_users)
    row_ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    items = np.concatenate([np.sort(rng.choice(n_items, d, replace=False)) for d in deg])
    ratings = rng.randint(1, 6, len(items)).astype(np.float64)
    eng = MFEngine((row_ptr, items, ratings), n_items, K, dtype="float64",
                   hyper=dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02,
                              reg_bi=.02, reg_pu=.02, reg_qi=.02,
                              global_mean=float(ratings.mean())))
    eng.set_factors(rng.normal(0, .1, (n_users, K)), rng.normal(0, .1, (n_items, K)))
    eng.run_epochs(2, ctx)
    f = eng.get_factors(ctx)
    res["engine_finite"] = bool(np.isfinite(f["qi"]).all() and np.isfinite(f["pu"]).all())
    ctx.barrier()
    ctx.dist.destroy_process_group()
    with open(out_path, "w") as fh:
        json.dump(res, fh)


if __name__ == "__main__":
    main()
