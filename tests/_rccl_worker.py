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
    res["exchange"] = forced_exchange(ctx, np, torch)
    ctx.barrier()
    ctx.dist.destroy_process_group()
    with open(out_path, "w") as fh:
        json.dump(res, fh)


def forced_exchange(ctx, np, torch):
    """The multi-rank exchange the driver's 8-GPU run takes first -- MFEngine.sync_items ->
    _delta_buffer / _delta_into -> ctx.all_reduce_sum (RCCL, device tensors) -> _apply -- forced
    at world 1 (engine option exchange=True):
      deterministic schedules, compared with the local fold on the same data and initial factors
      (3 epochs, fp64):
        SVD, checkpoint log, 3 chunks: the per-item sums and the next chunk's <p^2> ride in the
          buffer; one rank's all-reduce is the identity: factors equal the local fold's (1e-12);
        SVD++, q log, 3 chunks: the log sums plus y's affine composition (mf_item_affine) from
          the chunk-start snapshot: equal to the local fold (1e-9);
      SVD++'s float-atomic schedule (Hogwild q rows: two runs differ by the atomics' timing, so
      no two runs compare): each chunk's exchange must leave the tables as the chunk left them --
        q / b by mf_item_merge's recency rule (w = 1 with no later rank) and y by the affine
        composition, both from the chunk-start snapshots (1e-12 per chunk) -- with q's all-reduce
        overlapping the y fold (async RCCL, overlap_q: two collectives per chunk) and as one
        buffer (overlap_q=False)."""
    from surprise_amd.engine import MFEngine
    rng = np.random.RandomState(1)
    n_users, n_items, K = 400, 120, 16
    deg = rng.randint(2, 40, n_users)
    row_ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    items = np.concatenate([np.sort(rng.choice(n_items, d, replace=False)) for d in deg])
    ratings = rng.randint(1, 6, len(items)).astype(np.float64)
    pu0, qi0, yj0 = (rng.normal(0, .1, (n, K)) for n in (n_users, n_items, n_items))
    out = {}

    def hyper(algo):
        lr = .007 if algo == "svdpp" else .005
        return dict(lr_bu=lr, lr_bi=lr, lr_pu=lr, lr_qi=lr, lr_yj=lr, reg_bu=.02, reg_bi=.02,
                    reg_pu=.02, reg_qi=.02, reg_yj=.02, global_mean=float(ratings.mean()))

    def engine(algo, forced, **kw):
        eng = MFEngine((row_ptr, items, ratings), n_items, K, algo=algo, dtype="float64",
                       hyper=hyper(algo), exchange=True if forced else None, **kw)
        eng.set_factors(pu0, qi0, yj=yj0 if algo == "svdpp" else None)
        return eng

    def counting(fn):
        calls, asyncs = [0], [0]
        real, real_async = ctx.all_reduce_sum, ctx.all_reduce_sum_async

        def counted(t):
            assert t.is_cuda  # (RCCL: every exchange stays on the device)
            calls[0] += int(t.dtype == torch.float64)
            return real(t)

        def counted_async(t):
            assert t.is_cuda
            calls[0] += int(t.dtype == torch.float64)
            asyncs[0] += 1
            return real_async(t)
        ctx.all_reduce_sum, ctx.all_reduce_sum_async = counted, counted_async
        try:
            fn()
        finally:
            del ctx.all_reduce_sum
            del ctx.all_reduce_sum_async
        return calls[0], asyncs[0]

    # deterministic schedules: forced exchange vs local fold
    for name, algo, kw, tol in (("svd_log", "svd", dict(mode="log", n_chunks=3), 1e-12),
                                ("svdpp_qlog", "svdpp", dict(qlog=True, n_chunks=3), 1e-9)):
        got = {}
        for forced in (False, True):
            eng = engine(algo, forced, **kw)
            box = {}

            def run(eng=eng, box=box):
                eng.run_epochs(3, ctx)
                box["f"] = eng.get_factors(ctx)
            if forced:
                n_calls, n_async = counting(run)
            else:
                run()
            got[forced] = box["f"]
            if forced:
                out[name + "_allreduce_calls"] = n_calls
                out[name + "_overlap"] = n_async > 0
                out[name + "_buffer_elems"] = int(eng._delta_buffer()[0].numel())
                out[name + "_qlog"] = bool(getattr(eng, "qlog_pp", False))
        keys = ("pu", "qi", "bu", "bi") + (("yj",) if algo == "svdpp" else ())
        err = max(float(np.abs(got[True][k] - got[False][k]).max()) for k in keys)
        out[name + "_max_abs_diff"] = err
        out[name + "_equal"] = bool(err <= tol)
        out[name + "_chunks"] = kw["n_chunks"]
    # the float-atomic schedule: every chunk's exchange is the identity at world 1
    for name, ov in (("svdpp_atomic", True), ("svdpp_one_buffer", False)):
        eng = engine("svdpp", True, mode="atomic", n_chunks=2, overlap_q=ov)
        worst = [0.0]

        def run(eng=eng, worst=worst):
            eng._prepare(ctx)
            for _ in range(3):
                for c in range(eng.n_chunks):
                    eng.run_chunk(c)
                    torch.cuda.synchronize()
                    q0, y0 = eng.qb.clone(), eng.yj.clone()
                    eng.sync_items(ctx)
                    torch.cuda.synchronize()
                    worst[0] = max(worst[0], float((eng.qb - q0).abs().max()),
                                   float((eng.yj - y0).abs().max()))
        n_calls, n_async = counting(run)
        out[name + "_max_abs_diff"] = worst[0]
        out[name + "_equal"] = bool(worst[0] <= 1e-12)
        out[name + "_allreduce_calls"] = n_calls
        out[name + "_overlap"] = n_async > 0
        out[name + "_buffer_elems"] = int(eng._delta_buffer()[0].numel())
        out[name + "_chunks"] = 2
        out[name + "_finite"] = bool(np.isfinite(eng.get_factors(ctx)["yj"]).all())
    return out


if __name__ == "__main__":
    main()
