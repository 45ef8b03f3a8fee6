"""Round-5 probe (GPU box): two policy questions, one JSON line per measurement.

1. The SVD++ q log's drift with the number of epoch-chunks: C3 (ML-1M shape, KFold(5, rs=0)
   fold 0, SVD++ K=100 E=20 fp32) held-out RMSE vs the exact affine oracle, q log vs the atomic
   schedule at chunks 1, 2, 4, 8, 16, with fit times.
2. The deterministic (one wave, the reference's order) SVD fit's cost on u1 vs the parallel
   schedule (K=20 E=5, K=100 E=20).

Usage: python3 tools/probes/qlog_chunks_exact_speed.py OUT.jsonl [--no-c3] [--no-u1]
       [--chunks 1,2,4,8,16]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402


def rmse(preds):
    return float(np.sqrt(np.mean([(p.r_ui - p.est) ** 2 for p in preds])))


def main():
    out = open(sys.argv[1], "w")

    def emit(**kw):
        print(json.dumps(kw), flush=True)
        out.write(json.dumps(kw) + "\n")
        out.flush()

    import torch  # noqa: F401
    import conftest
    from surprise_amd import SVD, SVDpp
    golden_meta, _ = conftest.golden.__wrapped__()
    ts, test = conftest.u1.__wrapped__()
    for name in () if "--no-u1" in sys.argv else ("svd_k20_e5", "svd_k100_e20", "svd_k100_e20_unbiased"):
        case = golden_meta["cases"][name]
        for det in (False, True, False, True):  # (the first pair warms the code paths)
            t0 = time.perf_counter()
            a = SVD(**case["params"], dtype="float64", deterministic=det).fit(ts)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            r = rmse(a.test(test))
        emit(probe="u1_exact", case=name, deterministic=det, fit_s=dt,
             rmse=r, ref=case["rmse"], delta=r - case["rmse"])
        a = SVD(**case["params"], dtype="float64", deterministic=False).fit(ts)
        t0 = time.perf_counter()
        a = SVD(**case["params"], dtype="float64", deterministic=False).fit(ts)
        torch.cuda.synchronize()
        emit(probe="u1_parallel", case=name, fit_s=time.perf_counter() - t0,
             delta=rmse(a.test(test)) - case["rmse"])
    if "--no-c3" in sys.argv:
        return
    chunk_list = (1, 2, 4, 8, 16)
    if "--chunks" in sys.argv:
        chunk_list = tuple(int(x) for x in sys.argv[sys.argv.index("--chunks") + 1].split(","))
    from test_gpu_parity import _synthetic_fold, _oracle_rmse
    ts, test = _synthetic_fold("ml-1m")
    params = dict(n_factors=100, n_epochs=20, random_state=0)
    t0 = time.perf_counter()
    ref = _oracle_rmse("SVDpp", params, ts, test, affine=True)
    emit(probe="c3_oracle", rmse=ref, seconds=time.perf_counter() - t0)
    for chunks in chunk_list:
        for qlog in (False, True):
            a = SVDpp(**params, dtype="float32", chunks_per_epoch=chunks)
            a._engine_options = {"qlog": qlog}
            t0 = time.perf_counter()
            a.fit(ts)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            r = rmse(a.test(test))
            emit(probe="c3_chunks", chunks=chunks, qlog=qlog, fit_s=dt, rmse=r, delta=r - ref)


if __name__ == "__main__":
    main()
