"""Round-5 probe (GPU box): C3 (ML-1M fold, SVD++ K=100 E=20) held-out RMSE vs the exact affine
oracle for the hybrid launch's cold shares, fp32 and fp64."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402


def main():
    import torch
    from surprise_amd import SVDpp
    from test_gpu_parity import _synthetic_fold, _oracle_rmse
    out = open(sys.argv[1], "w")
    ts, test = _synthetic_fold("ml-1m")
    params = dict(n_factors=100, n_epochs=20, random_state=0)
    ref = _oracle_rmse("SVDpp", params, ts, test, affine=True)
    for dt in ("float32", "float64"):
        for cs in (0.0, 0.3, 0.5, 0.7):
            a = SVDpp(**params, dtype=dt, mode="atomic")
            a._engine_options = {"cold_share": cs}
            t0 = time.perf_counter()
            a.fit(ts)
            torch.cuda.synchronize()
            preds = a.test(test)
            r = float(np.sqrt(np.mean([(p.r_ui - p.est) ** 2 for p in preds])))
            rec = dict(dtype=dt, cold_share=cs, rmse=r, oracle=ref, delta=r - ref,
                       fit_s=time.perf_counter() - t0)
            print(json.dumps(rec), flush=True)
            out.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
