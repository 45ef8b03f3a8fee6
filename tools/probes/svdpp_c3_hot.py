"""Round-5 probe (GPU box): C3's hot-row replicas (engine option hot_rows) swept past the
policy's count: the auto policy (hot_items: items holding >= 0.15% of the ratings, at most 64),
then 0 / 32 / 64 / 128 / 256 / 512 replicas.  fp32 and fp64, ms per epoch over 3 x 10 epochs."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402


def main():
    import torch
    from surprise_amd.engine import MFEngine
    from test_gpu_parity import _synthetic_fold
    out = open(sys.argv[1], "w")
    ts, _ = _synthetic_fold("ml-1m")
    csr = ts.csr()
    hyper = dict(lr_bu=.007, lr_bi=.007, lr_pu=.007, lr_qi=.007, lr_yj=.007, reg_bu=.02,
                 reg_bi=.02, reg_pu=.02, reg_qi=.02, reg_yj=.02, global_mean=float(ts.global_mean))
    K = 100
    for dt in ("float32", "float64"):
        for hot in (None, 0, 32, 64, 128, 256, 512):
            rng = np.random.RandomState(0)
            kw = {} if hot is None else {"hot_rows": hot}
            eng = MFEngine(csr, ts.n_items, K, algo="svdpp", hyper=hyper, dtype=dt, mode="atomic",
                           **kw)
            eng.set_factors(rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K)),
                            yj=rng.normal(0, .1, (ts.n_items, K)))
            eng.run_epochs(2)
            torch.cuda.synchronize()
            ms = []
            for rep in range(3):
                t0 = time.perf_counter()
                eng.run_epochs(10)
                torch.cuda.synchronize()
                ms.append(round((time.perf_counter() - t0) / 10 * 1e3, 4))
            n_hot = int(eng.hot_flag.sum().item()) if getattr(eng, "hot_flag", None) is not None else 0
            r = dict(dtype=dt, hot_rows="auto" if hot is None else hot, replicas=n_hot,
                     ms_per_epoch=ms)
            print(json.dumps(r), flush=True)
            out.write(json.dumps(r) + "\n")
            del eng


if __name__ == "__main__":
    main()
