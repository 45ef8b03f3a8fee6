"""Experiment: SVD++ item-side schedules with the deferred y fold -- held-out RMSE delta vs the
fp64 affine-form oracle (BASELINE configs[2] shape, K=100, 5 epochs) and the epoch time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from exp_modes import oracle_rmse, synth  # noqa: E402
import torch  # noqa: E402
from surprise_amd import SVDpp, accuracy  # noqa: E402


def main():
    ts, test = synth("ml-1m")
    params = dict(n_factors=100, n_epochs=5, random_state=0)
    ref = oracle_rmse("SVDpp", params, ts, test, affine=True)
    print("oracle rmse %.5f" % ref, flush=True)
    for mode, chunks, ydefer in (("atomic", 1, "1"), ("atomic", 1, "0"), ("log", 1, "1"),
                                 ("log", 4, "1"), ("log", 1, "0"), ("log", 4, "0")):
        os.environ["SURPRISE_AMD_YDEFER"] = ydefer
        algo = SVDpp(**params, mode=mode, chunks_per_epoch=chunks)
        algo.fit(ts)  # warm (build + first launches)
        torch.cuda.synchronize()
        t = time.perf_counter()
        algo = SVDpp(**params, mode=mode, chunks_per_epoch=chunks).fit(ts)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / params["n_epochs"] * 1e3
        got = accuracy.rmse(algo.test(test), verbose=False)
        print("mode %-6s chunks %d ydefer %s: rmse %.5f delta %+.5f  fit %.3f ms/epoch (incl. setup)"
              % (mode, chunks, ydefer, got, got - ref, dt), flush=True)


if __name__ == "__main__":
    main()
