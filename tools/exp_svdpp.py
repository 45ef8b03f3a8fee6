"""Experiment: SVD++ item-side schedules on BASELINE configs[2]'s shape (K=100, E=20) -- held-out
RMSE delta vs the fp64 affine-form oracle and the fit time.
    python tools/exp_svdpp.py [epochs] [mode:chunks:ydefer:order,...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from exp_modes import oracle_rmse, synth  # noqa: E402
import torch  # noqa: E402
from surprise_amd import SVDpp, accuracy  # noqa: E402


def main():
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ts, test = synth("ml-1m")
    params = dict(n_factors=100, n_epochs=E, random_state=0)
    ref = oracle_rmse("SVDpp", params, ts, test, affine=True)
    print("oracle rmse %.5f (E=%d)" % (ref, E), flush=True)
    variants = [v.split(":") for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else
                ["atomic:1:1:deal", "atomic:2:1:band", "atomic:4:1:band", "atomic:2:0:band",
                 "atomic:4:0:band", "log:2:0:band", "log:4:0:band", "log:8:0:band"])]
    for v in variants:
        mode, chunks, ydefer, order = v[:4]
        waves = int(v[4]) if len(v) > 4 else 0
        chunks = int(chunks)
        os.environ["SURPRISE_AMD_YDEFER"] = ydefer
        os.environ["SURPRISE_AMD_CHUNK_ORDER"] = order
        algo = SVDpp(**params, mode=mode, chunks_per_epoch=chunks, n_waves=waves)
        algo.fit(ts)  # warm (build + first launches)
        torch.cuda.synchronize()
        t = time.perf_counter()
        algo = SVDpp(**params, mode=mode, chunks_per_epoch=chunks, n_waves=waves).fit(ts)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / params["n_epochs"] * 1e3
        got = accuracy.rmse(algo.test(test), verbose=False)
        eng = algo._engine
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            for c in range(eng.n_chunks):
                eng.run_chunk(c)
                eng.sync_items(None)
        torch.cuda.synchronize()
        ep = (time.perf_counter() - t) / 10 * 1e3
        print("mode %-6s chunks %d ydefer %s order %s waves %d: rmse %.5f delta %+.5f  epoch "
              "%.3f ms (fit %.3f ms/epoch incl. setup)" % (mode, chunks, ydefer, order, waves, got,
                                                          got - ref, ep, dt), flush=True)


if __name__ == "__main__":
    main()
