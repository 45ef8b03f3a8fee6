"""Probe (GPU box): the shader clock one wave sees (tools/probe_src/clock_probe.hip: cycle counter
vs the 100 MHz real-time counter over a dependent fp64 FMA chain) -- alone, and on a second stream
while the product SVD epochs (ML-1M shape, fp64 / fp32) run.  Build the probe first:
hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/probe_src/libclock_probe.so
tools/probe_src/clock_probe.hip"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from surprise_amd import Dataset, synthetic  # noqa: E402
from surprise_amd.engine import MFEngine  # noqa: E402
from surprise_amd.model_selection import KFold  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "probe_src", "libclock_probe.so"))
ps = torch.cuda.Stream()
outs = torch.zeros((64, 3), dtype=torch.int64, device="cuda")


def probes(n, iters=20000):
    for k in range(n):
        lib.clock_probe(ctypes.c_void_p(outs[k].data_ptr()), iters, ctypes.c_void_p(ps.cuda_stream))


def mhz(n):
    o = outs[:n].cpu().numpy().astype(np.float64)
    return o[:, 0] / (o[:, 1] / 100.0)  # cycles per us = MHz


probes(8)
torch.cuda.synchronize()
print("alone: shader clock %s MHz" % np.round(mhz(8)).astype(int).tolist(), flush=True)
u, i, r = synthetic.shape("ml-1m")
ts, _ = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
rp, it, rt = ts.csr()
for dt in ("float64", "float32"):
    rng = np.random.RandomState(0)
    eng = MFEngine((rp, it, rt), ts.n_items, 100, hyper=bench.hyper_for("svd", float(ts.global_mean)),
                   dtype=dt)
    eng.set_factors(rng.normal(0, .1, (ts.n_users, 100)), rng.normal(0, .1, (ts.n_items, 100)))
    eng._prepare(None)
    bench.run_steps(eng, None, 5, 2, torch, instrument=False)
    torch.cuda.synchronize()
    outs.zero_()
    for _ in range(400):
        eng.run_chunk(0)
        eng.sync_items(None)
    probes(40)
    torch.cuda.synchronize()
    m = mhz(40)
    print("%s epochs running: shader clock median %d MHz (min %d, max %d)"
          % (dt, np.median(m), m.min(), m.max()), flush=True)
    del eng
