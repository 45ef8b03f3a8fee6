"""Probe: one SVD log step (ML-1M shape, K=100, bench configuration) replayed as a HIP graph vs
launched eagerly.  Prints ms/step of both and whether the tables after the same number of
steps are bit-identical."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from surprise_amd import synthetic  # noqa: E402
from surprise_amd.engine import MFEngine  # noqa: E402
from surprise_amd.model_selection import KFold  # noqa: E402
from surprise_amd.trainset import Trainset  # noqa: E402

K = 100
U, I, N = synthetic.SHAPES["ml-1m"]
u, i, r = synthetic.population(0, U, I, N)
tr, _ = next(KFold(5, random_state=0).fold_indices(len(r)))
ts = Trainset.from_inner_arrays(u[tr], i[tr], r[tr], n_users=U, n_items=I)
csr = ts.csr()
gm = float(ts.global_mean)
hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02,
             reg_pu=.02, reg_qi=.02, global_mean=gm)
rng = np.random.RandomState(0)
pu0, qi0 = rng.normal(0, .1, (U, K)), rng.normal(0, .1, (I, K))
s = torch.cuda.Stream()


def make():
    with torch.cuda.stream(s):
        e = MFEngine(csr, I, K, hyper=hyper, mode="log")
        e.set_factors(pu0, qi0)
    return e


def step(e, n):
    with torch.cuda.stream(s):
        for _ in range(n):
            e.run_chunk(0)
            e.sync_items(None)


E = 40
eng = make()
step(eng, 4)
torch.cuda.synchronize()
t0 = time.perf_counter()
step(eng, E)
torch.cuda.synchronize()
eager = (time.perf_counter() - t0) / E * 1e3
ref = make()
step(ref, 4 + 2 * 10)
torch.cuda.synchronize()

g = make()
step(g, 2)
torch.cuda.synchronize()
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph, stream=s):
    step(g, 2)
torch.cuda.synchronize()
for _ in range(10):  # 2 + 2 (captured, not executed) ... the capture does not run the kernels
    graph.replay()
torch.cuda.synchronize()
same = all(torch.equal(getattr(ref, n), getattr(g, n)) for n in ("pu", "bu", "qb"))
mx = float((ref.qb - g.qb).abs().max())
t0 = time.perf_counter()
for _ in range(E // 2):
    graph.replay()
torch.cuda.synchronize()
gt = (time.perf_counter() - t0) / E * 1e3
print("eager %.4f ms/step   graph %.4f ms/step   bit-identical after 22 steps: %s (max|dq| %.2e)"
      % (eager, gt, same, mx), flush=True)
