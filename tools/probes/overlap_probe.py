"""Probe: does concurrent memory traffic slow the heaviest user's dependent chain?  (SVD, ML-1M
shape, K=100, log schedule.)  Times the epoch kernel over the heaviest user alone, then the same
launch beside a background launch on a second stream: the full checkpoint replay, a streaming
copy, the light users' epoch.  Prints one line per case (median of 10, microseconds)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from surprise_amd import Dataset, synthetic  # noqa: E402
from surprise_amd.engine import MFEngine  # noqa: E402
from surprise_amd.model_selection import KFold  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
u, i, r = synthetic.shape("ml-1m")
ts, _ = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
rp, it, rt = ts.csr()
hyper = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, reg_bu=.02, reg_bi=.02, reg_pu=.02,
             reg_qi=.02, global_mean=float(ts.global_mean))
eng = MFEngine((rp, it, rt), ts.n_items, K, hyper=hyper, mode="log", heavy=0)
rng = np.random.RandomState(0)
eng.set_factors(rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K)))
for _ in range(3):
    eng.run_chunk(0)
    eng.sync_items(None)
torch.cuda.synchronize()
order = eng.sched[0].cpu().numpy()
deg = np.diff(rp)
main = eng.stream
side = torch.cuda.Stream()
st_main = eng._st()
import ctypes  # noqa: E402
st_side = ctypes.c_void_p(side.cuda_stream)
top1 = torch.from_numpy(order[:1].copy()).cuda()
light = torch.from_numpy(order[64:].copy()).cuda()
big_a = torch.empty(1 << 28, dtype=torch.float32, device="cuda")  # 1 GiB
big_b = torch.empty_like(big_a)
lg = eng.logs[0]


def bg_replay(xm=0):
    eng._reduce_log(lg, eng.sums.data_ptr(), st_side, xm)


def bg_copy():
    with torch.cuda.stream(side):
        big_b.copy_(big_a)


def bg_light(xm=0):
    eng._epoch(light, light.numel(), eng.n_waves, 0, st_side, xm)


def bg_light_replay(xm=0):
    bg_light(xm)
    bg_replay(xm)


def timed(bg, xm_chain=0, reps=10):
    out_c, out_b = [], []
    for _ in range(reps + 2):
        e0, e1 = (torch.cuda.Event(enable_timing=True) for _ in range(2))
        e0.record(main)
        side.wait_event(e0)
        if bg is not None:
            bg()
        eb = torch.cuda.Event(enable_timing=True)
        eb.record(side)
        eng._epoch(top1, 1, 1, 0, st_main, xm_chain)
        e1.record(main)
        torch.cuda.synchronize()
        out_c.append(e0.elapsed_time(e1) * 1e3)
        out_b.append(e0.elapsed_time(eb) * 1e3)
    return float(np.median(out_c[2:])), float(np.median(out_b[2:]))


print("top user degree", int(deg[order[0]]), flush=True)
X0, XR = 0x01, 0xFE
for name, bg, xm in (("alone", None, 0), ("alone xcd0", None, X0),
                     ("replay", bg_replay, 0),
                     ("replay xcd1-7", lambda: bg_replay(XR), X0),
                     ("copy 1GiB", bg_copy, 0), ("copy 1GiB", bg_copy, X0),
                     ("light epoch", bg_light, 0),
                     ("light xcd1-7", lambda: bg_light(XR), X0),
                     ("light+replay", bg_light_replay, 0),
                     ("light+replay xcd1-7", lambda: bg_light_replay(XR), X0)):
    c, b = timed(bg, xm)
    print("%-22s chain(xmask %02x) %8.1f us  (%.1f ns/rating)   background %8.1f us" %
          (name, xm, c, c * 1e3 / deg[order[0]], b), flush=True)
