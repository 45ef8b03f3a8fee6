"""Round-5 probe (GPU box): does C3's helper-wave launch gain from keeping its heaviest users'
chains together on one XCD, away from the light chains?  The launch runs chain c as workgroup c,
and workgroups are dealt round-robin over the 8 XCDs, so chains c = 0 mod 8 share an XCD.  The
probe swaps engine.chain_schedule for a layout that gives the `top` heaviest users to chains
0, 8, 16, ... (one user each, `top` <= chains / 8) and deals the rest LPT over the other chains.
fp32 and fp64, ms per epoch over 10 epochs."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402


def xcd_schedule(top):
    def sched(users, row_ptr, n_chains, user_cost=16):
        import heapq
        users = np.asarray(users, np.int32)
        deg = np.diff(np.asarray(row_ptr, np.int64))[users]
        order = np.argsort(-deg, kind="stable")
        n_chains = max(1, min(int(n_chains), len(users)))
        lists = [[] for _ in range(n_chains)]
        x0 = [c for c in range(0, n_chains, 8)][:top]
        for c, x in zip(x0, order[:len(x0)]):
            lists[c].append(users[x])
        rest = [c for c in range(n_chains) if c not in set(x0)]
        heap = [(0, c) for c in rest]
        for x in order[len(x0):]:
            load, c = heapq.heappop(heap)
            lists[c].append(users[x])
            heapq.heappush(heap, (load + int(deg[x]) + user_cost, c))
        m = max(len(x) for x in lists)
        out = np.full((m, n_chains), -1, np.int32)
        for c, x in enumerate(lists):
            out[:len(x), c] = x
        return out.ravel()
    return sched


def main():
    import torch
    import surprise_amd.engine as E
    from test_gpu_parity import _synthetic_fold
    out = open(sys.argv[1], "w")
    ts, _ = _synthetic_fold("ml-1m")
    csr = ts.csr()
    hyper = dict(lr_bu=.007, lr_bi=.007, lr_pu=.007, lr_qi=.007, lr_yj=.007, reg_bu=.02,
                 reg_bi=.02, reg_pu=.02, reg_qi=.02, reg_yj=.02, global_mean=float(ts.global_mean))
    K = 100
    orig = E.chain_schedule
    for dt in ("float32", "float64"):
        for top in (0, 16, 32, 64):
            E.chain_schedule = xcd_schedule(top) if top else orig
            rng = np.random.RandomState(0)
            eng = E.MFEngine(csr, ts.n_items, K, algo="svdpp", hyper=hyper, dtype=dt, mode="atomic")
            eng.set_factors(rng.normal(0, .1, (ts.n_users, K)), rng.normal(0, .1, (ts.n_items, K)),
                            yj=rng.normal(0, .1, (ts.n_items, K)))
            eng.run_epochs(2)
            torch.cuda.synchronize()
            best = []
            for rep in range(3):
                t0 = time.perf_counter()
                eng.run_epochs(10)
                torch.cuda.synchronize()
                best.append((time.perf_counter() - t0) / 10 * 1e3)
            r = dict(dtype=dt, heavy_on_one_xcd=top, chains=int(eng.hx_chains),
                     ms_per_epoch=[round(x, 4) for x in best])
            print(json.dumps(r), flush=True)
            out.write(json.dumps(r) + "\n")
            del eng
    E.chain_schedule = orig


if __name__ == "__main__":
    main()
