"""Benchmark: rating-updates/sec of the SVD / SVD++ SGD hot path on MI355X.

Default (N=1): BASELINE configs[1] -- SVD n_factors=100 on the synthetic planted ML-1M shape
(6040 users x 3706 items x 1,000,209 ratings, surprise_amd.synthetic), KFold(5, random_state=0)
fold 0 -> 800,167 training ratings; one "step" = one epoch over them.  The headline computes in
fp64 (the reference's arithmetic, mf.pyx:207-227); an fp32 leg rides beside it (`f32_leg`).

--gpus N (one process per GPU; spawned here when WORLD_SIZE is unset, or launched by
torch.distributed.run): every rank holds ONLY its own user rows on its device.
  --shape ml-1m (default)  weak scaling: rank r trains user population r of one dataset (r = 0
                           is the single-GPU dataset above; every population is ML-1M-shaped and
                           rates the same 3706 items, synthetic.population) -- per-GPU work fixed
  --shape c4 | c5          strong scaling: BASELINE configs[3] / [4] (2M x 200k x 100M, SVD
                           K=128 / 10M x 1M x 1B, SVD++ K=128; 1% held out, fp32), sharded by
                           user range; each rank generates only its own rows
Item-side updates are SUM-all-reduced once per epoch-chunk (RCCL; `--backend gloo` only to
rehearse several ranks on one GPU).  The BASELINE scaling configs:
  C4 on 4 GPUs:  python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
                   --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 4 --shape c4
                 ~25M ratings and 500k users per rank, ~7.5 GB of device memory per rank; one
                 115 MB all-reduce per epoch (the per-item log sums, 200k x 144 fp32)
  C5 on 8 GPUs:  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
                   --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8 --shape c5
                 1.25M users / ~123M ratings per rank (the C5 shard: 5.2 GB measured on one
                 GPU, ~7.4 GB with the merge's snapshots and exchange buffer); 16 epoch-chunks,
                 each ONE 1.09 GB all-reduce (q deltas 1M x 144 + y maps 1M x 128, fp32)

Prints ONE JSON line on rank 0 with the contract fields plus:
  roofline      the dominant kernel's (the epoch kernel's launches): SURVEY 8(d) algorithmic
                bytes per launch / its average launch duration (HIP events on the stream it runs
                on), `traffic` its measured HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE,
                profiles/traffic_*.json); the whole step's figures beside it (step_*), and the
                per-phase GPU time of a step (phases_gpu_ms; N>1: the all-reduce per chunk)
  cpu_baseline  the fp64 C restatement of the reference loop (oracle/): 16 pinned processes (the
                box's CPU share) and one pinned core; the node's all-core figure is derived
  rmse          held-out RMSE of a full 20-epoch fit vs the fp64 sequential oracle (N=1; c4 / c5
                against the committed oracle values, tests/golden/scale_golden.json)
  svdpp_c3      BASELINE configs[2]: SVD++ K=100 epochs on the same fold (fp64 + fp32 legs)
  predict       test() / test_metrics() predictions/s of fitted SVD / SVD++
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md chip table); 6.3 TB/s achievable copy
# no-return float atomics (global_atomic_add_f32, one dword per lane) execute at the memory side:
# chip-wide ~1.3 TB/s of added bytes (MI355X_MICROARCH.md, "Global float atomics": 1.26-1.36)
ATOMIC_F32_GBS = 1300.0
PHASE_STEPS = 5  # epochs with HIP events around each phase, after the timed region
BOX_CPU_SHARE = 16  # host cores of one GPU's share on the GPU box (os.cpu_count() shows the host)
SHAPE_DEFAULTS = {  # shape -> (algo, n_factors, scaling)
    "ml-1m": ("svd", 100, "weak"),
    "c4": ("svd", 128, "strong"),
    "c5": ("svdpp", 128, "strong"),
}


_T0 = time.time()


def note(msg):
    """Progress on stderr (a long run keeps writing: the GPU pool's watchdog sees it alive)."""
    print("[bench %6.1fs] %s" % (time.time() - _T0, msg), file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--shape", default="ml-1m", choices=sorted(SHAPE_DEFAULTS))
    p.add_argument("--hot-rows", type=int, default=-1,
                   help="SVD++ helper-wave launch: q rows with a delta replica (-1: the engine's "
                        "policy, engine.hot_items)")
    p.add_argument("--replay-rows", type=int, default=0,
                   help="SVD checkpoint log: ratings per replay piece (0: the engine's policy, "
                        "engine.replay_piece_rows)")
    p.add_argument("--heavy", type=float, default=-1,
                   help="SVD checkpoint log: users in the heavy launch (MFEngine heavy; -1: the "
                        "engine's policy)")
    p.add_argument("--gram", type=int, default=-1,
                   help="SVD checkpoint log: the heavy users by the blocked solve (1) or the "
                        "lookahead chain (0); -1: the engine's policy")
    p.add_argument("--xcd-split", type=int, default=-1,
                   help="SVD checkpoint log: heavy launch on XCD 0, the rest on XCDs 1-7 (1 / 0; "
                        "-1: the engine's policy)")
    p.add_argument("--hx-helpers", type=int, default=0,
                   help="SVD++ helper-wave launch: helper waves per chain, 3 or 1 (0: the "
                        "engine default)")
    p.add_argument("--hx-chains", type=int, default=0,
                   help="SVD++ helper-wave launch: user chains per CU (0: the engine default)")
    p.add_argument("--algo", default=None, choices=["svd", "svdpp"])
    p.add_argument("--factors", type=int, default=None)
    p.add_argument("--mode", default="auto")
    p.add_argument("--dtype", default=None, choices=["f32", "f64"],
                   help="device arithmetic; default f64 (the reference's: mf.pyx:207-227) for "
                        "ml-1m, f32 for c4 / c5 (fp64 K=128 item rows exceed the 1 KiB "
                        "lookahead layout and the fp64 log would not fit C4 on one GPU)")
    p.add_argument("--chunks", type=int, default=0,
                   help="epoch-chunks (0: the engine's default, engine.default_chunks)")
    p.add_argument("--merge", default=None, choices=["count", "recency"],
                   help="log schedule's item fold (default: the engine's)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-rmse", action="store_true")
    p.add_argument("--no-svdpp", action="store_true", help="skip the SVD++ C3 leg")
    p.add_argument("--no-predict", action="store_true", help="skip the batched test() leg")
    p.add_argument("--no-chain-probe", action="store_true",
                   help="skip timing the heaviest user's chain alone (profiling runs: its extra "
                        "epoch-kernel launches would mix into the kernel's statistics)")
    p.add_argument("--top", type=int, default=-1,
                   help="split chunk: heavy users kept on the main stream, the rest of the heavy "
                        "launch beside them (engine option top; -1: the engine's default, 0: off)")
    p.add_argument("--qlog", type=int, nargs="?", const=1, default=-1,
                   help="SVD++: 1 (or bare --qlog) the q log (item rows read-only per chunk, "
                        "gradients logged and folded after it; engine option qlog), 0 the "
                        "float-atomic schedule; default: the engine's auto_qlog (the q log on one "
                        "rank with several chunks of <= 10 ratings per item: C5)")
    p.add_argument("--no-c4", action="store_true",
                   help="skip the C4 leg (BASELINE configs[3]'s shape on this GPU)")
    p.add_argument("--light-replay-wpc", type=int, default=-1,
                   help="split chunk: the light group's replay waves per CU (engine option "
                        "light_replay_wpc; -1: the engine's default)")
    p.add_argument("--log-nt", default="-1", choices=("-1", "0", "1", "heavy", "light"),
                   help="the log's stores non-temporal (engine option log_nt; -1: the engine's "
                        "size rule, 0 off, 1 on, heavy / light: that launch group only)")
    p.add_argument("--cold-share", type=float, default=-1,
                   help="SVD++ helper-wave launch: the least-rated items holding this share of a "
                        "chunk's ratings on the cold log (engine option cold_share; -1: the "
                        "engine's default)")
    p.add_argument("--bias-mirror", type=int, default=-1,
                   help="checkpoint log with SB rows: the item biases from a mirror array, rows "
                        "on 128-B lines (engine option bias_mirror; -1: the engine's default, on)")
    p.add_argument("--item-align", type=int, default=0,
                   help="item rows padded to a multiple of this many bytes (engine option "
                        "item_align, timing probes; 0: the engine's 64)")
    p.add_argument("--stagger", type=int, default=-1,
                   help="checkpoint log: the chunk's users in two staggered halves (engine option "
                        "stagger; -1: the engine's policy, 0 off, 1 on)")
    p.add_argument("--long-chain", type=int, default=-1,
                   help="epoch-chunk dealing: users of > 1/N of a chunk's ratings all in chunk 0 "
                        "(engine option long_chain; -1: the engine's 256, 0: round-robin)")
    p.add_argument("--users", type=int, default=0,
                   help="c4 / c5: train only the first N users of the shape (a user-prefix "
                        "subsample that keeps every item; 0 = all)")
    p.add_argument("--rmse-epochs", type=int, default=20)
    p.add_argument("--oracle", action="store_true",
                   help="c4 / c5 at N=1: also train the fp64 sequential oracle on the same CSR "
                        "and initial factors in the rmse leg (single host thread)")
    p.add_argument("--detail", default=None,
                   help="where the full result dictionary goes (the stdout line is its compact "
                        "summary, compact_line); default gpurun_out/bench_detail_<shape>_n<N>.json")
    p.add_argument("--backend", default="nccl",
                   help="torch.distributed backend for N>1 (nccl = RCCL; gloo only to rehearse "
                        "several ranks on one GPU)")
    a = p.parse_args()
    algo, K, scaling = SHAPE_DEFAULTS[a.shape]
    a.algo = a.algo or algo
    a.factors = a.factors or K
    a.scaling = scaling
    a.legs = a.dtype is None  # the default run adds the other precision's leg (N=1, ml-1m)
    a.dtype = a.dtype or ("f64" if a.shape == "ml-1m" else "f32")
    return a


TORCH_DTYPE = {"f32": "float32", "f64": "float64"}
ELEM_BYTES = {"f32": 4, "f64": 8}


def algorithmic_bytes_per_update(algo, K, s=4):
    """SVD 12 + 4 s (K+1); SVD++ adds one read + one write of y_j: + 2 s K."""
    b = 12 + 4 * s * (K + 1)
    if algo == "svdpp":
        b += 2 * s * K
    return b


def spawn_ranks(n):
    """--gpus N without a launcher: N fresh child processes (one per GPU), started before this
    process touches any GPU; exits with the first failing child's code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc]
    sys.exit(bad[0] if bad else 0)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ---------------------------------------------------------------------------- workloads
def workload(args, rank, world):
    """This rank's training CSR (rank-local rows), held-out triples (local user ids), item
    count, the rank's train-rating sum (for the global mean) and a description."""
    from surprise_amd import synthetic
    from surprise_amd.dist import shard_users
    from surprise_amd.model_selection import KFold
    from surprise_amd.trainset import Trainset
    if args.shape == "ml-1m":
        U, I, N = synthetic.SHAPES["ml-1m"]
        u, i, r = synthetic.population(rank, U, I, N)
        tr, te = next(KFold(5, random_state=0).fold_indices(len(r)))
        ts = Trainset.from_inner_arrays(u[tr], i[tr], r[tr], n_users=U, n_items=I)
        desc = ("ML-1M-shape user population %d of %d (%d users x %d items), KFold(5, rs=0) fold "
                "0" % (rank, world, U, I))
        return ts.csr(), (u[te], i[te], r[te]), I, U * world, desc
    U, I, N = synthetic.SHAPES[args.shape]
    truth = synthetic.sharded_truth(U, I, N)
    n_users = min(args.users, U) if args.users else U
    row_ptr = np.concatenate([[0], np.cumsum(truth["deg"][:n_users])])
    b = shard_users(row_ptr, world)
    csr, test = synthetic.sharded_rows(truth, int(b[rank]), int(b[rank + 1]),
                                       threads=max(1, min(16, len(os.sched_getaffinity(0)))))
    desc = ("%s shape (%d users x %d items x %d ratings, 1%% held out)%s, users [%d, %d) on this "
            "rank" % (args.shape, U, I, N, ", first %d users" % n_users if n_users < U else "",
                      b[rank], b[rank + 1]))
    workload.user_lo = int(b[rank])
    return csr, test, I, n_users, desc


def init_tables(shape, rank, n_users, n_items, K, svdpp, user_lo=0):
    """Initial factors: N(0, 0.1) as SVD.sgd draws them.  ML-1M: get_rng(0) pu then qi (then
    yj), the reference's own sequence (the rmse leg's oracle uses the same draws); other
    populations' users draw from their own stream.  c4 / c5: per user block (the generator's
    blocks), so that a user's initial row does not depend on the number of ranks."""
    if shape != "ml-1m":
        from surprise_amd.synthetic import BLOCK_USERS
        rng = np.random.RandomState([0, 6])
        qi = rng.normal(0, .1, (n_items, K))
        yj = rng.normal(0, .1, (n_items, K)) if svdpp else None
        hi = user_lo + n_users
        rows = []
        for b in range(user_lo // BLOCK_USERS, -(-hi // BLOCK_USERS)):
            b0 = b * BLOCK_USERS
            blk = np.random.RandomState([0, 5, b]).normal(0, .1, (BLOCK_USERS, K))
            rows.append(blk[max(user_lo - b0, 0):min(hi - b0, BLOCK_USERS)])
        pu = np.concatenate(rows) if rows else np.zeros((0, K))
        return pu, qi, yj
    rng = np.random.RandomState(0)
    pu = rng.normal(0, .1, (n_users, K))
    qi = rng.normal(0, .1, (n_items, K))
    yj = rng.normal(0, .1, (n_items, K)) if svdpp else None
    if rank > 0:  # other ranks' users: their own stream; item tables identical on every rank
        pu = np.random.RandomState([0, rank]).normal(0, .1, (n_users, K))
    return pu, qi, yj


def hyper_for(algo, gm):
    lr = .007 if algo == "svdpp" else .005  # SVDpp / SVD defaults (mf.pyx:398-407, :140-147)
    return dict(lr_bu=lr, lr_bi=lr, lr_pu=lr, lr_qi=lr, lr_yj=lr, reg_bu=.02, reg_bi=.02,
                reg_pu=.02, reg_qi=.02, reg_yj=.02, global_mean=float(gm))


# ---------------------------------------------------------------------------- timing
def run_steps(eng, ctx, steps, warmup, torch, instrument=True):
    """Warmup, then `steps` epochs between barriers + synchronize (no timing events inside the
    timed region), then -- instrument -- PHASE_STEPS more epochs carrying HIP events on the
    engine's stream around each phase (a recorded timing event idles the GPU for a few us).
    Returns (seconds of the timed region, phases of the instrumented epochs)."""
    for _ in range(warmup):
        for c in range(eng.n_chunks):
            eng.run_chunk(c)
            eng.sync_items(ctx)
    torch.cuda.synchronize()
    if ctx is not None:
        ctx.barrier()
    torch.cuda.synchronize()
    recs = []
    t0 = time.perf_counter()
    for step in range(steps):
        for c in range(eng.n_chunks):
            eng.run_chunk(c)
            eng.sync_items(ctx)
    t_enq = time.perf_counter() - t0  # (the host's enqueue time: below elapsed unless host-bound)
    torch.cuda.synchronize()
    if ctx is not None:
        ctx.barrier()
    elapsed = time.perf_counter() - t0
    multi = ctx is not None and ctx.world > 1
    for step in range(PHASE_STEPS if instrument else 0):
        for c in range(eng.n_chunks):
            ev = {k: torch.cuda.Event(enable_timing=True)
                  for k in ("begin", "start", "end", "end_h", "end_r", "done", "ar_begin",
                            "ar_end", "l_start", "l_end", "m_start", "m_end")}
            ev["begin"].record(eng.stream)
            eng.run_chunk(c, events=ev)
            if multi:  # (the collective of the chunk's exchange, bracketed on the stream)
                eng._sync_events = ev
            eng.sync_items(ctx)
            eng._sync_events = None
            ev["done"].record(eng.stream)
            ev["chunk"] = c
            recs.append(ev)
    torch.cuda.synchronize()
    phases = {"host_enqueue_ms": t_enq / max(steps, 1) * 1e3}
    if recs:
        span = lambda a, b: float(np.mean([e[a].elapsed_time(e[b]) for e in recs]))
        n = eng.n_chunks
        phases.update({"pre_ms": span("begin", "start") * n, "epoch_kernel_ms": span("start", "end") * n,
                  "replay_ms": span("end", "end_r") * n, "fold_sync_ms": span("end_r", "done") * n,
                  "step_gpu_ms": span("begin", "done") * n, "instrumented_steps": len(recs) // n})
        # the epoch kernel (the dominant kernel): each launch's span on its own stream, the
        # ratings it trains, and the kernel's wall span per chunk -- its launches of a split chunk
        # (heavy users on the main stream, the rest on the side stream) run concurrently, so
        # the span is from the first launch's start to the last one's end
        per_launch, spans = {}, []
        for e in recs:
            n_r = eng.epoch_launch_ratings(e["chunk"])
            t_main = e["start"].elapsed_time(e["end"])
            if len(n_r) > 1:
                t0 = e["start"].elapsed_time(e["l_start"])
                t1 = e["start"].elapsed_time(e["l_end"])
                per_launch.setdefault("heavy", []).append((t_main, n_r[0]))
                per_launch.setdefault("light", []).append((t1 - t0, n_r[1]))
                lo, hi = min(0.0, t0), max(t_main, t1)
                if len(n_r) > 2:  # (the heavy launch's rest on the third stream, engine `top`)
                    m0 = e["start"].elapsed_time(e["m_start"])
                    m1 = e["start"].elapsed_time(e["m_end"])
                    per_launch.setdefault("mid", []).append((m1 - m0, n_r[2]))
                    lo, hi = min(lo, m0), max(hi, m1)
                spans.append((hi - lo, sum(n_r)))
            else:
                per_launch.setdefault("all", []).append((t_main, n_r[0]))
                spans.append((t_main, n_r[0]))
        steps_i = max(len(recs) // n, 1)
        phases["epoch_kernel"] = {
            "span_ms_per_step": float(np.sum([t for t, _ in spans])) / steps_i,
            "ratings_per_step": float(np.sum([r for _, r in spans])) / steps_i,
            "launches": {k: {"per_step": len(v) / steps_i,
                             "avg_us": float(np.mean([t for t, _ in v])) * 1e3,
                             "ratings": float(np.mean([r for _, r in v]))}
                         for k, v in per_launch.items()}}
        if multi:  # the exchange: one SUM all-reduce per chunk (ms per chunk and per step)
            ar = span("ar_begin", "ar_end")
            phases.update({"allreduce_ms_per_chunk": ar, "allreduce_ms": ar * n,
                           "allreduce_bytes_per_chunk": int(eng._delta_buffer()[0].numel()
                                                            * eng._delta_buffer()[0].element_size())})
    return elapsed, phases


def max_over_ranks(ctx, x, torch):
    if ctx is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    ctx.all_reduce_max(t)
    return float(t.item())


def sum_over_ranks(ctx, xs, torch):
    if ctx is None:
        return list(xs)
    t = torch.tensor(list(xs), dtype=torch.float64, device="cuda")
    ctx.all_reduce_sum(t)
    return t.cpu().tolist()


def shape_key(shape, users=0):
    """Name of a workload's measured-traffic file: the shape, with _u<N> for a c4 / c5 user
    prefix (the C5 shard is c5_u1250000; the full 1B-rating C5 is c5)."""
    return shape + ("_u%d" % users if users and shape in ("c4", "c5") else "")


def traffic_for(algo, K, shape, dtype="f32", qlog=False):
    """Measured HBM-side bytes per step (profiles/traffic_<algo>_k<K>_<shape>[_f64][_qlog].json,
    written by tools/profile.sh from separate rocprofv3 --pmc passes; SVD++ on the q log has its
    own file -- the atomic schedule's bytes are not its)."""
    name = "traffic_%s_k%d_%s%s%s.json" % (algo, K, shape, "" if dtype == "f32" else "_" + dtype,
                                          "_qlog" if qlog else "")
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        t = json.load(f)
    return t.get("bytes_per_step"), t


# ---------------------------------------------------------------------------- CPU baseline
def physical_cores():
    """Physical cores of the host (distinct (package, core id) pairs of /proc/cpuinfo)."""
    seen, pkg = set(), None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                pkg = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                seen.add((pkg, line.split(":", 1)[1].strip()))
    except OSError:
        pass
    return len(seen) or os.cpu_count()


def cpu_baselines(csr, n_items, K, n_train):
    """The fp64 C restatement (oracle/) on this host: one pinned core (in-process affinity) for
    ~10 s, then every core of this process's share at once (one pinned child process per core,
    ~10 s each).  Bounded samples of the same workload: whole epochs over the same fold."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    row_ptr, items, ratings = csr
    cores = sorted(os.sched_getaffinity(0))
    share = cores[:BOX_CPU_SHARE]
    old = set(cores)
    os.sched_setaffinity(0, {share[0]})
    try:
        e, t1 = 0, 0.0
        while t1 < 10.0 and e < 2000:
            step = max(1, min(50, int(e * (10.0 - t1) / t1))) if t1 > 0 else 1
            t1 += orc.time_svd_epochs(row_ptr, items, ratings, n_items, K, step, seed=e)
            e += step
    finally:
        os.sched_setaffinity(0, old)
    rate1 = n_train * e / t1
    per_core_epochs = max(1, int(round(10.0 * rate1 / n_train)))
    with tempfile.TemporaryDirectory() as d:
        for name, a in (("row_ptr", row_ptr), ("items", items), ("ratings", ratings),
                        ("n_items", np.asarray(n_items))):
            np.save(os.path.join(d, name + ".npy"), a)
        w = os.path.join(ROOT, "oracle", "cpu_worker.py")
        t0 = time.perf_counter()
        procs = [subprocess.Popen([sys.executable, w, d, str(c), str(per_core_epochs), str(K)],
                                  stdout=subprocess.PIPE, text=True) for c in share]
        outs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in procs]
        wall = time.perf_counter() - t0
    ups = sum(o["updates"] for o in outs)
    compute = max(o["seconds"] for o in outs)
    cal = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["calibration"]
    ratio = cal["oracle_over_reference"]
    phys = physical_cores()
    per_core_loaded = ups / compute / len(share)
    return {
        "value": ups / compute, "unit": "rating-updates/s", "cores": len(share), "kind": "port",
        "sample": "fp64 C restatement of SVD.sgd (oracle/mf_oracle.c <- mf.pyx:241-262), SVD K=%d, "
                  "%d pinned processes x %d epochs over the same %d-rating train fold (wall incl. "
                  "process start %.1fs)" % (K, len(share), per_core_epochs, n_train, wall),
        "host_cpus": os.cpu_count(), "cpus_allowed": len(cores), "cpu_model": cpu_model(),
        "single_core": {"value": rate1, "cores": 1, "pinned": True,
                        "sample": "%d epochs on core %d (%.1fs)" % (e, share[0], t1),
                        "cython_equivalent_derived": rate1 / ratio},
        "node_physical_cores": phys,
        "all_cores_derived": {
            "value": per_core_loaded * phys, "cores": phys,
            "note": "NOT measured: the per-core rate under the %d-process load x the node's "
                    "physical cores. This pool caps one GPU's job at its CPU share (%d CPUs; "
                    "os.cpu_count() shows the whole host), so the node's other cores are not "
                    "ours to load; the extrapolation assumes linear scaling (optimistic for the "
                    "CPU: 128 processes share the memory system)" % (len(share), BOX_CPU_SHARE)},
        "calibration_oracle_over_cython": ratio,
        "calibration_note": "the restatement / compiled reference Cython rate, both timed in the "
                            "build container on the same fold (tests/golden/golden.json)",
    }


def cpu_baseline_svdpp(csr, n_items, K, n_train, target_s=8.0):
    """SVD++ C3 beside the GPU: the fp64 C restatement of SVDpp.sgd in the reference's
    per-rating form (oracle_svdpp_sgd <- mf.pyx:463-498: u_impl re-summed over I_u and every
    y_j of I_u stepped, per rating, so a user's epoch costs ~ n_u^2 K).  A whole full-fold epoch
    is minutes of CPU, so the bounded sample is one epoch over a user prefix of the same fold
    sized to ~target_s on one core; the full-fold epoch time is that time x sum_all(n_u^2) /
    sum_prefix(n_u^2) (the per-(rating x |I_u|) cost is flat: 485-486 ns at 100 and 300 users in
    the build container).  One pinned core, then one pinned process per core of the box's share
    on the same sample.  Context: the per-user affine form (O(K) per rating, the GPU kernels'
    algebra) on one core over the whole fold."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    row_ptr, items, ratings = (np.asarray(a) for a in csr)
    deg2 = np.diff(row_ptr).astype(np.float64) ** 2
    cum = np.cumsum(deg2)
    s_all = float(cum[-1])
    cores = sorted(os.sched_getaffinity(0))
    share = cores[:BOX_CPU_SHARE]
    old = set(cores)

    def prefix(s_target):
        nu = int(min(len(deg2), np.searchsorted(cum, s_target) + 1))
        k1 = int(row_ptr[nu])
        return nu, (row_ptr[:nu + 1], items[:k1], ratings[:k1]), float(cum[nu - 1])

    os.sched_setaffinity(0, {share[0]})
    try:
        nu0, sub0, s0 = prefix(2e6)
        t0 = orc.time_svdpp_epochs(*sub0, n_items, K, 1)
        nu, sub, s_smp = prefix(target_s * s0 / max(t0, 1e-6))
        t1 = orc.time_svdpp_epochs(*sub, n_items, K, 1)
        t_aff = orc.time_svdpp_epochs(row_ptr, items, ratings, n_items, K, 1, affine=True)
    finally:
        os.sched_setaffinity(0, old)
    full1 = t1 * s_all / s_smp  # one core's full-fold epoch (derived from the sample)
    with tempfile.TemporaryDirectory() as d:
        for name, a in zip(("row_ptr", "items", "ratings"), sub):
            np.save(os.path.join(d, name + ".npy"), a)
        np.save(os.path.join(d, "n_items.npy"), np.asarray(n_items))
        w = os.path.join(ROOT, "oracle", "cpu_worker.py")
        tw = time.perf_counter()
        procs = [subprocess.Popen([sys.executable, w, d, str(c), "1", str(K), "svdpp"],
                                  stdout=subprocess.PIPE, text=True) for c in share]
        outs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in procs]
        wall = time.perf_counter() - tw
    full_n = max(o["seconds"] for o in outs) * s_all / s_smp  # the slowest core's full epoch
    return {
        "value": len(share) * n_train / full_n, "unit": "rating-updates/s", "cores": len(share),
        "kind": "port",
        "sample": "fp64 C restatement of SVDpp.sgd in the reference's per-rating form "
                  "(oracle/mf_oracle.c oracle_svdpp_sgd <- mf.pyx:463-498), SVD++ K=%d: one epoch "
                  "over the first %d users (%d ratings, sum n_u^2 = %.3g of the fold's %.3g) on "
                  "each of %d pinned processes (wall incl. process start %.1fs); value = %d x "
                  "the fold's %d ratings / the slowest process's epoch time scaled by the "
                  "sum n_u^2 ratio (%.1f s per full-fold epoch per core)"
                  % (K, nu, int(sub[0][-1]), s_smp, s_all, len(share), wall, len(share),
                     n_train, full_n),
        "single_core": {"value": n_train / full1, "cores": 1, "pinned": True,
                        "full_fold_epoch_s_derived": full1,
                        "sample": "one epoch over the first %d users on core %d: %.2fs"
                                  % (nu, share[0], t1)},
        "affine_form_single_core": {
            "value": n_train / t_aff, "cores": 1, "pinned": True,
            "note": "context, not the reference's cost: the per-user affine reformulation "
                    "(oracle_svdpp_sgd_affine, O(K) per rating -- the algebra the GPU kernels "
                    "use), one full-fold epoch (%.2fs)" % t_aff},
        "host_cpus": os.cpu_count(), "cpus_allowed": len(cores), "cpu_model": cpu_model(),
    }


# ---------------------------------------------------------------------------- main
def layout_of(eng):
    """What the executed-byte model needs of an engine: element size, row strides, the log's
    form, and per epoch-kernel launch the ratings and users it trains (chunk 0 = every chunk's
    shape: chunks deal users round-robin)."""
    s = eng.pu.element_size()
    lay = {"s": s, "K": eng.K, "ldq": eng.ldq, "ld": eng.ld, "algo": eng.algo,
           "ckpt": bool(eng.ckpt), "narrow": bool(getattr(eng, "narrow", False)),
           "err_in_row": bool(eng.ckpt and eng.err_in_row),
           "ldc": int(getattr(eng, "ldc", eng.ldq)), "hx": bool(getattr(eng, "hx", False)),
           "n_items": eng.n_items, "n_chunks": eng.n_chunks, "launches": {}}
    deg = np.diff(eng._row_ptr_h)
    for c in range(eng.n_chunks):
        lg = eng.logs[c] if eng.ckpt else None
        groups = ([("heavy", lg["heavy"]), ("light", lg)] if lg is not None and lg["heavy"]
                  else [("all", lg)])
        if lg is not None and lg.get("mid") is not None:
            groups.append(("mid", lg["mid"]))
        for name, g in groups:
            us = (g["sched"] if g is not None else eng.sched[c]).cpu().numpy()
            us = us[us >= 0]
            d = lay["launches"].setdefault(name, {"ratings": 0, "users": 0, "pieces": 0})
            d["ratings"] += int(deg[us].sum())
            d["users"] += len(us)
            d["pieces"] += int(g["n_pieces"]) if g is not None else 0
    return lay


def executed_bytes(lay, ratings, users, pieces=0, whole_step=False):
    """Bytes the launch (or, whole_step, the whole step's kernels) must move by the work it
    executes -- every array it reads or writes once per use, caches ignored:
      SVD checkpoint log, epoch kernel: per rating the CSR entry (4 + s), the item row gather
        ((K + 2) s: factors, b_i, the constant column of the user bias; narrow rows: (K + 1) s)
        and half a packed checkpoint row (ldc s / 2, + s of elog when the errors are not in the
        rows); per user its row read and written once (2 (K + 1) s) + row_ptr / sched / user_sq;
        whole step adds the replay (per rating its pair's row ldc s + perm / ck / rpos 12 B
        (+ s elog); per piece the item row and the piece sums) and the fold (per piece the sums,
        per item its row read + written).
      SVD++ helper-wave launch: per rating the CSR entry, the q row read and its delta atomic
        (2 (K + 1) s) and the y row of the user's start-of-user implicit sum (K s); per user its
        row read + written and its y map (c_u) written; whole step adds the y fold (per rating
        the user's c_u row, per item its y row read + written).
    SURVEY 8(d)'s figure (12 + 4 s (K + 1) per update, + 2 s K for SVD++) also counts a p_u gather
    and scatter per rating, which the register-resident user row never performs."""
    s, K, ldq = lay["s"], lay["K"], lay["ldq"]
    if lay["algo"] == "svd" and lay["ckpt"]:
        q = (K + 1) * s if lay["narrow"] else (K + 2) * s
        log = lay["ldc"] * s / 2 + (0 if lay["err_in_row"] else s)
        b = ratings * (4 + s + q + log) + users * (2 * (K + 1) * s + 16 + 4 + 8)
        if whole_step:
            b += ratings * (lay["ldc"] * s + 12 + (0 if lay["err_in_row"] else s))
            b += pieces * ((K + 1) * s + 2 * ldq * s + 8)
            b += lay["n_chunks"] * lay["n_items"] * (2 * ldq * s + 8)
        return b
    if lay["algo"] == "svdpp":
        b = ratings * (4 + s + 2 * (K + 1) * s + K * s) + users * (2 * (K + 1) * s + K * s + 20)
        if whole_step:
            b += ratings * (K * s + 4) + lay["n_chunks"] * lay["n_items"] * 2 * lay["ld"] * s
        return b
    return ratings * algorithmic_bytes_per_update(lay["algo"], K, s)


def roofline_of(algo, K, dtype, n_train, ms_step, shape, phases=None, lay=None, chain=None,
                qlog=False):
    """The dominant kernel's roofline.  The dominant kernel is the epoch kernel; one "launch" in
    the contract's sense is its invocation over one step's ratings, whose launches of a split
    chunk (the heavy users' on XCD 0, the others' on XCDs 1-7) run concurrently -- so its
    duration is their wall span (HIP events on both streams, the instrumented epochs after the
    timed region) and kernel time per step never exceeds the step.  achieved = the executed
    bytes of that work (executed_bytes) / the span; each launch is also reported on its own
    (heavy = the critical path), the whole step beside it, and SURVEY 8(d)'s byte figure as a
    labelled rate (no frac: it counts traffic the kernel does not perform).  traffic = the
    kernel's measured HBM bytes per step (2 x FETCH_SIZE + WRITE_SIZE, profiles/traffic_*).
    chain: the heaviest user's chain timed alone -- the latency roof of the critical launch."""
    s = ELEM_BYTES[dtype]
    B8 = algorithmic_bytes_per_update(algo, K, s)
    traffic, tinfo = traffic_for(algo, K, shape, dtype, qlog)
    ek = (phases or {}).get("epoch_kernel")
    kname = ("mf_svdpp_qlog_kernel" if qlog else "mf_svdpp_hx_kernel") if algo == "svdpp" \
        else "mf_ckpt_epoch_kernel"
    gbs = lambda b, ms: b / (ms * 1e-3) / 1e9
    out = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    if not (ek and lay):
        a = gbs(B8 * n_train, ms_step)
        out.update(achieved=a, frac=a / HBM_PEAK_GBS, traffic=traffic)
        return out
    L = lay["launches"]
    tot_r = sum(v["ratings"] for v in L.values())
    tot_u = sum(v["users"] for v in L.values())
    tot_p = sum(v["pieces"] for v in L.values())
    ex = executed_bytes(lay, tot_r, tot_u)
    span = ek["span_ms_per_step"]
    k_traffic = None
    if tinfo and kname in (tinfo.get("per_kernel") or {}):
        k_traffic = tinfo["per_kernel"][kname]["bytes_per_step"]
    a = gbs(ex, span)
    out.update(achieved=a, frac=a / HBM_PEAK_GBS, traffic=k_traffic)
    if k_traffic:
        # the measured HBM bytes over the same span: where the executed bytes come largely from
        # L2 / MALL (ML-1M's item table is cache-resident) this is the HBM fraction proper
        out["traffic_frac"] = gbs(k_traffic, span) / HBM_PEAK_GBS
    launches = {}
    for name, v in ek["launches"].items():
        lv = L.get(name, {"users": 0})
        b = executed_bytes(lay, v["ratings"], lv["users"] / max(lay["n_chunks"], 1))
        launches[name] = {"avg_us": v["avg_us"], "per_step": v["per_step"],
                          "ratings": v["ratings"], "executed_bytes": b,
                          "achieved": gbs(b, v["avg_us"] * 1e-3),
                          "frac": gbs(b, v["avg_us"] * 1e-3) / HBM_PEAK_GBS}
    step_b = executed_bytes(lay, tot_r, tot_u, tot_p, whole_step=True)
    out["dominant_kernel"] = {
        "kernel": kname, "unit": "its invocation over one step's %d ratings (%d launch(es), "
                                 "concurrent when split)" % (tot_r, len(launches)),
        "span_us_per_step": span * 1e3, "executed_bytes_per_step": ex,
        "executed_bytes_per_update": ex / max(tot_r, 1), "traffic_per_step": k_traffic,
        "launches": launches}
    out["step"] = {"ms": ms_step, "executed_bytes": step_b, "achieved": gbs(step_b, ms_step),
                   "frac": gbs(step_b, ms_step) / HBM_PEAK_GBS, "traffic": traffic,
                   "traffic_frac": (gbs(traffic, ms_step) / HBM_PEAK_GBS) if traffic else None}
    out["survey_8d"] = {"bytes_per_update": B8, "rate_over_span": gbs(B8 * tot_r, span),
                        "rate_over_step": gbs(B8 * n_train, ms_step),
                        "note": "SURVEY 8(d)'s algorithmic figure, a rate only (no frac): it "
                                "counts a p_u gather + scatter per rating that the register-"
                                "resident user row never performs"}
    if chain:
        crit = launches.get("heavy", launches.get("all"))
        chain = dict(chain)
        if crit:
            chain["critical_launch_us"] = crit["avg_us"]
            chain["frac"] = chain["alone_us"] / crit["avg_us"]
        out["critical_path_bound"] = "chain latency: the heaviest user's ratings are sequential"
        out["chain_latency"] = chain
    if lay.get("hx"):
        # the SVD++ helper-wave launch adds each rating's q row (ldq columns: factors, b_i,
        # padding) by memory-side float atomics: its own roof is the chip's atomic rate
        # (factor columns filling whole 512-B lane groups: the bias rides beside them, K + 1
        # columns added; otherwise the whole padded row, ldq columns)
        cols = lay["K"] + 1 if (lay["K"] * s) % 512 == 0 else lay["ldq"]
        added = tot_r * cols * s
        a_at = gbs(added, span)
        out["atomic_roof"] = {
            "added_bytes_per_step": added, "achieved": a_at,
            "peak": ATOMIC_F32_GBS if s == 4 else None,
            "frac": a_at / ATOMIC_F32_GBS if s == 4 else None,
            "note": "float atomics' chip-wide added-byte rate (MI355X_MICROARCH.md, fp32 "
                    "global_atomic_add_f32); fp64 adds have no guide figure (null)"}
    out["traffic_breakdown"] = tinfo.get("per_kernel") if tinfo else None
    out["traffic_source"] = tinfo.get("source") if tinfo else None
    return out


def time_top_chain(eng, torch, reps=3):
    """The heaviest user's chain alone on the GPU (one wave, the product epoch kernel with its
    checkpoint rows): the latency roof of a launch that trains that user.  Run after the
    instrumented epochs (it moves that user's row and log rows; nothing reads them after)."""
    if not (eng.algo == "svd" and eng.ckpt):
        return None
    deg = np.diff(eng._row_ptr_h)
    top = int(np.argmax(deg))
    sched = torch.tensor([top], dtype=torch.int32, device=eng.dev)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(eng.stream)
        eng._heavy_epoch(sched, 1, eng._st())  # (the kernel the heavy launch uses)
        b.record(eng.stream)
        eng.stream.synchronize()
        ts.append(a.elapsed_time(b))
    t = float(np.median(ts)) * 1e3
    return {"top_user_ratings": int(deg[top]), "alone_us": t,
            "ns_per_rating": t * 1e3 / max(int(deg[top]), 1), "reps": reps,
            "kernel": "mf_svd_gram_kernel (blocked solve)" if eng.gram else
                      "mf_ckpt_epoch_kernel (lookahead chain)"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1:
        spawn_ranks(args.gpus)  # exits
    rank = int(os.environ.get("RANK", "0"))
    if args.shape in ("c4", "c5") and rank == 0:
        # the full C5 (1B ratings) spends minutes in host-side generation and in the engine's
        # per-chunk preparation: a heartbeat keeps the run visibly alive meanwhile
        import threading

        def beat():
            while True:
                time.sleep(45)
                note("alive")
        threading.Thread(target=beat, daemon=True).start()

    # host-side workload first (no GPU touched yet)
    csr, test, n_items, n_users_global, desc = workload(args, rank, world)
    row_ptr, items, ratings = csr
    n_train = int(row_ptr[-1])
    note("workload ready: %d training ratings on rank %d" % (n_train, rank))

    import torch
    from surprise_amd.dist import DistContext
    from surprise_amd.engine import MFEngine, default_ld
    ctx = None
    if world > 1:
        ctx = DistContext.from_env(args.backend)
    else:
        torch.cuda.set_device(0)
    # global mean of the training ratings over all ranks (one value for the model)
    tot, cnt = sum_over_ranks(ctx, [float(ratings.sum()), float(n_train)], torch)
    gm = tot / cnt
    K, algo = args.factors, args.algo
    mode = args.mode if args.mode != "auto" else ("atomic" if algo == "svdpp" else "log")
    n_users = len(row_ptr) - 1

    from surprise_amd.engine import default_chunks

    def make_engine(a=algo, k=K, md=mode, dt=args.dtype):
        pu, qi, yj = init_tables(args.shape, rank, n_users, n_items, k, a == "svdpp",
                                 getattr(workload, "user_lo", 0))
        eng = MFEngine(csr, n_items, k, algo=a, hyper=hyper_for(a, gm), mode=md,
                       dtype=TORCH_DTYPE[dt], world=world,
                       n_chunks=args.chunks or default_chunks(a, md, n_users_global, world),
                       **({"merge": args.merge} if args.merge else {}),
                       **({"hx_chains_per_cu": args.hx_chains} if args.hx_chains else {}),
                       **({"helpers": args.hx_helpers} if args.hx_helpers else {}),
                       **({"heavy": args.heavy} if args.heavy >= 0 else {}),
                       **({"hot_rows": args.hot_rows} if args.hot_rows >= 0 else {}),
                       **({"qlog": bool(args.qlog)} if args.qlog >= 0 and a == "svdpp"
                          else {}),
                       **({"top": args.top} if args.top >= 0 else {}),
                       **({"replay_rows": args.replay_rows} if args.replay_rows else {}),
                       **({"gram": bool(args.gram)} if args.gram >= 0 else {}),
                       **({"xcd_split": bool(args.xcd_split)} if args.xcd_split >= 0 else {}),
                       **({"long_chain": args.long_chain} if args.long_chain >= 0 else {}),
                       **({"stagger": bool(args.stagger)} if args.stagger >= 0 else {}),
                       **({"item_align": args.item_align} if args.item_align else {}),
                       **({"cold_share": args.cold_share} if args.cold_share >= 0 and
                          a == "svdpp" else {}),
                       **({"bias_mirror": bool(args.bias_mirror)} if args.bias_mirror >= 0
                          else {}),
                       **({"log_nt": args.log_nt if args.log_nt in ("heavy", "light")
                           else bool(int(args.log_nt))} if args.log_nt != "-1" else {}),
                       **({"light_replay_wpc": args.light_replay_wpc}
                          if args.light_replay_wpc >= 0 else {}))
        eng.set_factors(pu, qi, yj=yj)
        eng._prepare(ctx)  # global per-item counts (all ranks)
        return eng

    torch.cuda.reset_peak_memory_stats()
    eng = make_engine()
    note("engine ready")
    elapsed, phases = run_steps(eng, ctx, args.steps, args.warmup, torch)
    note("timed steps done")
    elapsed = max_over_ranks(ctx, elapsed, torch)
    dev_bytes = max_over_ranks(ctx, float(torch.cuda.max_memory_allocated()), torch)
    updates = sum_over_ranks(ctx, [float(n_train)], torch)[0] * args.steps
    value = updates / elapsed
    ms_step = elapsed / args.steps * 1e3
    headline = (algo, K, args.shape) == ("svd", 100, "ml-1m")

    result = {
        "metric": "rating-updates/sec/GPU, SVD n_factors=100; RMSE delta vs Cython ref"
        if headline else
        "rating-updates/sec, %s n_factors=%d (%s)" % (algo.upper(), K, args.shape),
        "value": value,
        "unit": "rating-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic planted ratings (surprise_amd.synthetic, seed 0): " + desc,
        "config": {"workload": "%s n_factors=%d %s, one epoch per step over %d training ratings "
                               "per GPU (rank 0), mode=%s, chunks/epoch=%d, %s scaling over %d "
                               "GPU(s)" % (algo.upper(), K, args.dtype, n_train,
                                           mode + ("+qlog" if getattr(eng, "qlog_pp", False)
                                                   else ""),
                                           eng.n_chunks, args.scaling, world),
                   "shape": args.shape, "algo": algo, "n_factors": K, "dtype": args.dtype,
                   "train_ratings_rank0": n_train, "users_total": n_users_global,
                   "items": n_items, "ld": default_ld(K, 1 if args.dtype == "f64" else 0),
                   "parallelism": "users sharded x%d (contiguous ranges), item tables replicated, "
                                  "one SUM all-reduce per epoch-chunk" % world},
        "per_gpu_value": value / world,
        "device_bytes_per_rank_max": dev_bytes,
    }
    lay = layout_of(eng)
    chain = time_top_chain(eng, torch) if args.shape == "ml-1m" and not args.no_chain_probe \
        else None
    qlog = bool(getattr(eng, "qlog_pp", False))
    rl = roofline_of(algo, K, args.dtype, n_train, ms_step, shape_key(args.shape, args.users),
                     phases, lay, chain, qlog=qlog)
    rl.update({
        "kernel": "dominant: %s; step (%s): %s" % (
            (rl.get("dominant_kernel") or {}).get("kernel"), mode,
            "mf_ckpt_epoch_kernel (heavy + light users) + log_replay_kernel (both groups) "
            "+ log_apply_kernel" if mode == "log" else
            "mf_svdpp_qlog_kernel + mf_svdpp_qlog_fold (log_reduce_kernel, y_piece_kernel, "
            "qlog_fold_kernel)" if qlog else "mf_svdpp_hx_kernel + y fold (+ merge)"),
        "phases_gpu_ms": phases, "note": ROOFLINE_NOTE})
    result["roofline"] = rl

    oracle_cache = {}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and algo == "svd":
        result["cpu_baseline"] = cpu_baselines(csr, n_items, K, n_train)
        cb = result["cpu_baseline"]
        cb["gpu_over_cpu_measured"] = value / cb["value"]  # (the 16 pinned processes)
        cb["gpu_over_cpu_all_cores_derived"] = value / cb["all_cores_derived"]["value"]
        cb["gpu_over_cython_equivalent_single"] = value / cb["single_core"]["cython_equivalent_derived"]
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and algo == "svdpp":
        result["cpu_baseline"] = cpu_baseline_svdpp(csr, n_items, K, n_train)
        result["cpu_baseline"]["gpu_over_cpu"] = value / result["cpu_baseline"]["value"]

    def reseed(e, a=algo, k=K):
        """The timed engine again from the initial factors (the rmse leg reuses its device
        layout instead of building another one: C5 / C4 host preparation takes minutes)."""
        pu, qi, yj = init_tables(args.shape, rank, n_users, n_items, k, a == "svdpp",
                                 getattr(workload, "user_lo", 0))
        e.set_factors(pu, qi, yj=yj)
        e._prepare(ctx)
        return e

    if not args.no_rmse:
        result["rmse"] = rmse_leg(args, ctx, csr, test, n_items, K, gm, mode, rank, world, torch,
                                  lambda: reseed(eng), oracle_cache)
        note("rmse leg done")

    small = world == 1 and args.shape == "ml-1m" and K == 100
    if small and args.legs and headline:
        # the other precision on the same fold and steps (the fp32 product option)
        other = "f32" if args.dtype == "f64" else "f64"
        eng = None
        e32 = make_engine(dt=other)
        el2, ph = run_steps(e32, None, args.steps, args.warmup, torch)
        lay2 = layout_of(e32)
        chain2 = None if args.no_chain_probe else time_top_chain(e32, torch)
        ms2 = el2 / args.steps * 1e3
        leg = {"dtype": other, "value": n_train * args.steps / el2, "ms_per_step": ms2,
               "roofline": roofline_of(algo, K, other, n_train, ms2, shape_key(args.shape, args.users), ph, lay2,
                                       chain2)}
        leg["roofline"]["phases_gpu_ms"] = ph
        if not args.no_rmse:
            leg["rmse"] = rmse_leg(args, ctx, csr, test, n_items, K, gm, mode, rank, world,
                                   torch, lambda: reseed(e32), oracle_cache)
        del e32
        result["%s_leg" % other] = leg

    if small and algo == "svd" and not args.no_svdpp:
        eng = None
        pp_legs = {}
        for dt in ([args.dtype] + ([d for d in ("f64", "f32") if d != args.dtype]
                                   if args.legs else [])):
            pp = make_engine("svdpp", 100, "atomic", dt)
            n2 = max(10, args.steps // 2)
            e2, ph2 = run_steps(pp, None, n2, 2, torch)
            lay_pp = layout_of(pp)
            del pp
            rl2 = roofline_of("svdpp", 100, dt, n_train, e2 / n2 * 1e3, args.shape, ph2, lay_pp)
            rl2["phases_gpu_ms"] = ph2
            pp_legs[dt] = {"value": n_train * n2 / e2, "unit": "rating-updates/s", "steps": n2,
                           "ms_per_step": e2 / n2 * 1e3, "roofline": rl2}
        result["svdpp_c3"] = dict(
            config="BASELINE configs[2]: SVD++ n_factors=100 (atomic q rows, deferred y fold) "
                   "on the same fold, one epoch per step", **pp_legs[args.dtype])
        for dt, leg in pp_legs.items():
            if dt != args.dtype:
                result["svdpp_c3"]["%s_leg" % dt] = leg
        if rank == 0 and not args.no_cpu_baseline:
            cb = cpu_baseline_svdpp(csr, n_items, 100, n_train)
            cb["gpu_over_cpu"] = result["svdpp_c3"]["value"] / cb["value"]
            result["svdpp_c3"]["cpu_baseline"] = cb
            note("svd++ cpu baseline done")

    if small and headline and args.legs and not args.no_predict:
        result["predict"] = predict_leg(csr, test, n_items, gm, torch)

    if small and headline and args.legs and not args.no_c4:
        eng = None
        legs = c4_leg(torch)
        result["c4"] = legs["f32"]
        result["c4_f64"] = legs.get("f64")
        note("c4 legs done")

    if rank == 0:
        detail = args.detail or os.path.join(
            ROOT, "gpurun_out", "bench_detail_%s_n%d.json" % (shape_key(args.shape, args.users),
                                                               world))
        try:
            os.makedirs(os.path.dirname(detail), exist_ok=True)
            with open(detail, "w") as f:
                json.dump(result, f, indent=1)
        except OSError as e:  # (the line itself never depends on the side file)
            note("could not write %s: %s" % (detail, e))
            detail = None
        print(json.dumps(compact_line(result, detail and os.path.relpath(detail, ROOT))),
              flush=True)
    if ctx is not None:
        ctx.barrier()
        ctx.dist.destroy_process_group()


LINE_LIMIT = 6000  # bytes of the stdout line (round 4's 21.9 KB line went unparsed by the driver)


def _sig(x, n=5):
    """Floats to n significant digits (the stdout line is a summary; the side file keeps all)."""
    if isinstance(x, float):
        return float("%.*g" % (n, x))
    if isinstance(x, dict):
        return {k: _sig(v, n) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_sig(v, n) for v in x]
    return x


def _pick(d, *keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and d.get(k) is not None}


def compact_roofline(rl):
    """The contract's roofline fields, the dominant kernel per launch, the step and the chain."""
    if not rl:
        return None
    out = _pick(rl, "bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_frac")
    dk = rl.get("dominant_kernel")
    if dk:
        out["dominant_kernel"] = dict(
            _pick(dk, "kernel", "span_us_per_step", "executed_bytes_per_update"),
            launches={k: _pick(v, "avg_us", "ratings", "frac")
                      for k, v in dk.get("launches", {}).items()})
    if rl.get("step"):
        out["step"] = _pick(rl["step"], "ms", "frac", "traffic_frac")
    if rl.get("chain_latency"):
        out["chain_latency"] = _pick(rl["chain_latency"], "top_user_ratings", "alone_us", "frac")
    if rl.get("atomic_roof"):
        out["atomic_roof"] = _pick(rl["atomic_roof"], "achieved", "frac")
    ph = rl.get("phases_gpu_ms") or {}
    keep = _pick(ph, "epoch_kernel_ms", "replay_ms", "fold_sync_ms", "step_gpu_ms",
                 "allreduce_ms_per_chunk", "allreduce_ms", "allreduce_bytes_per_chunk")
    if keep:
        out["phases_gpu_ms"] = keep
    return out


def compact_line(result, detail_path=None):
    """The ONE stdout JSON line: the contract fields, the headline's roofline / cpu_baseline /
    rmse, and one summary per leg (f32_leg, svdpp_c3, c4, predict); the full dictionary is in
    the side file `detail`.  Bounded by LINE_LIMIT (tests/test_host.py)."""
    out = {k: result[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup",
                                  "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
                                  "dtype", "data") if k in result}
    cfg = result.get("config", {})
    out["config"] = _pick(cfg, "workload", "shape", "algo", "n_factors", "dtype",
                          "train_ratings_rank0", "users_total", "items", "parallelism")
    out["device_bytes_per_rank_max"] = result.get("device_bytes_per_rank_max")
    out["roofline"] = compact_roofline(result.get("roofline"))
    cb = result.get("cpu_baseline")
    if cb:
        c = _pick(cb, "value", "unit", "cores", "kind", "sample", "gpu_over_cpu_measured",
                  "gpu_over_cpu")
        sc = cb.get("single_core") or {}
        c["single_core"] = _pick(sc, "value", "cores")
        if sc.get("cython_equivalent_derived"):
            c["cython_equivalent_single_core"] = sc["cython_equivalent_derived"]
            c["gpu_over_cython_single_core"] = cb.get("gpu_over_cython_equivalent_single")
        out["cpu_baseline"] = c
    if result.get("rmse"):
        out["rmse"] = _pick(result["rmse"], "gpu", "reference_oracle_fp64", "delta", "tolerance",
                            "global_mean_baseline", "below_global_mean")

    def leg(d):
        rl = d.get("roofline") or {}
        s = _pick(d, "dtype", "value", "ms_per_step", "steps")
        s["frac"] = rl.get("frac")
        if rl.get("traffic_frac") is not None:
            s["traffic_frac"] = rl["traffic_frac"]
        if (rl.get("atomic_roof") or {}).get("frac") is not None:
            s["atomic_frac"] = rl["atomic_roof"]["frac"]
        dk = rl.get("dominant_kernel") or {}
        if dk.get("span_us_per_step"):
            s["kernel_span_us"] = dk["span_us_per_step"]
        if d.get("rmse"):
            s["rmse_delta"] = d["rmse"].get("delta")
        return s

    for k in ("f32_leg", "f64_leg"):
        if result.get(k):
            out[k] = leg(result[k])
    if result.get("svdpp_c3"):
        pp = result["svdpp_c3"]
        s = leg(pp)
        for k, v in pp.items():
            if k.endswith("_leg"):
                s[k] = leg(v)
        if pp.get("cpu_baseline"):
            s["cpu_baseline"] = _pick(pp["cpu_baseline"], "value", "cores", "kind")
        out["svdpp_c3"] = s
    for k in ("c4", "c4_f64"):
        if result.get(k):
            out[k] = leg(result[k])
    if result.get("predict"):
        p = result["predict"]
        out["predict"] = {n: {k: p[n][k]["us_per_prediction"] for k in
                              ("test", "test_metrics", "test_metrics_columns") if k in p[n]}
                          for n in ("svd", "svdpp") if n in p}
    out["detail"] = detail_path
    rm = out.pop("rmse", None)
    out = _sig({k: v for k, v in out.items() if v is not None or k == "vs_baseline"})
    if rm:
        out["rmse"] = rm  # (full precision: tests compare the committed oracle value exactly)
    text = json.dumps(out)
    if len(text) > LINE_LIMIT:  # never lose the headline: drop the legs first
        for k in ("predict", "svdpp_c3", "f32_leg", "f64_leg", "c4_f64", "c4"):
            out.pop(k, None)
            if len(json.dumps(out)) <= LINE_LIMIT:
                break
    return out


ROOFLINE_NOTE = (
    "dominant kernel = the epoch kernel, one launch = its invocation over a step's ratings (a "
    "split chunk's heavy and light launches run concurrently on two streams: duration = their "
    "wall span). achieved = the bytes the executed work moves (executed_bytes(): per rating the "
    "CSR entry, the item row gather and half a packed checkpoint row; per user its row once) / "
    "that span; traffic = its measured HBM bytes per step (2 x FETCH_SIZE + WRITE_SIZE, "
    "separate --pmc passes); launches = each launch on its own (heavy = the critical path); "
    "step = every kernel of the step over ms_per_step; survey_8d = SURVEY 8(d)'s figure as a "
    "rate only. ML-1M's critical launch is bound by the heaviest user's sequential chain "
    "(chain_latency: that chain timed alone on the GPU), not by HBM: its item table is "
    "L2-resident; the HBM-bound configuration is the c4 leg")


def c4_leg(torch, steps=5, warmup=2, dtypes=("f32", "f64")):
    """BASELINE configs[3]'s shape on this one GPU (2M users x 200k items, 99M training ratings,
    SVD K=128, the checkpoint log, one epoch per step): the HBM-bound configuration (SURVEY
    8(d): its tables exceed the caches), with its own roofline and traffic (profiles/
    traffic_svd_k128_c4[_f64].json), in fp32 and -- the reference's arithmetic, mf.pyx:206-239 --
    fp64 (rows of 1088 B: the narrow checkpoint rows).  Held-out RMSE at E=20:
    tests/test_gpu_scale.py.  Returns {dtype: leg}."""
    from types import SimpleNamespace
    from surprise_amd.engine import MFEngine
    a = SimpleNamespace(shape="c4", users=0)
    t0 = time.perf_counter()
    csr, _, n_items, _, desc = workload(a, 0, 1)
    n_train = len(csr[1])
    gm = float(csr[2].sum()) / n_train
    K = 128
    pu, qi, _ = init_tables("c4", 0, len(csr[0]) - 1, n_items, K, False, 0)
    gen = time.perf_counter() - t0
    out = {}
    for dt in dtypes:
        t1 = time.perf_counter()
        eng = MFEngine(csr, n_items, K, algo="svd", hyper=hyper_for("svd", gm), mode="log",
                       dtype=TORCH_DTYPE[dt])
        eng.set_factors(pu, qi)
        eng._prepare(None)
        prep = time.perf_counter() - t1 + gen
        el, ph = run_steps(eng, None, steps, warmup, torch)
        lay = layout_of(eng)
        ms = el / steps * 1e3
        del eng
        torch.cuda.empty_cache()
        rl = roofline_of("svd", K, dt, n_train, ms, "c4", ph, lay)
        rl["phases_gpu_ms"] = ph
        rl["note"] = ROOFLINE_NOTE
        out[dt] = {"config": "BASELINE configs[3]'s shape on one GPU: " + desc + "; SVD K=128 "
                             "%s, checkpoint log, one epoch per step" % dt,
                   "value": n_train * steps / el, "unit": "rating-updates/s", "steps": steps,
                   "warmup": warmup, "ms_per_step": ms, "dtype": dt, "host_prep_s": prep,
                   "roofline": rl}
        note("c4 %s leg: %.2f ms/step" % (dt, ms))
    return out


def oracle_rmse(args, csr, test, n_items, K, gm, cache):
    """Held-out RMSE of the fp64 sequential oracle -- the reference loop restated (SVD:
    mf.pyx:241-262; SVD++: its exact per-user form of :463-498) -- on the same CSR and initial
    factors (computed once per run)."""
    if "rmse" in cache:
        return cache["rmse"], cache["seconds"]
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    E = args.rmse_epochs
    svdpp = args.algo == "svdpp"
    tu, ti, tr = test
    tu, ti = np.asarray(tu, np.int32), np.asarray(ti, np.int32)
    row_ptr, items, ratings = csr
    pu, qi, yj = init_tables(args.shape, 0, len(row_ptr) - 1, n_items, K, svdpp)
    h = hyper_for(args.algo, gm)
    hp = orc.hyper(**{k: v for k, v in h.items() if k != "global_mean"})
    t0 = time.perf_counter()
    if svdpp:
        pu, qi, yj, bu, bi = orc.svdpp_sgd(row_ptr, items, ratings, n_items, K, E, gm, hp, pu,
                                           qi, yj, affine=True)
        e = orc.svdpp_predict(tu, ti, row_ptr, items, K, gm, pu, qi, yj, bu, bi)
        imp = np.zeros(len(tu), bool)
    else:
        pu, qi, bu, bi = orc.svd_sgd(row_ptr, items, ratings, n_items, K, E, True, gm, hp,
                                     pu, qi)
        e, imp = orc.svd_predict(tu, ti, K, True, gm, pu, qi, bu, bi)
    cache["seconds"] = time.perf_counter() - t0
    cache["rmse"] = orc.rmse(tr, orc.finish_estimates(e, imp, gm, 0, (1, 5)))
    return cache["rmse"], cache["seconds"]


def data_fingerprint(csr, test):
    """sha256[:16] over the training CSR and the held-out triples (user, item as int32; rating
    as float64): ties a committed golden value to the exact synthetic data it was made on."""
    import hashlib
    h = hashlib.sha256()
    tu, ti, tr = test
    for a in (*csr, np.asarray(tu, np.int32), np.asarray(ti, np.int32), np.asarray(tr, np.float64)):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:16]


def scale_golden(args, E):
    """The committed fp64-oracle held-out RMSE of this c4 / c5-shard workload after E epochs
    (tests/golden/scale_golden.json, made by tests/golden/make_scale_golden.py), or None."""
    key = {"c4": "c4", "c5": "c5shard"}.get(args.shape)
    path = os.path.join(ROOT, "tests", "golden", "scale_golden.json")
    if key is None or not os.path.exists(path):
        return None
    data = json.load(open(path))
    g = data.get(key)
    if args.users and (g is None or (g["users"] or 0) != args.users):
        g = data.get("%s_u%d" % (args.shape, args.users))  # (a user-prefix miniature)
    if g is None or (g["users"] or 0) != (args.users or 0) or E > len(g["rmse_by_epoch"]):
        return None
    return g


def rmse_leg(args, ctx, csr, test, n_items, K, gm, mode, rank, world, torch, make_engine,
             oracle_cache):
    """A full fit (--rmse-epochs, 20 by default) through the same engine, held-out RMSE over all
    ranks; at N=1 on ML-1M (or with --oracle) also the fp64 sequential oracle on the same CSR and
    initial factors; c4 / c5-shard: the committed oracle value (scale_golden.json)."""
    E = args.rmse_epochs
    eng = make_engine()
    eng.run_epochs(E, ctx)
    tu, ti, tr = test
    tu, ti = np.asarray(tu, np.int32), np.asarray(ti, np.int32)
    svdpp = args.algo == "svdpp"
    est, _ = eng.predict(tu, ti, gm, imp=eng.user_implicit() if svdpp else None)
    est = np.clip(est, 1, 5)
    se, n, se_mu = sum_over_ranks(ctx, [float(((tr - est) ** 2).sum()), float(len(tr)),
                                        float(((tr - gm) ** 2).sum())], torch)
    out = {"gpu": (se / n) ** .5, "global_mean_baseline": (se_mu / n) ** .5,
           "below_global_mean": bool(se < se_mu),
           "fit": "%s K=%d E=%d %s (%s) through the bench engine, %d held-out ratings over %d "
                  "rank(s)" % (args.algo.upper(), K, E, eng.tdt,
                               mode + ("+qlog" if getattr(eng, "qlog_pp", False) else ""),
                               int(n), world)}
    del eng
    if world == 1 and (args.shape == "ml-1m" or args.oracle):
        ref, secs = oracle_rmse(args, csr, test, n_items, K, gm, oracle_cache)
        out["oracle_seconds"] = secs
        out["reference_oracle_fp64"] = ref
        out["delta"] = out["gpu"] - ref
        out["tolerance"] = 1e-3
    else:
        g = scale_golden(args, E)
        if g is not None and world == 1 and data_fingerprint(csr, test) != g["data_fingerprint"]:
            raise SystemExit("the %s workload differs from the one scale_golden.json was made on"
                             % args.shape)
        if g is not None:
            out["reference_oracle_fp64"] = g["rmse_by_epoch"][E - 1]
            out["reference_source"] = ("tests/golden/scale_golden.json (%s; data fingerprint %s)"
                                       % (g["generator"], g["data_fingerprint"]))
            out["delta"] = out["gpu"] - out["reference_oracle_fp64"]
            out["tolerance"] = 1e-3
    return out


def predict_leg(csr, test, n_items, gm, torch):
    """the batched device test() / test_metrics() of fitted SVD and SVD++ models
    (the public classes, default dtype) over the held-out fold, against the reference's
    per-prediction path (AlgoBase.predict -> estimate: algo_base.py:101-218, mf.pyx:269-299 /
    :506-522; 6.6 us per SVD prediction measured in the survey container)."""
    from surprise_amd import SVD, SVDpp
    from surprise_amd.trainset import Trainset
    row_ptr, items, ratings = csr
    ts = Trainset.from_csr(row_ptr, items, ratings, n_items)
    tu, ti, tr = test
    testset = list(zip(np.asarray(tu).tolist(), np.asarray(ti).tolist(),
                       np.asarray(tr, np.float64).tolist()))
    out = {"held_out": len(testset), "reference_us_per_prediction": 6.6,
           "reference_note": "SVD: AlgoBase.predict per rating (SURVEY 3.2, measured in the "
                             "build container); SVD++ re-sums y_j over I_u per call"}
    from surprise_amd.dataset import RatingColumns
    columns = RatingColumns(np.asarray(tu), np.asarray(ti), np.asarray(tr, np.float64))
    for name, klass, k in (("svd", SVD, 100), ("svdpp", SVDpp, 100)):
        algo = klass(n_factors=k, n_epochs=20, random_state=0).fit(ts)
        leg = {"dtype": algo.dtype}
        # test(): a list of Predictions (the reference's return type); test_metrics(): (rmse,
        # mae) from the device; *_columns: the same on a column-native testset (RatingColumns:
        # no Python object per rating on the way in)
        for key, fn, data in (("test", "test", testset), ("test_metrics", "test_metrics", testset),
                              ("test_metrics_columns", "test_metrics", columns)):
            getattr(algo, fn)(data[:1000])  # warm (device tables, implicit term)
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                r = getattr(algo, fn)(data)
            dt = (time.perf_counter() - t0) / reps
            leg[key] = {"seconds": dt, "predictions_per_s": len(testset) / dt,
                        "us_per_prediction": dt / len(testset) * 1e6}
            if fn == "test_metrics":
                leg[key]["rmse"] = r[0]
        leg["speedup_vs_reference_test"] = 6.6 / leg["test"]["us_per_prediction"]
        out[name] = leg
        del algo
    return out


if __name__ == "__main__":
    main()
