"""Multi-rank path on the GPU: ranks are separate processes, all on the box's one GPU, with gloo
for the collectives (RCCL needs one GPU per rank).  Every rank holds only its own user rows.
  * "log" mode: the multi-rank merge is the same arithmetic as one GPU processing every rank's
    users, so fp64 factors agree to rounding with the single-GPU fit;
  * "atomic" mode (SVD++'s default): q/b by the count-aware merge, y_j by the affine composition
    of the ranks' end-of-user maps -- held to the reference's golden RMSE (1e-3) and to the
    oracle's multi-rank schedule (tests/test_oracle_golden.py pins that rule);
  * random_state=None: rank 0 draws the initial factors and broadcasts them;
  * bench.py --gpus 2 spawns two ranks itself and reports the 2-GPU weak-scaling line."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ranks(tmp_path, world=2, **kw):
    out = str(tmp_path / "fit.npz")
    port = _port()
    args = []
    for k, v in kw.items():
        args += ["--" + k, str(v)]
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_worker.py"), "--rank",
                               str(r), "--world", str(world), "--port", str(port), "--out", out]
                              + args) for r in range(world)]
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0] * world, rcs
    return [dict(np.load(out.replace(".npz", "_r%d.npz" % r))) for r in range(world)]


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def _u1():
    sys.path.insert(0, HERE)
    from _dist_worker import dataset
    return dataset("u1")


def _single(algo, mode, **kw):
    from surprise_amd import SVD, SVDpp, accuracy
    ts, test = _u1()
    klass = SVD if algo == "SVD" else SVDpp
    a = klass(n_factors=20, n_epochs=5, random_state=0, dtype="float64", mode=mode, **kw).fit(ts)
    return a, accuracy.rmse(a.test(test), verbose=False)


def _same_on_every_rank(res, keys=("pu", "qi", "bu", "bi")):
    for k in keys:
        for r in res[1:]:
            np.testing.assert_array_equal(r[k], res[0][k], err_msg=k)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_n_ranks_log_mode_equals_one_gpu(torch, tmp_path, world):
    """2 / 4 / 8 ranks (all on the box's GPU, gloo): the log schedule's multi-rank fold is one
    GPU's arithmetic -- fp64 factors equal the single-GPU fit to 1e-9."""
    res = _ranks(tmp_path, world=world, algo="SVD", mode="log")
    _same_on_every_rank(res)
    a, rmse = _single("SVD", "log")
    for k in ("pu", "qi", "bu", "bi"):
        np.testing.assert_allclose(res[0][k], getattr(a, k), rtol=0, atol=1e-9, err_msg=k)
    assert abs(float(res[0]["rmse"]) - rmse) < 1e-9


@pytest.mark.parametrize("algo", ["SVD", "SVDpp"])
def test_two_ranks_atomic_mode_rmse_vs_reference(torch, tmp_path, golden, algo):
    """2 ranks, the default parallel schedules, K=20 E=20 on u1: within 1e-3 of the reference's
    own RMSE (golden: svd_k20 E=5 is the SVD case; svdpp_k20_e20 the SVD++ case)."""
    meta, _ = golden
    name, epochs = ("svd_k20_e5", 5) if algo == "SVD" else ("svdpp_k20_e20", 20)
    res = _ranks(tmp_path, algo=algo, mode="atomic", epochs=epochs, dtype="float32")
    keys = ("pu", "qi", "bu", "bi") + (("yj",) if algo == "SVDpp" else ())
    _same_on_every_rank(res, keys)
    assert abs(float(res[0]["rmse"]) - meta["cases"][name]["rmse"]) < 1e-3


@pytest.mark.parametrize("world", [2, 4, 8])
def test_n_ranks_svdpp_tracks_multirank_oracle(torch, tmp_path, golden, world):
    """The GPU's 2 / 4 / 8-rank SVD++ schedule (C5's path) against the oracle's statement of the
    same rule (oracle_svdpp_sgd_groups_merge, merge=3: q / b deltas carried through the later
    ranks' steps; merge_y=4) on u1, K=20, E=20, fp64."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    from surprise_amd.dist import shard_users
    res = _ranks(tmp_path, world=world, algo="SVDpp", mode="atomic", epochs=20)
    _same_on_every_rank(res, ("pu", "qi", "bu", "bi", "yj"))
    ts, test = _u1()
    row_ptr, items, ratings = ts.csr()
    rng = np.random.RandomState(0)
    pu, qi, yj = orc.init_factors(rng, ts.n_users, ts.n_items, 20, with_yj=True)
    hp = orc.hyper(lr_bu=.007, lr_bi=.007, lr_pu=.007, lr_qi=.007, lr_yj=.007, reg_bu=.02,
                   reg_bi=.02, reg_pu=.02, reg_qi=.02, reg_yj=.02)
    b = shard_users(row_ptr, world)
    g = (np.searchsorted(b, np.arange(ts.n_users), side="right") - 1).astype(np.int32)
    pu, qi, yj, bu, bi = orc.svdpp_sgd_groups_merge(row_ptr, items, ratings, ts.n_items, 20, 20,
                                                    ts.global_mean, hp, pu, qi, yj, g, world,
                                                    merge=3, merge_y=4)
    u = np.array([ts._raw2inner_id_users.get(x[0], -1) for x in test], np.int32)
    i = np.array([ts._raw2inner_id_items.get(x[1], -1) for x in test], np.int32)
    est = orc.svdpp_predict(u, i, row_ptr, items, 20, ts.global_mean, pu, qi, yj, bu, bi)
    est = orc.finish_estimates(est, np.zeros(len(u), bool), ts.global_mean, 0, (1, 5))
    rmse_orc = orc.rmse(np.array([x[2] for x in test]), est)
    assert abs(rmse_orc - golden[0]["cases"]["svdpp_k20_e20"]["rmse"]) < 1e-3
    assert abs(float(res[0]["rmse"]) - rmse_orc) < 5e-4, (float(res[0]["rmse"]), rmse_orc)


def test_two_ranks_random_state_none_share_initial_factors(torch, tmp_path):
    """random_state=None (the reference default): each process's global RNG differs, so rank 0
    draws and broadcasts; both ranks must end with one model that trains normally."""
    res = _ranks(tmp_path, algo="SVD", mode="log", seed="none")
    _same_on_every_rank(res)
    assert float(res[0]["rmse"]) < 1.1


def test_two_ranks_union_of_populations_equals_one_gpu(torch, tmp_path):
    """bench.py's 2-GPU data (two ML-1M-shape populations over one item set): the 2-rank "log"
    fit equals the single-GPU fit of the union (same arithmetic; fp32 rounding only)."""
    from surprise_amd import SVD, accuracy
    sys.path.insert(0, HERE)
    from _dist_worker import dataset
    res = _ranks(tmp_path, algo="SVD", mode="log", data="pop2", factors=100, epochs=20,
                 dtype="float32")
    ts, test = dataset("pop2")
    a = SVD(n_factors=100, n_epochs=20, random_state=0, mode="log", dtype="float32").fit(ts)
    rmse = accuracy.rmse(a.test(test), verbose=False)
    assert abs(float(res[0]["rmse"]) - rmse) < 2e-5, (float(res[0]["rmse"]), rmse)
    np.testing.assert_allclose(res[0]["qi"], a.qi, rtol=0, atol=2e-3)


def test_bench_two_ranks_spawned(torch):
    """`bench.py --gpus 2` (no launcher) spawns two ranks and prints ONE 2-GPU JSON line."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--backend", "gloo", "--steps", "4", "--warmup", "1", "--no-svdpp"],
                       capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["scaling"] == "weak"
    rl = r["roofline"]
    assert r["value"] > 0 and 0 < rl["frac"] <= 1.0
    assert rl["dominant_kernel"]["kernel"] == "mf_ckpt_epoch_kernel"
    # the kernel's time per step never exceeds the step; no launch passes the peak
    assert rl["dominant_kernel"]["span_us_per_step"] <= r["ms_per_step"] * 1e3
    assert all(0 < x["frac"] <= 1.0 for x in rl["dominant_kernel"]["launches"].values())
    assert rl["step"]["frac"] <= 1.0
    assert r["roofline"]["phases_gpu_ms"]["allreduce_ms_per_chunk"] > 0
    assert r["rmse"]["gpu"] < r["rmse"]["global_mean_baseline"]


def test_rccl_single_rank_collectives(torch, tmp_path):
    """The RCCL path (backend "nccl", device-resident collectives -- DistContext's
    non-host-staged branches) before the driver's 8-GPU run needs it: a world-size-1 process group
    joined through DistContext.from_env in a fresh child process; all_reduce_sum (fp32 / fp64),
    all_reduce_max, broadcast, all_gather_rows and check_agreement on device tensors, then an
    engine fit carrying the context.  (RCCL refuses two ranks on one GPU: the multi-rank merges
    are rehearsed over gloo above.)"""
    out = str(tmp_path / "rccl.json")
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, os.path.join(HERE, "_rccl_worker.py"), out], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.load(open(out))
    assert r["backend"] == "nccl" and r["world"] == 1 and r["rank"] == 0
    assert r["host_staged"] is False
    assert r["sum_float32"] and r["sum_float64"]
    assert r["max"] == [3, -7, 11] and r["broadcast"] == [2.5] * 5
    assert r["gather_equal"] and r["agreement"] and r["engine_finite"]
    # the device-resident exchange (sync_items -> _delta_into -> RCCL
    # all_reduce_sum -> _apply) forced at world 1: the deterministic schedules equal the local
    # fold; the float-atomic schedule's exchange leaves each chunk's tables unchanged
    x = r["exchange"]
    for name in ("svd_log", "svdpp_qlog", "svdpp_atomic", "svdpp_one_buffer"):
        assert x[name + "_equal"], (name, x[name + "_max_abs_diff"])
        # one collective per chunk and epoch (+ the SVD log's first-chunk <p^2> sum)
        assert x[name + "_allreduce_calls"] >= 3 * x[name + "_chunks"], x
        assert x[name + "_buffer_elems"] > 0
    assert x["svdpp_qlog_qlog"] and x["svdpp_atomic_finite"]
    # the overlapped exchange (q's part async beside the y fold, then y's part): two
    # collectives per chunk; overlap_q=False and the logs: one buffer
    assert x["svdpp_atomic_overlap"] and not x["svdpp_one_buffer_overlap"]
    assert not x["svd_log_overlap"] and not x["svdpp_qlog_overlap"]
    assert x["svdpp_atomic_allreduce_calls"] >= 2 * 3 * x["svdpp_atomic_chunks"], x
