"""BASELINE configs[3] / [4] on the box's one GPU, through bench.py (the same engine, data
generator and initial factors the scaling runs use), against the fp64 sequential oracle's
held-out RMSE committed in tests/golden/scale_golden.json (tests/golden/make_scale_golden.py ran
the oracle on the same data in the build container; nothing of the oracle runs here):

  * C4: SVD K=128 on the full 2M-user x 200k-item x 100M-rating shape at the reference's 20
    epochs, within 1e-3 of the oracle (the reference loop restated, mf.pyx:241-262), device
    memory under 35 GB, and the 2-rank sharded run (gloo rehearsal: each rank generates and
    holds only its user range) equal to the 1-rank run -- the "log" schedule's multi-rank merge
    is the same arithmetic;
  * C5: one rank's full share (1.25M users x 1M items, 123M ratings, SVD++ K=128) at 20 epochs
    within 1e-3 of the exact per-user oracle (mf.pyx:463-498), and on a user prefix the 2-rank
    run (SVD++'s affine y merge, count-aware q merge) within 1e-3 of the 1-rank run."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def _bench(*args, timeout=900):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--rmse-epochs", "2", "--no-cpu-baseline", "--no-svdpp", "--no-predict", *args]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def _golden(case):
    path = os.path.join(ROOT, "tests", "golden", "scale_golden.json")
    g = json.load(open(path)).get(case) if os.path.exists(path) else None
    if g is None or len(g["rmse_by_epoch"]) < 20:
        pytest.skip("tests/golden/scale_golden.json has no 20-epoch %s entry" % case)
    return g


@pytest.fixture(scope="module")
def c4_one(torch):
    return _bench("--shape", "c4", "--rmse-epochs", "20")


def test_c4_svd_k128_e20_within_1e3_of_committed_oracle(c4_one):
    """C4 (2M x 200k x 100M, SVD K=128) at the reference's 20 epochs against the fp64 sequential
    oracle's held-out RMSE, run in the build container on the same data (the bench checks the
    data fingerprint) and committed: no oracle runs here."""
    g = _golden("c4")
    r = c4_one
    assert r["config"]["n_factors"] == 128 and r["config"]["items"] == 200_000
    assert r["config"]["train_ratings_rank0"] == g["train_ratings"]
    assert r["rmse"]["reference_oracle_fp64"] == g["rmse_by_epoch"][19]
    assert abs(r["rmse"]["delta"]) < 1e-3, r["rmse"]
    assert r["rmse"]["gpu"] < r["rmse"]["global_mean_baseline"]


def test_c4_fp64_svd_k128_e20_within_1e3_of_committed_oracle(torch):
    """C4 at the reference's precision (fp64 arrays, mf.pyx:206-239): SVD K=128 in fp64 -- item
    rows of 1088 B, the narrow checkpoint log -- 20 epochs within 1e-3 of the committed fp64
    sequential oracle's held-out RMSE (scale_golden.json c4)."""
    g = _golden("c4")
    r = _bench("--shape", "c4", "--dtype", "f64", "--rmse-epochs", "20")
    assert r["dtype"] == "f64" and r["config"]["n_factors"] == 128
    assert r["config"]["train_ratings_rank0"] == g["train_ratings"]
    assert r["rmse"]["reference_oracle_fp64"] == g["rmse_by_epoch"][19]
    assert abs(r["rmse"]["delta"]) < 1e-3, r["rmse"]
    assert r["device_bytes_per_rank_max"] < 90e9, r["device_bytes_per_rank_max"]


def test_c4_device_memory_within_35gb(c4_one):
    """The packed checkpoint log (one row per pair of ratings) keeps C4 on one GPU under 35 GB."""
    assert c4_one["device_bytes_per_rank_max"] < 35e9, c4_one["device_bytes_per_rank_max"]


def test_c4_two_ranks_equal_one(torch, c4_one):
    r2 = _bench("--shape", "c4", "--gpus", "2", "--backend", "gloo", "--rmse-epochs", "20")
    assert r2["n_gpus"] == 2 and r2["scaling"] == "strong"
    # each rank holds about half of the ratings and only its pu rows
    assert r2["config"]["train_ratings_rank0"] < 0.51 * c4_one["config"]["train_ratings_rank0"]
    assert abs(r2["rmse"]["gpu"] - c4_one["rmse"]["gpu"]) < 1e-5, (r2["rmse"], c4_one["rmse"])


def test_c5_shard_svdpp_k128_e20_within_1e3_of_committed_oracle(torch):
    """One of 8 ranks' share of C5 (the first 1.25M users, every one of the 1M items, 123M
    ratings, SVD++ K=128) at 20 epochs on the float-atomic schedule (--qlog 0: on one rank the
    engine's default here is the q log, auto_qlog) against the committed exact per-user oracle
    value."""
    g = _golden("c5shard")
    r = _bench("--shape", "c5", "--users", "1250000", "--qlog", "0", "--rmse-epochs", "20",
               timeout=1100)
    assert "+qlog" not in r["config"]["workload"]
    assert r["config"]["algo"] == "svdpp" and r["config"]["items"] == 1_000_000
    assert r["config"]["train_ratings_rank0"] == g["train_ratings"]
    assert r["rmse"]["reference_oracle_fp64"] == g["rmse_by_epoch"][19]
    assert abs(r["rmse"]["delta"]) < 1e-3, r["rmse"]


def test_c5_shard_qlog_e20_within_1e3_of_committed_oracle(torch):
    """The C5 shard (1.25M users, 123M ratings, SVD++ K=128) on its default schedule on one rank,
    the q log (auto_qlog: 16 chunks of ~7.7 ratings per item; item rows read-only
    within each of the 16 chunks, gradients folded by the fused per-item fold, nt log stores) at
    20 epochs: within 1e-3 of the exact per-user oracle's held-out RMSE (scale_golden.json
    c5shard, mf.pyx:463-498)."""
    g = _golden("c5shard")
    r = _bench("--shape", "c5", "--users", "1250000", "--rmse-epochs", "20", timeout=1100)
    assert "+qlog" in r["config"]["workload"]  # (the default here: auto_qlog)
    assert r["rmse"]["reference_oracle_fp64"] == g["rmse_by_epoch"][19]
    assert abs(r["rmse"]["delta"]) < 1e-3, r["rmse"]


def test_c5_at_8_ranks_schedule_within_1e3_of_committed_oracle(torch):
    """C5@8's own schedule at shard scale (gloo rehearsal on the one GPU): the 1.25M-user shard
    split over 8 ranks exactly as bench.py --gpus 8 splits C5 (dist.shard_users), 2 epoch-chunks
    per epoch -- 625k users (78k per rank) per chunk, the users per chunk of C5@8 at its 16
    chunks over 10M users -- q / b carried through the later ranks' steps
    (MF_MERGE_RECENCY), y composed in rank order; 20 epochs within 1e-3 of the sequential
    reference loop's held-out RMSE (scale_golden.json c5shard), and within 1e-3 of the same
    schedule restated on the CPU (c5at8_c2_m3: oracle_svdpp_sgd_groups_merge(merge=3), final
    0.95164 vs the sequential 0.95182; the round-3 merge rule, c5at8_c2_m2, ends at -2.1e-3)."""
    g = _golden("c5shard")
    gm3 = _golden("c5at8_c2_m3")
    r = _bench("--shape", "c5", "--users", "1250000", "--gpus", "8", "--backend", "gloo",
               "--chunks", "2", "--rmse-epochs", "20", "--steps", "1", "--warmup", "0",
               timeout=1100)
    assert r["n_gpus"] == 8 and r["config"]["algo"] == "svdpp"
    assert "chunks/epoch=2" in r["config"]["workload"]
    assert r["rmse"]["reference_oracle_fp64"] == g["rmse_by_epoch"][19]
    assert abs(r["rmse"]["delta"]) < 1e-3, r["rmse"]
    assert abs(r["rmse"]["gpu"] - gm3["rmse_by_epoch"][19]) < 1e-3, (r["rmse"], gm3["rmse_by_epoch"][19])
    assert abs(gm3["rmse_by_epoch"][19] - g["rmse_by_epoch"][19]) < 1e-3
    ph = r["roofline"]["phases_gpu_ms"]
    assert ph["allreduce_bytes_per_chunk"] > 0 and ph["allreduce_ms_per_chunk"] > 0


C5_USERS = "60000"


def test_c5_miniature_long_chain_dealing_within_1e3_of_committed_oracle(torch):
    """dist.chunk_users' long-chain dealing (every user of > 1/256 of a
    chunk's ratings into chunk 0) pinned on a miniature where it fires: the first
    60k users of C5 at 8 epoch-chunks (8 such users, tests/test_dist.py), SVD++ K=128, 20 epochs,
    against the exact per-user oracle's held-out RMSE committed in scale_golden.json (c5_u60000,
    mf.pyx:463-498).  The round-robin dealing (long_chain=0, one long user per chunk) on the
    same data is held to the same bar, on the one-rank default schedule (the q log: auto_qlog,
    0.7 ratings per item and chunk) and on the float-atomic one; the deltas are printed."""
    g = _golden("c5_u60000")
    r = _bench("--shape", "c5", "--users", C5_USERS, "--chunks", "8", "--rmse-epochs", "20")
    r0 = _bench("--shape", "c5", "--users", C5_USERS, "--chunks", "8", "--rmse-epochs", "20",
                "--long-chain", "0")
    ra = _bench("--shape", "c5", "--users", C5_USERS, "--chunks", "8", "--rmse-epochs", "20",
                "--qlog", "0")
    print("c5_u60000 E=20: long-chain dealing %+.3e, round-robin %+.3e, atomic %+.3e (oracle %.6f)"
          % (r["rmse"]["delta"], r0["rmse"]["delta"], ra["rmse"]["delta"], g["rmse_by_epoch"][19]))
    assert "+qlog" in r["config"]["workload"] and "+qlog" not in ra["config"]["workload"]
    for x in (r, r0, ra):
        assert "chunks/epoch=8" in x["config"]["workload"]
        assert x["config"]["train_ratings_rank0"] == g["train_ratings"]
        assert x["rmse"]["reference_oracle_fp64"] == g["rmse_by_epoch"][19]
        assert abs(x["rmse"]["delta"]) < 1e-3, x["rmse"]


@pytest.fixture(scope="module")
def c5_small(torch):
    return _bench("--shape", "c5", "--users", C5_USERS, "--qlog", "0")  # (2 ranks: atomic)


def test_c5_two_ranks_within_1e3_of_one(torch, c5_small):
    """SVD++'s multi-rank merge (affine y composition, count-aware q) on C5's 1M-item tables and
    degree profile (a user prefix): 2 ranks within 1e-3 of 1 rank."""
    r2 = _bench("--shape", "c5", "--users", C5_USERS, "--gpus", "2", "--backend", "gloo")
    assert r2["n_gpus"] == 2
    assert abs(r2["rmse"]["gpu"] - c5_small["rmse"]["gpu"]) < 1e-3, (r2["rmse"], c5_small["rmse"])


# ------------------------------------------------------------------ item tables above 715 MB
# (the round-1 limit; now < 2 GiB, tools/probe_buffer_range.hip): 3,000 rated items spread over
# a table of ~800k rows, so gathers, stores and atomics reach offsets far past 715 MB.  Unrated
# rows never change, so the oracle runs on the compacted problem (rated items renumbered).

def _big_table_case(n_items, K, seed=11):
    import numpy as np
    rng = np.random.RandomState(seed)
    n_users, M = 1500, 3000
    ids = np.sort(rng.choice(n_items - 2, M - 2, replace=False))
    ids = np.concatenate([ids, [n_items - 2, n_items - 1]]).astype(np.int32)  # the last rows
    rows = [np.sort(rng.choice(M, rng.randint(5, 160), replace=False)) for _ in range(n_users)]
    row_ptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    local = np.concatenate(rows).astype(np.int32)
    ratings = rng.randint(1, 6, len(local)).astype(np.float64)
    pu0 = rng.normal(0, .1, (n_users, K))
    qc0 = rng.normal(0, .1, (M, K))
    yc0 = rng.normal(0, .1, (M, K))
    return ids, row_ptr, local, ratings, pu0, qc0, yc0


def _scatter_rows(ids, rows, n_items):
    import numpy as np
    full = np.zeros((n_items, rows.shape[1]))
    full[ids] = rows
    return full


HYPER = dict(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005, lr_yj=.005, reg_bu=.02,
             reg_bi=.02, reg_pu=.02, reg_qi=.02, reg_yj=.02)


@pytest.mark.parametrize("dtype,K,n_items", [("float32", 240, 800_000),
                                             ("float64", 100, 1_100_000)])
def test_svd_log_item_table_above_715mb(torch, dtype, K, n_items):
    """SVD, default log schedule: fp32 K=240 (1 KiB rows: the lookahead body + checkpoint
    replay, 819 MB table) and fp64 K=100 (915 MB, the direct body's gradient log) against the
    delta-log oracle on the compacted problem."""
    import numpy as np
    import oracle as orc
    from surprise_amd.engine import MFEngine
    ids, row_ptr, local, ratings, pu0, qc0, _ = _big_table_case(n_items, K)
    gm = float(ratings.mean())
    eng = MFEngine((row_ptr, ids[local], ratings), n_items, K, hyper=dict(HYPER, global_mean=gm),
                   dtype=dtype, mode="log")
    assert eng.qb.numel() * eng.qb.element_size() > 715 * 2 ** 20
    eng.set_factors(pu0, _scatter_rows(ids, qc0, n_items))
    eng.run_epochs(2)
    got = eng.get_factors()
    hp = orc.hyper(**HYPER)
    pu, qc, bu, bc = orc.svd_sgd_deltalog(row_ptr, local, ratings, len(ids), K, 2, True, gm, hp,
                                          pu0.copy(), qc0.copy(), merge=3)
    tol = 1e-9 if dtype == "float64" else 2e-5
    np.testing.assert_allclose(got["pu"], pu, rtol=0, atol=tol)
    np.testing.assert_allclose(got["qi"][ids], qc, rtol=0, atol=tol)
    np.testing.assert_allclose(got["bi"][ids], bc, rtol=0, atol=tol)
    np.testing.assert_allclose(got["bu"], bu, rtol=0, atol=tol)
    untouched = np.setdiff1d(np.arange(0, n_items, 9973), ids)
    assert not got["qi"][untouched].any() and not got["bi"][untouched].any()


def _svdpp_train_rmse(row_ptr, local, ratings, gm, pu, q, y, bu, b):
    import numpy as np
    n = np.diff(row_ptr)
    users = np.repeat(np.arange(len(n)), n)
    imp = np.add.reduceat(y[local], row_ptr[:-1], axis=0) / np.sqrt(n)[:, None]
    est = gm + bu[users] + b[local] + np.einsum("ij,ij->i", q[local], (pu + imp)[users])
    return float(np.sqrt(np.mean((ratings - est) ** 2)))


def test_svdpp_deterministic_item_tables_above_715mb(torch):
    """SVD++ in the reference's sequential order (one wavefront, plain stores), fp64 K=100:
    qb and yj of 915 MB each; factors within 1e-9 of the sequential oracle's."""
    import numpy as np
    import oracle as orc
    from surprise_amd.engine import MFEngine
    n_items, K = 1_100_000, 100
    ids, row_ptr, local, ratings, pu0, qc0, yc0 = _big_table_case(n_items, K, seed=12)
    gm = float(ratings.mean())
    eng = MFEngine((row_ptr, ids[local], ratings), n_items, K, algo="svdpp",
                   hyper=dict(HYPER, global_mean=gm), dtype="float64", deterministic=True)
    assert eng.yj.numel() * eng.yj.element_size() > 715 * 2 ** 20
    eng.set_factors(pu0, _scatter_rows(ids, qc0, n_items), yj=_scatter_rows(ids, yc0, n_items))
    eng.run_epochs(2)
    got = eng.get_factors()
    pu, qc, yc, bu, bc = orc.svdpp_sgd(row_ptr, local, ratings, len(ids), K, 2, gm,
                                       orc.hyper(**HYPER), pu0.copy(), qc0.copy(), yc0.copy())
    for name, a, b in (("pu", got["pu"], pu), ("qi", got["qi"][ids], qc),
                       ("yj", got["yj"][ids], yc), ("bu", got["bu"], bu), ("bi", got["bi"][ids], bc)):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-9, err_msg=name)
    untouched = np.setdiff1d(np.arange(0, n_items, 9973), ids)
    assert not got["qi"][untouched].any() and not got["yj"][untouched].any()


def test_svdpp_atomic_item_tables_above_715mb(torch):
    """SVD++ (float atomics on q, deferred y fold), fp32 K=240: qb 819 MB and yj 780 MB.  The
    parallel schedule is timing-dependent, so the big-table run is held to the same engine on
    the compacted table (3,000 rows): training RMSE within 2e-4 after 2 epochs."""
    import numpy as np
    from surprise_amd.engine import MFEngine
    n_items, K = 800_000, 240
    ids, row_ptr, local, ratings, pu0, qc0, yc0 = _big_table_case(n_items, K, seed=12)
    gm = float(ratings.mean())
    out = []
    for big in (True, False):
        n = n_items if big else len(ids)
        eng = MFEngine((row_ptr, (ids[local] if big else local), ratings), n, K, algo="svdpp",
                       hyper=dict(HYPER, global_mean=gm), dtype="float32", mode="atomic")
        if big:
            assert eng.yj.numel() * eng.yj.element_size() > 715 * 2 ** 20
            eng.set_factors(pu0, _scatter_rows(ids, qc0, n), yj=_scatter_rows(ids, yc0, n))
        else:
            eng.set_factors(pu0, qc0, yj=yc0)
        eng.run_epochs(2)
        f = eng.get_factors()
        sel = ids if big else slice(None)
        out.append(_svdpp_train_rmse(row_ptr, local, ratings, gm, f["pu"], f["qi"][sel],
                                     f["yj"][sel], f["bu"], f["bi"][sel]))
        if big:
            untouched = np.setdiff1d(np.arange(0, n_items, 9973), ids)
            assert not f["qi"][untouched].any() and not f["yj"][untouched].any()
    assert abs(out[0] - out[1]) < 2e-4, out
