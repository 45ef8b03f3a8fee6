"""BASELINE configs[3] / [4] on the box's one GPU, through bench.py (the same engine, data
generator and initial factors the scaling runs use), against the fp64 sequential oracle:

  * C4: SVD K=128 on the full 2M-user x 200k-item x 100M-rating shape, 2 epochs, held-out
    RMSE within 1e-3 of the oracle (the reference loop restated, mf.pyx:241-262), and the
    2-rank sharded run (gloo rehearsal: each rank generates and holds only its user range)
    equal to the 1-rank run -- the "log" schedule's multi-rank merge is the same arithmetic;
  * C5: SVD++ K=128 with C5's 1M-item tables (and its degree / popularity profile) on a
    user-prefix subsample, 2 epochs, within 1e-3 of the exact per-user oracle
    (mf.pyx:463-498), and the 2-rank run (SVD++'s affine y merge, count-aware q merge) within
    1e-3 of the 1-rank run."""
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


def _bench(*args, timeout=600):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--rmse-epochs", "2", "--no-cpu-baseline", "--no-svdpp", *args]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.fixture(scope="module")
def c4_one(torch):
    return _bench("--shape", "c4", "--oracle")


def test_c4_svd_k128_within_1e3_of_oracle(c4_one):
    r = c4_one
    assert r["config"]["n_factors"] == 128 and r["config"]["items"] == 200_000
    assert r["config"]["train_ratings_rank0"] > 98_000_000
    assert abs(r["rmse"]["delta"]) < 1e-3, r["rmse"]
    assert r["rmse"]["gpu"] < r["rmse"]["global_mean_baseline"]


def test_c4_two_ranks_equal_one(torch, c4_one):
    r2 = _bench("--shape", "c4", "--gpus", "2", "--backend", "gloo")
    assert r2["n_gpus"] == 2 and r2["scaling"] == "strong"
    # each rank holds about half of the ratings and only its pu rows
    assert r2["config"]["train_ratings_rank0"] < 0.51 * c4_one["config"]["train_ratings_rank0"]
    assert abs(r2["rmse"]["gpu"] - c4_one["rmse"]["gpu"]) < 1e-5, (r2["rmse"], c4_one["rmse"])


C5_USERS = "60000"


@pytest.fixture(scope="module")
def c5_one(torch):
    return _bench("--shape", "c5", "--users", C5_USERS, "--oracle")


def test_c5_svdpp_k128_subsample_within_1e3_of_oracle(c5_one):
    r = c5_one
    assert r["config"]["algo"] == "svdpp" and r["config"]["n_factors"] == 128
    assert r["config"]["items"] == 1_000_000
    assert abs(r["rmse"]["delta"]) < 1e-3, r["rmse"]
    assert r["rmse"]["gpu"] < r["rmse"]["global_mean_baseline"]


def test_c5_two_ranks_within_1e3_of_one(torch, c5_one):
    r2 = _bench("--shape", "c5", "--users", C5_USERS, "--gpus", "2", "--backend", "gloo")
    assert r2["n_gpus"] == 2
    assert abs(r2["rmse"]["gpu"] - c5_one["rmse"]["gpu"]) < 1e-3, (r2["rmse"], c5_one["rmse"])
