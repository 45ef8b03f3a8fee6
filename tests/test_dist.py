"""Multi-rank path on CPU (gloo, world_size 2): user sharding, per-chunk SUM all-reduce of
item deltas and the final user-row gather, driven by the product's ItemSync protocol
(surprise_amd/dist.py).  The per-rank compute is the oracle (the HIP kernel needs a GPU);
the result must equal oracle_svd_sgd_groups -- the G-group SUM schedule -- bit for bit."""
import os
import socket

import numpy as np
import pytest

from surprise_amd.dist import ItemSync, chunk_users, shard_users


def test_shard_users_balances_ratings():
    rng = np.random.RandomState(0)
    deg = rng.randint(1, 300, size=1000)
    row_ptr = np.concatenate([[0], np.cumsum(deg)])
    for world in (1, 2, 3, 4, 8):
        b = shard_users(row_ptr, world)
        assert b[0] == 0 and b[-1] == 1000 and np.all(np.diff(b) >= 0)
        per = np.diff(row_ptr[b])
        assert per.sum() == row_ptr[-1]
        assert per.max() - per.min() <= 2 * deg.max()


def test_chunk_users_partition():
    rng = np.random.RandomState(1)
    deg = rng.randint(0, 50, size=97)
    row_ptr = np.concatenate([[0], np.cumsum(deg)])
    users = np.arange(10, 90)
    chunks = chunk_users(users, row_ptr, 3)
    allu = np.sort(np.concatenate(chunks))
    np.testing.assert_array_equal(allu, users)
    for c in chunks:  # heaviest first inside a chunk
        assert np.all(np.diff(deg[c]) <= 0)


class OracleRankEngine(ItemSync):
    """CPU stand-in for MFEngine: same protocol, oracle compute (test infrastructure).  Holds
    only its rank's rows (a rank-local CSR), like the device engine."""

    def __init__(self, csr, n_items, K, hp, gm, n_chunks, pu, qi):
        import torch
        self.torch = torch
        self.row_ptr, self.items, self.ratings = csr
        self.n_items, self.K, self.hp, self.gm = n_items, K, hp, gm
        self.n_users = len(self.row_ptr) - 1
        self.n_chunks = n_chunks
        self.chunks = chunk_users(np.arange(self.n_users), self.row_ptr, n_chunks)
        self.pu, self.bu = pu.copy(), np.zeros(self.n_users)
        self.q_snap, self.b_snap = qi.copy(), np.zeros(n_items)
        self.q, self.b = qi.copy(), np.zeros(n_items)

    def run_chunk(self, c):
        import oracle as orc
        mask = np.zeros(self.n_users, bool)
        mask[self.chunks[c]] = True
        deg = np.diff(self.row_ptr) * mask
        rp = np.concatenate([[0], np.cumsum(deg)])
        keep = np.repeat(mask, np.diff(self.row_ptr))
        orc.svd_sgd(rp, self.items[keep], self.ratings[keep], self.n_items, self.K, 1, True,
                    self.gm, self.hp, self.pu, self.q, self.bu, self.b)

    def _delta_buffer(self):
        return self.torch.zeros(self.q.size + self.b.size, dtype=self.torch.float64)

    def _delta_into(self, buf):
        buf.copy_(self.torch.from_numpy(np.concatenate([(self.q - self.q_snap).ravel(),
                                                        self.b - self.b_snap])))

    def _apply(self, buf):
        d = buf.numpy()
        self.q_snap += d[:self.q.size].reshape(self.q.shape)
        self.b_snap += d[self.q.size:]
        self.q[...] = self.q_snap
        self.b[...] = self.b_snap

    def _merge_local(self):
        pass

    def gather_users(self, ctx):
        t = self.torch
        counts = ctx.all_gather_rows(t.tensor([[self.n_users]]), [1] * ctx.world)[:, 0].tolist()
        pu = ctx.all_gather_rows(t.from_numpy(self.pu), counts).numpy()
        bu = ctx.all_gather_rows(t.from_numpy(self.bu), counts).numpy()
        return pu, bu


def _worker(rank, world, port, n_chunks, out_dir):
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    sys.path.insert(0, root)
    import oracle as orc
    from surprise_amd.dist import DistContext, local_csr
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = DistContext()
    csr, n_items, K, gm, pu, qi = _problem()
    b = shard_users(csr[0], world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    hp = orc.hyper(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005,
                   reg_bu=.02, reg_bi=.02, reg_pu=.02, reg_qi=.02)
    eng = OracleRankEngine(local_csr(csr, lo, hi), n_items, K, hp, gm, n_chunks, pu[lo:hi], qi)
    eng.run_epochs(3, ctx)
    pu_all, bu_all = eng.gather_users(ctx)
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), pu=pu_all, bu=bu_all, qi=eng.q_snap,
             bi=eng.b_snap)
    dist.destroy_process_group()


def _problem():
    from surprise_amd import Dataset, synthetic
    from surprise_amd.model_selection import KFold
    u, i, r = synthetic.planted(200, 80, 6000, seed=3)
    ts, _ = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
    rng = np.random.RandomState(0)
    K = 6
    pu = rng.normal(0, .1, (ts.n_users, K))
    qi = rng.normal(0, .1, (ts.n_items, K))
    return ts.csr(), ts.n_items, K, ts.global_mean, pu, qi


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n_chunks", [1, 3])
def test_two_rank_gloo_equals_group_sum_schedule(tmp_path, n_chunks):
    import torch.multiprocessing as mp
    import oracle as orc
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), n_chunks, str(tmp_path)), nprocs=world,
             join=True)
    res = [dict(np.load(tmp_path / ("rank%d.npz" % r))) for r in range(world)]
    for k in ("pu", "bu", "qi", "bi"):  # every rank ends with the same full state
        np.testing.assert_array_equal(res[0][k], res[1][k])

    csr, n_items, K, gm, pu, qi = _problem()
    b = shard_users(csr[0], world)
    n_users = len(csr[0]) - 1
    group = np.searchsorted(b, np.arange(n_users), side="right") - 1
    chunk = np.zeros(n_users, np.int32)
    for r in range(world):
        for c, us in enumerate(chunk_users(np.arange(b[r], b[r + 1]), csr[0], n_chunks)):
            chunk[us] = c
    hp = orc.hyper(lr_bu=.005, lr_bi=.005, lr_pu=.005, lr_qi=.005,
                   reg_bu=.02, reg_bi=.02, reg_pu=.02, reg_qi=.02)
    epu, eqi, ebu, ebi = orc.svd_sgd_groups(*csr, n_items, K, 3, True, gm, hp, pu.copy(),
                                            qi.copy(), group, world, chunk, n_chunks)
    np.testing.assert_array_equal(res[0]["pu"], epu)
    np.testing.assert_array_equal(res[0]["bu"], ebu)
    np.testing.assert_allclose(res[0]["qi"], eqi, rtol=0, atol=1e-15)
    np.testing.assert_allclose(res[0]["bi"], ebi, rtol=0, atol=1e-15)


def test_chunk_users_groups_long_chains():
    """A few users whose chains outlast a chunk (> 1/256 of its ratings) all land in chunk 0
    (the full C5's 9 users of 200k-600k ratings); many such users, or one, leave the
    round-robin dealing unchanged."""
    rng = np.random.RandomState(2)
    deg = rng.randint(1, 100, size=100_000)
    deg[[5, 77, 900, 4242]] = [60_000, 50_000, 40_000, 30_000]
    row_ptr = np.concatenate([[0], np.cumsum(deg)])
    chunks = chunk_users(np.arange(len(deg)), row_ptr, 8)
    assert set(chunks[0][:4].tolist()) == {5, 77, 900, 4242}
    assert all(not ({5, 77, 900, 4242} & set(c.tolist())) for c in chunks[1:])
    np.testing.assert_array_equal(np.sort(np.concatenate(chunks)), np.arange(len(deg)))
    for c in chunks:
        assert np.all(np.diff(deg[c]) <= 0)
    deg[[5, 77, 900, 4242]] = 50  # no long chain: plain round-robin
    row_ptr = np.concatenate([[0], np.cumsum(deg)])
    srt = np.argsort(-deg, kind="stable")
    for c, us in enumerate(chunk_users(np.arange(len(deg)), row_ptr, 8)):
        np.testing.assert_array_equal(us, srt[c::8])


def test_chunk_users_long_chain_branch_fires_on_the_c5_miniature():
    """the C5 miniature the GPU test pins (the first 60k users of configs[4]'s
    shape at 8 epoch-chunks, bench.py --shape c5 --users 60000 --chunks 8) has 8 users above
    1/256 of a chunk's ratings: the long-chain branch puts all 8 in chunk 0; long_chain=0 (the
    engine option of the same name) deals them round-robin, one per chunk."""
    from surprise_amd import synthetic
    U, I, N = synthetic.SHAPES["c5"]
    deg = synthetic.sharded_truth(U, I, N)["deg"][:60_000]
    row_ptr = np.concatenate([[0], np.cumsum(deg)])
    thr = deg.sum() / 8 / 256
    long_users = set(np.flatnonzero(deg > thr).tolist())
    assert len(long_users) == 8
    chunks = chunk_users(np.arange(len(deg)), row_ptr, 8)
    assert set(chunks[0][:8].tolist()) == long_users
    old = chunk_users(np.arange(len(deg)), row_ptr, 8, long_chain=0)
    assert [len(long_users & set(c.tolist())) for c in old] == [1] * 8
    for cs in (chunks, old):
        np.testing.assert_array_equal(np.sort(np.concatenate(cs)), np.arange(len(deg)))
