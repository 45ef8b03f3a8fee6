"""Seeded synthetic (u, i, r) streams with planted structure.

There is no MovieLens data offline, and uniform random ratings carry no signal
(RMSE ~1.43), so every synthetic workload is drawn from a planted model:
  * user degrees: minimum 20 (like MovieLens) plus a lognormal share of the rest;
  * item popularity: Zipf-like weights, items drawn per user without repeats;
  * r = clip(round(mu + b_u + b_i + <p_u, q_i> + noise), 1, 5) with rank-10 factors
    ~N(0, 0.3), biases ~N(0, 0.5), mu = 3.58, noise ~N(0, 0.9).
Shapes: ml-100k (943 x 1682, 100,000), ml-1m (6040 x 3706, 1,000,209),
c4 (2M x 200k, 100M), c5 (10M x 1M, 1B), c5-shard (1.25M x 1M, 125M: c5's per-GPU share).  The stream is returned in a shuffled
"file order"; raw ids are ints.
"""
from __future__ import annotations

import numpy as np

SHAPES = {
    "tiny": (60, 40, 1200),
    "ml-100k": (943, 1682, 100_000),
    "ml-1m": (6040, 3706, 1_000_209),
    "c4": (2_000_000, 200_000, 100_000_000),
    "c5": (10_000_000, 1_000_000, 1_000_000_000),
    # one rank's shard of c5 on 8 GPUs: 1/8 of the users with their ratings, every item
    "c5-shard": (1_250_000, 1_000_000, 125_000_000),
}


def _user_degrees(rng, n_users, n_items, n_ratings, min_deg, sigma):
    min_deg = min(min_deg, n_items, n_ratings // max(n_users, 1))
    extra = n_ratings - min_deg * n_users
    w = rng.lognormal(0.0, sigma, n_users)  # MovieLens-like: mean/median ~1.7, long tail
    w /= w.sum()
    deg = min_deg + np.floor(extra * w).astype(np.int64)
    cap = max(min_deg, int(0.6 * n_items))
    deg = np.minimum(deg, cap)
    short = n_ratings - int(deg.sum())
    # hand the remainder out one by one to users below the cap, lightest first
    i = n_users - 1
    while short > 0 and i >= 0:
        room = cap - deg[i]
        take = min(room, short)
        deg[i] += take
        short -= take
        i -= 1
    return deg


def planted(n_users, n_items, n_ratings, rank=10, seed=0, min_deg=20, user_sigma=1.1,
            item_beta=0.75, mu=3.58, factor_std=0.3, bias_std=0.5, noise_std=0.9):
    """Returns (uid int32, iid int32, rating float64) in shuffled file order, no duplicate pairs."""
    rng = np.random.RandomState(seed)
    deg = _user_degrees(rng, n_users, n_items, n_ratings, min_deg, user_sigma)
    pop = np.arange(1, n_items + 1, dtype=np.float64) ** (-item_beta)
    rng.shuffle(pop)
    cdf = np.cumsum(pop)
    cdf /= cdf[-1]

    users = np.repeat(np.arange(n_users, dtype=np.int64), deg)
    items = np.searchsorted(cdf, rng.random_sample(len(users))).astype(np.int64)
    items = np.minimum(items, n_items - 1)
    # resample colliding (user, item) pairs until every pair is distinct; after a few
    # popularity-weighted rounds fall back to uniform draws (heavy users saturate the head)
    for rnd in range(1000):
        key = users * n_items + items
        order = np.argsort(key, kind="stable")
        ks = key[order]
        dup = np.zeros(len(ks), bool)
        dup[1:] = ks[1:] == ks[:-1]
        if not dup.any():
            break
        idx = order[dup]
        if rnd < 8:
            items[idx] = np.minimum(np.searchsorted(cdf, rng.random_sample(len(idx))), n_items - 1)
        else:
            items[idx] = rng.randint(0, n_items, len(idx))
    else:
        raise RuntimeError("could not draw distinct (user, item) pairs")

    P = rng.normal(0, factor_std, (n_users, rank))
    Q = rng.normal(0, factor_std, (n_items, rank))
    bu = rng.normal(0, bias_std, n_users)
    bi = rng.normal(0, bias_std, n_items)
    r = np.empty(len(users), np.float64)
    step = 1 << 22
    for s in range(0, len(users), step):
        u, i = users[s:s + step], items[s:s + step]
        r[s:s + step] = (mu + bu[u] + bi[i] + np.einsum("nk,nk->n", P[u], Q[i]) +
                         rng.normal(0, noise_std, len(u)))
    r = np.clip(np.rint(r), 1, 5)
    perm = rng.permutation(len(users))
    return users[perm].astype(np.int32), items[perm].astype(np.int32), r[perm]


def shape(name: str, seed: int = 0):
    U, I, N = SHAPES[name]
    return planted(U, I, N, seed=seed)


def kfold_first_fold(uid, iid, r, n_splits=5, random_state=0):
    """Fold 0 of KFold(n_splits, random_state) over the stream (split.py:103-122),
    as (train columns, test columns) in the reference's raw order."""
    from .model_selection import KFold
    train_idx, test_idx = next(KFold(n_splits, random_state=random_state).fold_indices(len(r)))
    return (uid[train_idx], iid[train_idx], r[train_idx]), (uid[test_idx], iid[test_idx],
                                                          r[test_idx])
