"""Seeded synthetic (u, i, r) streams with planted structure.

There is no MovieLens data offline, and uniform random ratings carry no signal
(RMSE ~1.43), so every synthetic workload is drawn from a planted model:
  * user degrees: minimum 20 (like MovieLens) plus a lognormal share of the rest;
  * item popularity: Zipf-like weights, items drawn per user without repeats;
  * r = clip(round(mu + b_u + b_i + <p_u, q_i> + noise), 1, 5) with rank-10 factors
    ~N(0, 0.3), biases ~N(0, 0.5), mu = 3.58, noise ~N(0, 0.9).
Shapes: ml-100k (943 x 1682, 100,000), ml-1m (6040 x 3706, 1,000,209),
c4 (2M x 200k, 100M), c5 (10M x 1M, 1B), c5-shard (1.25M x 1M, 125M: c5's per-GPU share).  The
stream is returned in a shuffled "file order"; raw ids are ints.
Multi-GPU: ``population`` gives weak scaling (population p = one more ML-1M-shape user set over
the same items; population 0 is the single-GPU dataset) and ``sharded_truth`` /
``sharded_rows`` give the C4 / C5 strong-scaling datasets, of which every rank generates only
its own user rows.
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
            item_beta=0.75, mu=3.58, factor_std=0.3, bias_std=0.5, noise_std=0.9,
            return_truth=False):
    """Returns (uid int32, iid int32, rating float64) in shuffled file order, no duplicate pairs
    (plus the planted item side {cdf, Q, bi} with return_truth)."""
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
    out = users[perm].astype(np.int32), items[perm].astype(np.int32), r[perm]
    if return_truth:
        return out + (dict(cdf=cdf, Q=Q, bi=bi),)
    return out


def _distinct_items(rng, users, n_items, cdf):
    """Popularity-weighted items for the rating slots `users` (sorted by user), resampled until
    every (user, item) pair is distinct (uniform draws after a few weighted rounds)."""
    items = np.minimum(np.searchsorted(cdf, rng.random_sample(len(users))), n_items - 1)
    items = items.astype(np.int64)
    for rnd in range(1000):
        key = users * n_items + items
        order = np.argsort(key)
        ks = key[order]
        dup = np.zeros(len(ks), bool)
        dup[1:] = ks[1:] == ks[:-1]
        if not dup.any():
            return items
        idx = np.sort(order[dup])
        if rnd < 3:
            items[idx] = np.minimum(np.searchsorted(cdf, rng.random_sample(len(idx))), n_items - 1)
        else:
            items[idx] = rng.randint(0, n_items, len(idx))
    raise RuntimeError("could not draw distinct (user, item) pairs")


def population(p, n_users, n_items, n_ratings, seed=0, rank=10, min_deg=20, user_sigma=1.1,
               mu=3.58, factor_std=0.3, bias_std=0.5, noise_std=0.9):
    """User population p of a weak-scaling dataset: population 0 IS planted(n_users, n_items,
    n_ratings, seed) (BASELINE configs[1]'s synthetic ML-1M); population p >= 1 draws its own
    users (degrees, items, factors, biases, noise; RandomState([seed, 1000 + p])) against the
    SAME planted item side, so the union of populations is one dataset over one item set.
    Returns (uid, iid, r) with population-local user ids, shuffled file order."""
    if p == 0:
        return planted(n_users, n_items, n_ratings, rank, seed, min_deg, user_sigma,
                       mu=mu, factor_std=factor_std, bias_std=bias_std, noise_std=noise_std)
    *_, truth = planted(n_users, n_items, n_ratings, rank, seed, min_deg, user_sigma, mu=mu,
                        factor_std=factor_std, bias_std=bias_std, noise_std=noise_std,
                        return_truth=True)
    rng = np.random.RandomState([seed, 1000 + p])
    deg = _user_degrees(rng, n_users, n_items, n_ratings, min_deg, user_sigma)
    users = np.repeat(np.arange(n_users, dtype=np.int64), deg)
    items = _distinct_items(rng, users, n_items, truth["cdf"])
    P = rng.normal(0, factor_std, (n_users, rank))
    bu = rng.normal(0, bias_std, n_users)
    r = (mu + bu[users] + truth["bi"][items] + np.einsum("nk,nk->n", P[users], truth["Q"][items])
         + rng.normal(0, noise_std, len(users)))
    r = np.clip(np.rint(r), 1, 5)
    perm = rng.permutation(len(users))
    return users[perm].astype(np.int32), items[perm].astype(np.int32), r[perm]


BLOCK_USERS = 1 << 16  # users per generation block of the sharded generator


def sharded_truth(n_users, n_items, n_ratings, seed=0, rank=10, min_deg=20, user_sigma=1.1,
                  item_beta=0.75, factor_std=0.3, bias_std=0.5):
    """Global side of a sharded planted dataset (C4 / C5 shapes): item popularity cdf, item
    factors / biases, and every user's degree.  Cheap next to the ratings (O(U + I))."""
    rng = np.random.RandomState([seed, 0])
    pop = np.arange(1, n_items + 1, dtype=np.float64) ** (-item_beta)
    rng.shuffle(pop)
    cdf = np.cumsum(pop)
    cdf /= cdf[-1]
    Q = rng.normal(0, factor_std, (n_items, rank))
    bi = rng.normal(0, bias_std, n_items)
    deg = _user_degrees(np.random.RandomState([seed, 1]), n_users, n_items, n_ratings, min_deg,
                        user_sigma)
    return dict(cdf=cdf, Q=Q, bi=bi, deg=deg, n_items=n_items, seed=seed, rank=rank)


def _block_rows(truth, b, lo, hi, holdout, mu, factor_std, bias_std, noise_std):
    I, rank, deg = truth["n_items"], truth["rank"], truth["deg"]
    b0, b1 = b * BLOCK_USERS, min((b + 1) * BLOCK_USERS, len(deg))
    rng = np.random.RandomState([truth["seed"], 2, b])
    d = deg[b0:b1]
    users = np.repeat(np.arange(b1 - b0, dtype=np.int64), d)
    items = _distinct_items(rng, users, I, truth["cdf"])
    P = rng.normal(0, factor_std, (b1 - b0, rank))
    bu = rng.normal(0, bias_std, b1 - b0)
    r = (mu + bu[users] + truth["bi"][items] +
         np.einsum("nk,nk->n", P[users], truth["Q"][items]) +
         rng.normal(0, noise_std, len(users)))
    r = np.clip(np.rint(r), 1, 5)
    test = rng.random_sample(len(users)) < holdout
    keep = (users + b0 >= lo) & (users + b0 < hi)
    tr, te = keep & ~test, keep & test
    n = np.bincount(users[tr], minlength=b1 - b0)[max(lo - b0, 0):min(hi, b1) - b0]
    return (items[tr].astype(np.int32), r[tr], n,
            (users[te] + b0 - lo, items[te].astype(np.int32), r[te]))


def sharded_rows(truth, lo, hi, holdout=0.01, mu=3.58, factor_std=0.3, bias_std=0.5,
                 noise_std=0.9, threads=8):
    """Users [lo, hi) of a sharded planted dataset, generated block by block (block b of
    BLOCK_USERS users from RandomState([seed, 2, b]): any rank regenerates exactly its own
    rows, independent of the world size; blocks run on `threads` host threads).  Returns the
    rank-local training CSR (row_ptr from 0, items int32, ratings float64, ratings of a user in
    draw order) and the held-out triples (local user id, item, rating): each rating is held
    out with probability `holdout`."""
    from concurrent.futures import ThreadPoolExecutor
    blocks = range(lo // BLOCK_USERS, -(-hi // BLOCK_USERS))
    job = lambda b: _block_rows(truth, b, lo, hi, holdout, mu, factor_std, bias_std, noise_std)
    with ThreadPoolExecutor(max(1, threads)) as ex:
        parts = list(ex.map(job, blocks))
    row_ptr = np.zeros(hi - lo + 1, np.int64)
    np.cumsum(np.concatenate([p[2] for p in parts]), out=row_ptr[1:])
    test = tuple(np.concatenate([p[3][x] for p in parts]) for x in range(3))
    csr = (row_ptr, np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
    return csr, test


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
