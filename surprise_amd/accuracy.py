"""Accuracy metrics, mirroring surprise/accuracy.py:22-143 (rmse, mae, fcp)."""

import numpy as np


def rmse(predictions, verbose=True):
    """sqrt(np.mean of squared errors) over (uid, iid, r_ui, est, details) tuples (accuracy.py:22-54)."""
    if not predictions:
        raise ValueError("Prediction list is empty.")
    mse = np.mean([float((true_r - est) ** 2) for (_, _, true_r, est, _) in predictions])
    rmse_ = np.sqrt(mse)
    if verbose:
        print("RMSE: {0:1.4f}".format(rmse_))
    return rmse_


def mae(predictions, verbose=True):
    """accuracy.py:57-88."""
    if not predictions:
        raise ValueError("Prediction list is empty.")
    mae_ = np.mean([float(abs(true_r - est)) for (_, _, true_r, est, _) in predictions])
    if verbose:
        print("MAE:  {0:1.4f}".format(mae_))
    return mae_



def fcp(predictions, verbose=True):
    """Fraction of Concordant Pairs (accuracy.py:91-143; Koren & Sill, 5.2).  Per user, over
    the ordered pairs of its predictions: concordant = est_i > est_j and r_i > r_j,
    discordant = est_i >= est_j and r_i < r_j.  As in the reference, each mean runs over the
    users with at least one pair of that kind; ValueError when neither kind occurs."""
    if not predictions:
        raise ValueError("Prediction list is empty.")
    by_user = {}
    for uid, _, true_r, est, _ in predictions:
        by_user.setdefault(uid, []).append((true_r, est))
    nc, nd = [], []
    for pairs in by_user.values():
        a = np.asarray(pairs, dtype=np.float64)
        r, e = a[:, 0], a[:, 1]
        c = int(np.count_nonzero((e[:, None] > e[None, :]) & (r[:, None] > r[None, :])))
        d = int(np.count_nonzero((e[:, None] >= e[None, :]) & (r[:, None] < r[None, :])))
        if c:
            nc.append(c)
        if d:
            nd.append(d)
    mc = np.mean(nc) if nc else 0
    md = np.mean(nd) if nd else 0
    if mc + md == 0:
        raise ValueError("cannot compute fcp on this list of prediction. Does every user have "
                         "at least two predictions?")
    fcp_ = mc / (mc + md)
    if verbose:
        print("FCP:  {0:1.4f}".format(fcp_))
    return fcp_
