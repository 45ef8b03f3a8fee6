"""Accuracy metrics, mirroring surprise/accuracy.py:22-143 (rmse, mae, fcp)."""
from collections import defaultdict

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
    """Fraction of concordant pairs (accuracy.py:91-143)."""
    if not predictions:
        raise ValueError("Prediction list is empty.")
    predictions_u = defaultdict(list)
    nc_u = defaultdict(int)
    nd_u = defaultdict(int)
    for u0, _, r0, est, _ in predictions:
        predictions_u[u0].append((r0, est))
    for u0, preds in predictions_u.items():
        for r0i, esti in preds:
            for r0j, estj in preds:
                if esti > estj and r0i > r0j:
                    nc_u[u0] += 1
                if esti >= estj and r0i < r0j:
                    nd_u[u0] += 1
    nc = np.mean(list(nc_u.values())) if nc_u else 0
    nd = np.mean(list(nd_u.values())) if nd_u else 0
    try:
        fcp_ = nc / (nc + nd)
    except ZeroDivisionError:
        raise ValueError("cannot compute fcp on this list of prediction. " +
                         "Does every user have at least two predictions?")
    if verbose:
        print("FCP:  {0:1.4f}".format(fcp_))
    return fcp_
