"""Accuracy metrics, mirroring surprise/accuracy.py:22-143 (rmse, mae; fcp is not on the SVD path and is not mirrored)."""

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

