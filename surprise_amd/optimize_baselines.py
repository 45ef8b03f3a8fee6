"""Baseline estimates on the device, mirroring
surprise/prediction_algorithms/optimize_baselines.pyx (baseline_als :14-54, baseline_sgd
:57-84).  Called by AlgoBase.compute_baselines (algo_base.py:220-254) with the algorithm as
``self``; ``bsl_options`` keys and defaults as in the reference."""
import numpy as np

from . import _lib


def _trainset(self):
    from .matrix_factorization import _as_trainset
    return _as_trainset(self.trainset)


def baseline_als(self):
    """b_i then b_u, n_epochs times (defaults n_epochs=10, reg_u=15, reg_i=10): one HIP launch
    per side per epoch (mf_baseline_als_epoch)."""
    from .engine import baseline_als_device
    ts = _trainset(self)
    o = self.bsl_options
    return baseline_als_device(ts.csr(), ts.csc(), ts.n_items, ts.global_mean,
                               int(o.get("n_epochs", 10)), float(o.get("reg_u", 15)),
                               float(o.get("reg_i", 10)))


def baseline_sgd(self):
    """SGD on the biases alone (defaults n_epochs=20, reg=0.02, learning_rate=0.005): the SVD
    epoch kernel with n_factors = 0, in its default race-free "log" schedule."""
    from .engine import MFEngine
    _lib.require_gpu()
    ts = _trainset(self)
    o = self.bsl_options
    lr, reg = float(o.get("learning_rate", .005)), float(o.get("reg", .02))
    hyper = dict(lr_bu=lr, lr_bi=lr, reg_bu=reg, reg_bi=reg, global_mean=float(ts.global_mean))
    eng = MFEngine(ts.csr(), ts.n_items, 0, hyper=hyper, biased=True, dtype="float64",
                   mode="log")
    eng.set_factors(np.zeros((ts.n_users, 0)), np.zeros((ts.n_items, 0)))
    eng.run_epochs(int(o.get("n_epochs", 20)))
    f = eng.get_factors()
    return f["bu"], f["bi"]
