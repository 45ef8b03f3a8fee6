"""BaselineOnly (surprise/prediction_algorithms/baseline_only.py): r_ui = mu + b_u + b_i, the
biases from AlgoBase.compute_baselines (ALS or SGD on the device)."""
from .algo_base import AlgoBase


class BaselineOnly(AlgoBase):
    """baseline_only.py:12-44."""

    def __init__(self, bsl_options={}):
        AlgoBase.__init__(self, bsl_options=bsl_options)

    def fit(self, trainset):
        AlgoBase.fit(self, trainset)
        self.bu, self.bi = self.compute_baselines()
        return self

    def estimate(self, u, i):
        est = self.trainset.global_mean
        if self.trainset.knows_user(u):
            est += self.bu[u]
        if self.trainset.knows_item(i):
            est += self.bi[i]
        return est
