"""AlgoBase -- the plugin API the hot path sits behind, mirroring
surprise/prediction_algorithms/algo_base.py:22-254 (fit / train / predict /
default_prediction / test / compute_baselines).  The similarity helpers (:256-334) belong to
the k-NN family and are out of scope.
"""
import warnings

import numpy as np

from .predictions import Prediction, PredictionImpossible


class AlgoBase:

    def __init__(self, **kwargs):
        self.bsl_options = kwargs.get("bsl_options", {})
        self.sim_options = kwargs.get("sim_options", {})
        if "user_based" not in self.sim_options:
            self.sim_options["user_based"] = True
        self.skip_train = False
        if (type(self).fit is AlgoBase.fit and type(self).train is not AlgoBase.train):
            warnings.warn("It looks like this algorithm (" + str(self.__class__) +
                          ") implements train() instead of fit(): train() is deprecated, "
                          "please use fit() instead.", UserWarning)

    def train(self, trainset):
        """Deprecated (algo_base.py:45-55)."""
        warnings.warn("train() is deprecated. Use fit() instead", UserWarning)
        self.skip_train = True
        self.fit(trainset)
        return self

    def fit(self, trainset):
        """algo_base.py:60-99: set self.trainset, reset baselines."""
        if type(self).train is not AlgoBase.train and not self.skip_train:
            self.train(trainset)
            return
        self.skip_train = False
        self.trainset = trainset
        self.bu = self.bi = None
        return self

    def _inner_ids(self, uid, iid):
        try:
            iuid = self.trainset.to_inner_uid(uid)
        except ValueError:
            iuid = "UKN__" + str(uid)
        try:
            iiid = self.trainset.to_inner_iid(iid)
        except ValueError:
            iiid = "UKN__" + str(iid)
        return iuid, iiid

    def predict(self, uid, iid, r_ui=None, clip=True, verbose=False):
        """algo_base.py:101-176: raw->inner ids ('UKN__' for unknown), estimate,
        PredictionImpossible -> default_prediction, subtract offset, clip."""
        iuid, iiid = self._inner_ids(uid, iid)
        details = {}
        try:
            est = self.estimate(iuid, iiid)
            if isinstance(est, tuple):
                est, details = est
            details["was_impossible"] = False
        except PredictionImpossible as e:
            est = self.default_prediction()
            details["was_impossible"] = True
            details["reason"] = str(e)
        est -= self.trainset.offset
        if clip:
            lower_bound, higher_bound = self.trainset.rating_scale
            est = min(higher_bound, est)
            est = max(lower_bound, est)
        pred = Prediction(uid, iid, r_ui, est, details)
        if verbose:
            print(pred)
        return pred

    def default_prediction(self):
        """algo_base.py:178-189: the trainset's global mean."""
        return self.trainset.global_mean

    def test(self, testset, verbose=False):
        """algo_base.py:191-218."""
        iterate_on = testset.tolist() if isinstance(testset, np.ndarray) else testset
        return [self.predict(uid, iid, r_ui_trans - self.trainset.offset, verbose=verbose)
                for (uid, iid, r_ui_trans) in iterate_on]

    def compute_baselines(self):
        """algo_base.py:220-254: baselines once per trainset, by bsl_options['method']
        ('als' default, or 'sgd'), computed on the device (optimize_baselines.py)."""
        if self.bu is not None:
            return self.bu, self.bi
        from .optimize_baselines import baseline_als, baseline_sgd
        method = dict(als=baseline_als, sgd=baseline_sgd)
        method_name = self.bsl_options.get('method', 'als')
        try:
            fn = method[method_name]
        except KeyError:
            raise ValueError('Invalid method ' + method_name +
                             ' for baseline computation.' +
                             ' Available methods are als and sgd.')
        self.bu, self.bi = fn(self)
        return self.bu, self.bi
