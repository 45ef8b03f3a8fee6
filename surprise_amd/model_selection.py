"""Cross-validation harness around the hot path, mirroring
surprise/model_selection/split.py (get_cv :44-55, KFold :58-122, PredefinedKFold
:654-685) and surprise/model_selection/validation.py (cross_validate :29-142,
fit_and_score :683-769).  ShuffleSplit / train_test_split / print_summary are not
on the SVD path (out of scope) and are not mirrored.

Index logic is the reference's, so a fold built here holds the same ratings in
the same order as the reference's fold for the same seed; array-native
datasets (``RatingColumns``) are indexed without Python tuples.
"""
import numbers
import time

import numpy as np

from . import accuracy
from .dataset import RatingColumns
from .utils import get_rng


def get_cv(cv):
    if cv is None:
        return KFold(n_splits=5)
    if isinstance(cv, numbers.Integral):
        return KFold(n_splits=cv)
    if hasattr(cv, "split") and not isinstance(cv, str):
        return cv
    raise ValueError("Wrong CV object. Expecting None, an int or CV iterator, "
                     "got a {}".format(type(cv)))


def _subset(raw, idx):
    if isinstance(raw, RatingColumns):
        return raw.take(np.asarray(idx, dtype=np.int64))
    return [raw[i] for i in idx]


class KFold:
    """split.py:58-122: shuffle np.arange(n) with get_rng(random_state), then
    contiguous folds; fold i gets one extra rating while i < n % n_splits."""

    def __init__(self, n_splits=5, random_state=None, shuffle=True):
        self.n_splits = n_splits
        self.shuffle = shuffle
        self.random_state = random_state

    def fold_indices(self, n):
        if self.n_splits > n or self.n_splits < 2:
            raise ValueError("Incorrect value for n_splits={0}. Must be >=2 and less than the "
                             "number of ratings".format(n))
        indices = np.arange(n)
        if self.shuffle:
            get_rng(self.random_state).shuffle(indices)
        start, stop = 0, 0
        for i_fold in range(self.n_splits):
            start = stop
            stop += n // self.n_splits
            if i_fold < n % self.n_splits:
                stop += 1
            yield np.concatenate([indices[:start], indices[stop:]]), indices[start:stop]

    def split(self, data):
        for train_idx, test_idx in self.fold_indices(len(data.raw_ratings)):
            raw_trainset = _subset(data.raw_ratings, train_idx)
            raw_testset = _subset(data.raw_ratings, test_idx)
            yield data.construct_trainset(raw_trainset), data.construct_testset(raw_testset)

    def get_n_folds(self):
        return self.n_splits


class PredefinedKFold:
    """split.py:654-685."""

    def split(self, data):
        self.n_splits = len(data.folds_files)
        for train_file, test_file in data.folds_files:
            raw_trainset = data.read_ratings(train_file)
            raw_testset = data.read_ratings(test_file)
            yield data.construct_trainset(raw_trainset), data.construct_testset(raw_testset)

    def get_n_folds(self):
        return self.n_splits


def fit_and_score(algo, trainset, testset, measures, return_train_measures=False,
                  crossfold_index=None):
    """validation.py:683-769 for a single list testset; returns the fork's 6-tuple
    (test_measures, train_measures, fit_time, test_time, num_tested, crossfold_index)."""
    start_fit = time.time()
    algo.fit(trainset)
    fit_time = time.time() - start_fit
    start_test = time.time()
    predictions = algo.test(testset)
    test_time = time.time() - start_test
    if not predictions:
        return {}, {}, 0, 0, 0, 0
    if return_train_measures:
        train_predictions = algo.test(trainset.build_testset())
    test_measures, train_measures = {}, {}
    for m in measures:
        f = getattr(accuracy, m.lower())
        test_measures[m] = f(predictions, verbose=0)
        if return_train_measures:
            train_measures[m] = f(train_predictions, verbose=0)
    return test_measures, train_measures, fit_time, test_time, {}, crossfold_index


def cross_validate(algo, data, measures=["rmse", "mae"], cv=None, return_train_measures=False,
                   n_jobs=1, pre_dispatch="2*n_jobs", verbose=False):
    """validation.py:29-142.  Folds run in this process (n_jobs is accepted for
    signature compatibility): one process owns the GPU, so the reference's joblib
    fan-out over folds (validation.py:109-112) would only oversubscribe it."""
    measures = [m.lower() for m in measures]
    cv = get_cv(cv)
    out = [fit_and_score(algo, trainset, testset, measures, return_train_measures)
           for (trainset, testset) in cv.split(data)]
    (test_measures_dicts, train_measures_dicts, fit_times, test_times, num_tested, _) = zip(*out)
    test_measures, train_measures, ret = {}, {}, {}
    for m in test_measures_dicts[0]:
        test_measures[m] = np.asarray([d[m] for d in test_measures_dicts])
        ret["test_" + m] = test_measures[m]
        if return_train_measures:
            train_measures[m] = np.asarray([d[m] for d in train_measures_dicts])
            ret["train_" + m] = test_measures[m]  # sic: validation.py:134
    ret["fit_time"] = fit_times
    ret["test_time"] = test_times
    ret["num_tested"] = [num_tested for _ in fit_times]
    if verbose:  # (the reference's print_summary table is not on the hot path)
        for m, vals in test_measures.items():
            print("{} (testset): mean {:1.4f} std {:1.4f}".format(m.upper(), np.mean(vals),
                                                                  np.std(vals)))
    return ret

