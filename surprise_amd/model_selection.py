"""Cross-validation harness around the hot path, mirroring
surprise/model_selection/split.py (get_cv :44-55, KFold :58-122, ShuffleSplit :422-540,
train_test_split :543-576, PredefinedKFold :654-685) and
surprise/model_selection/validation.py (cross_validate :29-142, fit_and_score :683-769,
print_summary :772-811).

Index logic is the reference's, so a fold built here holds the same ratings in
the same order as the reference's fold for the same seed; array-native
datasets (``RatingColumns``) are indexed without Python tuples.
"""
import math
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


class ShuffleSplit:
    """split.py:422-540: n_splits independent random (trainset, testset) splits.  test_size /
    train_size: a float is a proportion (test rounded up, train down), an int a count, None the
    complement of the other; permutations come from get_rng(random_state) (np.arange without
    shuffle).  The trainset takes the first train_size ratings of the permutation, the testset
    the next test_size."""

    def __init__(self, n_splits=5, test_size=.2, train_size=None, random_state=None,
                 shuffle=True):
        if n_splits <= 0:
            raise ValueError("n_splits = {0} should be strictly greater than 0.".format(n_splits))
        if test_size is not None and test_size <= 0:
            raise ValueError("test_size={0} should be strictly greater than 0".format(test_size))
        if train_size is not None and train_size <= 0:
            raise ValueError("train_size={0} should be strictly greater than 0".format(train_size))
        self.n_splits = n_splits
        self.test_size = test_size
        self.train_size = train_size
        self.random_state = random_state
        self.shuffle = shuffle

    def validate_train_test_sizes(self, test_size, train_size, n_ratings):
        """(train count, test count) for n_ratings ratings; ValueError as the reference."""
        for name, v in (("test_size", test_size), ("train_size", train_size)):
            if v is not None and v >= n_ratings:
                raise ValueError("{0}={1} should be less than the number of ratings {2}"
                                 .format(name, v, n_ratings))
        if np.asarray(test_size).dtype.kind == "f":
            test_size = math.ceil(test_size * n_ratings)
        if train_size is None:
            train_size = n_ratings - test_size
        elif np.asarray(train_size).dtype.kind == "f":
            train_size = math.floor(train_size * n_ratings)
        if test_size is None:
            test_size = n_ratings - train_size
        if train_size + test_size > n_ratings:
            raise ValueError("The sum of train_size and test_size ({0}) should be smaller than "
                             "the number of ratings {1}.".format(train_size + test_size,
                                                                 n_ratings))
        return int(train_size), int(test_size)

    def split(self, data):
        n = len(data.raw_ratings)
        n_train, n_test = self.validate_train_test_sizes(self.test_size, self.train_size, n)
        rng = get_rng(self.random_state)
        for _ in range(self.n_splits):
            perm = rng.permutation(n) if self.shuffle else np.arange(n)
            yield (data.construct_trainset(_subset(data.raw_ratings, perm[:n_train])),
                   data.construct_testset(_subset(data.raw_ratings,
                                                  perm[n_train:n_train + n_test])))

    def get_n_folds(self):
        return self.n_splits


def train_test_split(data, test_size=.2, train_size=None, random_state=None, shuffle=True):
    """split.py:543-576: one ShuffleSplit split -> (trainset, testset)."""
    return next(ShuffleSplit(n_splits=1, test_size=test_size, train_size=train_size,
                             random_state=random_state, shuffle=shuffle).split(data))


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
    if verbose:
        print_summary(algo, measures, test_measures, train_measures, fit_times, test_times,
                      cv.n_splits)
    return ret


def print_summary(algo, measures, test_measures, train_measures, fit_times, test_times,
                  n_splits):
    """validation.py:772-811: the per-fold table cross_validate(verbose=True) prints."""
    print("Evaluating {0} of algorithm {1} on {2} split(s).".format(
        ", ".join(m.upper() for m in measures), algo.__class__.__name__, n_splits))
    print()
    fmt = "{:<18}" + "{:<8}" * (n_splits + 2)

    def row(label, vals, f):
        return fmt.format(label, *[f.format(v) for v in vals] +
                          [f.format(np.mean(vals)), f.format(np.std(vals))])

    lines = [fmt.format("", *["Fold {0}".format(i + 1) for i in range(n_splits)] +
                        ["Mean", "Std"])]
    lines += [row(k.upper() + " (testset)", v, "{:1.4f}") for k, v in test_measures.items()]
    lines += [row(k.upper() + " (trainset)", v, "{:1.4f}") for k, v in train_measures.items()]
    lines += [row("Fit time", fit_times, "{:.2f}"), row("Test time", test_times, "{:.2f}")]
    print("\n".join(lines))

