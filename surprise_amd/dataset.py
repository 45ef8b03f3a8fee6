"""Datasets, mirroring surprise/dataset.py:47-375.

Inner ids are assigned by first appearance (dataset.py:219-234) -- done here
with ``pandas.factorize``, which numbers keys in order of first appearance --
and ratings keep their insertion order per user, so the resulting Trainset
iterates exactly like the reference's.  ``load_builtin`` never downloads (no
network): it reads the file if it is already at the reference's path.
"""
import itertools
import os
import random
import warnings

import numpy as np
import pandas as pd

from .reader import BUILTIN_DATASETS, Reader
from .trainset import Trainset


class RatingColumns:
    """Column-store raw ratings (uid, iid, rating[, timestamp]) for array-native
    datasets: the analogue of the reference's list of 4-tuples for data too large
    for Python objects.  Indexing by an int returns a 4-tuple, by an index array
    returns a RatingColumns; iteration yields (uid, iid, rating) 3-tuples, the
    shape of a testset."""

    def __init__(self, uid, iid, rating, timestamp=None):
        self.uid = np.asarray(uid)
        self.iid = np.asarray(iid)
        self.rating = np.asarray(rating, dtype=np.float64)
        self.timestamp = timestamp

    def __len__(self):
        return len(self.rating)

    def __getitem__(self, idx):
        if isinstance(idx, (int, np.integer)):
            return (self.uid[idx].item(), self.iid[idx].item(), float(self.rating[idx]), None)
        return RatingColumns(self.uid[idx], self.iid[idx], self.rating[idx])

    def __iter__(self):
        return zip(self.uid.tolist(), self.iid.tolist(), self.rating.tolist())

    def take(self, idx):
        return RatingColumns(self.uid[idx], self.iid[idx], self.rating[idx])


def _columns(raw):
    """(uid, iid, rating) columns of a raw rating collection (list of tuples,
    structured array or RatingColumns)."""
    if isinstance(raw, RatingColumns):
        return raw.uid, raw.iid, raw.rating
    if isinstance(raw, np.ndarray) and raw.dtype.names:
        return raw["uid"], raw["iid"], raw["rating"].astype(np.float64)
    if len(raw) == 0:
        return np.array([]), np.array([]), np.array([], np.float64)
    cols = list(zip(*raw))
    uid = np.empty(len(raw), dtype=object)
    uid[:] = cols[0]
    iid = np.empty(len(raw), dtype=object)
    iid[:] = cols[1]
    return uid, iid, np.asarray(cols[2], dtype=np.float64)


class Dataset:
    """Base class (dataset.py:47-56); use the load_* class methods."""

    def __init__(self, reader):
        self.reader = reader

    @classmethod
    def load_builtin(cls, name="ml-100k"):
        try:
            dataset = BUILTIN_DATASETS[name]
        except KeyError:
            raise ValueError("unknown dataset " + name + ". Accepted values are " +
                             ", ".join(BUILTIN_DATASETS.keys()) + ".")
        if not os.path.isfile(dataset.path):
            raise ValueError("Dataset " + name + " is not at " + dataset.path +
                             " and cannot be downloaded (no network).")
        reader = Reader(**dataset.reader_params)
        return cls.load_from_file(file_path=dataset.path, reader=reader)

    @classmethod
    def load_from_file(cls, file_path, reader):
        return DatasetAutoFolds(ratings_file=file_path, reader=reader)

    @classmethod
    def load_from_folds(cls, folds_files, reader):
        return DatasetUserFolds(folds_files=folds_files, reader=reader)

    @classmethod
    def load_from_df(cls, df, reader):
        return DatasetAutoFolds(reader=reader, df=df)

    @classmethod
    def load_from_arrays(cls, uid, iid, rating, reader=None):
        """Array-native dataset (no reference counterpart; SURVEY.md 7 step 3 ``fit_arrays``).
        Ratings are shifted by reader.offset like Reader.parse_line does."""
        reader = reader or Reader()
        return DatasetAutoFolds(reader=reader, columns=RatingColumns(
            uid, iid, np.asarray(rating, np.float64) + reader.offset))

    def read_ratings(self, file_name):
        with open(os.path.expanduser(file_name)) as f:
            raw_ratings = [self.reader.parse_line(line) for line in
                           itertools.islice(f, self.reader.skip_lines, None)]
        return raw_ratings

    def folds(self):
        warnings.warn("Using data.split() or using load_from_folds() without using a CV iterator "
                      "is now deprecated. ", UserWarning)
        for raw_trainset, raw_testset in self.raw_folds():
            yield self.construct_trainset(raw_trainset), self.construct_testset(raw_testset)

    def construct_trainset(self, raw_trainset):
        """dataset.py:201-250 (inner ids by first appearance, ur/ir insertion order)."""
        uid, iid, r = _columns(raw_trainset)
        ucodes, uniq_u = pd.factorize(uid, sort=False, use_na_sentinel=False)
        icodes, uniq_i = pd.factorize(iid, sort=False, use_na_sentinel=False)
        raw2inner_u = {k: n for n, k in enumerate(np.asarray(uniq_u).tolist())}
        raw2inner_i = {k: n for n, k in enumerate(np.asarray(uniq_i).tolist())}
        return Trainset.from_inner_arrays(
            ucodes.astype(np.int64), icodes.astype(np.int32), r, n_users=len(uniq_u),
            n_items=len(uniq_i), rating_scale=self.reader.rating_scale,
            offset=self.reader.offset, raw2inner_id_users=raw2inner_u,
            raw2inner_id_items=raw2inner_i)

    def construct_testset(self, raw_testset):
        """dataset.py:252-257."""
        if isinstance(raw_testset, RatingColumns):
            return raw_testset
        if isinstance(raw_testset, np.ndarray):
            return raw_testset[["uid", "iid", "rating"]]
        return [(ruid, riid, r_ui_trans) for (ruid, riid, r_ui_trans, _) in raw_testset]


class DatasetUserFolds(Dataset):
    """Predefined folds (dataset.py:260-280)."""

    def __init__(self, folds_files=None, reader=None):
        Dataset.__init__(self, reader)
        self.folds_files = folds_files
        for train_test_files in self.folds_files:
            for f in train_test_files:
                if not os.path.isfile(os.path.expanduser(f)):
                    raise ValueError("File " + str(f) + " does not exist.")

    def raw_folds(self):
        for train_file, test_file in self.folds_files:
            yield self.read_ratings(train_file), self.read_ratings(test_file)


class DatasetAutoFolds(Dataset):
    """Folds not predefined (dataset.py:283-375)."""

    def __init__(self, ratings_file=None, reader=None, df=None, columns=None):
        Dataset.__init__(self, reader)
        self.has_been_split = False
        if ratings_file is not None:
            self.ratings_file = ratings_file
            self.raw_ratings = self.read_ratings(self.ratings_file)
        elif df is not None:
            # the fork stores a structured array with int32 ids (dataset.py:295-304)
            self.raw_ratings = np.array(
                [(uid, iid, float(r) + self.reader.offset, 0)
                 for (uid, iid, r) in df.itertuples(index=False)],
                dtype=[("uid", "int32"), ("iid", "int32"), ("rating", float),
                       ("timestamp", bool)])
        elif columns is not None:
            self.raw_ratings = columns
        else:
            raise ValueError("Must specify ratings file or dataframe.")

    def build_full_trainset(self):
        return self.construct_trainset(self.raw_ratings)

    def raw_folds(self):
        if not self.has_been_split:
            self.split()

        def k_folds(seq, n_folds):
            start, stop = 0, 0
            for fold_i in range(n_folds):
                start = stop
                stop += len(seq) // n_folds
                if fold_i < len(seq) % n_folds:
                    stop += 1
                yield seq[:start] + seq[stop:], seq[start:stop]

        return k_folds(self.raw_ratings, self.n_folds)

    def return_raw_data(self):
        return self.raw_ratings

    def split(self, n_folds=5, shuffle=True):
        if n_folds > len(self.raw_ratings) or n_folds < 2:
            raise ValueError("Incorrect value for n_folds. Must be >=2 and less than the number "
                             "or entries")
        if shuffle:
            random.shuffle(self.raw_ratings)
        self.n_folds = n_folds
        self.has_been_split = True
