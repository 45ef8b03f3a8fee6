"""surprise_amd -- MI355X-native training path for Surprise's SVD / SVD++ (and, next to it,
NMF and the baseline estimates).

Drop-in for the hot path of nickmvincent/Surprise: ``SVD`` and ``SVDpp`` keep
the ``AlgoBase.fit()/estimate()`` plugin surface, and their SGD epochs run as
hand-written CDNA4 HIP kernels (libsurprise_amd.so, C ABI in
include/surprise_amd.h).  The data model and cross-validation harness around
the path (Reader, Dataset, Trainset, KFold, cross_validate, accuracy) mirror
the reference so that its test code reads the same.
"""
from . import accuracy, dump, model_selection
from .algo_base import AlgoBase
from .dataset import Dataset, RatingColumns
from .baseline_only import BaselineOnly
from .matrix_factorization import NMF, SVD, SVDpp
from .predictions import Prediction, PredictionImpossible
from .reader import Reader, get_dataset_dir
from .trainset import Trainset

__version__ = "0.1.0"

__all__ = ["AlgoBase", "SVD", "SVDpp", "NMF", "BaselineOnly", "PredictionImpossible", "Prediction", "Dataset",
           "RatingColumns", "Reader", "Trainset", "dump", "model_selection", "accuracy",
           "get_dataset_dir"]
