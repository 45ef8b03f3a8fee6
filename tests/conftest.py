import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # test infrastructure: the parity oracle


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: takes more than a few seconds")


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        meta = json.load(f)
    arrays = dict(np.load(os.path.join(GOLDEN, "golden_arrays.npz")))
    return meta, arrays


@pytest.fixture(scope="session")
def u1():
    """(trainset, testset) of the reference's u1 fixture through this repo's mirror."""
    from surprise_amd import Dataset, Reader
    from surprise_amd.model_selection import PredefinedKFold
    data = Dataset.load_from_folds([(os.path.join(GOLDEN, "u1_ml100k_train"),
                                     os.path.join(GOLDEN, "u1_ml100k_test"))], Reader("ml-100k"))
    return next(PredefinedKFold().split(data))
