"""Where a whole fit() spends its time (host setup vs epochs): cProfile of SVD / SVD++ fit on
the ML-1M shape, second fit (first one warms the library and the caching allocator)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from surprise_amd import SVD, SVDpp, Dataset, synthetic  # noqa: E402
from surprise_amd.model_selection import KFold  # noqa: E402

u, i, r = synthetic.shape("ml-1m")
ts, test = next(KFold(5, random_state=0).split(Dataset.load_from_arrays(u, i, r)))
for cls, ep in ((SVD, 20), (SVDpp, 20)):
    cls(n_factors=100, n_epochs=ep, random_state=0).fit(ts)
    torch.cuda.synchronize()
    t = time.perf_counter()
    pr = cProfile.Profile()
    pr.enable()
    cls(n_factors=100, n_epochs=ep, random_state=0).fit(ts)
    torch.cuda.synchronize()
    pr.disable()
    print("%s fit %d epochs: %.1f ms" % (cls.__name__, ep, (time.perf_counter() - t) * 1e3))
    pstats.Stats(pr).sort_stats("cumulative").print_stats(22)
