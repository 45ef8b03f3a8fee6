"""Child process of tests/test_gpu_ext.py::test_svdpp_helper_ring_failure_paths: an SVD++ fit
(u1, K=20, 20 epochs, the helper-wave launch) on the MF_HX_SPIN_TEST build of the library
(SURPRISE_AMD_LIB), whose bounded ring waits give up at once when the status word carries
0x100 (the helpers' wait for rows) / 0x200 (the chain's wait for ring room).
  argv[1] == "helper": both bits -- helpers time out (MF_HX_HELPER_TIMEOUT), the fit must raise
  argv[1] == "chain":  0x200 -- every bank of every chain takes the fallback
                       (MF_HX_CHAIN_FALLBACK), the fit must succeed with intact results"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dispatch_case(out):
    """The test build maps the XCD-masked launches' slot 1 onto slot 0 (MF_DISPATCH_FAULT_TEST):
    an SVD fit with the heavy users' launch on XCD 0 (heavy=16, xcd_split) trains one heavy user
    twice and another never; get_factors must raise (mf_dispatch_check)."""
    from surprise_amd import SVD, _lib
    from surprise_amd.synthetic import shape
    from surprise_amd.trainset import Trainset
    u, i, r = shape("ml-100k")
    ts = Trainset.from_inner_arrays(u, i, r, n_users=int(u.max()) + 1, n_items=int(i.max()) + 1)
    _lib.require_gpu()  # (torch's HIP context first; then the library's own calls)
    res = {"case": "dispatch", "layout": _lib.xcd_layout_ok()}
    algo = SVD(n_factors=20, n_epochs=2, random_state=0)
    algo._engine_options = {"heavy": 16, "xcd_split": True}
    try:
        algo.fit(ts)
        res["raised"] = None
    except _lib.SurpriseAMDError as e:
        res["raised"] = str(e)
    res["heavy_xcd"] = int(getattr(algo._engine, "heavy_xcd", -1)) if algo._engine else None
    with open(out, "w") as f:
        json.dump(res, f)


def main():
    case, out = sys.argv[1], sys.argv[2]
    if case == "dispatch":
        return dispatch_case(out)
    from surprise_amd import Dataset, Reader, SVDpp, _lib, accuracy, engine
    from surprise_amd.model_selection import PredefinedKFold
    assert _lib.LIB_PATH == os.environ["SURPRISE_AMD_LIB"]
    bits = 0x300 if case == "helper" else 0x200
    seen = {}
    orig = engine.MFEngine.set_factors

    def set_factors(self, *a, **k):
        orig(self, *a, **k)
        assert self.hx, "the helper-wave launch is off"
        self._hx_status.fill_(bits)
        seen["engine"] = self

    engine.MFEngine.set_factors = set_factors
    g = os.path.join(ROOT, "tests", "golden")
    data = Dataset.load_from_folds([(os.path.join(g, "u1_ml100k_train"),
                                     os.path.join(g, "u1_ml100k_test"))], Reader("ml-100k"))
    ts, test = next(PredefinedKFold().split(data))
    res = {"case": case}
    try:
        algo = SVDpp(n_factors=20, n_epochs=20, random_state=0, mode="atomic").fit(ts)
        res["raised"] = None
        res["rmse"] = accuracy.rmse(algo.test(test), verbose=False)
    except _lib.SurpriseAMDError as e:
        res["raised"] = str(e)
    seen["engine"].stream.synchronize()
    res["status"] = int(seen["engine"]._hx_status[0])
    with open(out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
