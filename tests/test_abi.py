"""The C-ABI library loads and exports every symbol include/surprise_amd.h declares (no GPU)."""
import ctypes
import os

import pytest

from surprise_amd import _lib


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        from surprise_amd import build
        build.build()
    return _lib.load()


def test_header_declares_expected_entry_points():
    syms = _lib.header_symbols()
    assert set(syms) == set(_lib.SIGNATURES), syms


def test_library_exports_every_header_symbol(lib):
    for name in _lib.header_symbols():
        assert hasattr(lib, name), name
        assert isinstance(getattr(lib, name), ctypes._CFuncPtr)


def test_version_and_error_without_device(lib):
    assert lib.mf_version() == 936
    rc = lib.mf_item_affine(None, None, 10, 16, None, None, None, 0, 0, None)
    assert rc == 1001 and b"bad argument" in lib.mf_last_error()
    # argument validation happens before any device call
    rc = lib.mf_item_merge(None, None, 10, 16, 10, 10, 1, 0, None, None, None, None, 0, 16,
                           None, None, 1, 0, None)
    assert rc == 1001
    assert b"bad item table" in lib.mf_last_error()
    csr = _lib.MfCsr(0, 0, 0, 0, 0)
    rc = lib.mf_svd_epoch(ctypes.byref(csr), None, 1, None, None, 16, None, 16, 10, 1, None,
                          0, None, None, 0, 0, 0, None)
    assert rc == 1001 and b"null csr" in lib.mf_last_error()
    rc = lib.mf_log_replay(None, None, 16, 10, None, None, None, None, None, None, 3, None, None,
                           None, 0, 0, None)
    assert rc == 1001 and b"null argument" in lib.mf_last_error()
    assert lib.mf_ckpt_interval() in (2, 4, 8, 16)
    rc = lib.mf_log_apply(None, 10, 16, 10, 10, None, None, None, None, None, None, None, 1, None,
                          1, None, None, 0, None, 0, None)
    assert rc == 1001 and b"count-aware rule needs" in lib.mf_last_error()
    rc = lib.mf_log_apply(None, 10, 16, 10, -1, None, None, None, None, None, None, None, 0, None,
                          1, None, None, 0, 1, 0, None)  # (bias_out without a bias column)
    assert rc == 1001 and b"bias_out needs apply and bias_col" in lib.mf_last_error()
    rc = lib.mf_log_reduce(None, 16, 11, None, None, 5, None, None, None, None, 0, None)
    assert rc == 1001 and b"null argument" in lib.mf_last_error()
    rec = _lib.MfRecency(0, 0, 0, 0)
    rc = lib.mf_log_reduce(1, 16, 11, 1, 1, 5, 1, None, None, ctypes.byref(rec), 0, None)
    assert rc == 1001 and b"recency weights need" in lib.mf_last_error()
    rc = lib.mf_svdpp_epoch(ctypes.byref(csr), None, 1, None, None, 16, None, 16, None, 10, None,
                            1, None, None, 0, 0, None, None, 0, None)
    assert rc == 1001 and b"null csr" in lib.mf_last_error()
    # the hybrid launch: its buffers, three helper waves, and q offsets below bit 31 (ring flag)
    rc = lib.mf_svdpp_epoch_mix(ctypes.byref(csr), None, 1, None, None, 16, None, 16, None, 10,
                                None, None, None, None, None, 0, 0, None, None, 0, None)
    assert rc == 1001 and b"needs cold_log" in lib.mf_last_error()
    rc = lib.mf_svdpp_epoch_mix(ctypes.byref(csr), None, 1, None, None, 16, None, 16, None, 10,
                                None, 1, 1, 1, 1, 0, 0, None, None, 0, None)
    assert rc == 1001 and b"three helpers" in lib.mf_last_error()
    big = _lib.MfCsr(1, 1, 1, 10, 1_100_000)  # 2 x 1.1M rows x 1 KiB: past 2 GiB with replicas
    rc = lib.mf_svdpp_epoch_mix(ctypes.byref(big), None, 1, None, None, 256, None, 256, None, 200,
                                None, 1, 1, 1, 1, 0, _lib.MF_EPOCH_SVDPP_HELPERS, None, 1, 0, None)
    assert rc != 0 and b"with replicas" in lib.mf_last_error()
    rc = lib.mf_sumsq(None, 4, 8, 4, None, 0, None)
    assert rc == 1001
    rc = lib.mf_svd_epoch_sq(ctypes.byref(csr), None, 1, None, None, 16, None, 16, 10, 1, None,
                             None, None, None, None, 0, 0, 0, None)
    assert rc == 1001 and b"needs elog and user_sq" in lib.mf_last_error()
    assert lib.mf_user_sq(None, 4, 8, 16, None, 0, None) == 1001
    assert lib.mf_user_sq_reduce(None, 4, 8, None, None) == 1001


def test_header_constants_match_python():
    text = open(_lib.HEADER_PATH).read()
    for name, val in (("MF_F32", 0), ("MF_F64", 1), ("MF_MODE_PLAIN", 0), ("MF_MODE_ATOMIC", 1),
                      ("MF_MODE_LOG", 2), ("MF_MERGE_SUM", 0), ("MF_MERGE_COUNT", 1), ("MF_MERGE_MEAN", 2),
                      ("MF_MERGE_RECENCY", 3), ("MF_EPOCH_DUP_ITEMS", 1), ("MF_HX_HELPER_TIMEOUT", 1),
                      ("MF_HX_CHAIN_FALLBACK", 2),
                      ("MF_MAX_FACTORS_F32", 512),
                      ("MF_MAX_FACTORS_F64", 256)):
        assert "#define %s" % name in text and str(val) in text.split("#define %s" % name)[1].split("\n")[0]


def test_library_hash_is_the_committed_sources(lib):
    """Build provenance: the loaded .so carries sha256 of mf_kernels.hip + surprise_amd.h + the
    compile lines, equal to the hash of the sources in this tree (_lib.load() enforces it)."""
    from surprise_amd import build
    assert lib.mf_source_hash().decode() == build.source_hash()
    assert build.embedded_hash() == build.source_hash()


def test_python_constants_equal_the_header_defines():
    """Every MF_* integer constant surprise_amd._lib mirrors equals its #define in
    include/surprise_amd.h (flags such as MF_EPOCH_SVDPP_ONE_HELPER cross the ABI as ints)."""
    import re
    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                       "surprise_amd.h")
    defines = {m.group(1): int(m.group(2), 0) for m in
               re.finditer(r"^#define\s+(MF_\w+)\s+(0x[0-9a-fA-F]+|\d+)\b", open(hdr).read(), re.M)}
    mirrored = {k: v for k, v in vars(_lib).items() if k.startswith("MF_") and isinstance(v, int)}
    assert mirrored, "no constants mirrored"
    missing = sorted(k for k in mirrored if k not in defines)
    assert not missing, missing
    for k, v in mirrored.items():
        assert defines[k] == v, (k, defines[k], v)
