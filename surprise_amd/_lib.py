"""Loader for libsurprise_amd.so, the C ABI declared in include/surprise_amd.h.

The library is built in-tree (``surprise_amd/libsurprise_amd.so``) by
``surprise_amd.build.build()`` with ``hipcc --offload-arch=gfx950``.  There is
no fallback: if the library is missing or the GPU is absent every training or
inference entry point raises ``SurpriseAMDError``.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SURPRISE_AMD_LIB") or os.path.join(_HERE, "libsurprise_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "surprise_amd.h")

MF_F32, MF_F64 = 0, 1
MF_MODE_PLAIN, MF_MODE_ATOMIC, MF_MODE_LOG = 0, 1, 2
MODES = {"plain": MF_MODE_PLAIN, "atomic": MF_MODE_ATOMIC, "log": MF_MODE_LOG}
MF_MERGE_SUM, MF_MERGE_COUNT, MF_MERGE_MEAN, MF_MERGE_RECENCY = 0, 1, 2, 3
MF_EPOCH_DUP_ITEMS = 1
MF_EPOCH_XCD_SHIFT = 8  # flags bits 8..15: XCD mask (include/surprise_amd.h)
MF_EPOCH_SVDPP_HELPERS = 2
MF_EPOCH_SVDPP_ONE_HELPER = 32
MF_EPOCH_ERR_IN_ROW = 4  # checkpoint log: errors in the checkpoint rows' padding
MF_EPOCH_CKPT_NARROW = 16  # checkpoint log: rows of the factor columns only (errors in elog)
MF_REPLAY_WPC_SHIFT = 16  # mf_log_replay flags bits 16..23: waves per CU (0: 16)
MF_EPOCH_LOG_NT = 64  # the epoch kernels' log stores non-temporal (streamed past L2 / MALL)
MF_FOLD_WORDS = 1024  # mf_launch_fold's arrival counters (uint32)
MF_SQ_PARTS_MIN = 65536  # users from which the <p^2> sum runs in MF_SQ_PARTS fixed-range parts
MF_SQ_PARTS = 256  # scratch doubles after a {sum, count} statistic buffer (from MF_SQ_PARTS_MIN rows)
MF_HX_HELPER_TIMEOUT, MF_HX_CHAIN_FALLBACK = 1, 2  # mf_svdpp_epoch status word bits


def ckpt_narrow_ld(K: int, dtype: int) -> int:
    """The MF_EPOCH_CKPT_NARROW checkpoint rows' stride (elements): K, fp32 rounded up to even."""
    return (K + 1) & ~1 if dtype == MF_F32 else K
MAX_FACTORS = {MF_F32: 512, MF_F64: 256}


class SurpriseAMDError(RuntimeError):
    """A HIP / library failure surfaced from the C ABI."""


class MfHyper(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "lr_bu", "lr_bi", "lr_pu", "lr_qi", "lr_yj",
        "reg_bu", "reg_bi", "reg_pu", "reg_qi", "reg_yj", "global_mean")]


class MfCsr(ctypes.Structure):
    _fields_ = [("row_ptr", ctypes.c_void_p), ("items", ctypes.c_void_p),
                ("ratings", ctypes.c_void_p), ("n_users", ctypes.c_int32),
                ("n_items", ctypes.c_int32)]


class MfFold(ctypes.Structure):
    """mf_fold_t (include/surprise_amd.h): the fold inside the next mf_log_replay launches."""
    _fields_ = [("qb", ctypes.c_void_p), ("ld", ctypes.c_int32), ("n_factors", ctypes.c_int32),
                ("bias_col", ctypes.c_int32), ("rule", ctypes.c_int32),
                ("sums", ctypes.c_void_p), ("item_piece_ptr", ctypes.c_void_p),
                ("sums2", ctypes.c_void_p), ("item_piece_ptr2", ctypes.c_void_p),
                ("totals", ctypes.c_void_p), ("hp", ctypes.c_void_p), ("p2stat", ctypes.c_void_p),
                ("stat_next", ctypes.c_void_p), ("user_sq", ctypes.c_void_p),
                ("n_users", ctypes.c_int64), ("bias_out", ctypes.c_void_p),
                ("item_count", ctypes.c_void_p), ("words", ctypes.c_void_p),
                ("role", ctypes.c_int32), ("n_launches", ctypes.c_int32)]


class MfRecency(ctypes.Structure):
    _fields_ = [("rpos", ctypes.c_void_p), ("pos0", ctypes.c_void_p), ("totals", ctypes.c_void_p),
                ("p2stat", ctypes.c_void_p)]


class MfQlogFold(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "perm", "rpos", "item_row_beg", "users", "hot_perm", "hot_rpos",
        "hot_users", "hot_piece_beg", "hot_piece_item", "hot_item_piece_ptr")] + \
        [("n_hot_pieces", ctypes.c_int64)] + \
        [(n, ctypes.c_void_p) for n in ("hot_sums", "hot_piece_c", "hot_piece_A")]


_vp, _i32, _i64, _dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double

# name -> argtypes (all return int except mf_last_error)
SIGNATURES = {
    "mf_svd_epoch": [ctypes.POINTER(MfCsr), _vp, _i64, _vp, _vp, _i32, _vp, _i32, _i32, _i32,
                     ctypes.POINTER(MfHyper), _i32, _vp, _vp, _i32, _i32, _i32, _vp],
    "mf_svdpp_epoch": [ctypes.POINTER(MfCsr), _vp, _i64, _vp, _vp, _i32, _vp, _i32, _vp, _i32,
                       ctypes.POINTER(MfHyper), _i32, _vp, _vp, _i32, _i32, _vp, _vp, _i32,
                       _vp],
    "mf_svdpp_epoch_mix": [ctypes.POINTER(MfCsr), _vp, _i64, _vp, _vp, _i32, _vp, _i32, _vp,
                           _i32, ctypes.POINTER(MfHyper), _vp, _vp, _vp, _vp, _i32, _i32, _vp,
                           _vp, _i32, _vp],
    "mf_svdpp_epoch_qlog": [ctypes.POINTER(MfCsr), _vp, _i64, _vp, _vp, _i32, _vp, _i32, _vp,
                            _i32, ctypes.POINTER(MfHyper), _vp, _vp, _vp, _vp, _i32, _i32, _i32,
                            _vp],
    "mf_svdpp_hot_fold": [_vp, _i32, _i32, _vp, _i32, _i32, _vp],
    "mf_svdpp_y_fold": [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _i32, _vp, _vp, _vp,
                        _i32, _vp],
    "mf_svd_epoch_sq": [ctypes.POINTER(MfCsr), _vp, _i64, _vp, _vp, _i32, _vp, _i32, _i32,
                        _i32, ctypes.POINTER(MfHyper), _vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp],
    "mf_svd_epoch_gram": [ctypes.POINTER(MfCsr), _vp, _i64, _vp, _vp, _i32, _vp, _i32, _i32,
                          _i32, ctypes.POINTER(MfHyper), _vp, _vp, _i32, _i32, _i32, _vp],
    "mf_sumsq": [_vp, _i64, _i32, _i32, _vp, _i32, _vp],
    "mf_user_sq": [_vp, _i64, _i32, _i32, _vp, _i32, _vp],
    "mf_user_sq_reduce": [_vp, _i64, _i32, _vp, _vp],
    "mf_log_reduce": [_vp, _i32, _i32, _vp, _vp, _i64, _vp, _vp, ctypes.POINTER(MfHyper),
                      ctypes.POINTER(MfRecency), _i32, _vp],
    "mf_log_replay": [_vp, _vp, _i32, _i32, ctypes.POINTER(MfCsr), _vp,
                      ctypes.POINTER(MfHyper), _vp, _vp, _vp, _i64, _vp, _vp,
                      ctypes.POINTER(MfRecency), _i32, _i32, _vp],
    "mf_ckpt_interval": [],
    "mf_svdpp_qlog_fold": [_vp, _i32, _i32, _vp, _i32, _vp, ctypes.POINTER(MfQlogFold), _vp,
                           _vp, ctypes.POINTER(MfHyper), _vp, _vp, _i32, _vp, _vp, _i64, _i32,
                           _vp],
    "mf_log_apply": [_vp, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp,
                     ctypes.POINTER(MfHyper), _vp, _i32, _vp, _i32, _vp, _vp, _i64, _vp, _i32,
                     _vp],
    "mf_item_merge": [_vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp,
                      ctypes.POINTER(MfHyper), _vp, _i32, _i32, _vp, _vp, _i32, _i32, _vp],
    "mf_item_apply": [_vp, _vp, _i32, _i32, _i32, _vp, _i32, _vp],
    "mf_item_affine": [_vp, _vp, _i32, _i32, _vp, _vp, _vp, _i32, _i32, _vp],
    "mf_nmf_user_pass": [ctypes.POINTER(MfCsr), _vp, _vp, _vp, _i32, _vp, _i32, _i32, _i32,
                         ctypes.POINTER(MfHyper), _vp, _vp, _vp, _i64, _vp, _vp, _vp, _i32, _vp],
    "mf_nmf_item_pass": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _i32, _i32, _i32, _i32,
                         ctypes.POINTER(MfHyper), _i32, _vp, _i64, _vp, _vp, _vp, _vp, _i32,
                         _vp],
    "mf_baseline_als_epoch": [ctypes.POINTER(MfCsr), _vp, _vp, _vp, _vp, _vp, _dbl, _dbl, _dbl,
                              _vp, _vp, _i32, _vp],
    "mf_predict": [_i64, _vp, _vp, _vp, _vp, _i32, _vp, _i32, _vp, _i32, _i32, _dbl, _vp, _vp,
                   _i32, _vp],
    "mf_rating_errors": [_i64, _vp, _vp, _vp, _dbl, _dbl, _dbl, _dbl, _vp, _i32, _vp],
    "mf_svdpp_user_implicit": [ctypes.POINTER(MfCsr), _vp, _i32, _vp, _i32, _i32, _vp],
    "mf_selftest_wave_sum": [_vp, _vp, _i32, _i32, _vp],
    "mf_selftest_xcc": [_vp, _i32, _vp],
    "mf_xcd_layout": [ctypes.POINTER(ctypes.c_int32)],
    "mf_dispatch_check": [ctypes.POINTER(ctypes.c_uint64)],
    "mf_event_create": [ctypes.POINTER(ctypes.c_void_p)],
    "mf_event_destroy": [_vp],
    "mf_event_record": [_vp, _vp],
    "mf_stream_wait_event": [_vp, _vp],
    "mf_launch_event": [_vp],
    "mf_launch_join": [_vp, _i32, ctypes.c_uint32],
    "mf_launch_fold": [ctypes.POINTER(MfFold)],
    "mf_version": [],
    "mf_last_error": [],
    "mf_source_hash": [],
}
_STR_RESULT = ("mf_last_error", "mf_source_hash")

_lib = None


def load(path: str = LIB_PATH):
    """Load the shared library (no GPU access happens here).  The product library must carry
    the source hash of the kernel source / header / compile lines next to it (build provenance:
    a stale or foreign .so is refused); SURPRISE_AMD_LIB (experiment variants) skips the check."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SurpriseAMDError(
            f"{path} is missing: build it with `python -c 'import surprise_amd.build as b; b.build()'`"
            " (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_char_p if name in _STR_RESULT else ctypes.c_int
    if not os.environ.get("SURPRISE_AMD_LIB"):
        from .build import source_hash
        have, want = lib.mf_source_hash().decode(), source_hash()
        if have != want:
            raise SurpriseAMDError(
                f"{path} was built from other sources (hash {have[:16]}, sources {want[:16]}): "
                "rebuild with surprise_amd.build.build()")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().mf_last_error()
        raise SurpriseAMDError(f"{what} failed with code {rc}: {msg.decode() if msg else ''}")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def require_gpu():
    """Return the torch module once a HIP device is confirmed; raise otherwise."""
    import torch
    if not torch.cuda.is_available():
        raise SurpriseAMDError(
            "surprise_amd needs a HIP GPU (MI355X, gfx950): torch.cuda.is_available() is False. "
            "There is no CPU fallback for the training path.")
    load()
    return torch


def xcd_layout_ok() -> bool:
    """The 8-XCD round-robin workgroup dispatch the XCD-masked launches assume (mf_xcd_layout,
    checked once per device on the GPU)."""
    ok = ctypes.c_int32(0)
    call("mf_xcd_layout", ctypes.byref(ok))
    return bool(ok.value)


def dispatch_check() -> None:
    """Raise unless every XCD-masked launch since the library was loaded gave each of its slots
    to exactly one wave (mf_dispatch_check: the device-side sum stays 0).  Synchronous."""
    s = ctypes.c_uint64(0)
    call("mf_dispatch_check", ctypes.byref(s))
    if s.value:
        raise SurpriseAMDError(
            "an XCD-masked launch did not deal its workgroups round-robin over the 8 XCDs "
            "(mf_dispatch_check sum %#x): some users were trained twice and others never; "
            "train with xcd_split=False" % s.value)


def header_symbols(path: str = HEADER_PATH):
    """Function names declared in include/surprise_amd.h (for the ABI test)."""
    import re
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(mf_\w+)\s*\(", text, re.M)))
