"""ctypes binding of libsqmp_w4a4.so (the C ABI declared in include/sqmp_w4a4.h).

The library is built in-tree by `smoothquant-mixedprecision_amd/build_ext.py` (or
`__graft_entry__.build()`).  There is deliberately no fallback: if the library cannot be
loaded, every quantized op raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

# SQMP_DIAG_LIB=1 loads the timing-diagnostics build (libsqmp_w4a4_diag.so, made by
# `SQMP_DIAG=1 python build_ext.py`: extra kernel variants selected by SQMP_*_DIAG, wrong
# results by design) -- tools only, never the product path
# SQMP_LIB_PATH: another build of the same C ABI (same-box A/B of two builds, tools only)
LIB_PATH = os.environ.get("SQMP_LIB_PATH") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)),
    "libsqmp_w4a4_diag.so" if os.environ.get("SQMP_DIAG_LIB") == "1" else "libsqmp_w4a4.so")

SQMP_OK, SQMP_EINVAL, SQMP_EUNSUPPORTED, SQMP_EHIP, SQMP_EWORKSPACE = 0, -1, -2, -3, -4

F32, F16, BF16 = 0, 1, 2
ACT_PER_TOKEN, ACT_PER_TENSOR, ACT_PER_GROUP, ACT_PER_GROUP_UNSORTED = 0, 1, 2, 3
ACT_PER_GROUP_MEAN3STD = 4
W_PER_CHANNEL, W_PER_TENSOR, W_PER_GROUP, W_PER_GROUP_UNSORTED, W_NONE = 0, 1, 2, 3, 4
W_PER_GROUP_MEAN3STD = 5
OUT_FP, OUT_INPLACE, OUT_F8, OUT_C4, OUT_H2 = 0, 2, 3, 5, 6
QA_CLEAN_WS, QA_REUSE_STATS, QA_STATS_GIVEN, QA_TILED, QA_TILED4 = 1, 2, 4, 8, 16
QA_TABLE_READY = 32
QA_WRITE_X = 64

_vp, _i, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
_ip = ctypes.POINTER(ctypes.c_int)



class Fq7Problem(ctypes.Structure):
    """sqmp_fq7_problem (include/sqmp_w4a4.h): one problem of sqmp_gemm_fq7_group."""
    _fields_ = [("a", ctypes.c_void_p), ("codes_t", ctypes.c_void_p),
                ("scale_t", ctypes.c_void_p), ("sal_t", ctypes.c_void_p),
                ("bias", ctypes.c_void_p), ("y", ctypes.c_void_p), ("colmax", ctypes.c_void_p),
                ("N", ctypes.c_int)]


# name -> (restype, argtypes); the authoritative list of exported symbols
SIGNATURES = {
    "sqmp_version": (ctypes.c_char_p, []),
    "sqmp_status_string": (ctypes.c_char_p, [_i]),
    "sqmp_weight_geometry": (_i, [_i, _i, _i, _i, _ip, _ip, _ip, _ip]),
    "sqmp_pack_workspace_bytes": (_sz, [_i, _i]),
    "sqmp_act_workspace_bytes": (_sz, [_i, _i, _i]),
    "sqmp_pack_weight": (_i, [_vp, _i, _i, _i, _i, _i, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp,
                              _vp, _vp, _vp, _sz, _vp]),
    "sqmp_dequant_weight": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _i,
                                 _vp, _vp]),
    "sqmp_dequant_weight_packed": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "sqmp_build_maps": (_i, [_i, _vp, _i, _vp, _vp, _vp, _vp, _i, _vp]),
    "sqmp_quant_act": (_i, [_vp, _i, _i, _i, _i, _i, _i, _vp, _i, _vp, _vp, _i, _i, _i, _vp,
                            _vp, _vp, _vp, _sz, _vp]),
    "sqmp_quant_act_v2": (_i, [_vp, _i, _i, _i, _i, _i, _i, _vp, _i, _vp, _vp, _i, _i, _vp, _i,
                               _i, _vp, _vp, _vp, _vp, _sz, _vp]),
    "sqmp_gemm_fq": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "sqmp_gemm_fq_colmax": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i,
                                 _vp, _vp]),
    "sqmp_pack_f8": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp]),
    "sqmp_gemm_f8": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i,
                          _vp]),
    "sqmp_gemm_f8_colmax": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i,
                                 _i, _vp, _vp]),
    "sqmp_quant_act_c4": (_i, [_vp, _i, _i, _i, _i, _i, _i, _vp, _i, _vp, _vp, _i, _i, _vp, _i,
                               _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _sz, _vp]),
    "sqmp_perm_weight_c4": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    "sqmp_gemm_fqt": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "sqmp_gemm_fqt7": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "sqmp_permute_act": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp]),
    "sqmp_gemm_fqt7j": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp,
                             _vp]),
    "sqmp_gemm_fqt7_colmax": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i,
                                   _vp, _vp]),
    "sqmp_fq7_sizes": (_i, [_i, _i, _i, _i, _i, ctypes.POINTER(_sz), ctypes.POINTER(_sz),
                            ctypes.POINTER(_sz)]),
    "sqmp_pack_fq7": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "sqmp_gemm_fq7": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp,
                           _vp]),
    "sqmp_quant_act_group": (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp, _i,
                                  _i, _i, _vp, _vp, _sz, _vp]),
    "sqmp_gemm_fq7_group": (_i, [ctypes.POINTER(Fq7Problem), _i, _i, _i, _i, _i, _i, _i, _i,
                                 _vp]),
    "sqmp_fq7_plan": (_i, [_i, _i, _ip, _i, _i, _i, _i, _ip, _ip]),
    "sqmp_reload_knobs": (_i, []),
    "sqmp_split2_f16": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp]),
    "sqmp_row_exp": (_i, [_vp, _i, _i, _vp, _vp]),
    "sqmp_gemm_h2": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
    "sqmp_pack_h2d": (_i, [_vp, _i, _i, _vp, _vp]),
    "sqmp_gemm_h2d": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
}

_lock = threading.Lock()
_lib = None


class SqmpError(RuntimeError):
    """A HIP runtime failure inside libsqmp_w4a4."""


def load():
    """Load (once) and return the ctypes library; raise RuntimeError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libsqmp_w4a4.so not found at {LIB_PATH}: build it with "
                "`python smoothquant-mixedprecision_amd/build_ext.py` (hipcc, gfx950). "
                "The W4A4 operator has no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(status: int, what: str):
    """Map a C status to the reference's exception types (ValueError for bad arguments /
    unsupported modes, RuntimeError for device failures)."""
    if status == SQMP_OK:
        return
    msg = load().sqmp_status_string(status).decode()
    if status in (SQMP_EINVAL, SQMP_EUNSUPPORTED):
        raise ValueError(f"{what}: {msg} (status {status})")
    raise SqmpError(f"{what}: {msg} (status {status})")


def version() -> str:
    return load().sqmp_version().decode()


_reload_hooks = []


def on_reload(fn):
    """Register a Python-side mirror of a library knob, refreshed by reload_knobs()."""
    _reload_hooks.append(fn)


def reload_knobs():
    """Re-read the library's SQMP_* launch knobs (read once at load) and their Python-side
    mirrors after os.environ changed: the in-process A/B tools and the tests that switch a
    launch variant call this."""
    if _lib is not None:
        _lib.sqmp_reload_knobs()
    for fn in _reload_hooks:
        fn()
