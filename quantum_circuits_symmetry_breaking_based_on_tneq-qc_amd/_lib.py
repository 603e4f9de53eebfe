"""ctypes binding of libtneqhip.so (C ABI in include/tneqhip.h).

The product path has no CPU fallback: if the library is missing or cannot be loaded the
import of :func:`lib` raises, and every backend / strategy entry point calls it.
torch is imported first so that libtneqhip.so binds to the HIP runtime torch already loaded
(same SONAME libamdhip64.so.7), giving one runtime per process.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TNEQHIP_LIB", os.path.join(_HERE, "lib", "libtneqhip.so"))

TQ_F32, TQ_F64, TQ_C64, TQ_C128 = 0, 1, 2, 3
TQ_OK, TQ_ERR_INVALID, TQ_ERR_HIP, TQ_ERR_ALLOC, TQ_ERR_UNSUPPORTED = 0, -1, -2, -3, -4

# every symbol the header declares (tests check the .so exports all of them)
EXPORTED = (
    "tq_version", "tq_last_error", "tq_device_synchronize", "tq_library_query", "tq_library_set", "tq_permute",
    "tq_gemm_batched",
    "tq_gemm_workspace_size", "tq_planes_gemm_workspace", "tq_planes_gemm_check", "tq_axpy", "tq_contract_pair_workspace", "tq_contract_pair",
    "tq_plan_create", "tq_plan_clone", "tq_plan_query", "tq_plan_set", "tq_plan_describe", "tq_plan_execute", "tq_plan_execute_group", "tq_plan_destroy",
    "tq_plan_profile", "tq_plan_profile_read", "tq_hermite_features", "tq_inverse_cdf_sample",
    "tq_sgdg_step", "tq_fidelity_forward", "tq_fidelity_backward",
)
TQ_SGDG_STIEFEL, TQ_SGDG_BUF_INIT, TQ_SGDG_RETRACT = 1, 2, 4
TQ_HERMITE_MAX_K, TQ_ICDF_MAX_GRID = 128, 8192
TQ_OP_PERMUTE, TQ_OP_GEMM, TQ_OP_APPLY, TQ_OP_AXPY, TQ_OP_SWEEP = 0, 1, 2, 3, 4


class TneqHipError(RuntimeError):
    """A HIP / library failure (maps TQ_ERR_HIP / TQ_ERR_UNSUPPORTED / TQ_ERR_ALLOC)."""


_lock = threading.Lock()
_lib = None

_c = ctypes
_i64p = _c.POINTER(_c.c_int64)
_i32p = _c.POINTER(_c.c_int32)
_vp = _c.c_void_p

_SIGS = {
    "tq_version": (_c.c_int, []),
    "tq_last_error": (_c.c_int, [_c.c_char_p, _c.c_size_t]),
    "tq_device_synchronize": (_c.c_int, []),
    "tq_library_query": (_c.c_int64, [_c.c_char_p]),
    "tq_library_set": (_c.c_int, [_c.c_char_p, _c.c_int64]),
    "tq_permute": (_c.c_int, [_c.c_int, _c.c_int, _i64p, _i64p, _vp, _vp, _c.c_double, _vp]),
    "tq_gemm_batched": (_c.c_int, [_c.c_int, _c.c_int, _c.c_int, _c.c_int64, _c.c_int64, _c.c_int64,
                                   _c.c_int64, _vp, _c.c_int64, _c.c_int64, _vp, _c.c_int64,
                                   _c.c_int64, _c.c_double, _vp, _c.c_int64, _c.c_int64, _vp,
                                   _c.c_size_t, _vp]),
    "tq_gemm_workspace_size": (_c.c_size_t, [_c.c_int, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int64]),
    "tq_planes_gemm_workspace": (_c.c_size_t, [_c.c_int64, _c.c_int64, _c.c_int64, _c.c_int64]),
    "tq_planes_gemm_check": (_c.c_int, [_c.c_int64, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int64,
                                        _c.c_size_t]),
    "tq_axpy": (_c.c_int, [_c.c_int, _c.c_int64, _vp, _vp, _c.c_double, _vp]),
    "tq_contract_pair_workspace": (_c.c_size_t, [_c.c_int, _c.c_int, _i64p, _i32p, _c.c_int, _i64p,
                                                 _i32p, _c.c_int, _i32p]),
    "tq_contract_pair": (_c.c_int, [_c.c_int, _c.c_int, _i64p, _i32p, _vp, _c.c_int, _i64p, _i32p,
                                    _vp, _c.c_int, _i32p, _vp, _vp, _c.c_size_t, _vp]),
    "tq_plan_create": (_c.c_int, [_c.POINTER(_vp), _c.c_int, _c.c_int, _i32p, _i32p, _i64p, _i64p,
                                  _c.c_int, _i32p, _c.c_int, _i32p, _c.c_int, _i32p]),
    "tq_plan_clone": (_c.c_int, [_vp, _c.POINTER(_vp)]),
    "tq_plan_query": (_c.c_int64, [_vp, _c.c_char_p]),
    "tq_plan_set": (_c.c_int, [_vp, _c.c_char_p, _c.c_int64]),
    "tq_plan_describe": (_c.c_int, [_vp, _c.c_char_p, _c.c_size_t]),
    "tq_plan_execute": (_c.c_int, [_vp, _c.POINTER(_vp), _vp, _c.c_int64, _c.c_int64, _c.c_int64,
                                   _c.c_int, _vp]),
    "tq_plan_execute_group": (_c.c_int, [_c.c_int, _c.POINTER(_vp), _c.POINTER(_c.POINTER(_vp)), _c.POINTER(_vp),
                                         _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int, _vp]),
    "tq_plan_destroy": (_c.c_int, [_vp]),
    "tq_plan_profile": (_c.c_int, [_vp, _c.c_int]),
    "tq_plan_profile_read": (_c.c_int, [_vp, _c.c_int, _c.POINTER(_c.c_double), _c.POINTER(_c.c_int64),
                                        _c.POINTER(_c.c_double), _c.POINTER(_c.c_double)]),
    "tq_hermite_features": (_c.c_int, [_c.c_int, _c.c_int64, _c.c_int, _vp, _c.POINTER(_c.c_double), _vp,
                                       _vp, _vp]),
    "tq_inverse_cdf_sample": (_c.c_int, [_c.c_int, _c.c_int64, _c.c_int64, _vp, _c.c_int64, _vp, _vp, _vp,
                                         _c.c_int64, _vp]),
    "tq_fidelity_forward": (_c.c_int, [_c.c_int, _c.c_int64, _vp, _vp, _vp, _vp, _vp]),
    "tq_fidelity_backward": (_c.c_int, [_c.c_int, _c.c_int64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "tq_sgdg_step": (_c.c_int, [_c.c_int, _c.c_int, _c.POINTER(_vp), _c.POINTER(_vp), _c.POINTER(_vp),
                                _i32p, _i32p, _i32p, _c.c_double, _c.c_double, _c.c_double,
                                _c.c_double, _c.c_int, _vp]),
}


def lib():
    """Load (once) and return the ctypes handle; raises if the native library is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (bind to torch's HIP runtime)
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libtneqhip.so not found at {LIB_PATH}: build it with "
                f"`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        h = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            f = getattr(h, name)
            f.restype = res
            f.argtypes = args
        _lib = h
    return _lib


def last_error() -> str:
    buf = ctypes.create_string_buffer(4096)
    lib().tq_last_error(buf, 4096)
    return buf.value.decode(errors="replace")


def check(rc: int, what: str = "") -> None:
    """Map a C status to the reference's exception types (ValueError / RuntimeError)."""
    if rc == TQ_OK:
        return
    msg = f"{what}: {last_error()}" if what else last_error()
    if rc == TQ_ERR_INVALID:
        raise ValueError(msg)
    if rc == TQ_ERR_ALLOC:
        raise MemoryError(msg)
    raise TneqHipError(msg)


def i64(seq):
    seq = [int(x) for x in seq]
    return (ctypes.c_int64 * max(1, len(seq)))(*seq)


def i32(seq):
    seq = [int(x) for x in seq]
    return (ctypes.c_int32 * max(1, len(seq)))(*seq)
