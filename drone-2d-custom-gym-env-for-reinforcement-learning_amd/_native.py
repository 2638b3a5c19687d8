"""ctypes binding of ``libdrone2d_hip.so`` -- the reference-side FFI stub for the C ABI.

This is the binding a maintainer of the reference would add (INTEGRATION.md shows it standalone).
There is deliberately NO fallback: if the HIP library is missing the import fails loudly, so a
parity test or a benchmark can never silently run on anything but the native HIP path.
"""
from __future__ import annotations

import ctypes as C
import os

from . import abi

LIB_NAME = "libdrone2d_hip.so"
LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
LIB_PATH = os.path.join(LIB_DIR, LIB_NAME)
# the exact-trig build of the same source (d2d_device.h D2D_EXACT_TRIG)
EXACT_LIB_PATH = os.path.join(LIB_DIR, "libdrone2d_hip_exact.so")

# every entry point of include/drone2d.h: name -> (restype, argtypes)
_VP = C.c_void_p
SIGNATURES = {
    "d2d_abi_version": (C.c_int32, []),
    "d2d_last_error": (C.c_char_p, []),
    "d2d_create": (C.c_int32, [C.POINTER(abi.D2DCfg), C.c_int32, C.c_int32, C.POINTER(_VP)]),
    "d2d_destroy": (None, [_VP]),
    "d2d_n_envs": (C.c_int32, [_VP]),
    "d2d_set_scenarios": (C.c_int32, [_VP, C.POINTER(abi.D2DScn), C.c_int32, C.POINTER(C.c_int32)]),
    "d2d_reset": (C.c_int32, [_VP, _VP, C.c_uint64, _VP, _VP]),
    "d2d_step": (C.c_int32, [_VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    "d2d_get_state": (C.c_int32, [_VP, _VP, _VP, _VP]),
    "d2d_set_state": (C.c_int32, [_VP, _VP, _VP, _VP]),
    "d2d_refresh_pool": (C.c_int32, [_VP, C.POINTER(abi.D2DScn), C.c_int32]),
    "d2d_get_env_scenarios": (C.c_int32, [_VP, _VP, _VP]),
    "d2d_set_env_scenarios": (C.c_int32, [_VP, _VP, _VP]),
    "d2d_episode_stats": (C.c_int32, [_VP, _VP, C.c_int32, _VP]),
    "d2d_selftest": (C.c_int32, [C.c_int32, C.c_int64, C.c_uint64, C.POINTER(C.c_uint64)]),
    "d2d_group_layout": (C.c_int32, [C.c_int32, _VP, C.c_int32, _VP, _VP]),
    "d2d_get_group_layout": (C.c_int32, [_VP, _VP, _VP]),
    "d2d_balanced_group_layout": (C.c_int32, [C.c_int32, _VP, C.c_int32, _VP, C.c_int32, _VP, _VP]),
    "d2d_pool_state": (C.c_int32, [_VP, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "d2d_restore_pool": (C.c_int32, [_VP, C.POINTER(abi.D2DScn), C.c_int32, C.c_int32, C.c_int32]),
    "d2d_set_curriculum": (C.c_int32, [_VP, C.POINTER(abi.D2DCurriculum)]),
    "d2d_fresh_recipes": (C.c_int32, [_VP, _VP, _VP, C.POINTER(C.c_int64), C.c_int32]),
    "d2d_get_scenario_table": (C.c_int32, [_VP, C.c_int32, C.c_int32, C.POINTER(abi.D2DScn)]),
    "d2d_generation": (C.c_int32, [_VP]),
    "d2d_set_scenario_costs": (C.c_int32, [_VP, C.POINTER(C.c_double), C.c_int32]),
}

_lib = None
_libs: dict = {}  # other builds, by path (one CDLL each)


class NativeError(RuntimeError):
    pass


def load(path: str | None = None) -> C.CDLL:
    """Load (once) the HIP library. Raises ``NativeError`` if it is absent or ABI-mismatched."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    if path is not None and path in _libs:
        return _libs[path]
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise NativeError(f"{p} not found: the HIP extension is not built "
                          f"(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    # torch must own the HIP runtime first: its bundled libamdhip64 has the same soname, so the
    # library below then binds to that one runtime (one HIP context for torch and the envs).
    import torch  # noqa: F401

    lib = C.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.d2d_abi_version()
    if v != abi.ABI_VERSION:
        raise NativeError(f"{p}: ABI version {v}, expected {abi.ABI_VERSION}")
    if path is None:
        _lib = lib
    else:
        _libs[path] = lib
    return lib


def check(code: int, what: str, lib: C.CDLL | None = None) -> None:
    """Raise ``NativeError`` for a non-OK status; the message is ``lib``'s (default: the main build's)
    thread-local ``d2d_last_error``."""
    if code != abi.E_OK:
        src = lib if lib is not None else _lib
        msg = src.d2d_last_error().decode() if src is not None else ""
        raise NativeError(f"{what} failed (code {code}): {msg}")
