"""Build the HIP extension in-tree (hipcc, gfx950) -- used by ``__graft_entry__.build()``."""
from __future__ import annotations

import glob
import os
import shutil
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
SRC = os.path.join(PKG_DIR, "csrc", "d2d_hip.hip")


def env_headers() -> list:
    """Every header the env library's source can include: all of csrc/*.h (globbed, so a new header
    cannot be forgotten) and the public ABI header."""
    return sorted(glob.glob(os.path.join(PKG_DIR, "csrc", "*.h"))) + [os.path.join(REPO, "include", "drone2d.h")]


HDRS = env_headers()
OUT = os.path.join(PKG_DIR, "_lib", "libdrone2d_hip.so")
# the same source with -DD2D_EXACT_TRIG=1: sin / cos / atan2 from d2d_pmath.h and the reference's
# bearing sequence (Drone2dVecEnv(exact_trig=True); bit-identical to the oracle's exact build)
EXACT_OUT = os.path.join(PKG_DIR, "_lib", "libdrone2d_hip_exact.so")
# the PPO update's fused element-wise kernels (include/d2d_ppo.h)
PPO_SRC = os.path.join(PKG_DIR, "csrc", "d2d_ppo.hip")
PPO_HDRS = [os.path.join(REPO, "include", "d2d_ppo.h")]
PPO_OUT = os.path.join(PKG_DIR, "_lib", "libd2d_ppo.so")

# -ffp-contract=off: the kernels follow the reference's NumPy evaluation order (explicit fma() only
# where NumPy/OpenBLAS fuses); no fast-math: IEEE inf/NaN semantics are part of the contract.
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
               "-fno-fast-math", "-Wall", "-Werror"]


def hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def needs_build(out: str = OUT, src: str = SRC, hdrs=None) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in [src, *(env_headers() if hdrs is None else hdrs)])


# the PPO update is float32 training arithmetic with no reference rounding to follow: FMAs contracted
# within an expression (-ffp-contract=on, which honours `#pragma clang fp contract(off)`: the rollout's
# GAE recursion keeps torch's operation-by-operation rounding; "fast" fuses across statements in the
# backend whatever the pragma says)
PPO_FLAGS = [f if f != "-ffp-contract=off" else "-ffp-contract=on" for f in HIPCC_FLAGS]


def _compile(src: str, out: str, verbose: bool, flags=None):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    cmd = [hipcc(), *(flags or HIPCC_FLAGS), "-I", os.path.join(REPO, "include"), src, "-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)


def build_exact(force: bool = False, verbose: bool = False) -> str:
    """The exact-trig build (libdrone2d_hip_exact.so), compiled only when asked for: by
    ``build(exact=True)`` (``__graft_entry__.build()``, which the tests rely on) or by the first
    ``Drone2dVecEnv(exact_trig=True)`` that finds it missing."""
    if force or needs_build(EXACT_OUT):
        _compile(SRC, EXACT_OUT, verbose, HIPCC_FLAGS + ["-DD2D_EXACT_TRIG=1"])
    return EXACT_OUT


def build(force: bool = False, verbose: bool = False, exact: bool = False) -> str:
    """The in-tree libraries: the env (libdrone2d_hip.so: every mode, one scenario layout), the PPO
    update kernels (libd2d_ppo.so) and, with ``exact``, the env's exact-trig build."""
    stale = os.path.join(PKG_DIR, "_lib", "libdrone2d_hip_rm.so")  # rounds 1-3's second layout build
    if os.path.exists(stale):
        os.remove(stale)
    if force or needs_build():
        _compile(SRC, OUT, verbose)
    if exact:
        build_exact(force, verbose)
    if force or needs_build(PPO_OUT, PPO_SRC, PPO_HDRS):
        _compile(PPO_SRC, PPO_OUT, verbose, PPO_FLAGS)
    return OUT
