"""Build the HIP extension in-tree (hipcc, gfx950) -- used by ``__graft_entry__.build()``."""
from __future__ import annotations

import os
import shutil
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
SRC = os.path.join(PKG_DIR, "csrc", "d2d_hip.hip")
HDRS = [os.path.join(PKG_DIR, "csrc", "d2d_device.h"), os.path.join(PKG_DIR, "csrc", "d2d_kernels.h"),
        os.path.join(REPO, "include", "drone2d.h")]
OUT = os.path.join(PKG_DIR, "_lib", "libdrone2d_hip.so")

# -ffp-contract=off: the kernels follow the reference's NumPy evaluation order (explicit fma() only
# where NumPy/OpenBLAS fuses); no fast-math: IEEE inf/NaN semantics are part of the contract.
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
               "-fno-fast-math", "-Wall", "-Werror"]


def hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in [SRC, *HDRS])


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = OUT + ".tmp"
    cmd = [hipcc(), *HIPCC_FLAGS, "-I", os.path.join(REPO, "include"), SRC, "-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT
