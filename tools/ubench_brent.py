#!/usr/bin/env python3
"""Brent-iteration micro-benchmark (diagnostic).  build: CPU container; run: GPU box.

    python tools/ubench_brent.py build
    python tools/ubench_brent.py run

Reports cycles per iteration (median over waves) for 1, 2 and 4 waves per SIMD, per knob variant.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "tools", "_abl")
VARIANTS = {"prod": [], "inl": ["UB_INLINE=1"]}


def lib(v):
    return os.path.join(OUT, f"libub_brent_{v}.so")


def build():
    os.makedirs(OUT, exist_ok=True)
    for v, d in VARIANTS.items():
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-ffp-contract=off", "-fno-fast-math", "-I", os.path.join(REPO, "include"),
                        *[f"-D{x}" for x in d], os.path.join(REPO, "tools", "ubench_brent.hip"), "-o", lib(v)],
                       check=True)
        print("built", lib(v))


def run():
    import torch  # noqa: F401  (HIP runtime shared with torch)

    import drone2d_amd  # noqa: F401
    from drone2d_amd import env as E
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    scn = E.build_scenarios(dict(ENV_TRAIN_CONFIG, scenario="corridor"))[0].to_c()
    rng = np.random.default_rng(0)
    n = 4096
    # off-path positions below the screen (the bench's dominant 43-iteration case) + near-path ones
    far = np.stack([rng.uniform(0, 1000, n // 2), rng.uniform(-3000, -500, n // 2)], 1)
    near = np.stack([rng.uniform(100, 900, n // 2), rng.uniform(200, 900, n // 2)], 1)
    res = {}
    only = os.environ.get("UB_ONLY", "").split(",") if os.environ.get("UB_ONLY") else list(VARIANTS)
    for name, pts in (("far", far), ("near", near)):
        pxy = np.ascontiguousarray(pts, dtype=np.float64)
        for v in only:
            L = C.CDLL(lib(v))
            L.ub_run.restype = C.c_int
            for wps in (1, 2, 4):
                nb = 1024 * wps
                u = np.zeros(64 * nb)
                cyc = np.zeros(nb, dtype=np.int64)
                it = np.zeros(nb, dtype=np.int32)
                rc = L.ub_run(C.byref(scn), nb, pxy.ctypes.data_as(C.c_void_p), len(pxy),
                              u.ctypes.data_as(C.c_void_p), cyc.ctypes.data_as(C.c_void_p),
                              it.ctypes.data_as(C.c_void_p))
                assert rc == 0, rc
                cpi = cyc / np.maximum(it, 1)
                res[f"{name}/{v}/{wps}"] = {"cyc_per_iter_med": float(np.median(cpi)), "iters_med": float(np.median(it)),
                                            "cycles_med": float(np.median(cyc))}
                print(name, v, wps, res[f"{name}/{v}/{wps}"], flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(REPO, "gpurun_out", "ubench_brent.json"), "w"), indent=1)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
