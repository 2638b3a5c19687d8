#!/usr/bin/env python3
"""Diagnostic: per-wave phase timeline of K1 from s_memtime stamps (timing-only build).

    python tools/stamps.py build        # CPU container
    python tools/stamps.py run [--scenario S] [--envs N]   # GPU box

Stamps per wave: 0 start, 1 after scenario staging, 2 end of phase-1 work, 3 after barrier 1,
4 end of phase-2 work, 5 after barrier 2, 6 end.  Reported in shader cycles per role (wave 0..3).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
LIB = os.path.join(REPO, "tools", "_abl", "libd2d_stamps.so")


def build():
    import drone2d_amd  # noqa: F401
    from drone2d_amd import _build

    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run([_build.hipcc(), *_build.HIPCC_FLAGS, "-DD2D_STAMPS", "-I", os.path.join(REPO, "include"),
                    _build.SRC, "-o", LIB], check=True)
    print("built", LIB)


def run(scenario, n, steps_warm):
    import numpy as np
    import torch

    import drone2d_amd as d2
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    venv = d2.Drone2dVecEnv(n, seed=3, with_info=False, native_lib=LIB, **dict(ENV_TRAIN_CONFIG, scenario=scenario))
    lib = venv._lib
    lib.d2d_debug_stamps.argtypes = [C.c_void_p, C.c_void_p]
    nw = (n + 63) // 64 * 4
    buf = torch.zeros(nw * 8, dtype=torch.int64, device=venv.device)
    venv.reset()
    for k in range(steps_warm):
        venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
    lib.d2d_debug_stamps(venv._h, C.c_void_p(buf.data_ptr()))
    venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
    torch.cuda.synchronize()
    s = buf.cpu().numpy().reshape(-1, 4, 8).astype(np.int64)
    t0 = s[:, :, 0].min()
    res = {"scenario": scenario, "envs": n, "kernel_span_cycles": int(s[:, :, 6].max() - t0)}
    names = ["stage", "phase1", "barrier1", "phase2", "barrier2", "phase3"]
    for w in range(4):
        d = np.diff(s[:, w, :7], axis=1)
        res[f"wave{w}"] = {nm: [int(np.median(d[:, k])), int(np.percentile(d[:, k], 95)), int(d[:, k].max())]
                           for k, nm in enumerate(names)}
        res[f"wave{w}"]["total"] = [int(np.median(s[:, w, 6] - s[:, w, 0])), int((s[:, w, 6] - s[:, w, 0]).max())]
    starts = s[:, 0, 0] - t0
    res["block_start_spread"] = [int(np.median(starts)), int(starts.max())]
    print(json.dumps(res, indent=1))
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("--scenario", default="corridor")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--warm", type=int, default=40)
    a = ap.parse_args()
    if a.mode == "build":
        build()
    else:
        out = [run(a.scenario, a.envs, a.warm), run(a.scenario, 16384, a.warm)]
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        json.dump(out, open(os.path.join(REPO, "gpurun_out", "stamps.json"), "w"), indent=1)
