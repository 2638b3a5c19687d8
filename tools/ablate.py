#!/usr/bin/env python3
"""Diagnostic ablation of the step kernel (timing-only builds, never shipped).

    python tools/ablate.py build          # CPU container: compile variants into tools/_abl/
    python tools/ablate.py run [--out F]  # GPU box: time every variant + occupancy sweep

Mask bits (D2D_ABLATE, csrc/d2d_device.h): 1 no Brent, 2 no sensing, 4 no joint iterations,
8 no collision test.  Outputs of ablated builds are wrong by construction; only times matter.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
ABL = os.path.join(REPO, "tools", "_abl")
MASKS = [0, 1, 2, 4, 8, 15]


def lib_for(mask):
    return os.path.join(ABL, f"libd2d_abl{mask}.so")


def build():
    import drone2d_amd  # noqa: F401
    from drone2d_amd import _build

    os.makedirs(ABL, exist_ok=True)
    for m in MASKS:
        cmd = [_build.hipcc(), *_build.HIPCC_FLAGS, f"-DD2D_ABLATE={m}", "-I", os.path.join(REPO, "include"),
               _build.SRC, "-o", lib_for(m)]
        subprocess.run(cmd, check=True)
        print("built", lib_for(m))


def time_variant(d2, torch, lib, n, scenario, steps=100, warmup=20):
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    venv = d2.Drone2dVecEnv(n, seed=1, with_info=False, native_lib=lib,
                            **dict(ENV_TRAIN_CONFIG, scenario=scenario))
    venv.reset()
    acts = [torch.rand(n, 2, device=venv.device) * 2 - 1 for _ in range(8)]
    for k in range(warmup):
        venv.step(acts[k % 8])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(steps):
        venv.step(acts[k % 8])
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    venv.close()
    return ms


def run(out):
    import torch

    import drone2d_amd as d2

    res = {}
    for m in MASKS:
        res[f"corridor_65536_mask{m}"] = time_variant(d2, torch, lib_for(m), 65536, "corridor")
        print(m, res[f"corridor_65536_mask{m}"], flush=True)
    full = lib_for(0)
    for n in (16384, 65536, 131072, 262144, 524288):
        res[f"corridor_{n}"] = time_variant(d2, torch, full, n, "corridor")
        print(n, res[f"corridor_{n}"], flush=True)
    for scn in ("large", "S_corridor", "corridor_free", "perpendicular", "impossible"):
        res[f"{scn}_65536"] = time_variant(d2, torch, full, 65536, scn)
        print(scn, res[f"{scn}_65536"], flush=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "ablate.json"))
    a = ap.parse_args()
    build() if a.mode == "build" else run(a.out)
