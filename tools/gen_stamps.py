#!/usr/bin/env python3
"""Diagnostic (not product): K5b's phase timeline from s_memtime stamps (a -DD2D_GEN_STAMPS build).

    python tools/variants.py build gst:D2D_GEN_STAMPS=1      # CPU container
    python tools/gen_stamps.py tools/_abl/libd2d_var_gst.so   # GPU box

Steps a 65 536-env fresh-curriculum batch (random actions) for the warmup, then records three steps'
K5b items (stamps per item: see below).  Prints the items of each step and per phase [median, p90,
max] shader cycles, plus the span of the slowest item.
"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402

lib = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 200
venv = d2.Drone2dVecEnv(n, seed=0, with_info=False, native_lib=lib,
                        **dict(ENV_TRAIN_CONFIG, mode="curriculum", scenario="curriculum", sim_num=0))
venv.reset(seed=0)
g = torch.Generator(device="cuda").manual_seed(0)
acts = [torch.rand(n, 2, device="cuda", generator=g) * 2 - 1 for _ in range(16)]
for k in range(warm):
    venv.step(acts[k % 16])
torch.cuda.synchronize()
venv.episode_stats()  # (clears the counters)
out = {"envs": n, "warmup": warm}
res = []
for rep in range(3):
    buf = torch.zeros(2 * n * 8, dtype=torch.int64, device="cuda")
    venv._lib.d2d_debug_stamps.argtypes = [C.c_void_p, C.c_void_p]
    venv._lib.d2d_debug_stamps(venv._h, C.c_void_p(buf.data_ptr()))
    venv.step(acts[rep % 16])
    torch.cuda.synchronize()
    venv._lib.d2d_debug_stamps(venv._h, None)
    s = buf.cpu().numpy().reshape(-1, 8)
    s = s[s[:, 0] != 0]
    r = {"items": int(len(s))}
    # 0 start, 1 Philox window, 2 path (waypoints, fit, knots + records), 4 obstacles (3 is unused),
    # 5 circles + scalars, 6 copied out
    def pct(d):
        return [int(np.median(d)), int(np.percentile(d, 90)), int(d.max())]
    r["window"] = pct(s[:, 1] - s[:, 0])
    r["path"] = pct(s[:, 2] - s[:, 1])
    r["obstacles"] = pct(s[:, 4] - s[:, 2])
    r["rest"] = pct(s[:, 5] - s[:, 4])
    r["copy"] = pct(s[:, 6] - s[:, 5])
    tot = s[:, 6] - s[:, 0]
    r["item_total"] = [int(np.median(tot)), int(np.percentile(tot, 90)), int(tot.max())]
    # the slowest item's phases
    k = int(np.argmax(tot))
    r["slowest_item_phases"] = [int(x) for x in np.diff(s[k, [0, 1, 2, 4, 5, 6]])]
    r["span_first_start_to_last_end"] = int(s[:, 6].max() - s[:, 0].min())
    r["start_spread"] = int(s[:, 0].max() - s[:, 0].min())
    res.append(r)
st1 = venv.episode_stats().cpu().numpy()
out["episodes_per_step"] = float(st1[1] / 3)
out["steps"] = res
print(json.dumps(out, indent=1))
