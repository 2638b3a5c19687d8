#!/usr/bin/env python3
"""Diagnostic: per-wave phase timeline of K1 from s_memtime stamps (timing-only build).

    python tools/stamps.py build        # CPU container
    python tools/stamps.py run [--scenario S] [--envs N]   # GPU box

Stamps per wave: 0 start, 1 after scenario staging, 2 end of the role's work, 3 after the barrier,
4/5 role-specific hand-off points (W0 physics done / CA received, W1 sensing done / joint sweep
received, W2 search done / reward part received, W3 reset part done / joint sweep received), 6 end.
Reported in shader cycles from stamp 1, per role (wave 0..3): [median, p95, max].
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


def lib_path(tag):
    return LIB if not tag else LIB.replace(".so", f"_{tag}.so")


def build(tag="", defines=()):
    import drone2d_amd  # noqa: F401
    from drone2d_amd import _build

    out = lib_path(tag)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run([_build.hipcc(), *_build.HIPCC_FLAGS, "-DD2D_STAMPS", *[f"-D{d}" for d in defines],
                    "-I", os.path.join(REPO, "include"), _build.SRC, "-o", out], check=True)
    print("built", out)


def run(scenario, n, steps_warm, lib=LIB):
    import numpy as np
    import torch

    import drone2d_amd as d2
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    venv = d2.Drone2dVecEnv(n, seed=3, with_info=False, native_lib=lib, **dict(ENV_TRAIN_CONFIG, scenario=scenario))
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
    # cumulative times from the wave's stamp 1 (after staging): [median, p95, max]
    marks = {0: {"physics_done": 4, "ca_received": 5},
             1: {"sensing_done": 4, "gs_received": 5},
             2: {"search_done": 4, "rp_raised": 5},
             3: {"reset_part_done": 4, "gs_received": 5}}
    for w in range(4):
        r = {"stage": [int(np.median(s[:, w, 1] - s[:, w, 0]))]}
        for nm, k in list(marks[w].items()) + [("role_done", 2), ("barrier", 3), ("end", 6)]:
            d = s[:, w, k] - s[:, w, 1]
            r[nm] = [int(np.median(d)), int(np.percentile(d, 95)), int(d.max())]
        res[f"wave{w}"] = r
    # placement: slot 7 = XCC_ID << 32 | HW_ID (wave, simd [5:4], cu [11:8], sh [12], se [15:13])
    hw = s[:, :, 7]
    xcc = (hw >> 32) & 0xF
    hid = hw & 0xFFFFFFFF
    simd = (hid >> 4) & 3
    cu = (xcc << 8) | (((hid >> 13) & 7) << 5) | (((hid >> 12) & 1) << 4) | ((hid >> 8) & 0xF)
    res["simd_of_wave_hist"] = [np.bincount(simd[:, w], minlength=4).tolist() for w in range(4)]
    # Brent waves (wave 2) sharing a SIMD, and W2's phase-A duration by that count
    key = cu * 4 + simd
    cnt = {}
    for b in range(s.shape[0]):
        cnt[key[b, 2]] = cnt.get(key[b, 2], 0) + 1
    share = np.array([cnt[key[b, 2]] for b in range(s.shape[0])])
    dA = s[:, 2, 2] - s[:, 2, 1]
    res["w2_by_simd_share"] = {int(k): [int((share == k).sum()), int(np.median(dA[share == k]))]
                               for k in np.unique(share)}
    res["blocks_per_cu"] = np.bincount(np.unique(cu[:, 0], return_inverse=True)[1]).tolist()[:8]
    # per-XCD clocks differ: span from per-XCD t0
    spans = []
    for x in np.unique(xcc[:, 0]):
        m = xcc[:, 0] == x
        spans.append(int(s[m, :, 6].max() - s[m, :, 0].min()))
    res["kernel_span_cycles_per_xcd"] = spans
    # slowest 5% of workgroups: which wave ends phase A last, relative to W2's end (cycles)
    tot = s[:, 0, 6] - s[:, :, 0].min(1)
    slow = np.argsort(tot)[-max(1, len(tot) // 20):]
    endA = s[slow, :, 2] - s[slow, 2, 2][:, None]
    res["slow_blocks"] = {"total_med": int(np.median(tot[slow])),
                          "last_wave_hist": np.bincount(np.argmax(s[slow, :, 2], 1), minlength=4).tolist(),
                          "endA_minus_w2_med": [int(np.median(endA[:, w])) for w in range(4)],
                          "w2_endA_from_start_med": int(np.median(s[slow, 2, 2] - s[slow, 2, 0])),
                          "after_A_med": int(np.median(s[slow, 0, 6] - s[slow, :, 2].max(1)))}
    print(json.dumps(res, indent=1))
    return res


def run_fill(scenario, n, steps_warm, lib=LIB):
    """K4's phase stamps (wave 0 sensing, waves 1-3 table re-check thirds, wave 1 continuation and
    path part) for one fill launch after ``steps_warm`` steps, in cycles from the block's stamp 0."""
    import numpy as np
    import torch

    import drone2d_amd as d2
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    venv = d2.Drone2dVecEnv(n, seed=3, with_info=False, native_lib=lib, **dict(ENV_TRAIN_CONFIG, scenario=scenario))
    lib = venv._lib
    lib.d2d_debug_stamps.argtypes = [C.c_void_p, C.c_void_p]
    nb = (n + 127) // 128
    base = 65536
    buf = torch.zeros(base + nb * 32 + nb, dtype=torch.int64, device=venv.device)
    venv.reset()
    k = 0
    while k < steps_warm or (k % 16) != 15:
        venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
        k += 1
    lib.d2d_debug_stamps(venv._h, C.c_void_p(buf.data_ptr()))
    venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)  # the 16th: K1 then K4
    torch.cuda.synchronize()
    b = buf.cpu().numpy()
    s = b[base:base + nb * 32].reshape(nb, 4, 8).astype(np.int64)
    tot = b[base + nb * 32:base + nb * 33]
    live = s[:, 0, 7] != 0  # blocks with work ran fill_split
    s, tot = s[live], tot[live]
    t0 = s[:, :, 0].min()
    res = {"scenario": scenario, "envs": n, "blocks_with_fills": int(live.sum()),
           "fills_per_block": [int(np.median(tot)), int(tot.max())],
           "kernel_span_cycles": int(s[:, :, 7].max() - t0),
           "block_start_spread": int(s[:, 0, 0].max() - t0)}
    names = {1: "staged", 2: "spawn", 3: "part1", 4: "barrier1", 5: "continuation", 6: "path", 7: "end"}
    for w in range(4):
        r = {}
        for k, nm in names.items():
            if w != 1 and k in (5, 6):
                continue
            d = s[:, w, k] - s[:, w, 0]
            r[nm] = [int(np.median(d)), int(np.percentile(d, 95)), int(d.max())]
        res[f"wave{w}"] = r
    print(json.dumps(res, indent=1))
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run", "fill"])
    ap.add_argument("--scenario", default="corridor")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--warm", type=int, default=40)
    ap.add_argument("--tag", default="", help="variant library suffix")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra -D for the variant")
    ap.add_argument("--small", type=int, default=16384, help="second (1 workgroup per CU) size; 0 = skip")
    a = ap.parse_args()
    if a.mode == "build":
        build(a.tag, a.defines)
    elif a.mode == "fill":
        out = [run_fill(s, a.envs, a.warm, lib_path(a.tag)) for s in a.scenario.split(",")]
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        json.dump(out, open(os.path.join(REPO, "gpurun_out", "fill_stamps.json"), "w"), indent=1)
    else:
        lib = lib_path(a.tag)
        out = [run(a.scenario, a.envs, a.warm, lib)]
        if a.small:
            out.append(run(a.scenario, a.small, a.warm, lib))
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        name = "stamps.json" if not a.tag else f"stamps_{a.tag}.json"
        json.dump(out, open(os.path.join(REPO, "gpurun_out", name), "w"), indent=1)
