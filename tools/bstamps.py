#!/usr/bin/env python3
"""Diagnostic (not product): where a Brent step's cycles go in K1's golden-march continuation.

    python tools/bstamps.py build                                  # CPU container: tools/_abl/libd2d_bst.so
    python tools/bstamps.py run [--scenario S] [--envs N] [--out F] # GPU box

The D2D_BSTAMP build (d2d_device.h) stamps s_memtime five times inside each continuation
`brent_step` of every path wave (wave 2; with `--scenario curriculum`, every step of the plain
search, whose tables are read per lane from global memory): entry, candidate computed (parabolic / golden arithmetic),
interval found (one compare, or the knot scan), probe evaluated (the interval's record from LDS +
the cubic's value, distance), state updated (scipy's compares and selects; the compiler schedules
them after the last stamp, so they are reported with the loop's own overhead).  Per phase the cycles
are summed over all stamped steps (first active lane of each wave; stamps also serialise the
stamped instructions a little, so the absolute total is a slight overestimate); the report gives
the median cycles per step of each phase, the loop's own gap between steps, and the share of steps
on the knot scan.
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
LIB = os.path.join(REPO, "tools", "_abl", "libd2d_bst.so")
BST_N = 1024 * 64 * 8


def build():
    import drone2d_amd  # noqa: F401
    from drone2d_amd import _build

    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run([_build.hipcc(), *_build.HIPCC_FLAGS, "-DD2D_BSTAMP", "-I", os.path.join(REPO, "include"),
                    _build.SRC, "-o", LIB], check=True)
    print("built", LIB)


def snapshot(venv, lib, n, torch):
    import numpy as np

    buf = np.zeros(BST_N, dtype=np.uint64)
    assert lib.d2d_debug_bstamps(None, 1) == 0
    venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
    torch.cuda.synchronize()
    assert lib.d2d_debug_bstamps(buf.ctypes.data_as(C.c_void_p), 0) == 0
    return buf.reshape(1024, 64, 8).astype(np.int64)


def analyse(s):
    import numpy as np

    t = s[:, :, :5]
    valid = t[:, :, 0] != 0
    d = np.diff(t[:, :, :4], axis=2)  # [wg][step][3]: candidate, interval, probe
    # the state update's selects are scheduled after the last stamp (they feed no stamp), so the
    # update is measured with the loop: the next step's entry - this step's probe stamp
    nxt = np.zeros_like(valid)
    nxt[:, :-1] = valid[:, 1:] & valid[:, :-1]
    upd = np.zeros(t.shape[:2], dtype=np.int64)
    upd[:, :-1] = t[:, 1:, 0] - t[:, :-1, 3]
    ok = nxt & (d.min(axis=2) >= 0) & (d.max(axis=2) < 100000) & (upd >= 0) & (upd < 100000)
    ph = np.concatenate([d, upd[:, :, None]], axis=2)[ok]
    per_wave = valid.sum(axis=1)
    scan = s[:, :, 6][ok]
    lanes = s[:, :, 7][ok]
    names = ["candidate", "interval", "probe", "update_and_loop"]
    res = {
        "stamped_steps": int(ok.sum()),
        "waves": int((per_wave > 0).sum()),
        "steps_per_wave_median_max": [int(np.median(per_wave[per_wave > 0])), int(per_wave.max())],
        "cycles_per_step_median": {k: int(np.median(ph[:, i])) for i, k in enumerate(names)},
        "cycles_per_step_mean": {k: round(float(ph[:, i].mean()), 1) for i, k in enumerate(names)},
        "step_total_median": int(np.median(ph.sum(axis=1))),
        "step_total_mean": round(float(ph.sum(axis=1).mean()), 1),
        "knot_scan_share": round(float(scan.mean()), 4),
        "active_lanes_median": int(np.median(lanes)),
    }
    if scan.any() and (~scan.astype(bool)).any():
        res["interval_median_fast_vs_scan"] = [int(np.median(ph[scan == 0, 1])), int(np.median(ph[scan == 1, 1]))]
    return res


def run(scenario, n, warm, reps, out):
    import numpy as np  # noqa: F401
    import torch

    import drone2d_amd as d2
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    kw = dict(ENV_TRAIN_CONFIG, scenario=scenario)
    if scenario == "curriculum":  # the fresh curriculum: the plain search over global-memory tables
        kw.update(mode="curriculum", sim_num=0)
    venv = d2.Drone2dVecEnv(n, seed=3, with_info=False, native_lib=LIB, **kw)
    lib = venv._lib
    lib.d2d_debug_bstamps.argtypes = [C.c_void_p, C.c_int32]
    lib.d2d_debug_bstamps.restype = C.c_int32
    venv.reset()
    for _ in range(warm):
        venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
    results = []
    for r in range(reps):
        res = analyse(snapshot(venv, lib, n, torch))
        res.update({"scenario": scenario, "envs": n, "rep": r})
        results.append(res)
        print(json.dumps(res))
    if out:
        with open(out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--scenario", default="corridor_free")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--warm", type=int, default=300)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.cmd == "build":
        build()
    else:
        run(a.scenario, a.envs, a.warm, a.reps, a.out)
