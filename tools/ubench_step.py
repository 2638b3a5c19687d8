#!/usr/bin/env python3
"""Cycles per Brent step of the plain closest-point search, one wave per SIMD (diagnostic).

    python tools/ubench_step.py build TAG[:DEF,DEF...] ...   # CPU container: tools/_abl/libub_step_<tag>.so
    python tools/ubench_step.py run TAG ... [--waves 64]      # GPU box

Each lane searches one point (uniform over the screen) on the corridor scenario; per wave the timed
loop runs max-over-lanes steps, so cycles / that max is the wave's per-step latency.  Reports the
median over waves, with the median steps per wave.
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
ABL = os.path.join(REPO, "tools", "_abl")


def lib_for(tag):
    return os.path.join(ABL, f"libub_step_{tag}.so")


def build(specs):
    os.makedirs(ABL, exist_ok=True)
    for spec in specs:
        tag, _, defs = spec.partition(":")
        d = [f"-D{x}" for x in defs.split(",") if x]
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fno-fast-math", "-fPIC", "-shared", *d, "-I", os.path.join(REPO, "include"),
                        os.path.join(REPO, "tools", "ubench_step.hip"), "-o", lib_for(tag)], check=True)
        print("built", lib_for(tag), d)


def run(tags, waves, scen):
    import numpy as np

    import drone2d_amd  # noqa: F401
    from drone2d_amd import scenarios

    sc = scenarios.scenario_to_c(scenarios.create_test_scenario(scen, 1300, 1300))
    rng = np.random.default_rng(7)
    n = 64 * waves
    pts = np.ascontiguousarray(rng.uniform(0.0, 1300.0, size=(n, 2)))
    res = {"scenario": scen, "waves": waves}
    for t in tags:
        lib = C.CDLL(lib_for(t))
        u = np.zeros(n)
        cyc = np.zeros(waves, dtype=np.uint64)
        st = np.zeros(n, dtype=np.int32)
        rc = lib.ub_run(C.byref(sc), pts.ctypes.data_as(C.c_void_p), n, waves, u.ctypes.data_as(C.c_void_p),
                        cyc.ctypes.data_as(C.c_void_p), st.ctypes.data_as(C.c_void_p))
        assert rc == 0, rc
        mx = st.reshape(waves, 64).max(1)
        per = cyc.astype(np.float64) / np.maximum(mx, 1)
        res[t] = {"cycles_per_step_median": float(np.median(per)), "steps_per_wave_median": float(np.median(mx)),
                  "cycles_per_search_median": float(np.median(cyc)), "u_checksum": float(np.sum(u))}
    print(json.dumps(res))
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--waves", type=int, default=64)
    ap.add_argument("--scenario", default="corridor")
    a = ap.parse_args()
    if a.mode == "build":
        build(a.specs)
    else:
        run([s.partition(":")[0] for s in a.specs], a.waves, a.scenario)
