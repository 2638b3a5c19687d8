#!/usr/bin/env python3
"""Diagnostic (GPU box): step time of the 65 536-env mixed batch under different env -> scenario
maps -- i mod 7 (BASELINE configs[4]), contiguous blocks, and single scenarios -- each timed like
bench.py (300 warmup steps, 16-step graph replays, HIP events).  One JSON line per case.

    python tools/mixed_probe.py [--envs 65536] [--steps 960]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

MIXED = ["perpendicular", "parallel", "S_parallel", "corridor", "S_corridor", "large", "impossible"]


def timed(venv, steps, warmup=300):
    import torch

    dev = venv.device
    g = torch.Generator(device=dev).manual_seed(1000)
    bank = [(torch.rand(venv.num_envs, 2, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)]
    venv.reset()
    for k in range(warmup):
        venv.step(bank[k % 16])
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for k in range(16):
            venv.step(bank[k])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps // 16):
        graph.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (steps // 16 * 16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=960)
    ap.add_argument("--cases", default="mod7,blocks,mod7_65408,heavy_light")
    a = ap.parse_args()
    import numpy as np
    import torch

    import drone2d_amd as d2
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    torch.cuda.set_device(0)
    kw = dict(ENV_TRAIN_CONFIG, scenario=MIXED)
    for case in a.cases.split(","):
        n = a.envs
        if case == "mod7":
            es = np.arange(n) % 7
        elif case == "blocks":
            es = (np.arange(n) * 7) // n
        elif case == "mod7_65408":
            n = 65408
            es = np.arange(n) % 7
        elif case == "heavy_light":
            # groups of 64 alternate heavy (S_parallel, S_corridor, large) / light scenarios
            heavy, light = [2, 4, 5], [0, 1, 3, 6]
            g = np.arange(n) // 64
            es = np.where(g % 2 == 0, np.array(heavy)[(g // 2) % 3], np.array(light)[(g // 2) % 4])
        else:
            raise SystemExit(case)
        venv = d2.Drone2dVecEnv(n, seed=12345, env_scenario=es.astype(np.int32), **kw)
        us = timed(venv, a.steps)
        venv.close()
        print(json.dumps({"case": case, "envs": n, "us_per_step": us, "env_steps_per_s": n / us * 1e6}), flush=True)


if __name__ == "__main__":
    main()
