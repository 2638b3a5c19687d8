#!/usr/bin/env python3
"""A/B timing of compile-time variants of the product library (diagnostic builds, never shipped).

    python tools/variants.py build base p0:D2D_PRIO=0     # CPU container: tools/_abl/libd2d_var_<tag>.so
    python tools/variants.py run base p0 [--envs N]        # GPU box: ms/step of each, interleaved rounds

A spec is TAG[:DEF[,DEF...]][::FLAG+FLAG][@PATCH]; DEF is passed as -DDEF, PATCH names a diagnostic
patch under tools/patches/ (e.g. ``r0:D2D_ABL=1@role_ablation``: the role ablations), applied to a
copy of the package sources before the build.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
ABL = os.path.join(REPO, "tools", "_abl")


def lib_for(tag):
    return os.path.join(ABL, f"libd2d_var_{tag}.so")


def build(specs):
    import drone2d_amd  # noqa: F401
    from drone2d_amd import _build

    os.makedirs(ABL, exist_ok=True)
    for spec in specs:
        spec, _, patch = spec.partition("@")
        spec, _, flags = spec.partition("::")   # TAG[:DEF,DEF][::flag+flag] (e.g. -mllvm+-misched=...)
        tag, _, defs = spec.partition(":")
        d = [f"-D{x}" for x in defs.split(",") if x] + [f for f in flags.split("+") if f]
        src, tmp = _build.SRC, None
        if patch:
            # the package sources + include/ copied, the patch applied to the copy (never to the tree)
            tmp = tempfile.mkdtemp(prefix="d2d_var_")
            pkg = os.path.basename(os.path.dirname(os.path.dirname(_build.SRC)))
            shutil.copytree(os.path.join(REPO, pkg, "csrc"), os.path.join(tmp, pkg, "csrc"))
            shutil.copytree(os.path.join(REPO, "include"), os.path.join(tmp, "include"))
            subprocess.run(["patch", "-s", "-p1", "-d", tmp, "-i",
                            os.path.join(REPO, "tools", "patches", patch + ".patch")], check=True)
            src = os.path.join(tmp, os.path.relpath(_build.SRC, REPO))
        subprocess.run([_build.hipcc(), *_build.HIPCC_FLAGS, *d, "-I", os.path.join(REPO, "include"), src,
                        "-o", lib_for(tag)], check=True)
        if tmp:
            shutil.rmtree(tmp)
        print("built", lib_for(tag), d, patch or "")


def time_variant(d2, torch, lib, n, scenario, steps=1000, warmup=300, auto_reset=True):
    import numpy as np

    from drone2d_amd.config import ENV_TRAIN_CONFIG

    es = None
    if scenario.startswith("mixed"):
        # mixed: env i -> scenario i mod 7; mixedblock: (i // 64) mod 7 (homogeneous 64-env blocks)
        es = (np.arange(n) // (64 if scenario == "mixedblock" else 1)) % 7
        from bench import MIXED as scenario
    venv = d2.Drone2dVecEnv(n, seed=1, with_info=False, native_lib=lib, auto_reset=auto_reset, env_scenario=es,
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


def run(tags, n, scenario, rounds, auto_reset=True, steps=1000, warmup=300):
    import torch

    import drone2d_amd as d2

    res = {t: [] for t in tags}
    for r in range(rounds):
        for t in tags:
            res[t].append(time_variant(d2, torch, lib_for(t), n, scenario, steps=steps, warmup=warmup,
                                       auto_reset=auto_reset))
    out = {t: {"ms_per_step_min": min(v), "ms_per_step_all": v} for t, v in res.items()}
    out = {"envs": n, "scenario": scenario, "auto_reset": auto_reset, "variants": out}
    print(json.dumps(out, indent=1))
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "variants.json"), "a") as f:
        f.write(json.dumps(out) + "\n")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run"])
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--scenario", default="corridor")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-auto-reset", action="store_true")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=300, help="untimed steps: the bench's steady state")
    a = ap.parse_args()
    if a.mode == "build":
        build(a.specs)
    else:
        run([s.partition("@")[0].partition("::")[0].partition(":")[0] for s in a.specs], a.envs, a.scenario, a.rounds, not a.no_auto_reset,
            a.steps, a.warmup)
