#!/usr/bin/env python3
"""Curriculum golden fixture from the reference's own code (run ONLY in the development container).

For every stage_1..stage_5 and seeds 0..S-1: seed Python's ``random`` and NumPy's global RNG, then
construct the reference's ``Drone2dEnv`` unmodified in ``mode='curriculum'`` (ref_shims for
pymunk / pygame / gym, as make_golden.py) and record what its reset generated: waypoints, QPMI2D
knots/coefficients, obstacle circles and the drone's spawn pose.  drone2d_amd.curriculum must
reproduce these bit for bit from ``RandomState(seed)`` / ``random.Random(seed)``.

Writes tests/golden/curriculum.npz (plain arrays, allow_pickle=False).
"""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _bodies, _import_reference  # noqa: E402

STAGES = ["stage_1", "stage_2", "stage_3", "stage_4", "stage_5"]
SEEDS = 24


def main():
    de, pp, rl_config, ts, shims = _import_reference()
    out = {}
    for stage in STAGES:
        for s in range(SEEDS):
            cfg = dict(rl_config.env_train_config)
            cfg.update(render_sim=False, render_path=False, render_shade=False, render_text=False,
                       mode="curriculum", scenario=stage)
            random.seed(s)
            np.random.seed(s)
            env = de.Drone2dEnv(**cfg)
            k = f"{stage}/{s}"
            out[k + "/wps"] = np.asarray(env.wps, dtype=np.float64)
            out[k + "/us"] = np.asarray(env.predef_path.us, dtype=np.float64)
            out[k + "/xp"] = np.asarray(env.predef_path.x_params, dtype=np.float64)
            out[k + "/yp"] = np.asarray(env.predef_path.y_params, dtype=np.float64)
            out[k + "/circles"] = np.array([[o.x_pos, o.y_pos, o.radius] for o in env.obstacles],
                                           dtype=np.float64).reshape(-1, 3)
            f = _bodies(env)[0]
            out[k + "/spawn"] = np.array([f.px, f.py, f.a], dtype=np.float64)
    np.savez(os.path.join(HERE, "curriculum.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
