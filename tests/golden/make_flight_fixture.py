#!/usr/bin/env python3
"""Fixture generator (run in the build container, where /root/reference exists): the flight paths
the reference recorded for agent 17 (``best_models_config_and_res/run17see3/res/<scenario>/
flight_paths``, JSON written by main.py:307-308 from ``info['flight_path']``: the frame position
(x, screen_height - y) after every step of each of the 100 test episodes), reduced to the positions
at a few fixed step counts and the final position of every episode (NaN where an episode ended
earlier).  Read with ``json`` only.

Output: tests/golden/agent_17_90_flights.npz
"""
import json
import os

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
RUN = "best_models_config_and_res/run17see3/res"
TIMES = np.array([1, 10, 25, 50, 100, 200, 400], np.int64)


def main():
    out = {"times": TIMES}
    resdir = os.path.join(REF, RUN)
    for scn in sorted(os.listdir(resdir)):
        f = os.path.join(resdir, scn, "flight_paths")
        if not os.path.exists(f):
            continue
        paths = json.load(open(f))
        at = np.full((len(paths), len(TIMES), 2), np.nan)
        fin = np.zeros((len(paths), 2))
        for i, p in enumerate(paths):
            p = np.asarray(p, np.float64)
            for j, t in enumerate(TIMES):
                if len(p) >= t:
                    at[i, j] = p[t - 1]
            fin[i] = p[-1]
        out[f"{scn}__at"] = at
        out[f"{scn}__final"] = fin
        out[f"{scn}__len"] = np.array([len(p) for p in paths], np.int64)
    np.savez_compressed(os.path.join(HERE, "agent_17_90_flights.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
