#!/usr/bin/env python3
"""Closed-loop distributional parity, GPU box.

Runs the shipped agent PFCA_see_3_obs_17_90 (weights: tests/golden/agent_17_90.npz) on every test
scenario with N envs each (stochastic policy, as the reference's ``model.predict(obs)``), writes the
reference's result files under gpurun_out/Tests/agent_17/<scenario>/ and compares success /
collision rates with the reference's own 100-run results (tests/golden/agent_17_90_results.json).

    python tools/closed_loop.py [--envs 2000] [--seed 0] [--config test|train]

Besides the rates, the per-episode distributions (flight time, APE, total reward) are compared with
the reference's own saved arrays (tests/golden/agent_17_90_episodes.npz): z of the mean difference
and the two-sample KS p-value; and the positions along the flights (after 1-400 steps and at the
end) with the reference's recorded flight paths (tests/golden/agent_17_90_flights.npz).
``--config`` picks the env kwargs: the reference's current
env_test_config (default) or its env_train_config (run17see3/env_train_config.txt): the two differ
in reward weights only (initial_throw / n_fall_steps are inert in the reference), so the flight time
and APE distributions must not move between them while the total rewards tell which configuration
the reference's saved results were produced with.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SCENARIOS = ["perpendicular", "parallel", "S_parallel", "corridor", "S_corridor", "large", "impossible"]


def flight_ks(fxy, time_spent, flights, scn):
    """Two-sample KS of the frame position (x and screen y) after t steps, over the episodes still
    flying at t, and of the final position, against the reference's own flight_paths of agent 17
    (tests/golden/agent_17_90_flights.npz)."""
    import numpy as np
    from scipy.stats import ks_2samp

    res = {}
    ref_at, ref_fin = flights[f"{scn}__at"], flights[f"{scn}__final"]
    for j, t in enumerate(flights["times"]):
        t = int(t)
        if t > fxy.shape[0]:
            break
        ours = fxy[t - 1][~np.isnan(fxy[t - 1, :, 0])]
        ref = ref_at[:, j][~np.isnan(ref_at[:, j, 0])]
        if len(ours) < 20 or len(ref) < 20:
            continue
        res[f"t{t}"] = {"n": [len(ours), len(ref)],
                        "ks_p_x": float(ks_2samp(ours[:, 0], ref[:, 0]).pvalue),
                        "ks_p_y": float(ks_2samp(ours[:, 1], ref[:, 1]).pvalue)}
    last = fxy[np.asarray(time_spent) - 1, np.arange(fxy.shape[1])]
    res["final"] = {"ks_p_x": float(ks_2samp(last[:, 0], ref_fin[:, 0]).pvalue),
                    "ks_p_y": float(ks_2samp(last[:, 1], ref_fin[:, 1]).pvalue)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--scenarios", default=",".join(SCENARIOS))
    ap.add_argument("--config", default="test", choices=["test", "train"])
    ap.add_argument("--flight-paths", action="store_true",
                    help="also write the reference's flight_paths JSON per scenario (large: ~24 B per env-step)")
    a = ap.parse_args()
    import torch  # noqa: F401

    import drone2d_amd as d2
    from drone2d_amd import harness
    from drone2d_amd.config import ENV_TEST_CONFIG

    ref = json.load(open(os.path.join(REPO, "tests", "golden", "agent_17_90_results.json")))
    import numpy as np
    from scipy.stats import ks_2samp

    eps = np.load(os.path.join(REPO, "tests", "golden", "agent_17_90_episodes.npz"))
    flights = np.load(os.path.join(REPO, "tests", "golden", "agent_17_90_flights.npz"))
    if a.config == "test":
        base = dict(ENV_TEST_CONFIG)
    else:
        base = dict(ENV_TEST_CONFIG, **{k: v for k, v in ref["env_config"].items() if not k.startswith("render")})
    pol = harness.MlpActor.from_npz(os.path.join(REPO, "tests", "golden", "agent_17_90.npz"))
    out = {}
    for scn in a.scenarios.split(","):
        t0 = time.perf_counter()
        venv = d2.Drone2dVecEnv(a.envs, seed=a.seed, with_info=True, **dict(base, scenario=scn))
        m = harness.run_first_episodes(venv, pol, seed=a.seed, flight_paths=True)
        venv.close()
        fxy = m.pop("flight_xy") if not a.flight_paths else m["flight_xy"]
        s = harness.write_results(m, os.path.join(REPO, "gpurun_out", "Tests", "agent_17_" + a.config, scn), scn, "17",
                                  ref["agent"])
        r = ref["results"][scn]
        p, q = s["Success rate"], r["Success rate"]
        n_ours, n_ref = s["Successes"] + s["Fails"], r["Successes"] + r["Fails"]
        se = math.sqrt(max(q * (1 - q), 0.01 * 0.99) / n_ref + max(p * (1 - p), 0.01 * 0.99) / max(n_ours, 1))
        out[scn] = {"ours": s, "reference": {k: r[k] for k in ("Success rate", "Collision rate", "Average APE",
                                                               "Average flight time")},
                    "runs": [n_ours, n_ref], "success_z": (p - q) / se, "unfinished": m["unfinished"],
                    "seconds": time.perf_counter() - t0}
        for k in ("time_spent", "apes", "rewards"):
            x, y = np.asarray(m[k], np.float64), eps[f"{scn}__{k}"].astype(np.float64)
            se_m = math.sqrt(x.var() / max(len(x), 1) + y.var() / len(y))
            out[scn][k] = {"ours": float(x.mean()), "ref": float(y.mean()),
                           "z": float((x.mean() - y.mean()) / max(se_m, 1e-12)),
                           "ks_p": float(ks_2samp(x, y).pvalue)}
        if f"{scn}__at" in flights:
            # where the drone is after t steps / at the end, against the reference's recorded flights
            out[scn]["flight"] = flight_ks(fxy, m["time_spent"], flights, scn)
        print(scn, json.dumps(out[scn]), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    json.dump({"config": a.config, "envs": a.envs, "seed": a.seed, "scenarios": out},
              open(os.path.join(REPO, "gpurun_out", f"closed_loop_{a.config}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
