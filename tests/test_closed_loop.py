"""Closed-loop distributional parity with the shipped agent -- needs an MI355X.

The reference publishes, for agent PFCA_see_3_obs_17_90, 100-run success / collision rates per test
scenario (best_models_config_and_res/run17see3/res/*/results.txt, in tests/golden/
agent_17_90_results.json).  The same actor (weights in tests/golden/agent_17_90.npz), sampled
stochastically as the reference's ``model.predict(obs)`` does, flies 1 000 first episodes per
scenario in the HIP env; the success rate must agree within 4 standard errors of the difference.
This is the one check of the (otherwise unpinned) Chipmunk-equivalent physics against the
reference's own behaviour.  Harness metrics are computed exactly as main.py:273-325 does.
"""
import json
import math
import os

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("scn", ["corridor", "large", "S_corridor", "impossible"])
def test_agent_success_rate_matches_reference(d2, scn):
    from drone2d_amd import harness
    from drone2d_amd.config import ENV_TEST_CONFIG

    ref = json.load(open(os.path.join(HERE, "golden", "agent_17_90_results.json")))["results"][scn]
    pol = harness.MlpActor.from_npz(os.path.join(HERE, "golden", "agent_17_90.npz"))
    venv = d2.Drone2dVecEnv(1000, seed=5, with_info=True, **dict(ENV_TEST_CONFIG, scenario=scn))
    m = harness.run_first_episodes(venv, pol, seed=5)
    venv.close()
    s = harness.summary(m)
    assert m["unfinished"] == 0 and s["Successes"] + s["Fails"] == 1000
    p, q = s["Success rate"], ref["Success rate"]
    se = math.sqrt(max(q * (1 - q), 0.0099) / 100 + max(p * (1 - p), 0.0099) / 1000)
    assert abs(p - q) < 4 * se, (scn, p, q)
    c, cq = s["Collision rate"], ref["Collision rate"]
    sec = math.sqrt(max(cq * (1 - cq), 0.0099) / 100 + max(c * (1 - c), 0.0099) / 1000)
    assert abs(c - cq) < 4 * sec, (scn, c, cq)


@pytest.mark.parametrize("scn", ["corridor", "large", "S_corridor", "impossible"])
def test_agent_episode_distributions_match_reference(d2, scn):
    """Per-episode flight time, APE and total reward against the reference's own saved arrays
    (run17see3/res/<scn>/{time_spent,apes,rewards}.npy, tests/golden/agent_17_90_episodes.npz):
    two-sample KS test, p > 1e-3.  The reference's saved rewards were produced with its
    env_train_config reward weights (PP_rew_max 3.5, abs_inv_CA_min_rew 1/6; tools/closed_loop.py
    --config train vs test, DESIGN.md "Closed-loop parity"), so this run uses those kwargs; the dynamics and
    observations do not depend on them."""
    import numpy as np
    from scipy.stats import ks_2samp

    from drone2d_amd import harness
    from drone2d_amd.config import ENV_TEST_CONFIG

    ref = json.load(open(os.path.join(HERE, "golden", "agent_17_90_results.json")))
    eps = np.load(os.path.join(HERE, "golden", "agent_17_90_episodes.npz"))
    kw = dict(ENV_TEST_CONFIG, **{k: v for k, v in ref["env_config"].items() if not k.startswith("render")})
    pol = harness.MlpActor.from_npz(os.path.join(HERE, "golden", "agent_17_90.npz"))
    venv = d2.Drone2dVecEnv(4096, seed=11, with_info=True, **dict(kw, scenario=scn))
    m = harness.run_first_episodes(venv, pol, seed=11)
    venv.close()
    assert m["unfinished"] == 0
    for k in ("time_spent", "apes", "rewards"):
        p = ks_2samp(np.asarray(m[k], np.float64), eps[f"{scn}__{k}"].astype(np.float64)).pvalue
        assert p > 1e-3, (scn, k, p)


def test_flight_paths_on_hip(d2):
    """info['flight_path'] from the HIP env (harness ``flight_paths=True``): one entry per env step,
    the first inside the spawn rectangle (screen coordinates, y flipped), every successful episode
    ending inside the reach-end box around the last waypoint (drone_2d_env.py:548-556)."""
    import numpy as np

    from drone2d_amd import harness
    from drone2d_amd.config import ENV_TEST_CONFIG

    kw = dict(ENV_TEST_CONFIG, scenario="corridor")
    pol = harness.MlpActor.from_npz(os.path.join(HERE, "golden", "agent_17_90.npz"))
    venv = d2.Drone2dVecEnv(1000, seed=7, with_info=True, **kw)
    scn = venv.scenarios[0]
    m = harness.run_first_episodes(venv, pol, seed=7, flight_paths=True)
    venv.close()
    H = float(kw["screensize_y"])
    xmin, xmax, ymin, ymax = scn.spawn
    tx, ty = float(scn.wps[-1][0]), H - float(scn.wps[-1][1])
    fps = harness.flight_path_lists(m)
    assert m["unfinished"] == 0 and len(fps) == 1000
    n_succ = 0
    for fp, T, col in zip(fps, m["time_spent"], m["collisions"]):
        assert len(fp) == T
        x0, y0 = fp[0]
        assert xmin - 2 <= x0 <= xmax + 2 and H - ymax - 2 <= y0 <= H - ymin + 2
        xl, yl = fp[-1]
        if abs(xl - tx) < 20 and abs(yl - ty) < 20:
            n_succ += 1
    assert n_succ >= m["successes"] > 0


@pytest.mark.parametrize("scn", ["corridor", "large", "S_corridor"])
def test_flight_positions_match_reference(d2, scn):
    """Where the drone is along its flights: the frame position after t steps (over the episodes
    still flying) and at the end, against the flight_paths the reference recorded for the same
    agent (run17see3/res/<scn>/flight_paths, reduced in tests/golden/agent_17_90_flights.npz by
    make_flight_fixture.py): two-sample KS, p > 1e-3 for x and y at every t."""
    import numpy as np
    from scipy.stats import ks_2samp

    from drone2d_amd import harness
    from drone2d_amd.config import ENV_TEST_CONFIG

    fl = np.load(os.path.join(HERE, "golden", "agent_17_90_flights.npz"))
    pol = harness.MlpActor.from_npz(os.path.join(HERE, "golden", "agent_17_90.npz"))
    venv = d2.Drone2dVecEnv(4000, seed=3, with_info=True, **dict(ENV_TEST_CONFIG, scenario=scn))
    m = harness.run_first_episodes(venv, pol, seed=3, flight_paths=True)
    venv.close()
    fxy = m["flight_xy"]
    ref_at = fl[f"{scn}__at"]
    checked = 0
    for j, t in enumerate(fl["times"]):
        ours = fxy[t - 1][~np.isnan(fxy[t - 1, :, 0])]
        ref = ref_at[:, j][~np.isnan(ref_at[:, j, 0])]
        if len(ours) < 20 or len(ref) < 20:
            continue
        for c in (0, 1):
            assert ks_2samp(ours[:, c], ref[:, c]).pvalue > 1e-3, (scn, int(t), c)
        checked += 1
    last = fxy[m["time_spent"] - 1, np.arange(fxy.shape[1])]
    for c in (0, 1):
        assert ks_2samp(last[:, c], fl[f"{scn}__final"][:, c]).pvalue > 1e-3, (scn, "final", c)
    assert checked >= 5
