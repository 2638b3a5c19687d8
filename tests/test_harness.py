"""Evaluation harness: the reference's test loop and results files, on CPU.

* ``write_results`` fed the reference's own saved per-episode arrays (collisions / rewards / apes /
  time_spent ``.npy`` of run17see3, tests/golden/agent_17_90_episodes.npz) and its success / fail
  counts must reproduce the reference's ``results.txt`` byte for byte (main.py:311-326) and save the
  same arrays.
* ``run_first_episodes`` over the oracle-backed batch (test infrastructure) with the shipped actor:
  every env finishes exactly one episode, the per-episode records agree with the info rows the
  batch emitted on its done step, and the summary obeys the reference's arithmetic.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle_backend import OracleVecBackend

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _ref():
    res = json.load(open(os.path.join(GOLD, "agent_17_90_results.json")))
    eps = np.load(os.path.join(GOLD, "agent_17_90_episodes.npz"))
    return res, eps


@pytest.mark.parametrize("scn", ["corridor", "S_corridor", "large", "impossible", "parallel",
                                 "perpendicular", "S_parallel", "stage_1", "stage_5"])
def test_results_txt_matches_reference(d2, tmp_path, scn):
    from drone2d_amd import harness

    res, eps = _ref()
    r = res["results"][scn]
    m = {"successes": int(r["Successes"]), "fails": int(r["Fails"]), "unfinished": 0}
    for k in ("collisions", "rewards", "apes", "time_spent"):
        m[k] = eps[f"{scn}__{k}"]
    # the reference's own arrays agree with its counts (one record per run)
    assert len(m["apes"]) == m["successes"] + m["fails"]
    s = harness.write_results(m, str(tmp_path), scn, "90", res["agent"])
    got = open(tmp_path / f"{scn}_90_results.txt").read()
    assert got == res["results_txt"][scn]
    assert s["Collisions"] == int(r["Collisions"])
    for k in ("collisions", "rewards", "apes", "time_spent"):
        np.testing.assert_array_equal(np.load(tmp_path / f"{k}.npy"), m[k])


def test_summary_edge_cases(d2):
    from drone2d_amd import harness

    empty = {"successes": 0, "fails": 0, "collisions": np.zeros(0, np.int64), "apes": np.zeros(0),
             "time_spent": np.zeros(0, np.int64), "rewards": np.zeros(0)}
    s = harness.summary(empty)
    assert s["Success rate"] == 0 and s["Collision rate"] == 0 and np.isnan(s["Average APE"])
    one = {"successes": 0, "fails": 1, "collisions": np.array([1]), "apes": np.array([2.5]),
           "time_spent": np.array([7]), "rewards": np.array([-3.0])}
    s = harness.summary(one)
    assert (s["Successes"], s["Fails"], s["Collisions"], s["Collision rate"]) == (0, 1, 1, 1.0)
    assert s["Average APE"] == 2.5 and s["Average flight time"] == 7.0


def test_first_episodes_on_oracle(d2):
    from drone2d_amd import harness
    from drone2d_amd.config import ENV_TEST_CONFIG

    n = 24
    pol = harness.MlpActor.from_npz(os.path.join(GOLD, "agent_17_90.npz"))
    be = OracleVecBackend(n, seed=3, **dict(ENV_TEST_CONFIG, scenario="corridor"))
    m = harness.run_first_episodes(be, pol, seed=3)
    be.close()
    assert m["unfinished"] == 0
    # every episode ends in exactly one of success / failure (main.py:273-276)
    assert m["successes"] + m["fails"] == n
    for k in ("collisions", "apes", "time_spent", "rewards"):
        assert len(m[k]) == n
    assert (m["time_spent"] >= 1).all() and (m["time_spent"] <= int(ENV_TEST_CONFIG["n_steps"]) + 1).all()
    assert (m["collisions"] >= 0).all() and (m["collisions"] <= 1).all()
    assert np.isfinite(m["apes"]).all() and (m["apes"] >= 0).all()
    s = harness.summary(m)
    assert s["Success rate"] == m["successes"] / n
    assert s["Collision rate"] == int(m["collisions"].sum()) / n

    # the same run again is identical (seeded policy noise and env resets)
    be2 = OracleVecBackend(n, seed=3, **dict(ENV_TEST_CONFIG, scenario="corridor"))
    m2 = harness.run_first_episodes(be2, pol, seed=3)
    be2.close()
    for k in ("collisions", "apes", "time_spent", "rewards"):
        np.testing.assert_array_equal(m[k], m2[k])


def test_actor_matches_npz_mlp(d2):
    """MlpActor's deterministic action = tanh MLP 27-64-64-2 of the shipped policy, clipped."""
    from drone2d_amd import harness

    w = dict(np.load(os.path.join(GOLD, "agent_17_90.npz")))
    pol = harness.MlpActor.from_npz(os.path.join(GOLD, "agent_17_90.npz"))
    x = np.random.default_rng(0).uniform(-1, 1, (32, 27)).astype(np.float32)
    h = np.tanh(x @ w["mlp_extractor_policy_net_0_weight"].T + w["mlp_extractor_policy_net_0_bias"])
    h = np.tanh(h @ w["mlp_extractor_policy_net_2_weight"].T + w["mlp_extractor_policy_net_2_bias"])
    ref = np.clip(h @ w["action_net_weight"].T + w["action_net_bias"], -1, 1)
    got = pol.act(torch.from_numpy(x), deterministic=True).numpy()
    np.testing.assert_allclose(got, ref, atol=1e-5)


class _Recording(OracleVecBackend):
    """Oracle batch that also keeps the fp64 frame position after every step (before auto-reset
    for the envs still running; done envs are reset inside the step, so their last position is
    not in the state)."""

    def step(self, actions):
        out = super().step(actions)
        st, _ = self.orc.get_state()
        self.trace.append(st[0:2].T.copy())
        return out


def test_flight_paths(d2, tmp_path):
    """info['flight_path'] per episode: one (x, H - y) entry per env step, the reference's JSON
    layout (main.py:278, 307-308; drone_2d_env.py:409-415, 984-986), positions within float32
    observation rounding of the fp64 body position."""
    from drone2d_amd import harness
    from drone2d_amd.config import ENV_TEST_CONFIG

    n = 12
    pol = harness.MlpActor.from_npz(os.path.join(GOLD, "agent_17_90.npz"))
    be = _Recording(n, seed=4, **dict(ENV_TEST_CONFIG, scenario="corridor"))
    be.trace = []
    m = harness.run_first_episodes(be, pol, seed=4, flight_paths=True)
    be.close()
    H = float(ENV_TEST_CONFIG["screensize_y"])
    fps = harness.flight_path_lists(m)
    assert m["unfinished"] == 0 and len(fps) == n
    for i, (fp, T) in enumerate(zip(fps, m["time_spent"])):
        assert len(fp) == T and all(len(p) == 2 for p in fp)
        ref = np.array([[x, H - y] for x, y in (be.trace[t][i] for t in range(T - 1))])
        np.testing.assert_allclose(np.array(fp[:-1]), ref.reshape(-1, 2), rtol=0, atol=2e-4)
        if T > 1:  # the last entry is the terminal position: one step from the one before
            assert np.hypot(*(np.array(fp[-1]) - np.array(fp[-2]))) < 40.0
    s = harness.write_results(m, str(tmp_path), "corridor", "17", "x")
    back = json.load(open(tmp_path / "flight_paths"))
    assert [len(p) for p in back] == list(m["time_spent"]) and back[0][0] == fps[0][0]
    assert s["Successes"] + s["Fails"] == n
