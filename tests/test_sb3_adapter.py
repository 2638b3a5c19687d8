"""SB3 VecEnv adapter (SURVEY.md §8(b) VecEnv row, §8(f)-1).

CPU: the adapter's contract over the oracle-backed batch (test infrastructure): shapes/dtypes,
SB3 auto-reset semantics (returned row = next episode's first obs, ``terminal_observation`` = last
obs), ``TimeLimit.truncated``, the reference's info keys.  GPU: the same adapter over the HIP batch
agrees with the oracle-backed one.
"""
import numpy as np
import pytest
import torch

from oracle_backend import OracleVecBackend
from parity_util import OBS_ATOL

REF_INFO_KEYS = {"reward", "collision_avoidance_reward", "path_adherence", "path_progression",
                 "collision_reward", "reach_end_reward", "agressive_alpha_reward", "env_steps",
                 "dist_closest_obs", "APE", "total_reward", "n_collisions", "n_successful_runs",
                 "n_failed_runs", "flight_path"}


def _kw(**over):
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    return dict(ENV_TRAIN_CONFIG, **over)


def _adapter(backend, infos):
    from drone2d_amd.sb3 import SB3VecEnv

    return SB3VecEnv(backend.num_envs, infos=infos, backend=backend)


@pytest.mark.parametrize("infos", ["full", "done", "none"])
def test_adapter_contract_on_oracle(d2, infos):
    n = 96
    be = OracleVecBackend(n, seed=4, **_kw(scenario=["corridor", "S_corridor", "large"]))
    ref = OracleVecBackend(n, seed=4, **_kw(scenario=["corridor", "S_corridor", "large"]))
    env = _adapter(be, infos)
    obs = env.reset()
    r_obs = ref.reset().numpy()
    assert obs.dtype == np.float32 and obs.shape == (n, 27)
    np.testing.assert_array_equal(obs, r_obs)
    rng = np.random.default_rng(0)
    seen_done = 0
    for t in range(120):
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        env.step_async(act)
        obs, rew, dones, inf = env.step_wait()
        r_obs, r_rew, r_term, r_trunc, r_info = ref.step(torch.from_numpy(act))
        assert obs.shape == (n, 27) and rew.shape == (n,) and dones.dtype == np.bool_ and len(inf) == n
        np.testing.assert_array_equal(obs, r_obs.numpy())
        np.testing.assert_array_equal(rew, r_rew.numpy())
        np.testing.assert_array_equal(dones, (r_term | r_trunc).numpy())
        tobs = ref.terminal_obs.numpy()
        for i in range(n):
            d = inf[i]
            assert d["TimeLimit.truncated"] is False
            if dones[i]:
                seen_done += 1
                np.testing.assert_array_equal(d["terminal_observation"], tobs[i])
                if infos != "none":
                    assert REF_INFO_KEYS <= set(d)
                    assert d["env_steps"] == int(r_info[i, 7])
            else:
                assert "terminal_observation" not in d
                if infos == "full":
                    assert REF_INFO_KEYS <= set(d)
    assert seen_done > 20
    env.close()
    ref.close()


def test_adapter_timelimit_truncation(d2):
    """With time-up reported as truncation, SB3's TimeLimit.truncated flag is set on those envs."""
    n = 32
    be = OracleVecBackend(n, seed=1, timeup_truncates=True, **_kw(scenario="large_free", n_steps=4))
    env = _adapter(be, "done")
    env.reset()
    for t in range(4):
        obs, rew, dones, inf = env.step(np.zeros((n, 2), np.float32))
    assert dones.all()
    assert all(d["TimeLimit.truncated"] is True for d in inf)
    assert all(d["env_steps"] == 4 for d in inf)
    env.close()


def test_adapter_api_surface(d2):
    be = OracleVecBackend(8, seed=0, **_kw(scenario="corridor"))
    env = _adapter(be, "none")
    assert env.num_envs == 8
    assert env.observation_space.shape == (27,) and env.action_space.shape == (2,)
    assert env.seed(7) == [7] * 8
    assert env.env_is_wrapped(object) == [False] * 8
    assert env.get_attr("num_envs", indices=[0, 1]) == [8, 8]
    env.reset()
    out = env.step(np.zeros((8, 2), np.float32))
    assert len(out) == 4
    env.close()


@pytest.mark.gpu
def test_adapter_hip_matches_oracle(d2):
    from drone2d_amd.sb3 import SB3VecEnv

    n = 512
    kw = _kw(scenario=["corridor", "S_corridor", "large", "parallel"])
    hip = SB3VecEnv(n, seed=9, infos="done", **kw)
    ref = _adapter(OracleVecBackend(n, seed=9, **kw), "done")
    np.testing.assert_allclose(hip.reset(), ref.reset(), rtol=0, atol=OBS_ATOL)
    rng = np.random.default_rng(3)
    dones_total = 0
    for t in range(90):
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        o1, r1, d1, i1 = hip.step(act)
        o2, r2, d2_, i2 = ref.step(act)
        np.testing.assert_array_equal(d1, d2_)
        np.testing.assert_allclose(o1, o2, rtol=0, atol=OBS_ATOL)
        np.testing.assert_allclose(r1, r2, rtol=1e-5, atol=1e-4)
        for i in np.nonzero(d1)[0]:
            dones_total += 1
            np.testing.assert_allclose(i1[i]["terminal_observation"], i2[i]["terminal_observation"], atol=OBS_ATOL)
            assert i1[i]["env_steps"] == i2[i]["env_steps"]
    assert dones_total > 0
    hip.close()
    ref.close()


def test_dist_closest_obs_in_curriculum_pool(d2):
    """Curriculum pool mode redraws each env's scenario at every reset (some stage_3 entries have
    no obstacles): info['dist_closest_obs'] must be the kernel's value for the episode's own
    scenario (+inf without obstacles), not one looked up from the initial env -> scenario map."""
    from drone2d_amd import abi

    n = 128
    kw = _kw(scenario="stage_3", mode="curriculum", curriculum_pool=32, curriculum_seed=3)
    be = OracleVecBackend(n, seed=5, **kw)
    n_free = sum(len(s.circles) == 0 for s in be.scenarios)
    assert 0 < n_free < len(be.scenarios)
    env = _adapter(be, "done")
    env.reset()
    rng = np.random.default_rng(0)
    seen = {True: 0, False: 0}
    for _ in range(400):
        env.step_async(rng.uniform(-1, 1, (n, 2)).astype(np.float32))
        _, _, dones, infos = env.step_wait()
        rows = be.orc.info
        for i in np.nonzero(dones)[0]:
            d = infos[i]["dist_closest_obs"]
            assert d == float(rows[i, abi.INFO_DCLOSE]) or (np.isinf(d) and np.isinf(rows[i, abi.INFO_DCLOSE]))
            seen[bool(np.isinf(d))] += 1
    assert seen[True] > 0 and seen[False] > 0
