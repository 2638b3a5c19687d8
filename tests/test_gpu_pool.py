"""Curriculum pool refresh, pool-mode checkpoints and failed scenario uploads -- needs an MI355X.

* ``d2d_refresh_pool``: running episodes keep their scenarios, later resets draw from the new pool;
  HIP vs the CPU oracle (same two-half pool semantics) teacher-forced across two refreshes.
* ``state_dict`` / ``load_state_dict`` (``d2d_get/set_env_scenarios``): a pool-mode batch restored
  into a fresh handle continues bit-identically.
* a rejected ``d2d_set_scenarios`` leaves the handle as it was (no freed tables behind it).
"""
import numpy as np
import pytest
import torch

from parity_util import OBS_ATOL, compare_step

pytestmark = pytest.mark.gpu


def _kw(**over):
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    return dict(dict(ENV_TRAIN_CONFIG, scenario="stage_5", mode="curriculum", curriculum_pool=16, curriculum_seed=5),
                **over)


def _pair(d2, n, seed, kw):
    import oracle
    from drone2d_amd.config import make_cfg

    venv = d2.Drone2dVecEnv(n, seed=seed, **kw)
    cfg = make_cfg(dict(kw))
    cfg.scn_pool = 1
    orc = oracle.OracleBatch(cfg, [s.to_c() for s in venv.scenarios], n, env_scenario=venv.env_scenario)
    np.testing.assert_allclose(venv.reset().cpu().numpy(), orc.reset(seed), rtol=0, atol=OBS_ATOL)
    return venv, orc


def test_refresh_pool_vs_oracle(d2):
    from drone2d_amd._native import NativeError

    n, rng = 1024, np.random.default_rng(11)
    venv, orc = _pair(d2, n, 21, _kw(n_steps=40))

    def run(steps):
        d = 0
        for _ in range(steps):
            compare_step(venv, orc, rng.uniform(-1, 1, (n, 2)).astype(np.float32))
            d += int(orc.term.sum())
        np.testing.assert_array_equal(venv.get_env_scenarios().cpu().numpy(), orc.get_env_scenarios())
        return d

    assert run(45) > 0
    old = venv.get_env_scenarios().cpu().numpy()
    assert old.max() < 16  # first half
    venv.refresh_curriculum(seed=100)
    assert orc.refresh_pool([s.to_c() for s in venv.scenarios]) == 0
    # running episodes keep their first-half scenarios; a second refresh now would overwrite them
    np.testing.assert_array_equal(venv.get_env_scenarios().cpu().numpy(), old)
    with pytest.raises(NativeError, match="still run episodes"):
        venv.refresh_curriculum(seed=101)
    run(45)  # > n_steps: every env has reset into the new (second) half since
    es = venv.get_env_scenarios().cpu().numpy()
    assert es.min() >= 16 and es.max() < 32
    venv.refresh_curriculum(seed=102)  # back into the first half
    assert orc.refresh_pool([s.to_c() for s in venv.scenarios]) == 0
    run(45)
    assert venv.get_env_scenarios().cpu().numpy().max() < 16
    venv.close()


def test_pool_checkpoint_restore(d2):
    """A pool-mode batch checkpointed mid-episode and restored into a new handle continues exactly."""
    n, rng = 512, np.random.default_rng(12)
    kw = _kw()
    a = d2.Drone2dVecEnv(n, seed=3, **kw)
    a.reset()
    for _ in range(150):
        a.step(torch.as_tensor(rng.uniform(-1, 1, (n, 2)).astype(np.float32)))
    sd = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in a.state_dict().items()}
    assert len(np.unique(sd["env_scn"].cpu().numpy())) > 1
    b = d2.Drone2dVecEnv(n, seed=999, **kw)  # another seed and initial map: all restored
    b.load_state_dict(sd)
    np.testing.assert_array_equal(b.get_env_scenarios().cpu().numpy(), sd["env_scn"].cpu().numpy())
    for _ in range(120):
        act = torch.as_tensor(rng.uniform(-1, 1, (n, 2)).astype(np.float32))
        oa, ra, ta, _, _ = a.step(act)
        ob, rb, tb, _, _ = b.step(act)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(ta, tb)
    a.close()
    b.close()


def test_pool_checkpoint_after_refresh(d2):
    """a checkpoint taken after refresh_curriculum (envs on both pool halves) restores
    into a handle whose own pool is different -- the saved pool halves come with the checkpoint --
    and continues bit-identically; indices into a pool half that was never filled are refused."""
    from drone2d_amd._native import NativeError

    n, rng = 512, np.random.default_rng(13)
    a = d2.Drone2dVecEnv(n, seed=3, **_kw(n_steps=60))
    a.reset()
    for _ in range(70):
        a.step(torch.as_tensor(rng.uniform(-1, 1, (n, 2)).astype(np.float32)))
    a.refresh_curriculum(seed=77)
    for _ in range(20):  # some envs reset into the new half, others still run first-half episodes
        a.step(torch.as_tensor(rng.uniform(-1, 1, (n, 2)).astype(np.float32)))
    sd = a.state_dict()
    es = sd["env_scn"].cpu().numpy()
    assert (es < 16).any() and (es >= 16).any() and sd["pool"]["active_base"] == 16
    assert sd["pool"]["valid_mask"] == 3
    b = d2.Drone2dVecEnv(n, seed=999, **_kw(n_steps=60, curriculum_seed=6))  # its own, different pool
    with pytest.raises(NativeError, match="no scenarios"):  # b never filled its second half
        b.set_env_scenarios(torch.full((n,), 20, dtype=torch.int32))
    b.load_state_dict(sd)
    for _ in range(100):
        act = torch.as_tensor(rng.uniform(-1, 1, (n, 2)).astype(np.float32))
        oa, ra, ta, _, _ = a.step(act)
        ob, rb, tb, _, _ = b.step(act)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(ta, tb)
    np.testing.assert_array_equal(a.get_env_scenarios().cpu().numpy(), b.get_env_scenarios().cpu().numpy())
    a.close()
    b.close()


def test_rejected_scenarios_leave_handle_usable(d2):
    from drone2d_amd import abi
    from drone2d_amd._native import NativeError
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    import oracle
    from drone2d_amd.config import make_cfg

    kw = dict(ENV_TRAIN_CONFIG, scenario="corridor")
    n = 256
    venv = d2.Drone2dVecEnv(n, seed=4, **kw)
    orc = oracle.OracleBatch(make_cfg(dict(kw)), [s.to_c() for s in venv.scenarios], n)
    venv.reset()
    orc.reset(4)
    bad = venv.scenarios[0].to_c()
    bad.n_wps = abi.MAX_WPS + 1
    arr = (abi.D2DScn * 1)(bad)
    with pytest.raises(NativeError):
        from drone2d_amd._native import check

        check(venv._lib.d2d_set_scenarios(venv._h, arr, 1, None), "d2d_set_scenarios")
    rng = np.random.default_rng(2)
    for _ in range(30):  # still the old scenario, still in parity
        compare_step(venv, orc, rng.uniform(-1, 1, (n, 2)).astype(np.float32))
    venv.close()
