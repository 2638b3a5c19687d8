"""HIP kernel parity (through the C ABI via the ctypes binding) -- needs an MI355X.

1. teacher-forced one-step parity against the golden vectors recorded from the reference,
2. HIP vs CPU oracle over natural trajectories with auto-reset (teacher-forced every step),
3. free-running agreement over the first steps,
4. full-size (65 536 envs) size-independent properties: determinism, shard invariance, finiteness,
   mask-reset isolation, episode statistics = sum of per-episode info rows.
"""
import numpy as np
import pytest
import torch

from conftest import SCENARIOS, load_golden
from parity_util import OBS_ATOL, REW_ATOL, REW_RTOL, compare_step, make_pair

pytestmark = pytest.mark.gpu


def _cfgkw(scenario="corridor", **over):
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    return dict(ENV_TRAIN_CONFIG, scenario=scenario, **over)


@pytest.mark.parametrize("which", ["traj", "crafted"])
def test_golden_teacher_forced(d2, which):
    from drone2d_amd import abi

    g = load_golden(which)
    M = len(g["rew"])
    venv = d2.Drone2dVecEnv(M, env_scenario=g["scn"], auto_reset=False, **_cfgkw(SCENARIOS))
    venv.reset(seed=0)
    st = torch.as_tensor(np.ascontiguousarray(g["pre"].T))
    ist = torch.zeros(3, M, dtype=torch.int32)
    ist[0] = torch.as_tensor(g["pre_i"][:, 0])
    ist[1] = torch.as_tensor(g["pre_i"][:, 1] | (g["pre_i"][:, 2] << 1))
    venv.set_state(st, ist)
    obs, rew, term, trunc, info = venv.step(torch.as_tensor(g["act"]))
    obs, rew, term, info = obs.cpu().numpy(), rew.cpu().numpy(), term.cpu().numpy(), info.cpu().numpy()
    np.testing.assert_array_equal(term.astype(int), g["done"])
    assert not trunc.any()
    np.testing.assert_allclose(obs, g["obs"], rtol=0, atol=OBS_ATOL)
    np.testing.assert_allclose(rew, g["rew"], rtol=1e-5, atol=1e-4)
    st2, ist2 = venv.get_state()
    np.testing.assert_allclose(st2.cpu().numpy().T, g["post"], rtol=1e-9, atol=1e-9)
    np.testing.assert_array_equal(ist2[0].cpu().numpy(), g["post_i"][:, 0])
    np.testing.assert_array_equal(ist2[1].cpu().numpy(), g["post_i"][:, 1] | (g["post_i"][:, 2] << 1))
    gi = g["info"]
    np.testing.assert_array_equal(info[:, abi.INFO_COLL], gi[:, 4])
    np.testing.assert_array_equal(info[:, abi.INFO_REACH], gi[:, 5])
    np.testing.assert_allclose(info[:, abi.INFO_PP], gi[:, 3], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(info[:, abi.INFO_CA], gi[:, 1], rtol=1e-5, atol=1e-4)
    venv.close()


@pytest.mark.parametrize("scn,n", [("corridor", 2048), ("S_corridor", 2048), ("large", 2048), ("mixed", 2048),
                                   ("corridor_free", 4096), ("corridor", 1000)])
def test_vs_oracle_teacher_forced(d2, scn, n):
    """HIP vs oracle with auto-reset, teacher-forced every step.  corridor_free at 4 096 envs is
    BASELINE configs[1] (no obstacles: obs 8..16 = (1, 0, 0) x 3, CA = 0); 1 000 envs end in a
    40-env workgroup (the obs tile's partial store)."""
    scenarios = SCENARIOS if scn == "mixed" else [scn]
    venv, orc = make_pair(d2, n, scenarios, seed=99, kwargs=_cfgkw())
    rng = np.random.default_rng(1)
    dones = 0
    for t in range(160):
        act = np.clip(rng.normal(0.0, 0.6, (venv.num_envs, 2)), -1, 1).astype(np.float32)
        compare_step(venv, orc, act)
        dones += int(orc.term.sum())
        if scn.endswith("_free"):
            np.testing.assert_array_equal(orc.obs[:, 8:17], np.tile([1.0, 0.0, 0.0], 3)[None].repeat(n, 0))
    assert dones > 50  # auto-resets were exercised
    venv.close()


def test_balanced_mixed_layout_full_size(d2):
    """65 536 mixed envs (BASELINE configs[4] per GPU): the layout in use is the host's co-residency
    balanced renumbering for this device's CU count (d2d_balanced_group_layout), not the natural
    order, and the full batch steps in parity with the oracle on it (teacher-forced, auto-resets)."""
    import ctypes as C

    from drone2d_amd.config import SCENARIO_STEP_COST

    n = FULL
    venv, orc = make_pair(d2, n, SCENARIOS, seed=17, kwargs=_cfgkw())
    se, gs = venv.group_layout()
    es = np.ascontiguousarray(venv.env_scenario, np.int32)
    cost = np.array([SCENARIO_STEP_COST[x] for x in SCENARIOS], np.float64)
    ng = (n + 63) // 64
    se_h, gs_h, se_n, gs_n = np.zeros(ng * 64, np.int32), np.zeros(ng, np.int32), np.zeros(ng * 64, np.int32), \
        np.zeros(ng, np.int32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    lib = venv._lib
    assert lib.d2d_balanced_group_layout(n, p(es), len(SCENARIOS), p(cost), n_cu, p(se_h), p(gs_h)) == ng
    assert lib.d2d_group_layout(n, p(es), len(SCENARIOS), p(se_n), p(gs_n)) == ng
    assert (se == se_h).all() and (gs == gs_h).all()
    assert n_cu % 8 or not (se == se_n).all()
    rng = np.random.default_rng(5)
    for t in range(24):
        compare_step(venv, orc, np.clip(rng.normal(0.0, 0.6, (n, 2)), -1, 1).astype(np.float32))
    venv.close()


def test_grouped_lane_map_irregular(d2):
    """Static mixed env -> scenario map with ragged groups: the step kernel's scenario-grouped lane
    map (partial groups padded, a scenario with 3 envs, one with none, n not a multiple of 64)."""
    rng = np.random.default_rng(7)
    n = 1001
    es = rng.choice(7, size=n, p=[0.3, 0.25, 0.2, 0.15, 0.1, 0.0, 0.0]).astype(np.int32)
    es[[5, 500, 1000]] = 5  # three envs of scenario 5, none of scenario 6
    venv, orc = make_pair(d2, n, SCENARIOS, seed=3, kwargs=_cfgkw(), env_scenario=es)
    dones = 0
    for t in range(120):
        act = np.clip(rng.normal(0.0, 0.6, (n, 2)), -1, 1).astype(np.float32)
        compare_step(venv, orc, act)
        dones += int(orc.term.sum())
    assert dones > 20
    venv.close()


def test_layout_change_keeps_state(d2):
    """d2d_set_scenarios with a new env -> scenario map moves the running state into the new slot
    layout (grouped -> regrouped -> identity): get_state in env order and the episode statistics are
    unchanged, and stepping continues in parity with the oracle."""
    rng = np.random.default_rng(9)
    n = 777
    es = rng.integers(0, 7, n).astype(np.int32)
    venv, orc = make_pair(d2, n, SCENARIOS, seed=4, kwargs=_cfgkw(), env_scenario=es)
    for _ in range(40):
        compare_step(venv, orc, np.clip(rng.normal(0.0, 0.6, (n, 2)), -1, 1).astype(np.float32))
    st0, ist0 = (x.cpu().numpy() for x in venv.get_state())
    stats0 = venv.episode_stats(clear=False).cpu().numpy()
    for new_map in (rng.permutation(es), np.zeros(n, np.int32), es):
        venv._upload_scenarios(new_map)
        st1, ist1 = (x.cpu().numpy() for x in venv.get_state())
        np.testing.assert_array_equal(st1, st0)
        np.testing.assert_array_equal(ist1, ist0)
        np.testing.assert_allclose(venv.episode_stats(clear=False).cpu().numpy(), stats0, rtol=1e-12)
    # back on the original map: keeps stepping in parity (the reset cache was dropped and refilled)
    for _ in range(30):
        compare_step(venv, orc, np.clip(rng.normal(0.0, 0.6, (n, 2)), -1, 1).astype(np.float32))
    venv.close()


def test_reset_cache_invalidation(d2):
    """The auto-reset observation cache (filled ahead of time by the fill kernel) must be dropped
    by a full reset with a new seed and by set_state (episode counters may change)."""
    venv, orc = make_pair(d2, 2048, ["corridor"], seed=99, kwargs=_cfgkw())
    rng = np.random.default_rng(4)

    def run(steps):
        d = 0
        for _t in range(steps):
            act = np.clip(rng.normal(0.0, 0.6, (venv.num_envs, 2)), -1, 1).astype(np.float32)
            compare_step(venv, orc, act)
            d += int(orc.term.sum())
        return d

    assert run(60) > 0
    obs_g = venv.reset(seed=123).cpu().numpy()
    obs_o = orc.reset(123)
    np.testing.assert_allclose(obs_g, obs_o, rtol=0, atol=OBS_ATOL)
    assert run(100) > 20
    st, ist = venv.get_state()
    ist[2] += 5  # jump every episode counter: cached spawns are stale
    venv.set_state(st, ist)
    orc.set_state(st.cpu().numpy(), ist.cpu().numpy())
    assert run(100) > 20
    venv.close()


@pytest.mark.parametrize("stage", ["stage_2", "stage_3", "stage_5"])
def test_curriculum_pool_vs_oracle(d2, stage):
    """Curriculum mode: every reset draws the env's next scenario from the pool on device; the
    oracle makes the same draws (teacher-forced over many auto-resets)."""
    import oracle
    from drone2d_amd.config import make_cfg

    kw = _cfgkw(stage, mode="curriculum", curriculum_pool=64, curriculum_seed=2)
    n = 2048
    venv = d2.Drone2dVecEnv(n, seed=17, **kw)
    assert venv.cfg.scn_pool == 1 and len(venv.scenarios) == 64
    cfg = make_cfg(dict(kw))
    cfg.scn_pool = 1
    orc = oracle.OracleBatch(cfg, [s.to_c() for s in venv.scenarios], n, env_scenario=venv.env_scenario)
    np.testing.assert_allclose(venv.reset().cpu().numpy(), orc.reset(17), rtol=0, atol=OBS_ATOL)
    rng = np.random.default_rng(6)
    dones = 0
    for t in range(120):
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        compare_step(venv, orc, act)
        dones += int(orc.term.sum())
    assert dones > 200
    venv.close()


def test_reset_cache_short_episodes(d2):
    """Episodes shorter than the cache fill: a mix of cached and synchronous reset observations."""
    venv, orc = make_pair(d2, 1024, SCENARIOS, seed=8, kwargs=_cfgkw(n_steps=3))
    rng = np.random.default_rng(5)
    dones = 0
    for t in range(30):
        act = rng.uniform(-1, 1, (venv.num_envs, 2)).astype(np.float32)
        compare_step(venv, orc, act)
        dones += int(orc.term.sum())
    assert dones >= 9 * 1000
    venv.close()


def test_free_running_agreement(d2):
    """No teacher forcing: both batches evolve independently from the same reset."""
    venv, orc = make_pair(d2, 1024, SCENARIOS, seed=5, kwargs=_cfgkw())
    rng = np.random.default_rng(2)
    for t in range(60):
        act = rng.uniform(-1, 1, (venv.num_envs, 2)).astype(np.float32)
        compare_step(venv, orc, act, teacher_force=False, check_state=False)
    venv.close()


def test_edge_actions(d2):
    """Unclipped / extreme actions (the env does not clip, drone_2d_env.py:400-401)."""
    venv, orc = make_pair(d2, 512, SCENARIOS, seed=3, kwargs=_cfgkw())
    vals = np.array([-1, 1, 0, -3.5, 2.25, 1e-30, -0.0], np.float32)
    rng = np.random.default_rng(3)
    for t in range(20):
        act = rng.choice(vals, (venv.num_envs, 2)).astype(np.float32)
        compare_step(venv, orc, act)
    venv.close()


def test_timeup_and_truncation_option(d2):
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    kw = dict(ENV_TRAIN_CONFIG, n_steps=5, scenario="large_free")
    for trunc_mode in (False, True):
        venv = d2.Drone2dVecEnv(64, timeup_truncates=trunc_mode, **kw)
        venv.reset(seed=0)
        hover = torch.zeros(64, 2, device=venv.device)
        for t in range(5):
            obs, rew, term, trunc, info = venv.step(hover)
        # all hovering envs end at t == n_steps (end_cond_4)
        if trunc_mode:
            assert trunc.all() and not term.any()
        else:
            assert term.all() and not trunc.any()
        assert torch.all(info[:, 7] == 5) and torch.all(info[:, 8] == 4)
        venv.close()


FULL = 65536


def _rollout(d2, n, seed, steps, scn="corridor", offset=0, env_scenario=None):
    venv = d2.Drone2dVecEnv(n, seed=seed, env_id_offset=offset, env_scenario=env_scenario, **_cfgkw(scn))
    obs0 = venv.reset().clone()
    g = torch.Generator(device="cpu").manual_seed(7)
    acts = (torch.rand(steps, FULL, 2, generator=g) * 2 - 1)[:, offset:offset + n].contiguous()
    outs = []
    for t in range(steps):
        obs, rew, term, trunc, info = venv.step(acts[t].to(venv.device))
        outs.append((obs.clone(), rew.clone(), term.clone()))
    st, ist = venv.get_state()
    stats = venv.episode_stats().clone()
    venv.close()
    return obs0, outs, st, ist, stats


def test_full_size_determinism_and_shard_invariance(d2):
    a = _rollout(d2, FULL, 11, 30)
    b = _rollout(d2, FULL, 11, 30)
    for (oa, ra, ta), (ob, rb, tb) in zip(a[1], b[1]):
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(ta, tb)
    assert torch.equal(a[2], b[2]) and torch.equal(a[4], b[4])
    # two shards with global env ids reproduce the single batch bit for bit
    h = FULL // 2
    s0 = _rollout(d2, h, 11, 30, offset=0)
    s1 = _rollout(d2, h, 11, 30, offset=h)
    for t in range(30):
        assert torch.equal(torch.cat([s0[1][t][0], s1[1][t][0]]), a[1][t][0])
        assert torch.equal(torch.cat([s0[1][t][1], s1[1][t][1]]), a[1][t][1])
    assert torch.equal(torch.cat([s0[2], s1[2]], 1), a[2])


@pytest.mark.parametrize("scn,n", [("corridor", FULL), ("large", FULL), ("S_corridor", FULL),
                                   ("corridor_free", 4096)])
def test_full_size_properties(d2, scn, n):
    """BASELINE sizes: 65 536 envs (configs[2], [3]) and configs[1]'s 4 096 obstacle-free envs."""
    obs0, outs, st, ist, stats = _rollout(d2, n, 3, 60, scn=scn)
    assert torch.isfinite(obs0).all()
    n_done = 0
    free = torch.tensor([1.0, 0.0, 0.0] * 3, device=obs0.device)
    for obs, rew, term in outs:
        assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
        if scn.endswith("_free"):  # no obstacles: the unfilled sensor slots (drone_2d_env.py:660-720)
            assert torch.equal(obs[:, 8:17], free.expand(n, 9))
        # sin/cos slots are in [-1, 1]; distance slots are 2d/diag - 1 >= -1 - r/diag
        sc = obs[:, [9, 10, 12, 13, 15, 16, 17, 18, 23, 24, 25, 26]]
        assert (sc.abs() <= 1.0 + 1e-6).all()
        n_done += int(term.sum())
    assert torch.isfinite(st).all()
    assert (ist[0] >= 0).all() and (ist[0] <= 1100).all()
    assert stats[1].item() == n_done  # every finished episode is counted once
    assert stats[2] + stats[3] >= stats[1]  # success or fail (both when reach + collide)


def test_reset_mask_isolation(d2):
    venv = d2.Drone2dVecEnv(4096, **_cfgkw(SCENARIOS))
    venv.reset(seed=1)
    for _ in range(5):
        venv.step(torch.rand(4096, 2, device=venv.device) * 2 - 1)
    st0, ist0 = venv.get_state()
    mask = torch.zeros(4096, dtype=torch.bool, device=venv.device)
    mask[::3] = True
    venv.reset(mask=mask)
    st1, ist1 = venv.get_state()
    keep = ~mask
    assert torch.equal(st0[:, keep], st1[:, keep]) and torch.equal(ist0[:, keep], ist1[:, keep])
    assert (ist1[0, mask] == 0).all() and (ist1[2, mask] == ist0[2, mask] + 1).all()
    venv.close()


def test_episode_stats_match_info_rows(d2):
    venv = d2.Drone2dVecEnv(8192, seed=4, **_cfgkw(SCENARIOS))
    venv.reset()
    ret = n = succ = ape = ln = 0.0
    for t in range(200):
        obs, rew, term, trunc, info = venv.step(torch.rand(8192, 2, device=venv.device) * 2 - 1)
        d = term | trunc
        if d.any():
            i = info[d].double()
            ret += i[:, 10].sum().item()
            n += d.sum().item()
            succ += ((i[:, 8].long() & 2) > 0).sum().item()
            ape += i[:, 9].sum().item()
            ln += i[:, 7].sum().item()
    s = venv.episode_stats().cpu().numpy()
    assert s[1] == n and s[2] == succ and s[6] == ln
    np.testing.assert_allclose(s[0], ret, rtol=1e-5, atol=1e-2)
    np.testing.assert_allclose(s[5], ape, rtol=1e-5)
    assert venv.episode_stats()[1].item() == 0  # cleared
    venv.close()


def test_single_env_api(d2):
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    env = d2.Drone2dEnv(**dict(ENV_TRAIN_CONFIG, scenario="corridor", render_path=True))
    obs = env.reset()
    assert obs.shape == (27,) and obs.dtype == np.float64
    done, steps = False, 0
    while not done and steps < 2000:
        obs, r, done, info = env.step([1.0, -1.0])  # spin -> AA termination
        steps += 1
    assert done and isinstance(r, float)
    for k in ("reward", "collision_avoidance_reward", "path_adherence", "path_progression", "collision_reward",
              "reach_end_reward", "agressive_alpha_reward", "env_steps", "dist_closest_obs", "APE",
              "n_collisions", "n_successful_runs", "n_failed_runs", "total_reward", "flight_path"):
        assert k in info
    assert info["n_failed_runs"] == 1 and len(info["flight_path"]) == steps
    _, _, done2, _ = env.step([0.0, 0.0])
    assert done2  # done is sticky until reset (drone_2d_env.py:594)
    env.close()


def test_step_accepts_every_action_form(d2):
    """``step()`` takes the fast host path for float32 contiguous device tensors of shape [N, 2] and
    converts everything else (numpy float64, CPU tensors, float64 / non-contiguous / flat device
    tensors): both paths give bit-identical steps, and each step writes the other output buffer."""
    n = 1000
    kw = _cfgkw()
    va = d2.Drone2dVecEnv(n, seed=21, **kw)
    vb = d2.Drone2dVecEnv(n, seed=21, **kw)
    va.reset()
    vb.reset()
    g = torch.Generator(device="cuda").manual_seed(3)
    forms = [lambda a: a.cpu().numpy().astype(np.float64), lambda a: a.cpu(), lambda a: a.double(),
             lambda a: a.t().contiguous().t(), lambda a: a.reshape(-1), lambda a: a.cpu().numpy().tolist()]
    prev = None
    for k in range(60):
        act = torch.rand(n, 2, device="cuda", generator=g) * 2 - 1
        oa, ra, ta, ua, ia = va.step(act)
        ob, rb, tb, ub, ib = vb.step(forms[k % len(forms)](act))
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(ta, tb) and torch.equal(ua, ub)
        assert torch.equal(ia, ib) and torch.equal(va.terminal_obs, vb.terminal_obs)
        if prev is not None:
            assert oa.data_ptr() != prev  # double-buffered outputs
        prev = oa.data_ptr()
    with pytest.raises(RuntimeError):
        va.step(torch.zeros(n + 1, 2, device="cuda"))  # wrong size: refused, not read past the end
    va.close()
    vb.close()


@pytest.mark.parametrize("which", [0, 1, 2])
def test_device_math_selftest(d2, which):
    """The kernels' shortcut fp64 routines (range-limited sqrt and division, division by a
    precomputed reciprocal) are bitwise equal to the IEEE operations on 2^26 random operands."""
    import ctypes as C

    from drone2d_amd import _native

    lib = _native.load()
    bad = C.c_uint64(123)
    assert lib.d2d_selftest(which, 1 << 26, 2024 + which, C.byref(bad)) == 0
    assert bad.value == 0


@pytest.mark.parametrize("per,gn", [(8192, 64), (512, 16)])
def test_closest_point_grid_bitwise(d2, per, gn):
    """Brent closest-point search over the whole plane and around every path, all 7 scenarios:
    the golden-march tables (golden-left / golden-right prefixes, resume at the first differing
    step) must give exactly the probe sequence of the plain search, so the closest / lookahead
    points (obs 19..22) and the accumulated path error are bit-identical to the C oracle (grouped
    layout: every 64-env group stages its scenario and probe table).  per = 512 (56 workgroups, fewer
    than CUs): the small-batch launch, whose continuation runs speculatively (brent_run_spec)."""
    from drone2d_amd import abi

    n = per * len(SCENARIOS)
    venv, orc = make_pair(d2, n, SCENARIOS, seed=5, kwargs=_cfgkw(), env_scenario=np.repeat(np.arange(7), per),
                          auto_reset=False)
    rng = np.random.default_rng(11)
    pts = []
    for s in venv.scenarios:
        g = np.linspace(-600.0, 1900.0, gn)
        grid = np.stack(np.meshgrid(g, g), -1).reshape(-1, 2)  # gn^2: behind, beyond, around the path
        L = float(s.path.us[-1])
        u = rng.uniform(-10.0, L + 10.0, per - len(grid))
        near = np.array([s.path(x) for x in u]) + rng.normal(0.0, 40.0, (len(u), 2))  # parabolic searches
        pts.append(np.concatenate([grid, near]))
    pts = np.concatenate(pts)
    st = np.zeros((abi.NSTATE, n))
    st[0], st[1] = pts[:, 0], pts[:, 1]
    st[6], st[7] = pts[:, 0] - 40.0, pts[:, 1]   # motors at frame -+ 40 (theta = 0, Drone.py:37,51)
    st[12], st[13] = pts[:, 0] + 40.0, pts[:, 1]
    ist = np.zeros((abi.NISTATE, n), np.int32)
    venv.set_state(torch.as_tensor(st), torch.as_tensor(ist))
    orc.set_state(st, ist)
    act = np.zeros((n, 2), np.float32)
    obs, rew, term, trunc, info = (x.cpu().numpy() for x in venv.step(torch.as_tensor(act, device=venv.device)))
    o_obs, o_rew, _, _, _ = orc.step(act)
    np.testing.assert_array_equal(obs[:, 19:23], o_obs[:, 19:23])
    np.testing.assert_allclose(obs, o_obs, rtol=0, atol=OBS_ATOL)
    st2 = venv.get_state()[0].cpu().numpy()
    o_st2 = orc.get_state()[0]
    np.testing.assert_array_equal(st2[abi.S_PATH_ERR], o_st2[abi.S_PATH_ERR])
    venv.close()


@pytest.mark.parametrize("radii", ["uniform", "mixed"])
def test_sensing_ties_and_radii(d2, radii):
    """Nearest-circle sensing: circles placed in mirror pairs (and a quad) around x = 600, frames on
    the mirror axis, so pairs of circles are exactly equidistant -- the squared-distance top-3 must
    fall back to the reference's index order on equal distances; with mixed radii the reference
    loop runs throughout.  HIP vs the oracle, teacher-forced."""
    import oracle
    from drone2d_amd.config import make_cfg
    from drone2d_amd.scenarios import Scenario

    base = d2.Drone2dVecEnv(1, **_cfgkw("corridor")).scenarios[0]
    cs = [(500.0, 600.0), (700.0, 600.0), (500.0, 800.0), (700.0, 800.0), (600.0, 400.0), (450.0, 700.0),
          (750.0, 700.0), (600.0, 1000.0)]
    r = [30.0] * len(cs) if radii == "uniform" else [30.0, 30.0, 25.0, 35.0, 30.0, 20.0, 20.0, 40.0]
    circ = np.array([(x, y, rr) for (x, y), rr in zip(cs, r)])
    scn = Scenario("mirror", base.wps, base.path, circ, (590.0, 610.0, 550.0, 850.0), base.spawn_angle)
    n = 512
    kw = dict(_cfgkw(), scenario=[scn])
    venv = d2.Drone2dVecEnv(n, seed=5, auto_reset=False, **kw)
    orc = oracle.OracleBatch(make_cfg(dict(kw), auto_reset=False), [scn.to_c()], n)
    venv.reset()
    orc.reset(5)
    st, ist = (x.cpu().numpy() for x in venv.get_state())
    rng = np.random.default_rng(3)
    st[0] = 600.0                                   # frame exactly on the mirror axis
    st[1] = rng.uniform(450.0, 950.0, n)
    st[1][:64] = 700.0                              # ... and on the horizontal mirror line
    st[2] = rng.uniform(-0.3, 0.3, n)
    for f in (3, 4, 5, 9, 10, 11, 15, 16, 17):
        st[f] = 0.0
    c, s_ = np.cos(st[2]), np.sin(st[2])
    st[6], st[7], st[8] = 600.0 - 40 * c, st[1] - 40 * s_, st[2]
    st[12], st[13], st[14] = 600.0 + 40 * c, st[1] + 40 * s_, st[2]
    venv.set_state(torch.as_tensor(st), torch.as_tensor(ist))
    act = np.zeros((n, 2), np.float32)              # hover-ish: positions barely move
    worst = compare_step(venv, orc, act)
    assert worst < OBS_ATOL
    venv.close()


def test_config5_size_on_one_gpu_windows(d2):
    """BASELINE configs[4]'s whole 524 288-env mixed batch (8 x 65 536, env i on scenario i mod 7)
    in ONE handle: 8 192 workgroups, i.e. eight rounds of the one-round 65 536-env launch.  Three
    windows (the first envs, an unaligned middle span, the last envs) are checked against oracle
    batches keyed by the same global env ids, teacher-forced every step with auto-reset on."""
    import oracle
    from drone2d_amd import shard
    from drone2d_amd.config import make_cfg

    n = 8 * FULL
    kw = _cfgkw(SCENARIOS)
    venv = shard.make_shard_venv(n, 0, 1, seed=21, **kw)
    obs = venv.reset().clone()
    m = 384
    wins = [0, n // 2 + 37, n - m]
    orcs = []
    for o in wins:
        cfg = make_cfg(dict(kw), auto_reset=True, env_id_base=o)
        orc = oracle.OracleBatch(cfg, [s.to_c() for s in venv.scenarios], m,
                                 env_scenario=venv.env_scenario[o:o + m])
        np.testing.assert_allclose(obs[o:o + m].cpu().numpy(), orc.reset(21), atol=OBS_ATOL)
        orcs.append(orc)
    rng = np.random.default_rng(5)
    dones = 0
    for t in range(40):
        st, ist = venv.get_state()
        for o, orc in zip(wins, orcs):
            orc.set_state(st[:, o:o + m].cpu().numpy().copy(), ist[:, o:o + m].cpu().numpy().copy())
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        obs, rew, term, trunc, info = venv.step(torch.as_tensor(act, device=venv.device))
        assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
        for o, orc in zip(wins, orcs):
            o_obs, o_rew, o_term, _, _ = orc.step(act[o:o + m])
            np.testing.assert_array_equal(term[o:o + m].cpu().numpy(), o_term)
            np.testing.assert_allclose(rew[o:o + m].cpu().numpy(), o_rew, rtol=REW_RTOL, atol=REW_ATOL)
            np.testing.assert_allclose(obs[o:o + m].cpu().numpy(), o_obs, rtol=0, atol=OBS_ATOL)
            dones += int(o_term.sum())
        if t == 0:
            assert not term.all()
    stats = venv.episode_stats()
    assert torch.isfinite(stats).all() and stats[1] > 0
    venv.close()


@pytest.mark.parametrize("scn", ["corridor", "large", "S_corridor"])
def test_bench_launch_windows(d2, scn):
    """The exact launch ``bench.py`` times (BASELINE configs[2] / [3], and S_corridor as the
    maximum-obstacle case): 65 536 envs of one scenario built as bench.py builds them
    (``make_shard_venv``, info rows off), i.e. the ungrouped ``d2d_step_kernel`` with the scenario and
    its golden-march tables staged in LDS, 1 024 workgroups, the three-way re-check off (more
    workgroups than CUs).  After 64 untested steps (the bench's steady-state mix of episode ages,
    reset-cache fills included), three windows of 384 envs (the first, an unaligned middle span, the
    last) are compared with oracle batches keyed by the same global env ids, teacher-forced every step
    for 40 steps with auto-reset on (drone_2d_env.py:394-615)."""
    import oracle
    from drone2d_amd import shard
    from drone2d_amd.config import make_cfg

    n = FULL
    kw = _cfgkw(scn)
    venv = shard.make_shard_venv(n, 0, 1, seed=12345, with_info=False, **kw)
    assert venv.group_layout() is None  # identity slot layout: the ungrouped kernel
    venv.reset()
    g = torch.Generator(device=venv.device).manual_seed(1000)
    for k in range(64):
        venv.step(torch.rand(n, 2, device=venv.device, generator=g) * 2 - 1)
    m = 384
    wins = [0, n // 2 + 37, n - m]
    cfg_for = lambda o: make_cfg(dict(kw), auto_reset=True, env_id_base=o)  # noqa: E731
    orcs = [oracle.OracleBatch(cfg_for(o), [s.to_c() for s in venv.scenarios], m) for o in wins]
    for o, orc in zip(wins, orcs):
        orc.reset(12345)
    rng = np.random.default_rng(8)
    dones = 0
    for t in range(40):
        st, ist = (x.cpu().numpy() for x in venv.get_state())
        for o, orc in zip(wins, orcs):
            orc.set_state(st[:, o:o + m].copy(), ist[:, o:o + m].copy())
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        obs, rew, term, trunc, _ = venv.step(torch.as_tensor(act, device=venv.device))
        obs, rew, term = obs.cpu().numpy(), rew.cpu().numpy(), term.cpu().numpy()
        assert np.isfinite(obs).all() and np.isfinite(rew).all()
        for o, orc in zip(wins, orcs):
            o_obs, o_rew, o_term, _, _ = orc.step(act[o:o + m])
            np.testing.assert_array_equal(term[o:o + m], o_term)
            np.testing.assert_allclose(rew[o:o + m], o_rew, rtol=REW_RTOL, atol=REW_ATOL)
            np.testing.assert_allclose(obs[o:o + m], o_obs, rtol=0, atol=OBS_ATOL)
            dones += int(o_term.sum())
    st2 = venv.get_state()[0].cpu().numpy()
    for o, orc in zip(wins, orcs):
        np.testing.assert_allclose(st2[:, o:o + m], orc.get_state()[0], rtol=1e-9, atol=1e-9)
    assert dones > 0  # auto-resets happened inside the windows
    venv.close()
