"""Fresh curriculum (cfg.scn_pool = 2): every curriculum episode runs on a scenario the device
generates for it (csrc/d2d_curriculum.h), as the reference's curriculum reset does
(drone_2d_env.py:199-215, 318-372) -- needs an MI355X.

* the device's scenario slots are bit-identical to the CPU oracle's restatement of the generator,
  and stepping is in parity with the oracle, teacher-forced, across many auto-resets and a stage
  change of the sim_num schedule;
* the stage follows the schedule through 700 k / 1 M / 1.6 M / 2 M with no host call but ``step``,
  and every episode gets its own scenario (distinct scenarios per n_steps steps >= num_envs);
* a checkpoint (slot recipes + state) restores into a new handle bit-identically.
"""
import numpy as np
import pytest
import torch

from parity_util import OBS_ATOL, compare_step

pytestmark = pytest.mark.gpu

FIELDS = ("n_wps", "n_circles", "us", "xa", "xb", "xc", "ya", "yb", "yc", "cx", "cy", "cr", "wp_last_x",
          "wp_last_y", "spawn_xmin", "spawn_xmax", "spawn_ymin", "spawn_ymax", "spawn_amin", "spawn_amax")


def _kw(**over):
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    return dict(ENV_TRAIN_CONFIG, mode="curriculum", scenario="curriculum", **over)


def _pair(d2, n, seed, kw):
    import oracle
    from drone2d_amd.config import make_cfg
    from drone2d_amd.env import make_curriculum

    venv = d2.Drone2dVecEnv(n, seed=seed, **kw)
    assert venv.cfg.scn_pool == 2 and venv.fresh
    cfg = make_cfg(dict(kw))
    cfg.scn_pool = 2
    orc = oracle.OracleBatch(cfg, [], n, curriculum=make_curriculum(kw, n))
    np.testing.assert_allclose(venv.reset().cpu().numpy(), orc.reset(seed), rtol=0, atol=OBS_ATOL)
    return venv, orc


def _tables_equal(venv, orc):
    n2 = 2 * venv.num_envs
    g, o = venv.scenario_table(0, n2), orc.scenario_table(0, n2)
    assert bytes(g) == bytes(o) or _diff(g, o)
    kg, cg, tg = venv.fresh_recipes()
    ko, co, to = orc.fresh_recipes()
    np.testing.assert_array_equal(kg, ko)
    np.testing.assert_array_equal(cg, co)
    assert tg == to


def _diff(g, o):
    for s in range(len(g)):
        for f in FIELDS:
            a, b = getattr(g[s], f), getattr(o[s], f)
            a = np.array(a[:] if hasattr(a, "__len__") else a)
            b = np.array(b[:] if hasattr(b, "__len__") else b)
            assert np.array_equal(a, b), (s, f, a, b)
    return True


def test_fresh_generator_bitwise_and_step_parity(d2):
    n, rng = 2048, np.random.default_rng(3)
    # sim_num = 1.95e6 + 2048 / step: stage 4 (on-path obstacles) -> stage 5 after 25 steps
    venv, orc = _pair(d2, n, 17, _kw(sim_num=1950000))
    _tables_equal(venv, orc)
    dones = 0
    for t in range(120):
        compare_step(venv, orc, rng.uniform(-1, 1, (n, 2)).astype(np.float32))
        dones += int(orc.term.sum())
        if t % 20 == 19:
            _tables_equal(venv, orc)
            np.testing.assert_array_equal(venv.get_env_scenarios().cpu().numpy(), 2 * np.arange(n) +
                                          ((venv.get_state()[1][2].cpu().numpy() - 1) & 1))
    assert dones > 300
    venv.close()


def _stage_of(sim):
    return 1 if sim <= 7e5 else 2 if sim <= 1e6 else 3 if sim <= 1.6e6 else 4 if sim <= 2e6 else 5


def test_fresh_stage_schedule_on_device(d2):
    """Only ``step`` is called: the device clock moves sim_num = steps x 4096 through every stage."""
    n, rng = 4096, np.random.default_rng(4)
    venv = d2.Drone2dVecEnv(n, seed=5, **_kw(sim_num=0))
    venv.reset()
    ep0 = venv.get_state()[1][2].clone()
    stages_seen = set()
    for t in range(1, 601):
        venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
        if t % 60 == 0:
            keys, clocks, clock = venv.fresh_recipes()
            assert clock == t
            tab = venv.scenario_table(0, 2 * n)
            for s in np.flatnonzero(keys >= 0)[::7]:
                st = _stage_of(float(clocks[s]) * n)
                stages_seen.add(st)
                sc = tab[s]
                box = (sc.spawn_xmin, sc.spawn_xmax, sc.spawn_ymin, sc.spawn_ymax) == (100.0, 1200.0, 100.0, 1200.0)
                assert box == (st == 2), (s, st)
                if st <= 2:
                    assert sc.n_circles == 0
                if st in (3, 4):
                    assert sc.n_circles <= 1
                if st != 2:
                    assert sc.spawn_xmin == sc.spawn_xmax  # spawn at the first waypoint
        if t == 540:  # every env started >= 1 episode in the last n_steps steps; each on its own path
            started = int((venv.get_state()[1][2] - ep0).sum())
            assert started >= n
    assert stages_seen == {1, 2, 3, 4, 5}
    tab = venv.scenario_table(0, 2 * n)
    keys = venv.fresh_recipes()[0]
    paths = {(round(tab[s].wp_last_x, 9), round(tab[s].wp_last_y, 9)) for s in np.flatnonzero(keys >= 0)}
    assert len(paths) == int((keys >= 0).sum())
    venv.close()


def test_fresh_checkpoint_restore(d2):
    n, rng = 1024, np.random.default_rng(6)
    kw = _kw(sim_num=2500000)
    a = d2.Drone2dVecEnv(n, seed=8, **kw)
    a.reset()
    for _ in range(80):
        a.step(torch.as_tensor(rng.uniform(-1, 1, (n, 2)).astype(np.float32)))
    sd = a.state_dict()
    b = d2.Drone2dVecEnv(n, seed=1, **kw)
    b.load_state_dict(sd)
    assert bytes(a.scenario_table()) == bytes(b.scenario_table())
    for _ in range(100):
        act = torch.as_tensor(rng.uniform(-1, 1, (n, 2)).astype(np.float32))
        oa, ra, ta, _, _ = a.step(act)
        ob, rb, tb, _, _ = b.step(act)
        assert torch.equal(oa, ob) and torch.equal(ra, rb) and torch.equal(ta, tb)
    a.close()
    b.close()


def test_set_curriculum_restarts_schedule(d2):
    """set_curriculum(sim_num=X) on an env that has stepped starts the schedule at X
    (the step clock is zeroed), so the next episodes are generated in X's stage."""
    n = 1024
    venv = d2.Drone2dVecEnv(n, seed=5, **_kw(sim_num=0))
    venv.reset()
    for _ in range(50):
        venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
    assert venv.fresh_recipes()[2] == 50
    venv.set_curriculum(sim_num=1_200_000)  # stage 3: one on-path obstacle, spawn at the first waypoint
    keys, clocks, clock = venv.fresh_recipes()
    assert clock == 0
    tab = venv.scenario_table(0, 2 * n)
    for s in np.flatnonzero(keys >= 0):
        assert clocks[s] == 0
        assert tab[s].n_circles <= 1 and tab[s].spawn_xmin == tab[s].spawn_xmax
    for _ in range(7):
        venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
    assert venv.fresh_recipes()[2] == 7
    venv.set_curriculum(sim_num=800_000)  # stage 2: the random spawn box, no obstacles
    keys, _, clock = venv.fresh_recipes()
    assert clock == 0
    tab = venv.scenario_table(0, 2 * n)
    for s in np.flatnonzero(keys >= 0):
        sc = tab[s]
        assert sc.n_circles == 0 and (sc.spawn_xmin, sc.spawn_xmax) == (100.0, 1200.0)
    venv.close()


def test_set_curriculum_seed_only_keeps_progress(d2):
    """set_curriculum(seed=...) alone on a fresh env carries the schedule's progress (the
    library zeroes its clock, the wrapper moves it into sim_num0): 690 000 + 50 x 1 024 = 741 200 is
    stage 2 (the random spawn box), where restarting at 690 000 would be stage 1."""
    n = 1024
    venv = d2.Drone2dVecEnv(n, seed=5, **_kw(sim_num=690000))
    venv.reset()
    for _ in range(50):
        venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
    venv.set_curriculum(seed=7)
    assert venv.kwargs["sim_num"] == 690000 + 50 * n
    keys, _, clock = venv.fresh_recipes()
    assert clock == 0
    tab = venv.scenario_table(0, 2 * n)
    for s in np.flatnonzero(keys >= 0):
        assert (tab[s].spawn_xmin, tab[s].spawn_xmax) == (100.0, 1200.0), s
    venv.close()


def test_set_curriculum_keeps_progress_non_stage_scenario(d2):
    """mode='curriculum' with a non-stage scenario (the reference's default train config,
    scenario='large') follows the sim_num schedule too (drone_2d_env.py:324-334), so set_curriculum()
    with neither stage nor sim_num carries the clock's progress into sim_num0 as well."""
    n = 1024
    venv = d2.Drone2dVecEnv(n, seed=5, **dict(_kw(sim_num=690000), scenario="large"))
    assert venv.fresh and venv.curriculum.stage == 0  # the schedule picks the stage
    venv.reset()
    for _ in range(50):
        venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
    venv.set_curriculum(seed=7)
    assert venv.kwargs["sim_num"] == 690000 + 50 * n
    keys, _, clock = venv.fresh_recipes()
    assert clock == 0
    tab = venv.scenario_table(0, 2 * n)
    for s in np.flatnonzero(keys >= 0):
        assert (tab[s].spawn_xmin, tab[s].spawn_xmax) == (100.0, 1200.0), s
    venv.set_curriculum()  # neither given again: still no restart of the schedule
    assert venv.kwargs["sim_num"] == 690000 + 50 * n
    venv.close()


def test_masked_fresh_reset_keeps_seed(d2):
    """a masked fresh reset with a new seed is refused (the envs it leaves running would
    keep old-seed scenarios that no checkpoint recipe regenerates); with the same seed it works."""
    n = 256
    venv = d2.Drone2dVecEnv(n, seed=5, **_kw(sim_num=0))
    venv.reset()
    for _ in range(5):
        venv.step(torch.rand(n, 2, device=venv.device) * 2 - 1)
    mask = torch.zeros(n, dtype=torch.bool, device=venv.device)
    mask[::3] = True
    with pytest.raises(RuntimeError, match="masked reset"):
        venv.reset(seed=99, mask=mask)
    assert venv.seed_value == 5  # the refused seed is not installed: state_dict() saves 5
    assert venv.state_dict()["seed"] == 5
    venv.reset(mask=mask)
    keys = venv.fresh_recipes()[0]
    ep = venv.get_state()[1][2].cpu().numpy()
    for i in range(n):  # every env's current slot stays tagged with its episode (checkpointable)
        assert keys[2 * i + ((ep[i] - 1) & 1)] == ep[i] - 1, i
    venv.close()


def test_fresh_graph_replay_keeps_every_slot(d2):
    """The fresh curriculum inside a captured HIP graph with other kernels between the steps (as PPO's
    rollout graph has them): after every replay each env's running and next slots hold its current
    and next episode's scenario (the slot ring K1 fills and K5 drains lost nothing, also after its
    indices wrapped: more than 2 n appends, FreshRing in d2d_kernels.h), and a handle restored from the
    recipes regenerates the same tables byte for byte."""
    n = 4096
    venv = d2.Drone2dVecEnv(n, seed=3, **_kw(sim_num=1950000))  # stage 4 -> 5 during the replays
    venv.reset()
    g = torch.Generator(device=venv.device).manual_seed(1)
    bank = [torch.rand(n, 2, device=venv.device, generator=g) * 2 - 1 for _ in range(16)]
    act = torch.empty(n, 2, device=venv.device)
    acc = torch.zeros((), dtype=torch.float64, device=venv.device)
    for k in range(16):
        venv.step(bank[k])
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for k in range(16):
            act.copy_(bank[k])
            _, rew, _, _, _ = venv.step(act)
            acc += rew.double().sum()
    dones = 0
    for _ in range(10):
        gr.replay()
        torch.cuda.synchronize()
        dones += int(venv.episode_stats()[1].item())
        keys = venv.fresh_recipes()[0]
        ep = venv.get_state()[1][2].cpu().numpy()
        slot = 2 * np.arange(n)
        np.testing.assert_array_equal(keys[slot + ((ep - 1) & 1)], ep - 1)
        np.testing.assert_array_equal(keys[slot + (ep & 1)], ep)
    # thousands of auto-resets inside the replays (~650 per replay); the reset's scan appended n, so
    # more than n resets have wrapped the ring of 2 n slots
    assert dones > n + 256
    b = d2.Drone2dVecEnv(n, seed=1, **_kw(sim_num=1950000))
    b.load_state_dict(venv.state_dict())
    assert bytes(venv.scenario_table()) == bytes(b.scenario_table())
    venv.close()
    b.close()


def test_fresh_search_bitwise(d2):
    """The fresh curriculum's closest-point search -- scipy's fminbound over each lane's own tables
    in global memory, run speculatively in K1's path wave (two probes per pass, csrc/d2d_device.h
    brent_run_spec) -- gives the oracle's closest and lookahead points (obs 19..22) and path error
    bit for bit, teacher-forced every step, across auto-resets and the stage 4 -> 5 change."""
    from drone2d_amd import abi
    from parity_util import sync_oracle

    n, rng = 4096, np.random.default_rng(8)
    venv, orc = _pair(d2, n, 23, _kw(sim_num=1990000))
    dones = 0
    for t in range(60):
        sync_oracle(venv, orc)
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        obs = venv.step(torch.as_tensor(act, device=venv.device))[0].cpu().numpy()
        o_obs, _, o_term, _, _ = orc.step(act)
        np.testing.assert_array_equal(obs[:, 19:23], o_obs[:, 19:23])
        st, o_st = venv.get_state()[0].cpu().numpy(), orc.get_state()[0]
        np.testing.assert_array_equal(st[abi.S_PATH_ERR], o_st[abi.S_PATH_ERR])
        dones += int(o_term.sum())
    assert dones > 50
    venv.close()
