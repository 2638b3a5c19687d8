"""Curriculum reset generator against the reference's own curriculum resets
(tests/golden/curriculum.npz, recorded by make_curriculum_golden.py from the unmodified
Drone2dEnv in mode='curriculum').  CPU only."""
import random

import numpy as np
import pytest

from conftest import load_golden

STAGES = ["stage_1", "stage_2", "stage_3", "stage_4", "stage_5"]


def _cfg():
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    return dict(ENV_TRAIN_CONFIG, mode="curriculum")


@pytest.mark.parametrize("stage", STAGES)
def test_generator_bit_exact_vs_reference(d2, stage):
    from drone2d_amd.curriculum import curriculum_scenario

    g = load_golden("curriculum")
    seeds = sorted({int(k.split("/")[1]) for k in g.files if k.startswith(stage + "/")})
    assert len(seeds) >= 8
    n_obs = 0
    for s in seeds:
        k = f"{stage}/{s}"
        sc = curriculum_scenario(stage, _cfg(), np.random.RandomState(s), random.Random(s))
        np.testing.assert_array_equal(sc.wps, g[k + "/wps"])
        np.testing.assert_array_equal(sc.path.us, g[k + "/us"])
        np.testing.assert_array_equal(np.asarray(sc.path.x_params), g[k + "/xp"])
        np.testing.assert_array_equal(np.asarray(sc.path.y_params), g[k + "/yp"])
        np.testing.assert_array_equal(sc.circles, g[k + "/circles"])
        n_obs += len(sc.circles)
        x, y, a = g[k + "/spawn"]
        xmin, xmax, ymin, ymax = sc.spawn
        assert xmin <= x <= xmax and ymin <= y <= ymax and abs(a) <= np.pi / 4
        if stage != "stage_2":
            assert (x, y) == (xmin, ymin) == (xmax, ymax)  # spawn at the first waypoint
    if stage in ("stage_4", "stage_5"):
        assert n_obs > 0


def test_pool_is_the_sequence_of_resets(d2):
    from drone2d_amd.curriculum import curriculum_pool, curriculum_scenario

    pool = curriculum_pool("stage_5", _cfg(), 6, seed=3)
    rs, py = np.random.RandomState(3), random.Random(3)
    for sc in pool:
        ref = curriculum_scenario("stage_5", _cfg(), rs, py)
        np.testing.assert_array_equal(sc.wps, ref.wps)
        np.testing.assert_array_equal(sc.circles, ref.circles)
    # every pool entry converts to the device table
    for sc in pool:
        sc.to_c()


def test_sim_num_schedule(d2):
    from drone2d_amd.curriculum import stage_for_sim_num

    assert stage_for_sim_num(0) == ("stage_1", None)
    assert stage_for_sim_num(800000) == ("stage_2", None)
    st, ch = stage_for_sim_num(1300000)
    assert st == "stage_3" and abs(ch - 0.4) < 1e-12
    st, ch = stage_for_sim_num(1800000)
    assert st == "stage_4" and abs(ch - 0.8) < 1e-12
    assert stage_for_sim_num(9000000) == ("stage_5", None)
    for gap in (700000, 1000000, 1600000, 2000000):
        with pytest.raises(ValueError):
            stage_for_sim_num(gap)


# ------------------------------------------------------------ fresh curriculum (device generator)
# The device draws every curriculum episode's scenario itself (csrc/d2d_curriculum.h); the oracle
# restates that generator (o_gen_curriculum) and the device must match it bit for bit (GPU tests).
# Here: the restatement against the reference-exact host generator above, distribution by
# distribution (two-sample KS / means), and its deterministic sin / cos / log against NumPy.
def _fresh(stage, n, seed=7):
    import oracle
    from drone2d_amd.env import make_curriculum

    c = make_curriculum(dict(_cfg(), scenario=stage), 1)
    return [oracle.gen_curriculum(c, 1300.0, 1300.0, seed, g, 3, 0.0) for g in range(n)]


@pytest.mark.parametrize("stage", STAGES)
def test_fresh_generator_matches_reference_distribution(d2, oracle_mod, stage):
    from scipy.stats import ks_2samp

    from drone2d_amd.curriculum import curriculum_pool
    from drone2d_amd.scenarios import QPMIPath

    dev = _fresh(stage, 2500)
    host = curriculum_pool(stage, _cfg(), 1200, seed=11)
    hc = [h.to_c() for h in host]
    feats = {
        "length": (lambda d: d.us[d.n_wps - 1]),
        "x0": (lambda d: d.spawn_xmin), "y0": (lambda d: d.spawn_ymin),
        "xmax": (lambda d: d.spawn_xmax), "wlast_x": (lambda d: d.wp_last_x), "wlast_y": (lambda d: d.wp_last_y),
        "u2": (lambda d: d.us[2]),
    }
    for k, f in feats.items():
        a, b = np.array([f(d) for d in dev]), np.array([f(h) for h in hc])
        if np.ptp(a) == 0 and np.ptp(b) == 0:
            assert a[0] == b[0], k
        else:
            assert ks_2samp(a, b).pvalue > 1e-3, k
    nd = np.array([d.n_circles for d in dev], float)
    nh = np.array([h.n_circles for h in hc], float)
    assert abs(nd.mean() - nh.mean()) < 4 * np.sqrt(nd.var() / len(nd) + nh.var() / len(nh)) + 1e-9
    if nh.sum() > 50:
        rd = np.concatenate([np.array(d.cr[:d.n_circles]) for d in dev])
        rh = np.concatenate([np.array(h.cr[:h.n_circles]) for h in hc])
        assert ks_2samp(rd, rh).pvalue > 1e-3
    # the fit: QPMI2D of the generated waypoints (recovered from the path) reproduces the record,
    # and the path passes through the last waypoint
    import oracle

    for d in dev[:50]:
        nw = d.n_wps
        L = d.us[nw - 1]
        x, y = oracle.path_eval(d, L)
        assert abs(x - d.wp_last_x) < 1e-7 and abs(y - d.wp_last_y) < 1e-7
        wps = np.array([oracle.path_eval(d, u) for u in d.us[:nw]])
        p = QPMIPath(wps)
        np.testing.assert_allclose(p.us, np.array(d.us[:nw]), rtol=1e-9, atol=1e-7)
        np.testing.assert_allclose(np.asarray(p.x_params)[:, 2], np.array(d.xc[:nw - 2]), rtol=1e-6, atol=1e-6)


def test_fresh_generator_stage_schedule(d2, oracle_mod):
    """The reference's sim_num thresholds (drone_2d_env.py:326-372) with the gaps taken by the stage
    below: spawn box in stage 2, obstacles only from stage 3, on the path in stage 4."""
    import oracle
    from drone2d_amd.env import make_curriculum

    c = make_curriculum(dict(_cfg(), scenario="curriculum"), 1)
    W = 1300.0
    for sim, stage in ((0, 1), (699999, 1), (700000, 1), (700001, 2), (1000000, 2), (1000001, 3),
                       (1600000, 3), (1600001, 4), (2000000, 4), (2000001, 5), (9e6, 5)):
        scn = [oracle.gen_curriculum(c, W, W, 5, g, 1, float(sim)) for g in range(300)]
        box = [(s.spawn_xmin, s.spawn_xmax) == (100.0, W - 100.0) for s in scn]
        nc = np.array([s.n_circles for s in scn])
        assert all(box) == (stage == 2) and (any(box) == (stage == 2)), sim
        if stage <= 2:
            assert nc.max() == 0, sim
        if stage == 4:
            assert nc.max() == 1 and nc.sum() > 150, sim  # chance 0.6 .. 1, one circle on the path
        if stage == 5:
            assert nc.max() > 2, sim


def test_pmath_matches_numpy(oracle_mod):
    """d2d_pmath.h (shared by the device generator and the oracle): <= 1 ulp from libm."""
    import ctypes as C
    import subprocess
    import tempfile

    from conftest import REPO

    src = r'''
#include <stdio.h>
#include "%s/drone-2d-custom-gym-env-for-reinforcement-learning_amd/csrc/d2d_pmath.h"
int main(void) { double x; while (scanf("%%lf", &x) == 1) { double s, c; d2d_pm_sincos(x, &s, &c);
  printf("%%.17g %%.17g %%.17g\n", s, c, x > 0 ? d2d_pm_log(x) : 0.0); } return 0; }
''' % REPO
    with tempfile.TemporaryDirectory() as td:
        open(f"{td}/p.c", "w").write(src)
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", f"{td}/p", f"{td}/p.c"], check=True)
        x = np.concatenate([np.random.default_rng(0).uniform(-8, 8, 20000),
                            np.random.default_rng(1).uniform(1e-12, 1, 20000)])
        out = subprocess.run([f"{td}/p"], input="\n".join(repr(float(v)) for v in x), capture_output=True,
                             text=True, check=True).stdout
    r = np.array([[float(t) for t in ln.split()] for ln in out.splitlines()])
    ulp = lambda a, b: np.abs(a - b) / np.spacing(np.abs(b))  # noqa: E731
    assert ulp(r[:, 0], np.sin(x)).max() <= 1.0 and ulp(r[:, 1], np.cos(x)).max() <= 1.0
    pos = x > 0
    assert ulp(r[pos, 2], np.log(x[pos])).max() <= 1.0
    del C


def test_fresh_oracle_backend_every_episode_new(d2, oracle_mod):
    """The oracle's fresh-curriculum protocol: every episode of every env runs on its own scenario
    (slot 2 i + (key & 1), regenerated one step ahead), and the stage follows the step clock."""
    from oracle_backend import OracleVecBackend
    import torch

    n = 64
    be = OracleVecBackend(n, seed=9, **dict(_cfg(), scenario="curriculum", sim_num=650000), envs_total=1000)
    be.reset()
    rng = np.random.default_rng(0)
    seen = set()
    for t in range(150):
        be.step(torch.as_tensor(rng.uniform(-1, 1, (n, 2)).astype(np.float32)))
        keys, clocks, clock = be.orc.fresh_recipes()
        assert clock == t + 1
        tab = be.orc.scenario_table(0, 2 * n)
        for s in range(2 * n):
            if keys[s] >= 0:
                seen.add((s // 2, int(keys[s]), round(tab[s].wp_last_x, 9)))
    # distinct (env, episode) pairs and distinct paths
    assert len(seen) > n and len({p for _, _, p in seen}) == len(seen)
    # the clock crossed 700 000 (stage 1 -> 2) at step 50: stage-2 spawn boxes appear
    tab = be.orc.scenario_table(0, 2 * n)
    assert any(tab[s].spawn_xmin == 100.0 and tab[s].spawn_xmax == 1200.0 for s in range(2 * n))
    be.close()


def _fresh_oracle(n, sim_num=0):
    import oracle

    import drone2d_amd  # noqa: F401
    from drone2d_amd.config import ENV_TRAIN_CONFIG, make_cfg
    from drone2d_amd.env import make_curriculum

    kw = dict(ENV_TRAIN_CONFIG, mode="curriculum", scenario="curriculum", sim_num=sim_num)
    cfg = make_cfg(dict(kw))
    cfg.scn_pool = 2
    return oracle.OracleBatch(cfg, [], n, curriculum=make_curriculum(kw, n)), kw


def test_oracle_set_curriculum_restarts_clock():
    """d2d_set_curriculum's contract, restated by the oracle: the step clock restarts at
    zero, so the schedule starts at the new sim_num0, not at sim_num0 + the steps already taken."""
    from drone2d_amd.env import make_curriculum

    n = 16
    orc, kw = _fresh_oracle(n)
    orc.reset(3)
    rng = np.random.default_rng(0)
    for _ in range(7):
        orc.step(rng.uniform(-1, 1, (n, 2)).astype(np.float32))
    assert orc.fresh_recipes()[2] == 7
    orc.set_curriculum(make_curriculum(dict(kw, sim_num=1_200_000), n))
    assert orc.fresh_recipes()[2] == 0
    orc.reset(3)
    keys, clocks, clock = orc.fresh_recipes()
    tab = orc.scenario_table(0, 2 * n)
    for s in np.flatnonzero(keys >= 0):  # generated at clock 0 of sim_num 1.2e6: stage 3
        assert clocks[s] == 0 and tab[s].n_circles <= 1 and tab[s].spawn_xmin == tab[s].spawn_xmax
    orc.close()


def test_oracle_masked_fresh_reset_keeps_seed():
    """A masked fresh-curriculum reset must pass the previous full reset's seed (d2d_reset's rule):
    the envs it leaves running would otherwise keep scenarios no (key, clock) recipe regenerates."""
    n = 8
    orc, _ = _fresh_oracle(n)
    mask = np.zeros(n, np.uint8)
    mask[::2] = 1
    with pytest.raises(RuntimeError):
        orc.reset(5, mask)  # no full reset yet
    orc.reset(5)
    with pytest.raises(RuntimeError):
        orc.reset(6, mask)
    orc.reset(5, mask)
    orc.close()
