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
