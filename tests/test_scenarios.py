"""Host scenario builder vs the reference's own test_scenarios.py output (golden, bit-exact)."""
import numpy as np
import pytest

from conftest import SCENARIOS


@pytest.mark.parametrize("name", SCENARIOS)
def test_scenario_geometry_bit_exact(d2, golden_scn, name):
    from drone2d_amd.scenarios import create_test_scenario

    s = create_test_scenario(name, 1300, 1300)
    np.testing.assert_array_equal(s.wps, golden_scn[f"{name}/wps"])
    np.testing.assert_array_equal(s.path.us, golden_scn[f"{name}/us"])
    np.testing.assert_array_equal(np.asarray(s.path.x_params), golden_scn[f"{name}/x_params"])
    np.testing.assert_array_equal(np.asarray(s.path.y_params), golden_scn[f"{name}/y_params"])
    np.testing.assert_array_equal(s.circles, golden_scn[f"{name}/circles"])
    np.testing.assert_array_equal(np.asarray(s.spawn), golden_scn[f"{name}/spawn"])


def test_scenario_table_matches_survey(d2):
    """SURVEY.md §8(d) scenario table: wps / path length / circles / radius."""
    from drone2d_amd.scenarios import create_test_scenario

    expect = {"perpendicular": (10, 900, 6, 20), "parallel": (10, 900, 6, 30), "S_parallel": (6, 1500, 20, 15),
              "corridor": (10, 900, 18, 35), "S_corridor": (7, 1200, 58, 16.67), "large": (14, 1434.96, 1, 260),
              "impossible": (10, 900, 20, 15.71)}
    for name, (nw, L, nc, r) in expect.items():
        s = create_test_scenario(name, 1300, 1300)
        assert len(s.wps) == nw
        assert abs(float(s.path.length) - L) < 0.01
        assert len(s.circles) == nc
        assert abs(float(s.circles[0, 2]) - r) < 0.01


def test_to_c_roundtrip(d2):
    from drone2d_amd.scenarios import create_test_scenario

    s = create_test_scenario("S_corridor", 1300, 1300)
    c = s.to_c()
    assert c.n_wps == 7 and c.n_circles == 58
    assert c.us[6] == float(s.path.us[6])
    assert c.cr[57] == float(s.circles[57, 2])
    assert (c.wp_last_x, c.wp_last_y) == (float(s.wps[-1][0]), float(s.wps[-1][1]))


def test_limits(d2):
    from drone2d_amd.scenarios import Scenario, scenario_to_c, QPMIPath

    wps = np.stack([np.arange(20) * 50.0, np.zeros(20)], 1)
    with pytest.raises(ValueError):
        scenario_to_c(Scenario("x", wps, QPMIPath(wps), np.zeros((0, 3)), (0, 1, 0, 1)))
    wps = wps[:5]
    with pytest.raises(ValueError):
        scenario_to_c(Scenario("x", wps, QPMIPath(wps), np.zeros((65, 3)), (0, 1, 0, 1)))
