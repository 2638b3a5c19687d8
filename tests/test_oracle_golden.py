"""Pin the CPU oracle against golden vectors recorded from the reference's own Python.

Pinned here (reference code executed by tests/golden/make_golden.py): QPMI2D evaluation, scipy
fminbound closest point, lookahead, k-nearest sensing, the 27-dim observation, the reward terms,
termination, info counters, the path-error / total-reward bookkeeping and the reset observation.
The physics step inside those vectors is the ref_shims restatement of Chipmunk2D (parity
unpinned); the oracle restates it independently in C and must agree.
"""
import numpy as np
import pytest

from conftest import SCENARIOS

OBS_ATOL = 1e-6      # oracle emits float32 obs; golden is float64
# Post-step state.  The golden physics is ref_shims.py's unfused Python restatement of Chipmunk; the
# oracle (like the HIP kernels) contracts every a + b*c of the step into one fma (DESIGN.md
# "Arithmetic"), so the two differ by rounding only.  Measured over traj + crafted (round 6):
# positions / angles <= 3.1e-14 relative, velocities <= 4.9e-12, jAcc <= 4.0e-11 (Gauss-Seidel
# cancellation), total_reward <= 5.0e-11 (one crafted CA case amplifies a velocity difference).
STATE_RTOL = 1e-12   # positions, angles
DYN_RTOL = 1e-10     # velocities, jAcc, path_error, total_reward
POS_COLS = [0, 1, 2, 6, 7, 8, 12, 13, 14]
DYN_COLS = [c for c in range(32) if c not in POS_COLS]


def _flags(pre_i):
    return (pre_i[:, 1].astype(np.int32) * 1) | (pre_i[:, 2].astype(np.int32) * 2)


def run_one_step_batch(oracle_mod, d2, scenarios_c, g, auto_reset=False):
    """Teacher forcing: every recorded step becomes one env of a batch, stepped once."""
    from drone2d_amd.config import ENV_TRAIN_CONFIG, make_cfg

    cfg = make_cfg(dict(ENV_TRAIN_CONFIG), auto_reset=auto_reset)
    M = len(g["rew"])
    b = oracle_mod.OracleBatch(cfg, scenarios_c, M, env_scenario=g["scn"])
    st = np.ascontiguousarray(g["pre"].T)
    ist = np.zeros((3, M), np.int32)
    ist[0] = g["pre_i"][:, 0]
    ist[1] = _flags(g["pre_i"])
    b.set_state(st, ist)
    obs, rew, term, trunc, info = b.step(g["act"])
    st2, ist2 = b.get_state()
    return obs, rew, term, trunc, info, st2, ist2


@pytest.mark.parametrize("which", ["traj", "crafted"])
def test_one_step_teacher_forced(oracle_mod, d2, scenarios_c, which):
    from conftest import load_golden
    from drone2d_amd import abi

    g = load_golden(which)
    obs, rew, term, trunc, info, st2, ist2 = run_one_step_batch(oracle_mod, d2, scenarios_c, g)
    np.testing.assert_array_equal(term.astype(int), g["done"])
    assert not trunc.any()
    np.testing.assert_allclose(obs, g["obs"], rtol=0, atol=OBS_ATOL)
    np.testing.assert_allclose(rew, g["rew"], rtol=1e-6, atol=1e-5)
    # post-step physics state and bookkeeping
    np.testing.assert_allclose(st2.T[:, POS_COLS], g["post"][:, POS_COLS], rtol=STATE_RTOL, atol=1e-9)
    np.testing.assert_allclose(st2.T[:, DYN_COLS], g["post"][:, DYN_COLS], rtol=DYN_RTOL, atol=1e-9)
    np.testing.assert_array_equal(ist2[0], g["post_i"][:, 0])
    np.testing.assert_array_equal(ist2[1], _flags(g["post_i"]))
    # info terms (keys: see make_golden.INFO_KEYS)
    gi = g["info"]
    np.testing.assert_allclose(info[:, abi.INFO_REWARD], gi[:, 0], rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(info[:, abi.INFO_CA], gi[:, 1], rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(info[:, abi.INFO_PA], gi[:, 2], rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(info[:, abi.INFO_PP], gi[:, 3], rtol=1e-6, atol=1e-5)
    np.testing.assert_array_equal(info[:, abi.INFO_COLL], gi[:, 4])
    np.testing.assert_array_equal(info[:, abi.INFO_REACH], gi[:, 5])
    np.testing.assert_allclose(info[:, abi.INFO_AA], gi[:, 6], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(info[:, abi.INFO_DCLOSE], gi[:, 7], rtol=1e-6, atol=1e-4)
    np.testing.assert_array_equal(info[:, abi.INFO_STEPS], gi[:, 8])
    done = g["done"] == 1
    np.testing.assert_allclose(info[done, abi.INFO_APE], gi[done, 9], rtol=1e-6)
    np.testing.assert_allclose(info[done, abi.INFO_TOTREW], gi[done, 10], rtol=1e-6, atol=1e-4)
    # the info counters of drone_2d_env.py:593-610 follow from the cause bits
    cause = info[:, abi.INFO_CAUSE].astype(int)
    c1, c2 = (cause & 1) > 0, (cause & 2) > 0
    c4, c5 = (cause & 4) > 0, (cause & 8) > 0
    ncol = c1 & ~c2 & ~c4 & ~c5
    np.testing.assert_array_equal(ncol[done].astype(int), gi[done, 11])
    np.testing.assert_array_equal(c2[done].astype(int), gi[done, 12])
    np.testing.assert_array_equal((c1 | c4 | c5)[done].astype(int), gi[done, 13])


@pytest.mark.parametrize("which", ["traj", "crafted"])
def test_observation_fp64(oracle_mod, scenarios_c, ref_cfg, which):
    """The fp64 observation of the post-step state equals the reference's.

    Exact except where Brent's converged u moves within its own tolerance: the reference's
    ``u**2`` is glibc ``pow(u, 2.0)``, which differs from the correctly rounded ``u*u`` in ~0.08 %
    of inputs; near the minimum that flips a comparison of nearly equal f values and moves the
    result by << xtol (1e-6), i.e. <= ~1e-10 in the normalised closest/lookahead terms."""
    from conftest import load_golden

    g = load_golden(which)
    worst = 0.0
    for k in range(len(g["rew"])):
        flags = int(g["pre_i"][k, 2]) * 2  # LA lock before the step; observe may set it
        obs, f = oracle_mod.observe_state(ref_cfg, scenarios_c[int(g["scn"][k])], g["post"][k], flags)
        worst = max(worst, float(np.max(np.abs(obs - g["obs"][k]))))
        assert (f >> 1) == int(g["post_i"][k, 2])
    assert worst < 1e-9, worst


def test_reset_observation(oracle_mod, scenarios_c, ref_cfg, golden_traj):
    g = golden_traj
    idx = np.nonzero(g["is_reset"] == 1)[0]
    assert len(idx) > 5
    for k in idx:
        obs, _ = oracle_mod.observe_state(ref_cfg, scenarios_c[int(g["scn"][k])], g["reset_state"][k], 0)
        np.testing.assert_allclose(obs, g["reset_obs"][k], rtol=0, atol=1e-12)
        # spawn geometry: motors rigidly at +-40 along the body axis, all at rest
        s = g["reset_state"][k]
        assert np.all(s[[3, 4, 5, 9, 10, 11, 15, 16, 17]] == 0) and np.all(s[18:32] == 0)


@pytest.mark.parametrize("name", SCENARIOS)
def test_path_eval_and_closest_point(oracle_mod, scenarios_c, golden_probe, name):
    """QPMI2D.__call__ and fminbound vs the reference (predef_path.py + scipy 1.15.3).

    Bit-exact except for the reference's ``u**2`` = glibc pow(u, 2.0), which is not correctly
    rounded in ~0.08 % of inputs (1 ulp); the oracle uses u*u.  So: >= 99 % of evaluations and of
    closest-u results are bitwise equal, and every one is within 4 ulp / within xtol."""
    scn = scenarios_c[SCENARIOS.index(name)]
    g = golden_probe
    exact = total = 0
    for u, xy in zip(g[f"{name}/u"], g[f"{name}/xy"]):
        x, y = oracle_mod.path_eval(scn, u)
        np.testing.assert_allclose([x, y], xy, rtol=4e-16 * 4, atol=1e-12)
        exact += (x, y) == (xy[0], xy[1])
        total += 1
    L = scn.us[scn.n_wps - 1]
    for p, cu, cxy, lxy in zip(g[f"{name}/pts"], g[f"{name}/closest_u"], g[f"{name}/closest_xy"],
                               g[f"{name}/lookahead_xy"]):
        u, nf = oracle_mod.closest_u(scn, p[0], p[1])
        assert abs(u - cu) <= 1e-6, (p, u, cu)  # xtol of get_closest_u
        assert 1 < nf < 500
        ula = L if u + 220 > L else u + 220
        np.testing.assert_allclose(oracle_mod.path_eval(scn, u), cxy, atol=1e-6)
        np.testing.assert_allclose(oracle_mod.path_eval(scn, ula), lxy, atol=1e-6)
        exact += u == cu
        total += 1
    assert exact >= 0.99 * total, (exact, total)


def test_free_running_trajectories(oracle_mod, scenarios_c, golden_traj):
    """Run each recorded episode from its first state with the recorded actions (no forcing)."""
    from drone2d_amd.config import ENV_TRAIN_CONFIG, make_cfg

    g = golden_traj
    cfg = make_cfg(dict(ENV_TRAIN_CONFIG), auto_reset=False)
    starts = [0] + [k + 1 for k in np.nonzero(g["done"] == 1)[0] if k + 1 < len(g["rew"])]
    # also episode starts at scenario boundaries
    starts += [k for k in range(1, len(g["rew"])) if g["scn"][k] != g["scn"][k - 1]]
    starts = sorted(set(starts))
    checked = 0
    for si, k0 in enumerate(starts):
        k1 = starts[si + 1] if si + 1 < len(starts) else len(g["rew"])
        b = oracle_mod.OracleBatch(cfg, scenarios_c, 1, env_scenario=[g["scn"][k0]])
        ist = np.array([[g["pre_i"][k0, 0]], [g["pre_i"][k0, 1] | (g["pre_i"][k0, 2] << 1)], [0]], np.int32)
        b.set_state(g["pre"][k0][:, None], ist)
        for k in range(k0, k1):
            obs, rew, term, _, _ = b.step(g["act"][k][None])
            np.testing.assert_allclose(obs[0], g["obs"][k], atol=1e-5)
            np.testing.assert_allclose(rew[0], g["rew"][k], rtol=1e-5, atol=1e-4)
            assert int(term[0]) == g["done"][k]
            checked += 1
            if term[0]:
                break
    assert checked > 1000
