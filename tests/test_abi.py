"""C-ABI checks that need no GPU: struct layout of include/drone2d.h vs the ctypes mirror, the
HIP library loads and exports every entry point the header declares, Philox KAT."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "drone2d.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(d2d_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_api():
    fns = header_functions()
    for f in ("d2d_create", "d2d_destroy", "d2d_set_scenarios", "d2d_reset", "d2d_step", "d2d_get_state",
              "d2d_set_state", "d2d_episode_stats", "d2d_last_error", "d2d_abi_version", "d2d_n_envs"):
        assert f in fns


def test_struct_layout_matches_ctypes(tmp_path, d2):
    from drone2d_amd import abi
    from drone2d_amd.ppo import D2DPPORollout

    ppo_h = os.path.join(REPO, "include", "d2d_ppo.h")
    prog = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', f'#include "{ppo_h}"',
            "int main(void){"]
    structs = (("d2d_cfg", abi.D2DCfg), ("d2d_scn", abi.D2DScn), ("d2d_curriculum", abi.D2DCurriculum),
               ("d2d_ppo_rollout", D2DPPORollout))
    for cname, cls in structs:
        prog.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            prog.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    for k in ("D2D_NSTATE", "D2D_NISTATE", "D2D_INFO_DIM", "D2D_NSTATS", "D2D_OBS_DIM", "D2D_MAX_WPS",
              "D2D_MAX_CIRCLES", "D2D_ABI_VERSION"):
        prog.append(f'printf("{k} %d\\n", (int){k});')
    prog.append("return 0;}")
    c = tmp_path / "probe.c"
    c.write_text("\n".join(prog))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-o", str(exe), str(c)], check=True)
    out = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                                check=True).stdout.splitlines())
    for cname, cls in structs:
        assert int(out[cname]) == C.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert int(out[f"{cname}.{fname}"]) == getattr(cls, fname).offset, (cname, fname)
    assert int(out["D2D_NSTATE"]) == abi.NSTATE and int(out["D2D_NISTATE"]) == abi.NISTATE
    assert int(out["D2D_INFO_DIM"]) == abi.INFO_DIM and int(out["D2D_NSTATS"]) == abi.NSTATS
    assert int(out["D2D_OBS_DIM"]) == abi.OBS_DIM and int(out["D2D_MAX_WPS"]) == abi.MAX_WPS
    assert int(out["D2D_MAX_CIRCLES"]) == abi.MAX_CIRCLES and int(out["D2D_ABI_VERSION"]) == abi.ABI_VERSION


@pytest.fixture(scope="module")
def hip_lib(d2):
    from drone2d_amd import _build, _native

    _build.build()
    return _native.load()


def test_hip_library_exports_every_header_symbol(hip_lib):
    from drone2d_amd import _native, abi

    for f in header_functions():
        assert hasattr(hip_lib, f), f
        assert f in _native.SIGNATURES, f  # and the ctypes binding declares it
    assert hip_lib.d2d_abi_version() == abi.ABI_VERSION == 5


def test_hip_library_is_gfx950(d2):
    from drone2d_amd import _build

    data = open(_build.OUT, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in data  # the embedded code-object bundle id


def test_exact_trig_library_exports_the_same_abi(d2):
    """The exact-trig build (Drone2dVecEnv(exact_trig=True)) is the same source and ABI; asking for it
    together with another library is refused before anything is loaded."""
    import ctypes

    from drone2d_amd import _build, _native

    _build.build(exact=True)  # (built only on request)
    lib = ctypes.CDLL(_native.EXACT_LIB_PATH)
    for f in header_functions():
        assert hasattr(lib, f), f
    with pytest.raises(ValueError):
        d2.Drone2dVecEnv(4, device="cpu", exact_trig=True, native_lib=_native.LIB_PATH)


def test_errors_without_device(hip_lib):
    """Argument validation happens before any device call."""
    from drone2d_amd import abi
    from drone2d_amd.config import ENV_TRAIN_CONFIG, make_cfg

    h = C.c_void_p()
    cfg = make_cfg(dict(ENV_TRAIN_CONFIG))
    assert hip_lib.d2d_create(C.byref(cfg), 0, 0, C.byref(h)) == abi.E_ARG
    assert b"n_envs" in hip_lib.d2d_last_error()
    assert hip_lib.d2d_step(None, None, None, None, None, None, None, None, None) == abi.E_ARG
    assert hip_lib.d2d_reset(None, None, 0, None, None) == abi.E_ARG
    assert hip_lib.d2d_n_envs(None) == -1


@pytest.mark.parametrize("case", ["mod7", "ragged", "single", "tiny"])
def test_group_layout_properties(hip_lib, case):
    """The grouped slot layout of d2d_set_scenarios (host code): a bijection env <-> slot with no
    padding between scenarios (ceil(n/64) groups), every pure group's envs of its scenario, at most
    n_scn - 1 straddling groups, groups numbered by first env id, (scenario, id) order inside a group."""
    import numpy as np

    rng = np.random.default_rng(11)
    if case == "mod7":
        n, k = 65536, 7
        es = np.arange(n) % k
    elif case == "ragged":
        n, k = 1001, 7
        es = rng.choice(k, size=n, p=[0.3, 0.25, 0.2, 0.15, 0.1, 0.0, 0.0])
        es[[5, 500, 1000]] = 5
    elif case == "single":
        n, k = 300, 3
        es = np.full(n, 2)
    else:
        n, k = 5, 4
        es = np.array([3, 0, 3, 1, 0])
    es = np.ascontiguousarray(es, dtype=np.int32)
    ng = (n + 63) // 64
    slot_env = np.zeros(ng * 64, np.int32)
    group_scn = np.zeros(ng, np.int32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    assert hip_lib.d2d_group_layout(n, p(es), k, p(slot_env), p(group_scn)) == ng
    valid = slot_env[slot_env >= 0]
    assert sorted(valid.tolist()) == list(range(n))              # bijection
    assert (slot_env >= 0).sum() == n and (g_pad := (slot_env < 0).sum()) == ng * 64 - n, g_pad
    g = slot_env.reshape(ng, 64)
    straddle = 0
    for j in range(ng):
        e = g[j][g[j] >= 0]
        if group_scn[j] >= 0:
            assert (es[e] == group_scn[j]).all()
        elif group_scn[j] <= -2:                                 # exactly scenarios s, s + 1
            straddle += 1
            s = -int(group_scn[j]) - 2
            assert set(es[e].tolist()) == {s, s + 1}
        else:                                                    # three or more
            straddle += 1
            assert group_scn[j] == -1 and len(set(es[e].tolist())) > 2
    assert straddle <= k - 1
    firsts = g[:, 0]
    assert (np.diff(firsts) > 0).all()                           # numbered by first env id
    for j in range(ng):                                          # (scenario, id) order in a group
        e = g[j][g[j] >= 0]
        key = [(int(es[x]), int(x)) for x in e]
        assert key == sorted(key)
    bad = np.array([0, 9], np.int32)
    assert hip_lib.d2d_group_layout(2, p(bad), 3, p(slot_env), p(group_scn)) == -1
    assert b"out of range" in hip_lib.d2d_last_error()


def _xcd_group(b, nb):
    per, rem, x, k = nb // 8, nb % 8, b % 8, b // 8
    return x * (per + 1) + k if x < rem else rem * (per + 1) + (x - rem) * per + k


@pytest.mark.parametrize("n,n_cu", [(65536, 256), (32768, 256), (65536 + 37, 256), (1001, 256), (65536, 0),
                                    (65536, 100)])
def test_balanced_group_layout(hip_lib, n, n_cu):
    """d2d_balanced_group_layout (what d2d_set_scenario_costs installs): the same groups as
    d2d_group_layout, renumbered only inside each XCD chunk, dealt so that the workgroups sharing a
    CU (blocks congruent mod n_cu) carry a balanced cost: on the mixed batch no CU holds more heavy
    groups than the even share rounded up, and the straddling groups sit on distinct CUs.  With
    n_cu = 0, n_cu not a multiple of 8, or more groups than 4 n_cu: the natural order."""
    import numpy as np

    from drone2d_amd.config import SCENARIO_STEP_COST

    names = ["perpendicular", "parallel", "S_parallel", "corridor", "S_corridor", "large", "impossible"]
    k = len(names)
    cost = np.array([SCENARIO_STEP_COST[x] for x in names], np.float64)
    es = np.ascontiguousarray(np.arange(n) % k, dtype=np.int32)
    ng = (n + 63) // 64
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    se0, gs0 = np.zeros(ng * 64, np.int32), np.zeros(ng, np.int32)
    se, gs = np.zeros(ng * 64, np.int32), np.zeros(ng, np.int32)
    assert hip_lib.d2d_group_layout(n, p(es), k, p(se0), p(gs0)) == ng
    assert hip_lib.d2d_balanced_group_layout(n, p(es), k, p(cost), n_cu, p(se), p(gs)) == ng
    nat = {tuple(r): j for j, r in enumerate(se0.reshape(ng, 64))}
    new_of = np.array([nat[tuple(r)] for r in se.reshape(ng, 64)])   # same groups, renumbered
    assert sorted(new_of.tolist()) == list(range(ng)) and (gs == gs0[new_of]).all()
    if n_cu == 0 or n_cu % 8 or ng > 4 * n_cu:
        assert (new_of == np.arange(ng)).all()
        return
    per, rem = ng // 8, ng % 8
    chunk = np.concatenate([np.full(per + (x < rem), x) for x in range(8)])
    assert (chunk[new_of] == chunk[np.arange(ng)]).all()               # XCD chunks kept
    cu_groups = {}
    for b in range(ng):
        cu_groups.setdefault(b % n_cu, []).append(_xcd_group(b, ng))
    heavy = {2, 4, 5}
    hv = [sum(1 for g in gl if gs[g] in heavy or gs[g] < 0) for gl in cu_groups.values()]
    if n >= 32768:
        share = -(-sum(1 for x in gs if x in heavy or x < 0) // len(cu_groups))
        assert max(hv) <= share, (max(hv), share)
        strad = [c for c, gl in cu_groups.items() for g in gl if gs[g] < 0]
        assert len(strad) == len(set(strad))


def test_philox_known_answers(oracle_mod):
    """Random123 Philox4x32-10 KAT vectors (the spawn RNG spec shared by kernel and oracle)."""
    assert oracle_mod.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    m = 0xFFFFFFFF
    assert oracle_mod.philox([m, m, m, m], [m, m]) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert oracle_mod.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_spawn_uniforms_range(oracle_mod):
    import numpy as np

    u = np.array([oracle_mod.spawn_uniforms(7, i, e) for i in range(200) for e in range(3)])
    assert u.min() >= 0 and u.max() < 1
    assert abs(u.mean() - 0.5) < 0.05


def test_ppo_library_exports_every_header_symbol(d2):
    """libd2d_ppo.so (include/d2d_ppo.h, the PPO update's kernels): every declared entry point is
    exported and bound; argument checks run before any device call."""
    import ctypes as C

    from drone2d_amd import _build, ppo

    _build.build()
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", "d2d_ppo.h")).read(), flags=re.S)
    fns = sorted(set(re.findall(r"\b(d2d_ppo_[a-z_]+)\s*\(", src)))
    assert len(fns) >= 8
    lib = ppo.ppo_native()
    for f in fns:
        assert hasattr(lib, f), f
        assert getattr(lib, f).argtypes is not None, f  # declared in ppo_native's signatures
    assert lib.d2d_ppo_abi_version() == 6
    assert b"gfx950" in open(_build.PPO_OUT, "rb").read()
    # v4: the shuffles and the fused rollout step check their arguments before any launch
    assert lib.d2d_ppo_permute(0, 3, 1, None, None, None) == 0
    assert lib.d2d_ppo_permute(100, 3, 1, None, None, None) == 1
    r = ppo.D2DPPORollout(n=64, t=0, T=16)
    assert lib.d2d_ppo_rollout_step(C.byref(r), None, None) == 1
    assert lib.d2d_ppo_rollout_step(C.byref(r), (C.c_void_p * 12)(), None) == 1  # no obs / buffers
    r.n = 0
    assert lib.d2d_ppo_rollout_step(C.byref(r), (C.c_void_p * 12)(), None) == 0
    # out-of-range shapes are refused (hipErrorInvalidValue = 1) without a launch
    assert lib.d2d_ppo_adam(0, None, None, None, None, None, 1e-3, 0.9, 0.999, 1e-5, 0.5, None) == 0  # no launch
    assert lib.d2d_ppo_adam(1 << 20, None, None, None, None, None, 1e-3, 0.9, 0.999, 1e-5, 0.5, None) == 1
    one = (C.c_int32 * 1)(65)
    ptr = (C.c_void_p * 1)(None)
    assert lib.d2d_ppo_wgrad(64, 1, ptr, one, ptr, one, one, one, one, one, 100, None, None, None) == 1
    assert lib.d2d_ppo_wgrad(0, 1, ptr, one, ptr, one, one, one, one, one, 100, None, None, None) == 0

