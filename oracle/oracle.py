"""ctypes wrapper of the CPU parity oracle ``oracle/libd2d_oracle.so``.

TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).  The oracle
is a plain C restatement of the reference's hot path; see d2d_oracle.c for the per-function
reference citations and the parity-pinning status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libd2d_oracle.so")
# sin / cos / atan2 from d2d_pmath.h: the oracle of the HIP library's exact-trig build
LIB_EXACT = os.path.join(HERE, "libd2d_oracle_exact.so")


def build(force: bool = False) -> str:
    src = [os.path.join(HERE, f) for f in ("d2d_oracle.c", "d2d_oracle.h", "Makefile")]
    src.append(os.path.join(HERE, "..", "include", "drone2d.h"))
    src.append(os.path.join(HERE, "..", "drone-2d-custom-gym-env-for-reinforcement-learning_amd", "csrc", "d2d_pmath.h"))
    if force or any(not os.path.exists(o) or any(os.path.getmtime(s) > os.path.getmtime(o) for s in src)
                    for o in (LIB, LIB_EXACT)):
        subprocess.run(["make", "-s", "-C", HERE, "-B" if force else "all"], check=True)
    return LIB


def _abi():
    import drone2d_amd.abi as abi  # ctypes structs only; does not load the HIP library

    return abi


_libs = {}


def load(exact_trig: bool = False) -> C.CDLL:
    path = LIB_EXACT if exact_trig else LIB
    if path not in _libs:
        if not os.path.exists(path):
            build()
        abi = _abi()
        lib = C.CDLL(path)
        P, VP, I32, D = C.POINTER, C.c_void_p, C.c_int32, C.c_double
        sigs = {
            "d2dcpu_create": (VP, [P(abi.D2DCfg), I32]),
            "d2dcpu_destroy": (None, [VP]),
            "d2dcpu_set_scenarios": (I32, [VP, P(abi.D2DScn), I32, VP]),
            "d2dcpu_reset": (I32, [VP, VP, C.c_uint64, VP]),
            "d2dcpu_refresh_pool": (I32, [VP, P(abi.D2DScn), I32]),
            "d2dcpu_get_env_scenarios": (I32, [VP, VP]),
            "d2dcpu_step": (I32, [VP, VP, VP, VP, VP, VP, VP, VP]),
            "d2dcpu_step_mt": (I32, [VP, VP, VP, VP, VP, VP, VP, VP, I32]),
            "d2dcpu_get_state": (I32, [VP, VP, VP]),
            "d2dcpu_set_state": (I32, [VP, VP, VP]),
            "d2dcpu_episode_stats": (I32, [VP, VP, I32]),
            "d2dcpu_path_eval": (None, [P(abi.D2DScn), D, P(D), P(D)]),
            "d2dcpu_closest_u": (D, [P(abi.D2DScn), D, D, P(C.c_int)]),
            "d2dcpu_observe_state": (None, [P(abi.D2DCfg), P(abi.D2DScn), VP, P(I32), VP]),
            "d2dcpu_physics_step": (I32, [P(abi.D2DCfg), P(abi.D2DScn), VP, D, D, I32]),
            "d2dcpu_moment_box": (D, [D, D, D]),
            "d2dcpu_spawn_uniforms": (None, [C.c_uint64, C.c_uint32, C.c_uint32, P(D)]),
            "d2dcpu_philox": (None, [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]),
            "d2dcpu_set_curriculum": (I32, [VP, P(abi.D2DCurriculum)]),
            "d2dcpu_fresh_recipes": (I32, [VP, VP, VP, P(C.c_int64), I32]),
            "d2dcpu_get_scenario_table": (I32, [VP, I32, I32, P(abi.D2DScn)]),
            "d2dcpu_gen_curriculum": (None, [P(abi.D2DCurriculum), D, D, C.c_uint64, C.c_uint32, C.c_uint32, D,
                                             P(abi.D2DScn)]),
        }
        for name, (res, args) in sigs.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _libs[path] = lib
    return _libs[path]


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


class OracleBatch:
    """Host-side batch with the same call shapes as the HIP library (numpy buffers)."""

    def __init__(self, cfg, scenarios_c, n_envs: int, env_scenario=None, curriculum=None, exact_trig: bool = False):
        """``curriculum``: a D2DCurriculum for the fresh curriculum (cfg.scn_pool = 2; no scenarios).
        ``exact_trig``: the exact-trig build (the oracle of ``Drone2dVecEnv(exact_trig=True)``)."""
        self.lib = load(exact_trig)
        abi = _abi()
        self.abi = abi
        self.n = int(n_envs)
        self.cfg = cfg
        self.h = self.lib.d2dcpu_create(C.byref(cfg), self.n)
        if curriculum is not None:
            self._cur = curriculum
            if self.lib.d2dcpu_set_curriculum(self.h, C.byref(curriculum)) != 0:
                raise ValueError("d2dcpu_set_curriculum: cfg.scn_pool must be 2")
        else:
            arr = (abi.D2DScn * len(scenarios_c))(*scenarios_c)
            self._scn = arr
            es = None
            if env_scenario is not None:
                es = np.ascontiguousarray(np.asarray(env_scenario, dtype=np.int32))
            self.lib.d2dcpu_set_scenarios(self.h, arr, len(scenarios_c), _p(es))
        n = self.n
        self.obs = np.zeros((n, abi.OBS_DIM), np.float32)
        self.rew = np.zeros(n, np.float32)
        self.term = np.zeros(n, np.uint8)
        self.trunc = np.zeros(n, np.uint8)
        self.info = np.zeros((n, abi.INFO_DIM), np.float32)
        self.tobs = np.zeros((n, abi.OBS_DIM), np.float32)

    def close(self):
        if self.h:
            self.lib.d2dcpu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def reset(self, seed: int, mask=None):
        m = None if mask is None else np.ascontiguousarray(np.asarray(mask, dtype=np.uint8))
        rc = self.lib.d2dcpu_reset(self.h, _p(m), C.c_uint64(seed & (2 ** 64 - 1)), _p(self.obs))
        if rc != 0:
            raise RuntimeError(f"d2dcpu_reset: error {rc}")
        return self.obs.copy()

    def step(self, actions, nthreads: int = 1):
        a = np.ascontiguousarray(np.asarray(actions, dtype=np.float32).reshape(self.n, 2))
        self.lib.d2dcpu_step_mt(self.h, _p(a), _p(self.obs), _p(self.rew), _p(self.term), _p(self.trunc),
                                _p(self.info), _p(self.tobs), nthreads)
        return self.obs.copy(), self.rew.copy(), self.term.astype(bool), self.trunc.astype(bool), self.info.copy()

    def get_state(self):
        st = np.zeros((self.abi.NSTATE, self.n), np.float64)
        ist = np.zeros((self.abi.NISTATE, self.n), np.int32)
        self.lib.d2dcpu_get_state(self.h, _p(st), _p(ist))
        return st, ist

    def set_state(self, st, ist):
        st = np.ascontiguousarray(st, dtype=np.float64)
        ist = np.ascontiguousarray(ist, dtype=np.int32)
        self.lib.d2dcpu_set_state(self.h, _p(st), _p(ist))

    def refresh_pool(self, scenarios_c) -> int:
        arr = (self.abi.D2DScn * len(scenarios_c))(*scenarios_c)
        self._scn_refresh = arr
        return self.lib.d2dcpu_refresh_pool(self.h, arr, len(scenarios_c))

    def get_env_scenarios(self):
        out = np.zeros(self.n, np.int32)
        self.lib.d2dcpu_get_env_scenarios(self.h, _p(out))
        return out

    def scenario_table(self, first: int, count: int):
        out = (self.abi.D2DScn * count)()
        if self.lib.d2dcpu_get_scenario_table(self.h, first, count, out) != 0:
            raise ValueError("scenario table range")
        return out

    def set_curriculum(self, curriculum):
        """d2dcpu_set_curriculum (as d2d_set_curriculum: empties the slots and zeroes the step clock)."""
        self._cur = curriculum
        if self.lib.d2dcpu_set_curriculum(self.h, C.byref(curriculum)) != 0:
            raise ValueError("d2dcpu_set_curriculum: cfg.scn_pool must be 2")

    def fresh_recipes(self, keys=None, clocks=None, clock=None):
        """get (no arguments) -> (keys int32[2n], clocks int64[2n], clock); set with all three."""
        n2 = 2 * self.n
        if keys is None:
            k, c, t = np.zeros(n2, np.int32), np.zeros(n2, np.int64), C.c_int64()
            self.lib.d2dcpu_fresh_recipes(self.h, _p(k), _p(c), C.byref(t), 0)
            return k, c, t.value
        k = np.ascontiguousarray(keys, np.int32)
        c = np.ascontiguousarray(clocks, np.int64)
        t = C.c_int64(int(clock))
        self.lib.d2dcpu_fresh_recipes(self.h, _p(k), _p(c), C.byref(t), 1)

    def episode_stats(self, clear=True):
        out = np.zeros(self.abi.NSTATS, np.float64)
        self.lib.d2dcpu_episode_stats(self.h, _p(out), 1 if clear else 0)
        return out


# ------------------------------------------------------------------------------ single probes
def path_eval(scn_c, u: float):
    x, y = C.c_double(), C.c_double()
    load().d2dcpu_path_eval(C.byref(scn_c), float(u), C.byref(x), C.byref(y))
    return x.value, y.value


def closest_u(scn_c, px: float, py: float):
    nf = C.c_int()
    u = load().d2dcpu_closest_u(C.byref(scn_c), float(px), float(py), C.byref(nf))
    return u, nf.value


def observe_state(cfg, scn_c, state, flags: int = 0):
    st = np.ascontiguousarray(state, dtype=np.float64)
    obs = np.zeros(27, np.float64)
    f = C.c_int32(flags)
    load().d2dcpu_observe_state(C.byref(cfg), C.byref(scn_c), _p(st), C.byref(f), _p(obs))
    return obs, f.value


def physics_step(cfg, scn_c, state, fL: float, fR: float, collided: int = 0):
    st = np.array(state, dtype=np.float64)
    hit = load().d2dcpu_physics_step(C.byref(cfg), C.byref(scn_c), _p(st), float(fL), float(fR), int(collided))
    return st, int(hit)


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    load().d2dcpu_philox(c, k, o)
    return list(o)


def spawn_uniforms(seed: int, env_id: int, episode: int):
    u = (C.c_double * 3)()
    load().d2dcpu_spawn_uniforms(C.c_uint64(seed), env_id, episode, u)
    return list(u)


def gen_curriculum(cur, W: float, H: float, seed: int, gid: int, key: int, sim: float):
    """One fresh-curriculum scenario (the oracle's restatement of the device generator)."""
    out = _abi().D2DScn()
    load().d2dcpu_gen_curriculum(C.byref(cur), float(W), float(H), C.c_uint64(seed & (2 ** 64 - 1)), gid, key,
                                 float(sim), C.byref(out))
    return out
