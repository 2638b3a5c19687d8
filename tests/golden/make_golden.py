#!/usr/bin/env python3
"""Generate the golden fixtures under ``tests/golden/`` from the reference's own Python.

Run ONLY in the development container (``/root/reference`` does not exist on the GPU box):

    python tests/golden/make_golden.py

What is executed from the reference, unmodified (imported from /root/reference):
  * ``predef_path.py`` (QPMI2D fit, ``__call__``, ``get_closest_u`` -> scipy ``fminbound``,
    ``get_closest_position``, ``get_lookahead_point``) and ``transformations.py``;
  * ``test_scenarios.py`` / ``obstacles.py`` (the 7 deterministic test scenarios);
  * ``drone_2d_env.py`` + ``Drone.py`` (spawn, ``step``, ``get_observation``, reward,
    termination, ``info``, ``reset``), with the ``ref_shims`` modules standing in for
    pymunk / pygame / gym.  The shim's ``Space.step`` is a restatement of Chipmunk2D
    (see ``ref_shims.py``) -- the physics recorded here is therefore parity-unpinned.

Fixtures written (all plain ``.npz``, loadable with ``allow_pickle=False``):
  scenarios.npz     geometry of the 7 test scenarios (+ spawn rectangles)
  path_probe.npz    QPMI2D evaluations and fminbound closest-u / lookahead on every path
  traj.npz          random-action trajectories with SB3-style auto-reset, per step:
                    pre-state, f32 action, obs (f64), reward, done, info terms, post-state
  crafted.npz       one-step cases from crafted states (collisions, reach-end, AA, time-up,
                    LA lock, danger-range CA/lambda) across all scenarios
"""
from __future__ import annotations

import contextlib
import io
import os
import random
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/drone_2d_custom_gym_env"
SCENARIOS = ["perpendicular", "parallel", "S_parallel", "corridor", "S_corridor", "large", "impossible"]

# state layout (matches include/drone2d.h D2D_S_*): 3 bodies x (px,py,a,vx,vy,w), 6 x jAcc(2),
# path_error, total_reward
NSTATE = 32
INFO_KEYS = ["reward", "collision_avoidance_reward", "path_adherence", "path_progression",
             "collision_reward", "reach_end_reward", "agressive_alpha_reward", "dist_closest_obs",
             "env_steps", "APE", "total_reward", "n_collisions", "n_successful_runs", "n_failed_runs"]


def _import_reference():
    sys.path.insert(0, HERE)
    import ref_shims  # noqa: E402

    ref_shims.install()
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.path.insert(0, REF)
    import drone_2d_env  # noqa: E402  (reference, unmodified)
    import predef_path  # noqa: E402
    import rl_config  # noqa: E402
    import test_scenarios  # noqa: E402
    return drone_2d_env, predef_path, rl_config, test_scenarios, ref_shims


def _bodies(env):
    d = env.drone
    return [d.frame_shape.body, d.left_motor_shape.body, d.right_motor_shape.body]


def _joints(env):
    d = env.drone
    return [d.left_1, d.left_2, d.left_3, d.right_1, d.right_2, d.right_3]


def get_state(env):
    s = np.zeros(NSTATE)
    for bi, b in enumerate(_bodies(env)):
        s[bi * 6:bi * 6 + 6] = [b.px, b.py, b.a, b.vx, b.vy, b.w]
    for ji, j in enumerate(_joints(env)):
        s[18 + 2 * ji:20 + 2 * ji] = j.jAcc
    s[30] = env.path_error
    s[31] = env.total_reward
    ints = np.array([env.current_time_step, int(bool(env.space.collison)), int(bool(env.LA_in_last_wp))],
                    dtype=np.int64)
    return s, ints


def set_state(env, s, ints):
    for bi, b in enumerate(_bodies(env)):
        b.px, b.py = float(s[bi * 6]), float(s[bi * 6 + 1])
        b.angle = float(s[bi * 6 + 2])
        b.vx, b.vy, b.w = float(s[bi * 6 + 3]), float(s[bi * 6 + 4]), float(s[bi * 6 + 5])
    for ji, j in enumerate(_joints(env)):
        j.jAcc = [float(s[18 + 2 * ji]), float(s[19 + 2 * ji])]
    env.path_error = float(s[30])
    env.total_reward = float(s[31])
    env.current_time_step = int(ints[0])
    env.space.collison = bool(ints[1])
    env.LA_in_last_wp = bool(ints[2])
    env.space.curr_dt = 1.0 / 60  # mid-episode: warm start active (dt_coef = 1)


def info_vec(info):
    out = np.zeros(len(INFO_KEYS))
    for i, k in enumerate(INFO_KEYS):
        out[i] = float(info.get(k, np.nan))
    return out


def make_cfg(rl_config, scenario):
    cfg = dict(rl_config.env_train_config)
    cfg.update(render_sim=False, render_path=False, render_shade=False, render_text=False,
               mode="test", scenario=scenario)
    return cfg


def gen_scenarios(de, pp, rl_config, ts, shims):
    out = {}
    W = rl_config.env_train_config["screensize_x"]
    H = rl_config.env_train_config["screensize_y"]
    for si, name in enumerate(SCENARIOS):
        space = shims.Space()
        wps, path, obstacles = ts.create_test_scenario(space, name, W, H)
        circ = np.array([[o.x_pos, o.y_pos, o.radius] for o in obstacles], dtype=np.float64)
        out[f"{name}/wps"] = np.asarray(wps, dtype=np.float64)
        out[f"{name}/us"] = np.asarray(path.us, dtype=np.float64)
        out[f"{name}/x_params"] = np.asarray(path.x_params, dtype=np.float64)
        out[f"{name}/y_params"] = np.asarray(path.y_params, dtype=np.float64)
        out[f"{name}/circles"] = circ.reshape(-1, 3)
        # spawn rectangle exactly as the env computes it (drone_2d_env.py:221-311):
        env = de.Drone2dEnv(**make_cfg(rl_config, name))
        xmin, ymin, width, height = env.spawn_rect
        out[f"{name}/spawn"] = np.array([xmin, xmin + width, ymin, height], dtype=np.float64)
    return out


def gen_path_probe(pp, scen_npz, rng):
    out = {}
    for name in SCENARIOS:
        wps = scen_npz[f"{name}/wps"]
        path = pp.QPMI2D(wps)
        L = float(path.length)
        # path evaluation incl. extrapolation branches and exact knots
        us = np.concatenate([rng.uniform(-30.0, L + 30.0, 300), path.us, path.us - 0.0005,
                             [-10.0, L + 10.0, path.us[-2] - 0.001, path.us[-2] - 0.0011]])
        xy = np.array([path(float(u)) for u in us])
        # closest point / lookahead from points all over the screen and near the path
        pts = np.concatenate([rng.uniform(-100.0, 1400.0, (150, 2)),
                              xy[:150] + rng.normal(0.0, 40.0, (150, 2))])
        cu = np.array([path.get_closest_u([float(p[0]), float(p[1])]) for p in pts])
        cp = np.array([path.get_closest_position([float(p[0]), float(p[1])]) for p in pts])
        la = np.array([path.get_lookahead_point([float(p[0]), float(p[1])], 220) for p in pts])
        out[f"{name}/u"] = us
        out[f"{name}/xy"] = xy
        out[f"{name}/pts"] = pts
        out[f"{name}/closest_u"] = cu
        out[f"{name}/closest_xy"] = cp
        out[f"{name}/lookahead_xy"] = la
    return out


class _Rec:
    def __init__(self):
        self.cols = {k: [] for k in ["scn", "pre", "pre_i", "act", "obs", "rew", "done", "info", "post",
                                     "post_i", "reset_obs", "reset_state", "is_reset"]}

    def add(self, **kw):
        for k, v in kw.items():
            self.cols[k].append(v)

    def arrays(self, prefix):
        out = {}
        for k, v in self.cols.items():
            if v:
                out[f"{prefix}{k}"] = np.asarray(v)
        return out


def gen_traj(de, rl_config, steps=300, seed=0):
    rec = _Rec()
    for si, name in enumerate(SCENARIOS):
        random.seed(1000 + si + seed)
        arng = np.random.default_rng(2000 + si + seed)
        env = de.Drone2dEnv(**make_cfg(rl_config, name))
        obs = env.reset()
        for t in range(steps):
            pre, pre_i = get_state(env)
            # mildly biased random thrust so some episodes live long enough to reach obstacles
            a = np.clip(arng.normal(0.0, 0.55, 2) + arng.choice([0.0, 0.15, -0.15]), -1, 1).astype(np.float32)
            o, r, d, info = env.step(a)
            post, post_i = get_state(env)
            ro = np.full(27, np.nan)
            rs = np.full(NSTATE, np.nan)
            if d:  # SB3 worker auto-reset
                ro = np.asarray(env.reset(), dtype=np.float64)
                rs, _ = get_state(env)
            rec.add(scn=si, pre=pre, pre_i=pre_i, act=a, obs=np.asarray(o, np.float64), rew=float(r),
                    done=int(bool(d)), info=info_vec(info), post=post, post_i=post_i, reset_obs=ro,
                    reset_state=rs, is_reset=int(bool(d)))
    return rec.arrays("")


def _crafted_state(rng, scn_circles, wps, spawn, kind):
    """A plausible mid-episode drone state designed to hit one reference branch."""
    s = np.zeros(NSTATE)
    if kind == "near_obstacle" and len(scn_circles):
        c = scn_circles[rng.integers(len(scn_circles))]
        ang = rng.uniform(-np.pi, np.pi)
        rad = c[2] + rng.uniform(-5.0, 160.0)
        x, y = c[0] + rad * np.cos(ang), c[1] + rad * np.sin(ang)
    elif kind == "near_target":
        x, y = wps[-1][0] + rng.uniform(-30, 30), wps[-1][1] + rng.uniform(-30, 30)
    elif kind == "near_path_end":
        x, y = wps[-2][0] + rng.uniform(-60, 60), wps[-2][1] + rng.uniform(-60, 60)
    else:
        x, y = rng.uniform(-50.0, 1350.0), rng.uniform(-50.0, 1350.0)
    th = rng.uniform(-1.7, 1.7) if kind != "tilted" else rng.choice([-1, 1]) * rng.uniform(0.7, 1.7)
    vx, vy, w = rng.uniform(-500, 500), rng.uniform(-500, 500), rng.uniform(-8, 8)
    s[0:6] = [x, y, th, vx, vy, w]
    for bi, sign in ((1, -1.0), (2, 1.0)):
        jit = rng.normal(0.0, 0.05, 2)
        s[bi * 6:bi * 6 + 6] = [x + sign * 40.0 * np.cos(th) + jit[0], y + sign * 40.0 * np.sin(th) + jit[1],
                                th + rng.normal(0.0, 0.01), vx + rng.normal(0, 2.0), vy + rng.normal(0, 2.0),
                                w + rng.normal(0, 0.2)]
    s[18:30] = rng.normal(0.0, 3.0, 12)
    s[30] = rng.uniform(0.0, 20000.0)
    s[31] = rng.uniform(-500.0, 500.0)
    t = int(rng.integers(0, 1100)) if kind != "time_up" else 1099
    ints = np.array([t, 0, int(rng.random() < 0.2)], dtype=np.int64)
    return s, ints


def gen_crafted(de, rl_config, scen_npz, per_scn=150, seed=7):
    rec = _Rec()
    rng = np.random.default_rng(seed)
    kinds = ["random", "near_obstacle", "near_obstacle", "near_target", "near_path_end", "tilted", "time_up"]
    for si, name in enumerate(SCENARIOS):
        random.seed(3000 + si)
        env = de.Drone2dEnv(**make_cfg(rl_config, name))
        env.reset()
        circ = scn_npz_circles = scen_npz[f"{name}/circles"]
        wps = scen_npz[f"{name}/wps"]
        for i in range(per_scn):
            env.reset()
            env.step(np.zeros(2, np.float32))  # so that space.curr_dt != 0 (warm start on)
            kind = kinds[i % len(kinds)]
            pre, pre_i = _crafted_state(rng, scn_npz_circles, wps, scen_npz[f"{name}/spawn"], kind)
            set_state(env, pre, pre_i)
            env.done = False
            env.info = {k: 0 for k in env.info}
            a = rng.uniform(-1, 1, 2).astype(np.float32)
            o, r, d, info = env.step(a)
            post, post_i = get_state(env)
            rec.add(scn=si, pre=pre, pre_i=pre_i, act=a, obs=np.asarray(o, np.float64), rew=float(r),
                    done=int(bool(d)), info=info_vec(info), post=post, post_i=post_i)
        del circ
    return rec.arrays("")


def main():
    de, pp, rl_config, ts, shims = _import_reference()
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp, contextlib.redirect_stdout(io.StringIO()):
        os.chdir(tmp)  # the env globs logs/rl_model_*.zip relative to cwd (drone_2d_env.py:79)
        try:
            scen = gen_scenarios(de, pp, rl_config, ts, shims)
            probe = gen_path_probe(pp, scen, np.random.default_rng(11))
            traj = gen_traj(de, rl_config)
            crafted = gen_crafted(de, rl_config, scen)
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "scenarios.npz"), **scen)
    np.savez_compressed(os.path.join(HERE, "path_probe.npz"), **probe)
    np.savez_compressed(os.path.join(HERE, "traj.npz"), **traj)
    np.savez_compressed(os.path.join(HERE, "crafted.npz"), **crafted)
    print("traj steps", len(traj["rew"]), "resets", int(traj["is_reset"].sum()),
          "crafted steps", len(crafted["rew"]), "crafted done", int(crafted["done"].sum()))


if __name__ == "__main__":
    main()
