"""Curriculum reset generator: the reference's ``mode == 'curriculum'`` episodes.

In the reference every reset of a curriculum env draws a fresh random 12-waypoint path
(``generate_random_waypoints_2d``, predef_path.py:307-363, from one of four screen corners,
drone_2d_env.py:199-215), fits QPMI2D, and places obstacles by stage (drone_2d_env.py:324-372,
``generate_obstacles_around_path`` obstacles.py:58-89).  The schedule is the env's checkpoint-step
counter ``sim_num`` (stage_1 < 700k, stage_2 < 1M, stage_3 < 1.6M, stage_4 < 2M, then stage_5) or
an explicit ``scenario='stage_k'``.

Here generation stays host-side (reset-time work, with the reference's NumPy / ``random`` calls in
the reference's order, so a generator seeded like the reference reproduces its scenarios bit for
bit -- tests/test_curriculum.py pins it against the reference's own functions).  A *pool* of P
scenarios is generated per stage and uploaded once; at every (auto-)reset the kernel draws the
env's next pool entry from its Philox stream keyed by (seed, global env id, episode), so each
episode gets an independent uniformly chosen path + obstacle set.  The spawn point is the path's
first waypoint (stage 2: uniform in [100, W-100] x [100, H-100]); the spawn angle U(-pi/4, pi/4)
is drawn in-kernel as for the test scenarios.
"""
from __future__ import annotations

import random

import numpy as np

from .scenarios import QPMIPath, Scenario

CORNERS = {1: "DL", 2: "DR", 3: "UL", 4: "UR"}


def random_waypoints(nwaypoints, distance, scen, screen_x, screen_y, rs: np.random.RandomState) -> np.ndarray:
    """generate_random_waypoints_2d (predef_path.py:307-363) on an explicit RandomState."""
    if scen == "DL":
        x1, y1 = rs.uniform(100, 180), rs.uniform(100, 180)
        lo, hi = 0, np.pi / 2
    elif scen == "UL":
        x1, y1 = rs.uniform(100, 180), rs.uniform(screen_y - 180, screen_y - 100)
        lo, hi = 0, -np.pi / 2
    elif scen == "DR":
        x1, y1 = rs.uniform(screen_x - 180, screen_x - 100), rs.uniform(100, 180)
        lo, hi = np.pi / 2, np.pi
    elif scen == "UR":
        x1, y1 = rs.uniform(screen_x - 180, screen_x - 100), rs.uniform(screen_y - 180, screen_y - 100)
        lo, hi = -np.pi / 2, -np.pi
    else:
        raise ValueError(scen)
    waypoints = [np.array([x1, y1])]
    for i in range(nwaypoints - 1):
        azimuth = rs.uniform(lo, hi)
        x = waypoints[i][0] + distance * np.cos(azimuth)
        y = waypoints[i][1] + distance * np.sin(azimuth)
        waypoints.append(np.array([x, y]))
    return np.array(waypoints)


def obstacles_around_path(n, path: QPMIPath, mean, std, rs: np.random.RandomState, on_path=False) -> list:
    """generate_obstacles_around_path (obstacles.py:58-89): list of (x, y, r)."""
    out = []
    num = 0
    L = path.length
    while num < n:
        u_obs = rs.uniform(0.20 * L, 0.90 * L)
        path_angle = path.direction_angle(u_obs)
        dist = rs.normal(mean, std)
        x, y = path(u_obs)
        on = np.array([x, y])
        pos = on + dist * np.array([np.cos(path_angle - np.pi / 2), np.sin(path_angle - np.pi / 2)])
        size = rs.uniform(10, 50)
        if np.linalg.norm(pos - on) > size + 10 and not on_path:
            out.append((pos[0], pos[1], size))
            num += 1
        elif on_path:
            out.append((on[0], on[1], size))
            num += 1
    return out


def stage_for_sim_num(sim_num: int) -> tuple[str, float | None]:
    """(stage, obstacle spawn chance) of the reference's step-counter schedule (:326-372); the
    chance is the linear ramp of stages 3 and 4 (None where the stage has no draw)."""
    if 0 <= sim_num < 700000:
        return "stage_1", None
    if 700000 < sim_num < 1000000:
        return "stage_2", None
    if 1000000 < sim_num < 1600000:
        return "stage_3", (sim_num - 1000000) * (0.6 - 0.2) / (1600000 - 1000000) + 0.2
    if 1600000 < sim_num < 2000000:
        return "stage_4", (sim_num - 1600000) * (1 - 0.6) / (2000000 - 1600000) + 0.6
    if sim_num > 2000000:
        return "stage_5", None
    # exactly 700 000 / 1e6 / 1.6e6 / 2e6 (and negative counts) match no branch in the reference,
    # no drone is created and the env fails with AttributeError (SURVEY.md §8(b) Errors)
    raise ValueError(f"sim_num {sim_num} falls in a gap of the reference's curriculum schedule")


def curriculum_scenario(stage: str, kwargs: dict, rs: np.random.RandomState, py: random.Random,
                        spawn_chance: float | None = None) -> Scenario:
    """One reset of a curriculum env (drone_2d_env.py:199-215, 318-372) with the reference's draws:
    ``py`` stands in for Python's ``random`` (corner, angle, stage-2 spawn), ``rs`` for
    ``np.random`` (path, obstacle chance, obstacles)."""
    W, H = kwargs["screensize_x"], kwargs["screensize_y"]
    if kwargs.get("random_path_spawn", True) is True:
        a, b = kwargs["spawn_corners"]
        scen = CORNERS[py.randint(a, b)]
    else:
        scen = "DR"
    wps = random_waypoints(kwargs["n_wps"], kwargs["path_segment_length"], scen, W, H, rs)
    path = QPMIPath(wps)
    py.uniform(-np.pi / 4, np.pi / 4)  # angle_rand (:322); the kernel draws its own spawn angle
    x1, y1 = float(wps[0][0]), float(wps[0][1])
    spawn = (x1, x1, y1, y1)
    circles = []
    if stage == "stage_1":
        pass
    elif stage == "stage_2":
        py.uniform(100, W - 100)
        py.uniform(100, H - 100)
        spawn = (100.0, float(W - 100), 100.0, float(H - 100))
    elif stage == "stage_3":
        chance = 0.6 if spawn_chance is None else spawn_chance
        if rs.binomial(1, chance) == 1:
            circles = obstacles_around_path(1, path, 0, 100, rs, on_path=False)
    elif stage == "stage_4":
        chance = 1 if spawn_chance is None else spawn_chance
        if rs.binomial(1, chance) == 1:
            circles = obstacles_around_path(1, path, 0, 0, rs, on_path=True)
    elif stage == "stage_5":
        n_obs = rs.normal(1, 4)
        if n_obs < 0 and n_obs > -3:
            n_obs = 1
        if n_obs < -3:
            n_obs = 0
        if n_obs != 0:
            circles = obstacles_around_path(n_obs, path, 0, 100, rs)
            circles.append(obstacles_around_path(1, path, 0, 0, rs, on_path=True)[0])
    else:
        raise ValueError(f"unknown curriculum stage {stage!r}")
    circ = np.array([[float(c[0]), float(c[1]), float(c[2])] for c in circles], dtype=np.float64).reshape(-1, 3)
    return Scenario(stage, wps, path, circ, spawn, meta={"corner": scen})


def curriculum_pool(stage: str, kwargs: dict, n: int, seed: int = 0, spawn_chance: float | None = None,
                    max_circles: int = 64) -> list[Scenario]:
    """n consecutive curriculum resets from one seeded stream (the pool the kernel samples from).
    Stage 5 can draw more obstacles than the device table holds (n_obs ~ N(1, 4)); such rare draws
    (P(n_obs > 63) < 1e-50) would raise in scenario_to_c."""
    rs = np.random.RandomState(seed)
    py = random.Random(seed)
    return [curriculum_scenario(stage, kwargs, rs, py, spawn_chance) for _ in range(n)]


__all__ = ["random_waypoints", "obstacles_around_path", "stage_for_sim_num", "curriculum_scenario",
           "curriculum_pool", "CORNERS"]
