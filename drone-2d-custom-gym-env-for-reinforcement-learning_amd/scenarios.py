"""Host-side scenario construction: QPMI2D path fit, the 7 test scenarios and spawn rectangles.

This is reset-time work (run once per scenario, uploaded to HBM by ``d2d_set_scenarios``); it is
not on the per-step hot path.  Every function restates the reference with the same NumPy calls in
the same order, so the uploaded coefficients are bit-identical to the reference's
(``tests/test_scenarios.py`` checks them against ``tests/golden/scenarios.npz``).

Reference anchors:
  QPMI2D fit            predef_path.py:9-50
  QPMI2D.__call__       predef_path.py:88-142   (host copy, used only to place obstacles)
  calculate_gradient    predef_path.py:145-188
  get_direction_angle   predef_path.py:216-223
  waypoints             test_scenarios.py:87-167
  obstacles             test_scenarios.py:4-84
  create_test_scenario  test_scenarios.py:169-246
  spawn rectangles      drone_2d_env.py:221-311
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .abi import MAX_CIRCLES, MAX_SEGS, MAX_WPS, D2DScn


class QPMIPath:
    """QPMI2D: blended piecewise quadratics through waypoints (predef_path.py:9-142)."""

    def __init__(self, waypoints):
        self.waypoints = np.asarray(waypoints)
        diff = np.diff(self.waypoints, axis=0)
        seg_lengths = np.cumsum(np.sqrt(np.sum(diff ** 2, axis=1)))
        self.us = np.array([0, *seg_lengths[:]])
        self.length = self.us[-1]
        self.x_params = []
        self.y_params = []
        for n in range(1, len(self.waypoints) - 1):
            wp_prev, wp_n, wp_next = self.waypoints[n - 1], self.waypoints[n], self.waypoints[n + 1]
            u_prev, u_n, u_next = self.us[n - 1], self.us[n], self.us[n + 1]
            U_n = np.vstack([np.hstack([u_prev ** 2, u_prev, 1]),
                             np.hstack([u_n ** 2, u_n, 1]),
                             np.hstack([u_next ** 2, u_next, 1])])
            self.x_params.append(np.linalg.inv(U_n).dot(np.array([wp_prev[0], wp_n[0], wp_next[0]])))
            self.y_params.append(np.linalg.inv(U_n).dot(np.array([wp_prev[1], wp_n[1], wp_next[1]])))

    def _u_index(self, u):
        n = 0
        while n < len(self.us) - 1:
            if u <= self.us[n + 1]:
                break
            n += 1
        return n

    def _mu(self, u):
        n = self._u_index(u)
        return (u - self.us[n]) / (self.us[n + 1] - self.us[n]), (self.us[n + 1] - u) / (self.us[n + 1] - self.us[n])

    def __call__(self, u):
        xp, yp, us = self.x_params, self.y_params, self.us
        if u >= us[0] and u <= us[1]:
            x = xp[0][0] * u ** 2 + xp[0][1] * u + xp[0][2]
            y = yp[0][0] * u ** 2 + yp[0][1] * u + yp[0][2]
        elif (u >= us[-2] - 0.001 and u <= us[-1]) or self._u_index(u) == len(us) - 1:
            x = xp[-1][0] * u ** 2 + xp[-1][1] * u + xp[-1][2]
            y = yp[-1][0] * u ** 2 + yp[-1][1] * u + yp[-1][2]
        else:
            n = self._u_index(u)
            mu_r, mu_f = self._mu(u)
            x1 = xp[n - 1][0] * u ** 2 + xp[n - 1][1] * u + xp[n - 1][2]
            y1 = yp[n - 1][0] * u ** 2 + yp[n - 1][1] * u + yp[n - 1][2]
            x2 = xp[n][0] * u ** 2 + xp[n][1] * u + xp[n][2]
            y2 = yp[n][0] * u ** 2 + yp[n][1] * u + yp[n][2]
            x = mu_r * x2 + mu_f * x1
            y = mu_r * y2 + mu_f * y1
        return np.array([x, y])

    def gradient(self, u):
        xp, yp, us = self.x_params, self.y_params, self.us
        if u >= us[0] and u <= us[1]:
            return np.array([xp[0][0] * u * 2 + xp[0][1], yp[0][0] * u * 2 + yp[0][1]])
        if u >= us[-2]:
            return np.array([xp[-1][0] * u * 2 + xp[-1][1], yp[-1][0] * u * 2 + yp[-1][1]])
        n = self._u_index(u)
        mu_r, mu_f = self._mu(u)
        dx1 = xp[n - 1][0] * u * 2 + xp[n - 1][1]
        dy1 = yp[n - 1][0] * u * 2 + yp[n - 1][1]
        dx2 = xp[n][0] * u * 2 + xp[n][1]
        dy2 = yp[n][0] * u * 2 + yp[n][1]
        return np.array([mu_r * dx2 + mu_f * dx1, mu_r * dy2 + mu_f * dy1])

    def direction_angle(self, u):
        dx, dy = self.gradient(u)[:]
        return np.arctan2(dy, dx)


# --------------------------------------------------------------------------------------------
def scen_waypoints(nwaypoints, distance, scen, screen_x=None, screen_y=None, offset=0):
    """generate_scen_waypoints_2d, test_scenarios.py:87-167."""
    waypoints = []
    if scen in ("perpendicular", "parallel", "impossible", "corridor"):
        x1 = screen_x / 2 - distance * (nwaypoints - 1) / 2
        y1 = screen_y / 2 + (offset if scen == "corridor" else 0)
        waypoints = [np.array([x1, y1])]
        for i in range(nwaypoints - 1):
            azimuth = 0
            waypoints.append(np.array([waypoints[i][0] + distance * np.cos(azimuth),
                                       waypoints[i][1] + distance * np.sin(azimuth)]))
    elif scen in ("S_parallel", "S_corridor"):
        x1 = screen_x / 10 if scen == "S_parallel" else screen_x / 7
        y1 = screen_y / 2 + (offset if scen == "S_corridor" else 0)
        waypoints = [np.array([x1, y1])]
        phase = np.pi / 4
        for i in range(nwaypoints - 1):
            azimuth = -phase if i % 2 == 0 else phase
            waypoints.append(np.array([waypoints[i][0] + distance * np.cos(azimuth),
                                       waypoints[i][1] + distance * np.sin(azimuth)]))
    elif scen == "large":
        nwaypoints = int(screen_x / 100)
        obs_rad = screen_x / 5
        margin = 80
        circle_to_follow_radius = obs_rad + margin
        circumference = 2 * np.pi * circle_to_follow_radius
        half_circumference = circumference / 2
        circ_seg_lengths = half_circumference / (nwaypoints - 3)
        distance = screen_x / 10
        x1 = screen_x / 2 - obs_rad - margin - distance
        y1 = screen_y / 2 - margin
        waypoints = [np.array([x1, y1]), np.array([x1 + distance, y1])]
        for i in range(1, nwaypoints - 1):
            azimuth = np.pi / 2 - (i - 1) * np.pi / (nwaypoints - 3)
            waypoints.append(np.array([waypoints[i][0] + circ_seg_lengths * np.cos(azimuth),
                                       waypoints[i][1] + circ_seg_lengths * np.sin(azimuth)]))
        waypoints.append(np.array([waypoints[-1][0] + distance, waypoints[-1][1]]))
    return np.array(waypoints)


def scen_obstacles(n, scen, path: QPMIPath, obs_size, screen_x=None, screen_y=None):
    """generate_scen_obstacles, test_scenarios.py:4-84. Returns [(x, y, r), ...]."""
    out = []
    if scen == "perpendicular":
        half = path.length / 2
        path_angle = path.direction_angle(half)
        x, y = path(half)
        on_path = np.array([x, y])
        start = n * obs_size - obs_size
        for i in range(0, n):
            p = on_path + (start - i * obs_size * 2) * np.array([np.cos(path_angle - np.pi / 2),
                                                                   np.sin(path_angle - np.pi / 2)])
            out.append((p[0], p[1], obs_size))
    elif scen in ("parallel", "S_parallel"):
        space_occupied = n * obs_size * 2
        offset = (path.length - space_occupied) / 2 - (obs_size if scen == "parallel" else 0)
        for i in range(1, n + 1):
            x, y = path(offset + i * obs_size * 2)
            out.append((x, y, obs_size))
    elif scen in ("corridor", "S_corridor"):
        if scen == "corridor":
            n = 10
        free_end_space = 100
        space_to_fill = path.length - free_end_space * 2
        obs_size = space_to_fill / (n * 2)
        for i in range(1, n):
            x, y = path(i * obs_size * 2 + free_end_space)
            out.append((x, y, obs_size))
    elif scen == "impossible":
        r_goal = 100
        obs_size = 2 * np.pi * r_goal / (n * 2)
        path_angle = path.direction_angle(path.length)
        x, y = path(path.length)
        on_path = np.array([x, y])
        pi_update = 2 * np.pi / n
        for i in range(1, n + 1):
            p = on_path + r_goal * np.array([np.cos(path_angle - i * pi_update), np.sin(path_angle - i * pi_update)])
            out.append((p[0], p[1], obs_size))
    elif scen == "large":
        out.append((screen_x / 2, screen_y / 2, obs_size))
    return out


# spawn rectangles (xmin, xmax, ymin, ymax) as functions of the screen, drone_2d_env.py:221-311
def _spawn_rect(scen, W, H):
    table = {
        "perpendicular": (50, W / 2 - 100, 50, H - 100),
        "parallel": (50, W / 2 - 300, 150, H - 300),
        "S_parallel": (50, W / 2 - 300, 150, H - 300),
        "corridor": (50, W / 2 - 400, 150, H - 300),
        "S_corridor": (50, W / 2 - 450, 150, H - 300),
        "large": (50, W / 2 - W / 4 - 50, 150, H - 300),
        "impossible": (50, W / 2, 150, H - 300),
    }
    return table[scen]


@dataclass
class Scenario:
    name: str
    wps: np.ndarray
    path: QPMIPath
    circles: np.ndarray                      # [n, 3] (x, y, r)
    spawn: tuple                             # (xmin, xmax, ymin, ymax)
    spawn_angle: tuple = (-np.pi / 4, np.pi / 4)
    meta: dict = field(default_factory=dict)

    def to_c(self) -> D2DScn:
        return scenario_to_c(self)


def create_test_scenario(scen: str, screen_x: int, screen_y: int, offset: int = 0, obs_size: int = 30,
                         n_wps: int = 10, n_obs: int = 6) -> Scenario:
    """create_test_scenario, test_scenarios.py:169-246 (+ the env's spawn rectangle)."""
    circles = []
    if scen == "perpendicular":
        wps = scen_waypoints(n_wps, 100, scen, screen_x, screen_y)
        path = QPMIPath(wps)
        circles = scen_obstacles(6, scen, path, 20)
    elif scen == "parallel":
        wps = scen_waypoints(n_wps, 100, scen, screen_x, screen_y)
        path = QPMIPath(wps)
        circles = scen_obstacles(n_obs, scen, path, obs_size)
    elif scen == "S_parallel":
        wps = scen_waypoints(6, 300, scen, screen_x, screen_y)
        path = QPMIPath(wps)
        circles = scen_obstacles(20, scen, path, 15)
    elif scen == "corridor":
        wps = scen_waypoints(n_wps, 100, scen, screen_x, screen_y)
        path = QPMIPath(wps)
        po = QPMIPath(scen_waypoints(n_wps, 100, scen, screen_x, screen_y, 100))
        mo = QPMIPath(scen_waypoints(n_wps, 100, scen, screen_x, screen_y, -100))
        circles = scen_obstacles(n_obs, scen, po, obs_size) + scen_obstacles(n_obs, scen, mo, obs_size)
    elif scen == "S_corridor":
        wps = scen_waypoints(7, 200, scen, screen_x, screen_y)
        path = QPMIPath(wps)
        po = QPMIPath(scen_waypoints(7, 200, scen, screen_x, screen_y, 150))
        mo = QPMIPath(scen_waypoints(7, 200, scen, screen_x, screen_y, -150))
        circles = scen_obstacles(30, scen, po, None) + scen_obstacles(30, scen, mo, None)
    elif scen == "impossible":
        wps = scen_waypoints(n_wps, 100, scen, screen_x, screen_y)
        path = QPMIPath(wps)
        circles = scen_obstacles(20, scen, path, obs_size)
    elif scen == "large":
        wps = scen_waypoints(n_wps, 100, scen, screen_x, screen_y)
        path = QPMIPath(wps)
        circles = scen_obstacles(1, scen, path, screen_x / 5, screen_x, screen_y)
    else:
        raise ValueError(f"unknown test scenario {scen!r}")
    circ = np.array([[float(c[0]), float(c[1]), float(c[2])] for c in circles], dtype=np.float64).reshape(-1, 3)
    return Scenario(scen, wps, path, circ, tuple(float(v) for v in _spawn_rect(scen, screen_x, screen_y)))


def free_flight(scen: Scenario) -> Scenario:
    """BASELINE config 2: the same path with no obstacles (obs[8:17] = (1,0,0)x3, CA = 0)."""
    return Scenario(scen.name + "_free", scen.wps, scen.path, np.zeros((0, 3)), scen.spawn, scen.spawn_angle)


def scenario_to_c(s: Scenario) -> D2DScn:
    n = len(s.path.us)
    if not (3 <= n <= MAX_WPS):
        raise ValueError(f"path with {n} waypoints: supported 3..{MAX_WPS}")
    if len(s.circles) > MAX_CIRCLES:
        raise ValueError(f"{len(s.circles)} circles: supported up to {MAX_CIRCLES}")
    c = D2DScn()
    c.n_wps = n
    c.n_circles = len(s.circles)
    for i in range(n):
        c.us[i] = float(s.path.us[i])
    for k in range(n - 2):
        c.xa[k], c.xb[k], c.xc[k] = (float(v) for v in s.path.x_params[k])
        c.ya[k], c.yb[k], c.yc[k] = (float(v) for v in s.path.y_params[k])
    assert n - 2 <= MAX_SEGS
    for i, (x, y, r) in enumerate(s.circles):
        c.cx[i], c.cy[i], c.cr[i] = float(x), float(y), float(r)
    c.wp_last_x, c.wp_last_y = float(s.wps[-1][0]), float(s.wps[-1][1])
    c.spawn_xmin, c.spawn_xmax, c.spawn_ymin, c.spawn_ymax = s.spawn
    c.spawn_amin, c.spawn_amax = (float(v) for v in s.spawn_angle)
    return c
