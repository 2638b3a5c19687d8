"""Environment kwargs: the same dict surface as the reference's ``rl_config.py``.

``Drone2dEnv`` in the reference reads 29 required keys by subscript
(``drone_2d_env.py:34-66``), so a missing key raises ``KeyError``; ``make_cfg`` keeps that
behaviour.  Render keys are accepted and ignored (rendering is out of scope), and
``initial_throw`` / ``n_fall_steps`` are accepted and inert exactly as in the reference, where
``initial_movement()`` (``drone_2d_env.py:917-946``) is never called.
"""
from __future__ import annotations

import math

from .abi import D2DCfg

# rl_config.py:5-8
RL_CONFIG = {
    "total_timesteps": 9000000,
    "ent_coef": 0.01,
}

# rl_config.py:10-44 (values of the snapshot; runs 17/19/20 used a few different ones, see
# best_models_config_and_res/run*/env_train_config.txt)
ENV_TRAIN_CONFIG = {
    "render_sim": False,
    "render_path": False,
    "render_shade": False,
    "render_text": False,
    "shade_distance": 75,
    "n_steps": 1100,
    "n_fall_steps": 5,
    "change_target": False,
    "initial_throw": True,
    "random_path_spawn": True,
    "path_segment_length": 100,
    "n_wps": 12,
    "screensize_x": 1300,
    "screensize_y": 1300,
    "lookahead": 220,
    "spawn_corners": (1, 4),
    "danger_range": 150,
    "danger_angle": 20,
    "abs_inv_CA_min_rew": 1 / 8,
    "PA_band_edge": 40,
    "PA_scale": 2,
    "PP_vel_scale": 0.08,
    "PP_rew_max": 2.5,
    "PP_rew_min": -1,
    "rew_collision": -50,
    "reach_end_radius": 20,
    "rew_reach_end": 30,
    "AA_angle": math.pi / 2,
    "AA_band": math.pi / 4,
    "rew_AA": -1,
    "use_Lambda": True,
    "mode": "test",
    "scenario": "large",
}

# rl_config.py:63-79 (visualisation variant)
ENV_TEST_CONFIG = dict(ENV_TRAIN_CONFIG, render_sim=True, render_path=True, render_shade=True,
                       render_text=True, initial_throw=False, n_fall_steps=0)

# keys read by Drone2dEnv.__init__ (drone_2d_env.py:34-66), in the reference's order
REQUIRED_KEYS = (
    "render_sim", "render_path", "render_shade", "shade_distance", "render_text", "n_steps",
    "n_fall_steps", "change_target", "initial_throw", "random_path_spawn", "path_segment_length",
    "n_wps", "screensize_x", "screensize_y", "lookahead", "spawn_corners", "danger_range",
    "danger_angle", "abs_inv_CA_min_rew", "PA_band_edge", "PA_scale", "PP_vel_scale", "PP_rew_max",
    "PP_rew_min", "rew_collision", "reach_end_radius", "rew_reach_end", "AA_angle", "AA_band",
    "rew_AA", "use_Lambda", "mode", "scenario",
)

TEST_SCENARIOS = ("perpendicular", "parallel", "S_parallel", "corridor", "S_corridor", "large", "impossible")
CURRICULUM_STAGES = ("stage_1", "stage_2", "stage_3", "stage_4", "stage_5")

# Relative step-kernel cost of each test scenario (us per step at 65 536 envs of that scenario alone,
# MI355X, docs/DESIGN_HISTORY.md "Every test scenario alone"): the grouped layout deals its 64-env groups over the
# CUs by these weights (d2d_set_scenario_costs; placement only, never results).
SCENARIO_STEP_COST = {"perpendicular": 31.2, "parallel": 31.3, "S_parallel": 43.8, "corridor": 32.4,
                      "S_corridor": 45.1, "large": 41.5, "impossible": 32.4}

FORCE_SCALE = 1000.0   # drone_2d_env.py:150
SPACE_DAMPING = 1.0    # body.damping = 0.9 (drone_2d_env.py:376-380) has no effect in pymunk 6


def make_cfg(kwargs: dict, *, auto_reset: bool = True, timeup_truncates: bool = False,
             damping: float = SPACE_DAMPING, env_id_base: int = 0) -> D2DCfg:
    """Build the C ``d2d_cfg`` from reference-style kwargs (KeyError on a missing key)."""
    for k in REQUIRED_KEYS:
        kwargs[k]  # noqa: B018 -- same KeyError as drone_2d_env.py:34-66
    c = D2DCfg()
    c.screen_w = float(kwargs["screensize_x"])
    c.screen_h = float(kwargs["screensize_y"])
    c.lookahead = float(kwargs["lookahead"])
    c.danger_range = float(kwargs["danger_range"])
    c.danger_angle = float(kwargs["danger_angle"])
    c.abs_inv_ca_min_rew = float(kwargs["abs_inv_CA_min_rew"])
    c.pa_band_edge = float(kwargs["PA_band_edge"])
    c.pa_scale = float(kwargs["PA_scale"])
    c.pp_vel_scale = float(kwargs["PP_vel_scale"])
    c.pp_rew_max = float(kwargs["PP_rew_max"])
    c.pp_rew_min = float(kwargs["PP_rew_min"])
    c.rew_collision = float(kwargs["rew_collision"])
    c.reach_end_radius = float(kwargs["reach_end_radius"])
    c.rew_reach_end = float(kwargs["rew_reach_end"])
    c.aa_angle = float(kwargs["AA_angle"])
    c.aa_band = float(kwargs["AA_band"])
    c.rew_aa = float(kwargs["rew_AA"])
    c.force_scale = FORCE_SCALE
    c.damping = float(damping)
    c.n_steps = int(kwargs["n_steps"])
    c.use_lambda = 1 if kwargs["use_Lambda"] is True else 0
    c.auto_reset = 1 if auto_reset else 0
    c.timeup_truncates = 1 if timeup_truncates else 0
    c.env_id_base = int(env_id_base)
    return c
