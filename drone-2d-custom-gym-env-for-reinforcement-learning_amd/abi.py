"""ctypes mirror of ``include/drone2d.h`` (the C ABI of ``libdrone2d_hip.so``).

Kept field-for-field identical to the header; ``tests/test_abi.py`` checks sizes and offsets
against a compiled probe of the header.
"""
from __future__ import annotations

import ctypes as C

ABI_VERSION = 5

MAX_WPS = 16
MAX_SEGS = MAX_WPS - 2
MAX_CIRCLES = 64
OBS_DIM = 27
ACT_DIM = 2
K_OBS = 3

# fp64 SoA state fields (D2D_S_*)
S_F, S_L, S_R, S_J = 0, 6, 12, 18
S_PATH_ERR, S_TOT_REW = 30, 31
NSTATE = 32
# int32 SoA state fields (D2D_I_*)
I_T, I_FLAGS, I_EPISODE = 0, 1, 2
NISTATE = 3
FLAG_COLLIDED, FLAG_LA_LOCK = 1, 2

# info row (D2D_INFO_*)
INFO_CA, INFO_PA, INFO_PP, INFO_COLL, INFO_REACH, INFO_AA = 0, 1, 2, 3, 4, 5
INFO_DCLOSE, INFO_STEPS, INFO_CAUSE, INFO_APE, INFO_TOTREW, INFO_REWARD = 6, 7, 8, 9, 10, 11
INFO_DIM = 12
END_COLLISION, END_REACH, END_TIMEUP, END_AA = 1, 2, 4, 8

# episode statistics (D2D_ST_*)
ST_RETURN, ST_EPISODES, ST_SUCCESS, ST_FAIL, ST_COLLISION, ST_APE, ST_LEN = range(7)
NSTATS = 8

E_OK, E_ARG, E_HIP, E_STATE, E_NOMEM = 0, 1, 2, 3, 4


class D2DCfg(C.Structure):
    _fields_ = [
        ("screen_w", C.c_double), ("screen_h", C.c_double),
        ("lookahead", C.c_double),
        ("danger_range", C.c_double), ("danger_angle", C.c_double),
        ("abs_inv_ca_min_rew", C.c_double),
        ("pa_band_edge", C.c_double), ("pa_scale", C.c_double),
        ("pp_vel_scale", C.c_double), ("pp_rew_max", C.c_double), ("pp_rew_min", C.c_double),
        ("rew_collision", C.c_double),
        ("reach_end_radius", C.c_double), ("rew_reach_end", C.c_double),
        ("aa_angle", C.c_double), ("aa_band", C.c_double), ("rew_aa", C.c_double),
        ("force_scale", C.c_double),
        ("damping", C.c_double),
        ("n_steps", C.c_int32),
        ("use_lambda", C.c_int32),
        ("auto_reset", C.c_int32),
        ("timeup_truncates", C.c_int32),
        ("env_id_base", C.c_int32),
        ("scn_pool", C.c_int32),
    ]


class D2DScn(C.Structure):
    _fields_ = [
        ("n_wps", C.c_int32), ("n_circles", C.c_int32),
        ("us", C.c_double * MAX_WPS),
        ("xa", C.c_double * MAX_SEGS), ("xb", C.c_double * MAX_SEGS), ("xc", C.c_double * MAX_SEGS),
        ("ya", C.c_double * MAX_SEGS), ("yb", C.c_double * MAX_SEGS), ("yc", C.c_double * MAX_SEGS),
        ("cx", C.c_double * MAX_CIRCLES), ("cy", C.c_double * MAX_CIRCLES), ("cr", C.c_double * MAX_CIRCLES),
        ("wp_last_x", C.c_double), ("wp_last_y", C.c_double),
        ("spawn_xmin", C.c_double), ("spawn_xmax", C.c_double),
        ("spawn_ymin", C.c_double), ("spawn_ymax", C.c_double),
        ("spawn_amin", C.c_double), ("spawn_amax", C.c_double),
    ]


class D2DCurriculum(C.Structure):
    """d2d_curriculum: the fresh curriculum generator's parameters (cfg.scn_pool = 2)."""
    _fields_ = [
        ("stage", C.c_int32), ("n_wps", C.c_int32),
        ("segment_length", C.c_double),
        ("random_path_spawn", C.c_int32), ("corner_lo", C.c_int32), ("corner_hi", C.c_int32),
        ("pad", C.c_int32),
        ("sim_num0", C.c_double), ("envs_total", C.c_double),
    ]
