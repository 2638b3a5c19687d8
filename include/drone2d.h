/*
 * drone2d.h -- C ABI of the MI355X-native batched Drone2dEnv (libdrone2d_hip.so).
 *
 * This is the drop-in boundary for the reference's hot path, ``Drone2dEnv.step()`` /
 * ``reset()`` (reference: drone_2d_custom_gym_env/drone_2d_env.py:394-615, :908-912), which the
 * reference reaches only from Python (gym.Env, SB3 SubprocVecEnv, main.py:88-101, 181-210).
 * The reference has no FFI of its own; the binding a maintainer adds is the ctypes stub shown in
 * INTEGRATION.md, and the package's ``_native.py`` is exactly that stub.
 *
 * Conventions
 *  - Plain C types only; the HIP stream is passed as an opaque ``void*`` (a hipStream_t, or NULL
 *    for the null stream).  Every call is stream-ordered on that stream; no call synchronises
 *    the device except d2d_create / d2d_set_scenarios / d2d_destroy (allocation + upload).
 *  - ``*_dev`` pointers are device pointers on the handle's device (e.g. torch.Tensor.data_ptr()).
 *  - Every entry point returns 0 on success, otherwise a D2D_E_* code; the message is in the
 *    thread-local d2d_last_error().  Numeric edge cases (e.g. the CA reward's division by
 *    d + k*R, drone_2d_env.py:503) produce IEEE inf/NaN exactly as the reference's NumPy does.
 *  - One handle per GPU per process; a handle is not re-entrant.  Multi-GPU = one process per GPU,
 *    each with its own shard of envs (see DESIGN.md "Multi-GPU").
 *
 * Units/semantics are the reference's: pixels, seconds (dt = 1/60), radians; the observation is
 * the 27-vector of drone_2d_env.py:765-773, the reward the 6-term sum of :572.
 */
#ifndef DRONE2D_H
#define DRONE2D_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define D2D_ABI_VERSION 5

#define D2D_MAX_WPS 16                    /* largest test path: 'large' has 14 waypoints   */
#define D2D_MAX_SEGS (D2D_MAX_WPS - 2)    /* QPMI2D fits n_wps-2 quadratics (predef_path.py:34) */
#define D2D_MAX_CIRCLES 64                /* largest obstacle set: 'S_corridor' has 58 circles */
#define D2D_OBS_DIM 27                    /* drone_2d_env.py:160 */
#define D2D_ACT_DIM 2                     /* drone_2d_env.py:155 */
#define D2D_K_OBS 3                       /* drone_2d_env.py:67 */

/* Per-env fp64 state, struct-of-arrays: field f of env i lives at state[f * n_envs + i].
 * Bodies are the three Chipmunk bodies of Drone.py:9-95 (frame, left motor, right motor);
 * jAcc are the accumulated impulses of the 6 PivotJoints in space.add order (Drone.py:61-95). */
enum {
    D2D_S_F = 0,      /* frame body:  px, py, angle, vx, vy, w  (fields 0..5)   */
    D2D_S_L = 6,      /* left motor:  px, py, angle, vx, vy, w  (fields 6..11)  */
    D2D_S_R = 12,     /* right motor: px, py, angle, vx, vy, w  (fields 12..17) */
    D2D_S_J = 18,     /* jAcc[k].x, jAcc[k].y for k = 0..5      (fields 18..29) */
    D2D_S_PATH_ERR = 30,  /* self.path_error   (drone_2d_env.py:589)           */
    D2D_S_TOT_REW = 31,   /* self.total_reward (drone_2d_env.py:592)           */
    D2D_NSTATE = 32
};
/* Per-env int32 state, SoA: istate[f * n_envs + i]. */
enum {
    D2D_I_T = 0,          /* self.current_time_step (drone_2d_env.py:407)              */
    D2D_I_FLAGS = 1,      /* bit0 space.collison (sticky), bit1 LA_in_last_wp (sticky) */
    D2D_I_EPISODE = 2,    /* episodes started by this env (RNG stream position)         */
    D2D_NISTATE = 3
};
#define D2D_FLAG_COLLIDED 1u
#define D2D_FLAG_LA_LOCK 2u

/* info row per env (float32, [n_envs][D2D_INFO_DIM]); keys of drone_2d_env.py:575-613 */
enum {
    D2D_INFO_CA = 0,        /* info['collision_avoidance_reward'] = CA * lambda_CA */
    D2D_INFO_PA = 1,        /* info['path_adherence']            = PA * lambda_PA */
    D2D_INFO_PP = 2,        /* info['path_progression']                        */
    D2D_INFO_COLL = 3,      /* info['collision_reward']                        */
    D2D_INFO_REACH = 4,     /* info['reach_end_reward']                        */
    D2D_INFO_AA = 5,        /* info['agressive_alpha_reward']                  */
    D2D_INFO_DCLOSE = 6,    /* info['dist_closest_obs'] (inf without obstacles) */
    D2D_INFO_STEPS = 7,     /* info['env_steps']                               */
    D2D_INFO_CAUSE = 8,     /* done causes bitmask D2D_END_* (0 while running) */
    D2D_INFO_APE = 9,       /* info['APE'] (written at done)                   */
    D2D_INFO_TOTREW = 10,   /* info['total_reward'] (written at done)          */
    D2D_INFO_REWARD = 11,   /* info['reward'] (fp32 copy of the step reward)   */
    D2D_INFO_DIM = 12
};
#define D2D_END_COLLISION 1   /* end_cond_1 */
#define D2D_END_REACH 2       /* end_cond_2 */
#define D2D_END_TIMEUP 4      /* end_cond_4 */
#define D2D_END_AA 8          /* end_cond_5 */

/* episode statistics vector (float64, D2D_NSTATS): reduced over envs by d2d_episode_stats */
enum {
    D2D_ST_RETURN = 0,    /* sum of total_reward over finished episodes        */
    D2D_ST_EPISODES = 1,  /* finished episodes                                 */
    D2D_ST_SUCCESS = 2,   /* info['n_successful_runs'] == 1                     */
    D2D_ST_FAIL = 3,      /* info['n_failed_runs'] == 1                         */
    D2D_ST_COLLISION = 4, /* info['n_collisions'] == 1                          */
    D2D_ST_APE = 5,       /* sum of APE                                        */
    D2D_ST_LEN = 6,       /* sum of episode lengths (env_steps at done)         */
    D2D_ST_PAD = 7,
    D2D_NSTATS = 8
};

/* Environment parameters: the numeric kwargs of rl_config.py:10-44 read at drone_2d_env.py:34-66
 * plus the constants hard-coded in the env (force_scale :150, damping :376-380). */
typedef struct d2d_cfg {
    double screen_w, screen_h;         /* screensize_x, screensize_y            */
    double lookahead;                  /* lookahead                             */
    double danger_range, danger_angle; /* danger_range, danger_angle (degrees)  */
    double abs_inv_ca_min_rew;         /* abs_inv_CA_min_rew                    */
    double pa_band_edge, pa_scale;     /* PA_band_edge, PA_scale                */
    double pp_vel_scale, pp_rew_max, pp_rew_min;
    double rew_collision;
    double reach_end_radius, rew_reach_end;
    double aa_angle, aa_band, rew_aa;  /* AA_angle, AA_band, rew_AA            */
    double force_scale;                /* 1000 (drone_2d_env.py:150)            */
    double damping;                    /* Space.damping; 1.0 (docs/DESIGN_HISTORY.md) */
    int32_t n_steps;                   /* max episode steps (1100)              */
    int32_t use_lambda;                /* use_Lambda                            */
    int32_t auto_reset;                /* 1: SB3 VecEnv auto-reset inside d2d_step */
    int32_t timeup_truncates;          /* 0: reference (time-up is 'terminated')   */
    int32_t env_id_base;               /* global id of env 0: the Philox spawn stream is keyed by
                                          (seed, env_id_base + i, episode), so a sharded run draws
                                          the same spawns as one big batch               */
    int32_t scn_pool;                  /* 0: env i always runs scenario env_scn[i] (test mode);
                                          1: curriculum pool -- at every reset env i draws its next
                                          scenario uniformly from the n_scn uploaded, from its
                                          Philox stream (counter (gid, episode, 2, 0));
                                          2: fresh curriculum -- every reset runs on a scenario
                                          generated on the device for that episode alone
                                          (d2d_set_curriculum), as the reference's reset does */
} d2d_cfg;

/* Curriculum generator parameters (cfg.scn_pool = 2): the kwargs the reference's curriculum reset
 * reads (rl_config.py:10-44; drone_2d_env.py:199-215, 318-372) plus the stage clock. */
typedef struct d2d_curriculum {
    int32_t stage;              /* 1..5: a fixed stage (scenario='stage_k'); 0: the sim_num schedule */
    int32_t n_wps;              /* n_wps                                                         */
    double segment_length;      /* path_segment_length                                           */
    int32_t random_path_spawn;  /* 1: corner from spawn_corners (random.randint), 0: 'DR'        */
    int32_t corner_lo, corner_hi;  /* spawn_corners: 1 DL, 2 DR, 3 UL, 4 UR                     */
    int32_t pad;
    double sim_num0;            /* schedule: sim_num = sim_num0 + clock * envs_total, clock = the  */
    double envs_total;          /* number of d2d_step calls since this d2d_set_curriculum (which   */
                                /* zeroes it), all ranks' envs: envs_total                         */
} d2d_curriculum;

/* One scenario: a QPMI2D path + circle obstacles + spawn distribution.
 * Built on the host once (test_scenarios.py:169-246, predef_path.py:20-50). */
typedef struct d2d_scn {
    int32_t n_wps;                     /* 3..D2D_MAX_WPS                      */
    int32_t n_circles;                 /* 0..D2D_MAX_CIRCLES                  */
    double us[D2D_MAX_WPS];            /* QPMI2D.us (arc length at each wp)   */
    double xa[D2D_MAX_SEGS], xb[D2D_MAX_SEGS], xc[D2D_MAX_SEGS];  /* x_params[n] = (a,b,c) */
    double ya[D2D_MAX_SEGS], yb[D2D_MAX_SEGS], yc[D2D_MAX_SEGS];  /* y_params[n] = (a,b,c) */
    double cx[D2D_MAX_CIRCLES], cy[D2D_MAX_CIRCLES], cr[D2D_MAX_CIRCLES]; /* circles (x, y, r) */
    double wp_last_x, wp_last_y;       /* wps[-1]: target and LA lock point   */
    double spawn_xmin, spawn_xmax;     /* test-mode spawn rect (drone_2d_env.py:221-311) */
    double spawn_ymin, spawn_ymax;
    double spawn_amin, spawn_amax;     /* spawn angle range (+-pi/4)          */
} d2d_scn;

typedef struct d2d_handle d2d_t;

/* Library / build identification. */
int32_t d2d_abi_version(void);
const char* d2d_last_error(void);

/* Allocate a batch of n_envs environments on HIP device `device`.  State is zeroed; call
 * d2d_set_scenarios then d2d_reset before stepping. (replaces Drone2dEnv.__init__, :33-165) */
int32_t d2d_create(const d2d_cfg* cfg, int32_t n_envs, int32_t device, d2d_t** out);
void d2d_destroy(d2d_t* h);
int32_t d2d_n_envs(const d2d_t* h);

/* Upload n_scn scenarios (host array) and the env->scenario map (host int32[n_envs], NULL = all
 * envs use scenario 0).  (replaces create_test_scenario + QPMI2D fit in init_pymunk, :218-311) */
int32_t d2d_set_scenarios(d2d_t* h, const d2d_scn* scns, int32_t n_scn, const int32_t* env_scn_host);

/* Relative step cost of each scenario of the last d2d_set_scenarios (test mode; default 1.0 each).
 * With a grouped layout (several scenarios), the groups are renumbered so that the workgroups that
 * share a CU carry a balanced load (d2d_get_group_layout; the state moves along, cached reset
 * observations are recomputed, d2d_generation changes).  Placement only: results do not depend
 * on it.
 * Synchronises. */
int32_t d2d_set_scenario_costs(d2d_t* h, const double* cost, int32_t n_scn);

/* Reset the envs whose mask byte is non-zero (mask_dev NULL = all envs) and write their
 * observation rows into obs_dev (float32 [n_envs][27]; NULL = do not write).  Spawn draws come
 * from a counter-based Philox4x32-10 stream keyed by (seed, env id, episode number), so results
 * do not depend on the batch size or the sharding.  The seed is kept for auto-resets.  Fresh
 * curriculum (cfg.scn_pool = 2): a masked reset must pass the seed of the previous full reset
 * (D2D_E_ARG otherwise: the envs left running would keep scenarios no recipe regenerates).
 * (replaces Drone2dEnv.reset, :908-912) */
int32_t d2d_reset(d2d_t* h, const uint8_t* mask_dev, uint64_t seed, float* obs_dev, void* stream);

/* One environment step for every env (replaces Drone2dEnv.step, :394-615).
 *   act_dev   float32 [n_envs][2]   (not clipped, as in the reference)
 *   obs_dev   float32 [n_envs][27]  next observation (after auto-reset, if enabled)
 *   rew_dev   float32 [n_envs]
 *   term_dev  uint8   [n_envs]      done (terminated)
 *   trunc_dev uint8   [n_envs]      time-limit truncation (always 0 unless timeup_truncates)
 *   info_dev  float32 [n_envs][D2D_INFO_DIM] or NULL
 *   term_obs_dev float32 [n_envs][27] or NULL: the pre-reset observation of envs that finished
 *             (SB3 info['terminal_observation']); rows of running envs are left untouched. */
int32_t d2d_step(d2d_t* h, const float* act_dev, float* obs_dev, float* rew_dev, uint8_t* term_dev,
                 uint8_t* trunc_dev, float* info_dev, float* term_obs_dev, void* stream);

/* Teacher forcing / checkpointing: copy the SoA state out of / into the handle.
 * state_dev: float64 [D2D_NSTATE][n_envs], istate_dev: int32 [D2D_NISTATE][n_envs]. */
int32_t d2d_get_state(d2d_t* h, double* state_dev, int32_t* istate_dev, void* stream);
int32_t d2d_set_state(d2d_t* h, const double* state_dev, const int32_t* istate_dev, void* stream);

/* Curriculum pool mode only: replace the pool by n_scn fresh scenarios (n_scn = the size given to
 * d2d_set_scenarios) without stopping the running episodes.  The handle keeps two pool halves:
 * the new scenarios go into the half not used by the current pool, resets from now on draw from it,
 * and episodes that started earlier finish on their own scenarios.  Returns D2D_E_STATE if an env
 * still runs an episode drawn before the previous refresh (refresh at most once per cfg.n_steps
 * steps).  Synchronises the device.  (The reference draws a fresh path and obstacle set at every
 * curriculum reset, drone_2d_env.py:199-215, 324-372; refreshing the pool regularly approaches
 * that distribution.) */
int32_t d2d_refresh_pool(d2d_t* h, const d2d_scn* scns, int32_t n_scn);

/* Checkpointing in curriculum pool mode (cfg.scn_pool = 1), where every reset rewrites the env's
 * scenario index: copy the per-env scenario map (int32 [n_envs], env order) out of / into the handle,
 * alongside d2d_get_state / d2d_set_state, so a restored episode continues on its own path and
 * obstacles (the reference keeps them in the env object until reset, drone_2d_env.py:199-215).
 * d2d_set_env_scenarios is for pool mode only (a static map is changed by d2d_set_scenarios, which
 * re-lays the state out) and synchronises `stream` to range-check the indices on the host. */
int32_t d2d_get_env_scenarios(d2d_t* h, int32_t* env_scn_dev, void* stream);
int32_t d2d_set_env_scenarios(d2d_t* h, const int32_t* env_scn_dev, void* stream);
/* Pool-mode checkpoints: *active_base = the table index resets draw from (0 or pool_n), *valid_mask
 * bit h = half h holds uploaded scenarios (d2d_set_env_scenarios rejects indices into an empty
 * half).  d2d_restore_pool writes both halves (2 * pool_n ABI records, read back with
 * d2d_get_scenario_table; a half whose bit is clear in valid_mask stays empty) and selects the
 * active half, so a restored batch draws and runs exactly what the saved one did.  Synchronises. */
int32_t d2d_pool_state(d2d_t* h, int32_t* active_base, int32_t* valid_mask);
int32_t d2d_restore_pool(d2d_t* h, const d2d_scn* scns, int32_t n_total, int32_t active_base, int32_t valid_mask);

/* Fresh curriculum (cfg.scn_pool = 2), the reference's curriculum reset: the episode that env i
 * starts with episode counter k runs on scenario G(seed, gid i, k, stage) -- a random 12-waypoint
 * path (predef_path.py:307-363) with its QPMI2D fit (:20-50), the stage's obstacles
 * (drone_2d_env.py:318-372, obstacles.py:58-89) and spawn -- generated on the device from a Philox
 * stream keyed by (seed, gid, k) one step ahead of the reset that needs it (after every d2d_step
 * and around d2d_reset), with the stage of the clock at generation time.  Replaces
 * d2d_set_scenarios in this mode (allocates 2 scenario slots per env; captured graphs must be
 * recaptured after it, d2d_generation changes).  */
int32_t d2d_set_curriculum(d2d_t* h, const d2d_curriculum* c);
/* Checkpointing in fresh mode: each env's two scenario slots are described by their recipe
 * (episode key, -1 = empty; clock at generation); get copies them to host int32[2 n] / int64[2 n]
 * (slot 2 i + (key & 1) of env i) and the current clock to *clock; set uploads them (and the clock)
 * and regenerates every slot from its recipe, so restored episodes continue on their own paths.
 * Synchronises the device. */
int32_t d2d_fresh_recipes(d2d_t* h, int32_t* keys, int64_t* clocks, int64_t* clock, int32_t set);
/* Copy scenario slots [first, first + count) of the device table (pool or fresh mode) to the host as
 * ABI records (parity tests hand them to the CPU oracle).  Synchronises the device. */
int32_t d2d_get_scenario_table(d2d_t* h, int32_t first, int32_t count, d2d_scn* out);
/* Bumped by every call that frees or re-allocates what a captured step graph points at
 * (d2d_set_scenarios, d2d_set_curriculum): a caller holding a captured graph re-captures it. */
int32_t d2d_generation(const d2d_t* h);

/* Reduce the per-env finished-episode accumulators into out_dev (float64 [D2D_NSTATS]) with a
 * fixed-order (bitwise reproducible) block reduction; clear != 0 zeroes the accumulators after. */
int32_t d2d_episode_stats(d2d_t* h, double* out_dev, int32_t clear, void* stream);

/* Device arithmetic self-check (no reference counterpart): runs n seeded random cases of one of the
 * kernels' shortcut fp64 routines against the IEEE operation on the current device and stores the
 * number of bitwise mismatches in *mismatches (host pointer).  which: D2D_SELFTEST_*. */
#define D2D_SELFTEST_SQRT 0      /* range-limited sqrt (Brent distance) vs sqrt()        */
#define D2D_SELFTEST_DIV 1       /* range-limited division (parabolic step) vs '/'       */
#define D2D_SELFTEST_RECIP_DIV 2 /* division by a precomputed reciprocal (path blend)    */
int32_t d2d_selftest(int32_t which, int64_t n, uint64_t seed, uint64_t* mismatches);

/* The internal slot layout d2d_set_scenarios builds for a static env->scenario map with several
 * scenarios (host-only, no device needed; for tests and diagnostics, no reference counterpart):
 * envs sorted by (scenario, id) are cut into ceil(n/64) groups of 64 slots; slot_env[64 g + l] is
 * the env in slot l of group g (-1: padding at the end), group_scn[g] the group's scenario, or
 * -(s + 2) if it straddles exactly scenarios s and s + 1, or -1 if it holds three or more.  slot_env: int32[ceil(n/64) * 64], group_scn: int32[ceil(n/64)].
 * Returns the number of groups, or -1 on bad arguments (d2d_last_error says which). */
int32_t d2d_group_layout(int32_t n, const int32_t* env_scn, int32_t n_scn, int32_t* slot_env, int32_t* group_scn);
/* The slot layout the handle uses now (slot_env [ns], group_scn [n_groups], as d2d_group_layout
 * describes them): d2d_group_layout's groups renumbered by d2d_set_scenario_costs so that each CU's
 * co-resident workgroups carry a balanced load (no effect on results).  Returns the number of
 * groups, 0 for the identity layout (outputs untouched), -1 on error.  Added in ABI v5. */
int32_t d2d_get_group_layout(d2d_t* h, int32_t* slot_env, int32_t* group_scn);
/* The renumbering itself, host-only (tests): d2d_group_layout's groups dealt over n_cu CUs by
 * cost[n_scn] -- what d2d_set_scenario_costs installs on a device with n_cu compute units (n_cu not a
 * multiple of 8, or more groups than 4 x n_cu: d2d_group_layout's order).  Added in ABI v5. */
int32_t d2d_balanced_group_layout(int32_t n, const int32_t* env_scn, int32_t n_scn, const double* cost, int32_t n_cu,
                                  int32_t* slot_env, int32_t* group_scn);

/* Error codes */
#define D2D_OK 0
#define D2D_E_ARG 1
#define D2D_E_HIP 2
#define D2D_E_STATE 3
#define D2D_E_NOMEM 4

#ifdef __cplusplus
}
#endif
#endif /* DRONE2D_H */
