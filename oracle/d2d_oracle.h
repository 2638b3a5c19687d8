/* d2d_oracle.h -- CPU parity oracle (TEST INFRASTRUCTURE ONLY, see d2d_oracle.c header).
 * Same call shapes as include/drone2d.h with host pointers and a `d2dcpu_` prefix. */
#ifndef D2D_ORACLE_H
#define D2D_ORACLE_H
#include "../include/drone2d.h"

#ifdef __cplusplus
extern "C" {
#endif
typedef struct d2dcpu d2dcpu_t;

d2dcpu_t* d2dcpu_create(const d2d_cfg* cfg, int32_t n_envs);
void d2dcpu_destroy(d2dcpu_t* h);
int32_t d2dcpu_set_scenarios(d2dcpu_t* h, const d2d_scn* scns, int32_t n_scn, const int32_t* env_scn);
int32_t d2dcpu_refresh_pool(d2dcpu_t* h, const d2d_scn* scns, int32_t n_scn);
int32_t d2dcpu_get_env_scenarios(const d2dcpu_t* h, int32_t* env_scn);
int32_t d2dcpu_reset(d2dcpu_t* h, const uint8_t* mask, uint64_t seed, float* obs);
int32_t d2dcpu_step(d2dcpu_t* h, const float* act, float* obs, float* rew, uint8_t* term,
                    uint8_t* trunc, float* info, float* term_obs);
int32_t d2dcpu_step_mt(d2dcpu_t* h, const float* act, float* obs, float* rew, uint8_t* term,
                       uint8_t* trunc, float* info, float* term_obs, int32_t nthreads);
int32_t d2dcpu_get_state(const d2dcpu_t* h, double* state, int32_t* istate);
int32_t d2dcpu_set_state(d2dcpu_t* h, const double* state, const int32_t* istate);
int32_t d2dcpu_episode_stats(d2dcpu_t* h, double* out, int32_t clear);
/* fresh curriculum (cfg.scn_pool = 2): the device protocol of d2d_set_curriculum / d2d_fresh_recipes */
int32_t d2dcpu_set_curriculum(d2dcpu_t* h, const d2d_curriculum* c);
int32_t d2dcpu_fresh_recipes(d2dcpu_t* h, int32_t* keys, int64_t* clocks, int64_t* clock, int32_t set);
int32_t d2dcpu_get_scenario_table(const d2dcpu_t* h, int32_t first, int32_t count, d2d_scn* out);
void d2dcpu_gen_curriculum(const d2d_curriculum* c, double W, double H, uint64_t seed, uint32_t gid,
                           uint32_t key, double sim, d2d_scn* s);

/* single-function probes */
void d2dcpu_path_eval(const d2d_scn* s, double u, double* x, double* y);
double d2dcpu_fminbound(const d2d_scn* s, double px, double py, double x1, double x2, double xatol,
                        int maxfun, int* nfev);
double d2dcpu_closest_u(const d2d_scn* s, double px, double py, int* nfev);
void d2dcpu_observe_state(const d2d_cfg* cfg, const d2d_scn* s, const double* st, int32_t* flags,
                          double* obs);
int32_t d2dcpu_physics_step(const d2d_cfg* cfg, const d2d_scn* s, double* st, double fL, double fR,
                            int32_t collided);
double d2dcpu_moment_box(double m, double w, double h);
void d2dcpu_spawn_uniforms(uint64_t seed, uint32_t env_id, uint32_t episode, double u[3]);
uint32_t d2dcpu_pool_pick(uint64_t seed, uint32_t env_id, uint32_t episode, uint32_t n_scn);
void d2dcpu_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
#ifdef __cplusplus
}
#endif
#endif
