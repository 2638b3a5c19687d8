/* d2d_ppo.h -- C ABI of libd2d_ppo.so: one PPO minibatch update in five launches
 * (drone2d_amd.ppo.ManualStep).  The reference trains with
 * Stable-Baselines3 2.1's PPO.train (main.py:181-210); these kernels restate its loss head, the
 * backward pass through the two MLPs and clip_grad_norm_ + torch.optim.Adam over one flat
 * parameter buffer.
 *
 * All pointers are device pointers (float32 unless stated), every call is stream-ordered on
 * `stream` (a hipStream_t; NULL = the default stream) and launches without synchronising, so a
 * sequence of calls captures into a HIP graph.  Return value: 0, or a hipError_t code.
 */
#ifndef D2D_PPO_H
#define D2D_PPO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define D2D_PPO_ABI_VERSION 6  /* v6 (round 4): d2d_ppo_adam_spread / d2d_ppo_wgrad_head_adam removed */
#define D2D_PPO_HEAD_BLOCK 64  /* v1: 256 */

int32_t d2d_ppo_abi_version(void);

/* Advantage statistics of the minibatch (SB3 normalize_advantage: mean and unbiased std of
 * adv[idx[0..m)]): per-workgroup double partial sums ws[2 b] = sum, ws[2 b + 1] = sum of squares,
 * b < ceil(m / D2D_PPO_HEAD_BLOCK); d2d_ppo_mlp_backward finishes them. */
int32_t d2d_ppo_adv_stats(int32_t m, const int64_t* idx, const float* adv, double* ws, void* stream);

/* Reduces the head's partials: log_std_grad[d] = sum_b partial[b][3 + d] - ent_coef, and adds the
 * minibatch statistics to acc[0..3] (policy loss, value loss, entropy, clip fraction).  One
 * workgroup. */
int32_t d2d_ppo_head_finish(int32_t m, int32_t n_blocks, const float* partial, const float* log_std, float ent_coef,
                            float* log_std_grad, float* acc_pl, float* acc_vl, float* acc_ent, float* acc_clip,
                            void* stream);

/* clip_grad_norm_(max_norm) then one torch.optim.Adam step (betas b1, b2, eps; bias corrections
 * from the step counter *t, which is incremented) over n parameters p with gradients g and
 * moments m1, m2; g is clipped in place, as torch clips .grad.  One workgroup, n <= 16 384 (the
 * policy has ~10 k parameters). */
int32_t d2d_ppo_adam(int32_t n, float* p, float* g, float* m1, float* m2, float* t, float lr, float b1, float b2,
                     float eps, float max_norm, void* stream);

/* Weight and bias gradients of up to D2D_PPO_WGRAD_MAX linear layers in one launch (+ one reduce):
 * for problem k, g[w_off[k] + i q + j] = sum_r a_k[r][i] b_k[r][j] (i < p[k], j < q[k]; rows r < m;
 * a_k row stride lda[k], b_k ldb[k]; p, q <= 64) and g[b_off[k] + i] = sum_r a_k[r][i].  `a` and `b`
 * are host arrays of device pointers.  partial: device scratch of
 * d2d_ppo_wgrad_chunks(m) x row_len floats; g[0 .. row_len) is overwritten (entries no problem
 * covers become 0). */
#define D2D_PPO_WGRAD_MAX 8
int32_t d2d_ppo_wgrad(int32_t m, int32_t n_problems, const float* const* a, const int32_t* lda, const float* const* b,
                      const int32_t* ldb, const int32_t* p, const int32_t* q, const int32_t* w_off,
                      const int32_t* b_off, int32_t row_len, float* partial, float* g, void* stream);
/* d2d_ppo_wgrad and d2d_ppo_head_finish in two launches instead of three (the reduce's last
 * workgroup finishes the head; log_std_grad must point at two slots inside g[0 .. row_len), which
 * the reduce leaves to the head).  Added in ABI v2. */
int32_t d2d_ppo_wgrad_head(int32_t m, int32_t n_problems, const float* const* a, const int32_t* lda,
                           const float* const* b, const int32_t* ldb, const int32_t* p, const int32_t* q,
                           const int32_t* w_off, const int32_t* b_off, int32_t row_len, float* partial, float* g,
                           int32_t n_blocks, const float* head_partial, const float* log_std, float ent_coef,
                           float* log_std_grad, float* acc_pl, float* acc_vl, float* acc_ent, float* acc_clip,
                           void* stream);
int32_t d2d_ppo_wgrad_chunks(int32_t m);

/* The two MLPs (policy 27-64-64-2, value 27-64-64-1, tanh) per minibatch sample, four threads per
 * (sample, net) each owning a quarter of every layer's units.  weights: 12 device pointers, per net (policy, then value): W1 [64][27], b1 [64],
 * W2 [64][64], b2 [64], W3 [od][64], b3 [od].  bufs: 10 device pointers, per net: h1 [m][64],
 * h2 [m][64], out [m][od] (the action mean / the value), g1 [m][64], g2 [m][64].
 * mlp_forward: the rollout rows idx[0..m) of obs [.][27] through both nets (h1, h2, out) and the
 * gathered observations into xg [m][27].  mlp_backward: the loss head below (gout[0] =
 * d loss / d mean [m][2], gout[1] = d loss / d value [m]; partial[d2d_ppo_mlp_partial_rows(m)][5],
 * finished by d2d_ppo_head_finish with n_blocks = d2d_ppo_mlp_partial_rows(m)) and the hidden layers' output gradients g2, g1.
 * The head: Gaussian log-density of act under (mean, exp(log_std)), ratio = exp(logp - old_logp),
 * clipped surrogate with advantages normalised by d2d_ppo_adv_stats' partials (normalize != 0),
 * squared value error scaled by vf_coef. */
int32_t d2d_ppo_mlp_forward(int32_t m, const int64_t* idx, const float* obs, const float* const* weights,
                            float* const* bufs, float* xg, void* stream);
/* mlp_forward plus d2d_ppo_adv_stats' partials into ws from the same launch (adv != NULL; the
 * matrix-core forward's workgroups each take D2D_PPO_HEAD_BLOCK rows).  Added in ABI v2. */
int32_t d2d_ppo_mlp_forward_adv(int32_t m, const int64_t* idx, const float* obs, const float* adv,
                                const float* const* weights, float* const* bufs, float* xg, double* ws, void* stream);
int32_t d2d_ppo_mlp_partial_rows(int32_t m);
int32_t d2d_ppo_mlp_backward(int32_t m, const int64_t* idx, const float* act, const float* old_logp, const float* adv,
                             const float* ret, const float* log_std, const double* ws, int32_t normalize, float clip,
                             float vf_coef, const float* const* weights, float* const* bufs, float* const* gout,
                             float* partial, void* stream);

/* The per-epoch minibatch shuffles of one update (SB3 PPO.train: RolloutBuffer.get draws
 * np.random.permutation(buffer_size) every epoch): out[e n + i] = pi_e(i) for e < n_perm, i < n, each
 * pi_e a bijection of [0, n) -- an 8-round keyed Feistel network on the next power of two >= n, walked
 * back into [0, n) -- keyed by (seed, *counter + e).  A one-thread launch after it advances *counter
 * (one uint64 in device memory) by n_perm, so a captured graph draws new shuffles on every replay.
 * Two launches, replacing torch.randperm's sort (~0.24 ms per 1 M-sample epoch).  Added in ABI v4. */
int32_t d2d_ppo_permute(int64_t n, int32_t n_perm, uint64_t seed, uint64_t* counter, int64_t* out, void* stream);

/* One step of SB3 OnPolicyAlgorithm.collect_rollouts over n envs in one launch (ABI v4): both MLPs
 * on the observations of step t, the Gaussian action a = mean + exp(log_std) noise (stored
 * unclipped, clipped to [-1, 1] into act_env for the env), its log-density and the value into row t of
 * the rollout buffers ([T][n] rows, row t = samples t n .. t n + n - 1); for t >= 1 also step t-1's
 * env outputs (reward, done = terminated | truncated) into row t-1 and per-workgroup episode
 * statistics of step t-1.  t == T: the bootstrap value of obs, step T-1's env outputs, then
 * RolloutBuffer.compute_returns_and_advantage (GAE(gamma, gae_lambda) with the episode starts, same
 * operation order as the torch restatement) into adv_buf / ret_buf.  Time-limit bootstrapping of
 * truncated episodes is not done here (the reference never truncates). */
/* The minibatch gradient in one launch (ABI v5): what d2d_ppo_mlp_forward_adv + d2d_ppo_mlp_backward +
 * d2d_ppo_wgrad compute, with every per-sample activation and gradient kept on chip.  Workgroup
 * (x, net) handles the 64-sample chunks x, x + R, ... (R = d2d_ppo_fused_rows(m)) of rows idx[0..m) and
 * writes its net's weight / bias gradient sums into row x of wpart ([R][row_len], at offsets[6 net
 * + k] for W1, b1, W2, b2, W3, b3 of net 0 = policy, 1 = value) and its loss-head sums into row x
 * (policy) / R + x (value) of hpart ([2 R][5], d2d_ppo_mlp_backward's partial-row meaning).  ws: the
 * minibatch's d2d_ppo_adv_stats partials (normalize != 0).  d2d_ppo_grad_reduce then adds the rows
 * into g and finishes the head (log_std gradient, statistics) as d2d_ppo_wgrad_head does. */
int32_t d2d_ppo_fused_rows(int32_t m);
int32_t d2d_ppo_fused_grad(int32_t m, const int64_t* idx, const float* obs, const float* act, const float* old_logp,
                           const float* adv, const float* ret, const float* log_std, const double* ws, int32_t normalize,
                           float clip, float vf_coef, const float* const* weights, const int32_t* offsets,
                           int32_t row_len, float* wpart, float* hpart, void* stream);
int32_t d2d_ppo_grad_reduce(int32_t n_rows, int32_t row_len, const float* partial, float* g, int32_t n_blocks,
                            const float* head_partial, int32_t m, const float* log_std, float ent_coef,
                            float* log_std_grad, float* acc_pl, float* acc_vl, float* acc_ent, float* acc_clip,
                            void* stream);

typedef struct d2d_ppo_rollout {
    int32_t n;            /* envs */
    int32_t t;            /* rollout step of obs: 0 .. T */
    int32_t T;            /* rollout length */
    int32_t info_dim;     /* row length of prev_info (D2D_INFO_DIM) */
    int32_t info_totrew;  /* column of the episode return in prev_info (D2D_INFO_TOTREW) */
    float gamma;
    float gae_lambda_gamma; /* gamma * gae_lambda, rounded to float as torch rounds the scalar */
    int32_t pad;
    const float* obs;        /* [n][27] observations of step t (the env's output tensor) */
    const float* noise;      /* [n][2] N(0, 1) draws of step t (t < T) */
    const float* log_std;    /* [2] */
    const float* prev_rew;   /* step t-1's env outputs (t >= 1): reward [n] */
    const uint8_t* prev_term;   /* [n] 0 / 1 */
    const uint8_t* prev_trunc;  /* [n] 0 / 1 */
    const float* prev_info;  /* [n][info_dim], or NULL (episode returns not summed) */
    float* obs_buf;          /* [T][n][27] */
    float* act_buf;          /* [T][n][2] unclipped actions */
    float* logp_buf;         /* [T][n] */
    float* val_buf;          /* [T][n] */
    float* rew_buf;          /* [T][n] */
    uint8_t* done_buf;       /* [T][n] */
    uint8_t* start0;         /* [n] episode starts of step 0; t == T: replaced by done of step T-1 */
    float* act_env;          /* [n][2] */
    float* adv_buf;          /* [T][n] (t == T) */
    float* ret_buf;          /* [T][n] (t == T) */
    double* stats;           /* [T][ceil(n / 64)][2]: per workgroup, (episodes ended, sum of their returns) at
                                step t-1 */
} d2d_ppo_rollout;
int32_t d2d_ppo_rollout_step(const d2d_ppo_rollout* r, const float* const* weights, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* D2D_PPO_H */
