// Fused element-wise parts of one PPO minibatch update (include/d2d_ppo.h; drone2d_amd.ppo.ManualStep).
// SB3 2.1 PPO.train's loss head, the tanh backward and clip_grad_norm_ + Adam, each as one launch
// instead of the ~80 small element-wise kernels the same math costs as separate torch ops.  The
// GEMMs of the two 27-64-64 MLPs stay on hipBLASLt (torch.addmm / bmm).
#include <hip/hip_runtime.h>

#include <cmath>

#include "d2d_ppo.h"

namespace {

constexpr float HALF_LOG_2PI = 0.91893853320467274f;  // 0.5 * log(2 pi)

// sum over the 64 lanes of a wave (every lane gets the total)
__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// sum over a workgroup of `nt` threads (nt a multiple of 64, <= 1024); every thread gets the total
__device__ __forceinline__ double block_sum(double x, double* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    x = wave_sum(x);
    __syncthreads();  // red may still be read by a previous call
    if (lane == 0) red[w] = x;
    __syncthreads();
    double t = 0.0;
    for (int k = 0; k < nw; ++k) t += red[k];
    return t;
}

// per-workgroup (sum, sum of squares) of adv[idx[i]] in double: ws[2 b], ws[2 b + 1]
__global__ __launch_bounds__(D2D_PPO_HEAD_BLOCK) void adv_stats_kernel(int m, const int64_t* __restrict__ idx,
                                                                       const float* __restrict__ adv,
                                                                       double* __restrict__ ws) {
    __shared__ double red[D2D_PPO_HEAD_BLOCK / 64];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const double x = i < m ? (double)adv[idx[i]] : 0.0;
    const double s = block_sum(x, red), q = block_sum(x * x, red);
    if (threadIdx.x == 0) {
        ws[2 * blockIdx.x] = s;
        ws[2 * blockIdx.x + 1] = q;
    }
}

__global__ __launch_bounds__(D2D_PPO_HEAD_BLOCK) void head_kernel(int m, const int64_t* idx, const float* mean,
                                                                  const float* value, const float* act,
                                                                  const float* old_logp, const float* adv,
                                                                  const float* ret, const float* log_std,
                                                                  const double* ws, int normalize, float clip,
                                                                  float vf_coef, float* g_mean, float* g_v,
                                                                  float* partial) {
    __shared__ double red[D2D_PPO_HEAD_BLOCK / 64];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float adv_mean = 0.0f, adv_inv = 1.0f;
    if (normalize) {
        // mean and unbiased std of the minibatch's advantages from adv_stats_kernel's partials
        const int nb = gridDim.x;
        double s = 0.0, q = 0.0;
        for (int b = threadIdx.x; b < nb; b += blockDim.x) {
            s += ws[2 * b];
            q += ws[2 * b + 1];
        }
        s = block_sum(s, red);
        q = block_sum(q, red);
        const double mu = s / m, var = (q - s * mu) / (m > 1 ? m - 1 : 1);
        adv_mean = (float)mu;
        adv_inv = 1.0f / ((float)sqrt(var > 0.0 ? var : 0.0) + 1e-8f);
    }
    double p_min = 0.0, p_err = 0.0, p_clip = 0.0, p_l0 = 0.0, p_l1 = 0.0;
    if (i < m) {
        const int64_t j = idx[i];
        const float ls0 = log_std[0], ls1 = log_std[1];
        const float is0 = expf(-ls0), is1 = expf(-ls1);
        const float z0 = (act[2 * j] - mean[2 * i]) * is0, z1 = (act[2 * j + 1] - mean[2 * i + 1]) * is1;
        const float logp = (-0.5f * z0 * z0 - ls0 - HALF_LOG_2PI) + (-0.5f * z1 * z1 - ls1 - HALF_LOG_2PI);
        const float a = normalize ? (adv[j] - adv_mean) * adv_inv : adv[j];
        const float ratio = expf(logp - old_logp[j]);
        const float s1 = a * ratio, s2 = a * fminf(fmaxf(ratio, 1.0f - clip), 1.0f + clip);
        // d(-mean min(s1, s2)) / d logp: the unclipped branch's a * ratio where it is the minimum
        // (ties: both branches' derivatives are a * ratio)
        const float g_lp = (s1 <= s2) ? a * ratio * (-1.0f / m) : 0.0f;
        g_mean[2 * i] = g_lp * z0 * is0;
        g_mean[2 * i + 1] = g_lp * z1 * is1;
        const float err = ret[j] - value[i];
        g_v[i] = err * (-2.0f * vf_coef / m);
        p_min = fminf(s1, s2);
        p_err = (double)err * err;
        p_clip = fabsf(ratio - 1.0f) > clip ? 1.0 : 0.0;
        p_l0 = (double)g_lp * (z0 * z0 - 1.0f);
        p_l1 = (double)g_lp * (z1 * z1 - 1.0f);
    }
    const double v0 = block_sum(p_min, red), v1 = block_sum(p_err, red), v2 = block_sum(p_clip, red);
    const double v3 = block_sum(p_l0, red), v4 = block_sum(p_l1, red);
    if (threadIdx.x == 0) {
        float* o = partial + (size_t)blockIdx.x * 5;
        o[0] = (float)v0;
        o[1] = (float)v1;
        o[2] = (float)v2;
        o[3] = (float)v3;
        o[4] = (float)v4;
    }
}

__global__ __launch_bounds__(256) void head_finish_kernel(int m, int nb, const float* partial, const float* log_std,
                                                          float ent_coef, float* ls_grad, float* acc_pl,
                                                          float* acc_vl, float* acc_ent, float* acc_clip) {
    __shared__ double red[4];
    double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
#pragma unroll
        for (int k = 0; k < 5; ++k) s[k] += partial[(size_t)b * 5 + k];
    }
    double t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] = block_sum(s[k], red);
    if (threadIdx.x == 0) {
        ls_grad[0] = (float)t[3] - ent_coef;
        ls_grad[1] = (float)t[4] - ent_coef;
        *acc_pl += (float)(-t[0] / m);
        *acc_vl += (float)(t[1] / m);
        *acc_clip += (float)(t[2] / m);
        *acc_ent += (0.5f + HALF_LOG_2PI + log_std[0]) + (0.5f + HALF_LOG_2PI + log_std[1]);
    }
}

__global__ void tanh_grad_kernel(int64_t n, const float* h, float* g) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const float x = h[i];
        g[i] = g[i] * (1.0f - x * x);
    }
}

constexpr int ADAM_THREADS = 1024, ADAM_PER_THREAD = 16;  // n <= 16 384 parameters
__global__ __launch_bounds__(ADAM_THREADS) void adam_kernel(int n, float* __restrict__ p, float* __restrict__ g,
                                                            float* __restrict__ m1, float* __restrict__ m2,
                                                            float* __restrict__ t, float lr, float b1, float b2,
                                                            float eps, float max_norm) {
    __shared__ double red[ADAM_THREADS / 64];
    float gv[ADAM_PER_THREAD];
    double q = 0.0;
#pragma unroll
    for (int k = 0; k < ADAM_PER_THREAD; ++k) {
        const int i = threadIdx.x + k * ADAM_THREADS;
        gv[k] = i < n ? g[i] : 0.0f;
        q += (double)gv[k] * gv[k];
    }
    const double norm = sqrt(block_sum(q, red));
    // torch.nn.utils.clip_grad_norm_: clip_coef = max_norm / (norm + 1e-6), clamped to 1
    const float coef = fminf((float)(max_norm / (norm + 1e-6)), 1.0f);
    const float step = t[0] + 1.0f;
    const float bc1 = 1.0f - powf(b1, step), bc2s = sqrtf(1.0f - powf(b2, step));
    const float lr_t = lr / bc1;
#pragma unroll
    for (int k = 0; k < ADAM_PER_THREAD; ++k) {
        const int i = threadIdx.x + k * ADAM_THREADS;
        if (i < n) {
            const float gi = gv[k] * coef;
            g[i] = gi;
            const float a0 = m1[i], v0 = m2[i];
            const float a = a0 + (1.0f - b1) * (gi - a0);  // exp_avg.lerp_(grad, 1 - beta1)
            const float v = v0 * b2 + (1.0f - b2) * gi * gi;
            m1[i] = a;
            m2[i] = v;
            p[i] -= a * lr_t / (sqrtf(v) / bc2s + eps);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) t[0] = step;
}

// ---------------------------------------------------------------------------- weight gradients
// Every weight / bias gradient of the two MLPs in one launch: problem k (blockIdx.y) is
// W_k.grad = a_k^T b_k (a_k [m][p_k] the layer-output gradient, b_k [m][q_k] the layer input, p, q <=
// 64) and bias_k.grad = sum_rows a_k.  Workgroup (c, k) sums rows [c R, c R + R) in 64-row LDS tiles,
// each thread a 4 x 4 block of the output, and writes its partial sums at the gradient's offsets in
// a row of `partial` ([n_chunks][row_len], the flat gradient buffer's layout); wgrad_reduce_kernel
// adds the rows up into the gradient buffer.
struct WgradProblem {
    const float* a;
    const float* b;
    int lda, ldb, p, q, w_off, b_off;
};
struct WgradProblems {
    WgradProblem k[D2D_PPO_WGRAD_MAX];
};
constexpr int WG_TILE = 64, WG_ROWS = 256;

__global__ __launch_bounds__(256) void wgrad_kernel(WgradProblems P, int m, int row_len, float* __restrict__ partial) {
    __shared__ float ta[WG_TILE][64 + 4];
    __shared__ float tb[WG_TILE][64 + 4];
    const WgradProblem& pr = P.k[blockIdx.y];
    const int p = pr.p, q = pr.q;
    const int pi = (threadIdx.x >> 4) * 4, qi = (threadIdx.x & 15) * 4;  // this thread's 4 x 4 block
    float acc[4][4] = {};
    float bsum[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const int r0 = blockIdx.x * WG_ROWS, r1 = min(m, r0 + WG_ROWS);
    for (int rt = r0; rt < r1; rt += WG_TILE) {
        __syncthreads();
        for (int e = threadIdx.x; e < WG_TILE * 64; e += 256) {
            const int r = e >> 6, c = e & 63, row = rt + r;
            ta[r][c] = (row < r1 && c < p) ? pr.a[(size_t)row * pr.lda + c] : 0.0f;
            tb[r][c] = (row < r1 && c < q) ? pr.b[(size_t)row * pr.ldb + c] : 0.0f;
        }
        __syncthreads();
        if (pi < p && qi < q) {
#pragma unroll 8
            for (int r = 0; r < WG_TILE; ++r) {
                const float4 av = *reinterpret_cast<const float4*>(&ta[r][pi]);
                const float4 bv = *reinterpret_cast<const float4*>(&tb[r][qi]);
                const float a4[4] = {av.x, av.y, av.z, av.w}, b4[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
                for (int x = 0; x < 4; ++x) {
#pragma unroll
                    for (int y = 0; y < 4; ++y) acc[x][y] += a4[x] * b4[y];
                }
                if (qi == 0) {
#pragma unroll
                    for (int x = 0; x < 4; ++x) bsum[x] += a4[x];
                }
            }
        }
    }
    float* out = partial + (size_t)blockIdx.x * row_len;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
        if (pi + x >= p) continue;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            if (qi + y < q) out[pr.w_off + (pi + x) * q + qi + y] = acc[x][y];
        }
        if (qi == 0) out[pr.b_off + pi + x] = bsum[x];
    }
}

// g[e] = sum over the n_chunks rows of partial[.][e], e < row_len
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(int n_chunks, int row_len, const float* __restrict__ partial,
                                                           float* __restrict__ g) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= row_len) return;
    float s = 0.0f;
    for (int c = 0; c < n_chunks; ++c) s += partial[(size_t)c * row_len + e];
    g[e] = s;
}

inline int32_t rc(hipError_t e) { return e == hipSuccess ? 0 : (int32_t)e; }

}  // namespace

extern "C" {

int32_t d2d_ppo_abi_version(void) { return D2D_PPO_ABI_VERSION; }

int32_t d2d_ppo_adv_stats(int32_t m, const int64_t* idx, const float* adv, double* ws, void* stream) {
    if (m <= 0) return 0;
    const int nb = (m + D2D_PPO_HEAD_BLOCK - 1) / D2D_PPO_HEAD_BLOCK;
    hipLaunchKernelGGL(adv_stats_kernel, dim3(nb), dim3(D2D_PPO_HEAD_BLOCK), 0, (hipStream_t)stream, m, idx, adv, ws);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_head(int32_t m, const int64_t* idx, const float* mean, const float* value, const float* act,
                     const float* old_logp, const float* adv, const float* ret, const float* log_std,
                     const double* ws, int32_t normalize, float clip, float vf_coef, float* g_mean, float* g_v,
                     float* partial, void* stream) {
    if (m <= 0) return 0;
    const int nb = (m + D2D_PPO_HEAD_BLOCK - 1) / D2D_PPO_HEAD_BLOCK;
    hipLaunchKernelGGL(head_kernel, dim3(nb), dim3(D2D_PPO_HEAD_BLOCK), 0, (hipStream_t)stream, m, idx, mean, value,
                       act, old_logp, adv, ret, log_std, ws, normalize, clip, vf_coef, g_mean, g_v, partial);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_head_finish(int32_t m, int32_t n_blocks, const float* partial, const float* log_std, float ent_coef,
                            float* log_std_grad, float* acc_pl, float* acc_vl, float* acc_ent, float* acc_clip,
                            void* stream) {
    if (m <= 0) return 0;
    hipLaunchKernelGGL(head_finish_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, m, n_blocks, partial, log_std,
                       ent_coef, log_std_grad, acc_pl, acc_vl, acc_ent, acc_clip);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_tanh_grad(int64_t n, const float* h, float* g, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(tanh_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, h,
                       g);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_adam(int32_t n, float* p, float* g, float* m1, float* m2, float* t, float lr, float b1, float b2,
                     float eps, float max_norm, void* stream) {
    if (n <= 0) return 0;
    if (n > ADAM_THREADS * ADAM_PER_THREAD) return (int32_t)hipErrorInvalidValue;
    hipLaunchKernelGGL(adam_kernel, dim3(1), dim3(ADAM_THREADS), 0, (hipStream_t)stream, n, p, g, m1, m2, t, lr, b1,
                       b2, eps, max_norm);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_wgrad(int32_t m, int32_t n_problems, const float* const* a, const int32_t* lda, const float* const* b,
                      const int32_t* ldb, const int32_t* p, const int32_t* q, const int32_t* w_off,
                      const int32_t* b_off, int32_t row_len, float* partial, float* g, void* stream) {
    if (m <= 0 || n_problems <= 0) return 0;
    if (n_problems > D2D_PPO_WGRAD_MAX) return (int32_t)hipErrorInvalidValue;
    WgradProblems P{};
    for (int k = 0; k < n_problems; ++k) {
        if (p[k] < 1 || p[k] > 64 || q[k] < 1 || q[k] > 64) return (int32_t)hipErrorInvalidValue;
        P.k[k] = WgradProblem{a[k], b[k], lda[k], ldb[k], p[k], q[k], w_off[k], b_off[k]};
    }
    const int nc = (m + WG_ROWS - 1) / WG_ROWS;
    hipLaunchKernelGGL(wgrad_kernel, dim3(nc, n_problems), dim3(256), 0, (hipStream_t)stream, P, m, row_len, partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int32_t)e;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((row_len + 255) / 256), dim3(256), 0, (hipStream_t)stream, nc,
                       row_len, partial, g);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_wgrad_chunks(int32_t m) { return (m + WG_ROWS - 1) / WG_ROWS; }

}  // extern "C"
