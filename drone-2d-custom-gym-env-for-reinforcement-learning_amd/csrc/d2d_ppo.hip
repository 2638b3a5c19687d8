// One PPO minibatch update in seven launches (include/d2d_ppo.h; drone2d_amd.ppo.ManualStep): SB3 2.1
// PPO.train's loss, its gradient through the policy and value MLPs (27-64-64 tanh), clip_grad_norm_
// and Adam, instead of ~190 autograd / optimiser kernels.
#include <hip/hip_runtime.h>

#include <cmath>

#include "d2d_ppo.h"

namespace {

constexpr float HALF_LOG_2PI = 0.91893853320467274f;  // 0.5 * log(2 pi)
typedef float f32x16 __attribute__((ext_vector_type(16)));  // a 32 x 32 f32 MFMA accumulator

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

// block_sum of N values at once (one barrier pair); red holds N x (threads / 64) doubles
template <int N>
__device__ __forceinline__ void block_sum_n(double (&x)[N], double* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = wave_sum(x[k]);
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < N; ++k) red[k * nw + w] = x[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; ++k) {
        double t = 0.0;
        for (int j = 0; j < nw; ++j) t += red[k * nw + j];
        x[k] = t;
    }
}

// per-workgroup (sum, sum of squares) of adv[idx[i]] in double: ws[2 b], ws[2 b + 1]
__global__ __launch_bounds__(D2D_PPO_HEAD_BLOCK) void adv_stats_kernel(int m, const int64_t* __restrict__ idx,
                                                                       const float* __restrict__ adv,
                                                                       double* __restrict__ ws) {
    __shared__ double red[2 * (D2D_PPO_HEAD_BLOCK / 64)];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const double x = i < m ? (double)adv[idx[i]] : 0.0;
    double sq[2] = {x, x * x};
    block_sum_n(sq, red);
    if (threadIdx.x == 0) {
        ws[2 * blockIdx.x] = sq[0];
        ws[2 * blockIdx.x + 1] = sq[1];
    }
}

// the head's partial rows finished by one 256-thread workgroup (head_finish_kernel, or the last
// workgroup of wgrad_reduce_kernel)
struct HeadArgs {
    int m, nb;
    const float* partial;  // nullptr: no head work
    const float* log_std;
    float ent_coef;
    float* ls_grad;
    float *acc_pl, *acc_vl, *acc_ent, *acc_clip;
};
__device__ __forceinline__ void head_finish_body(const HeadArgs& H) {
    __shared__ double red[5 * 4];
    const int m = H.m, nb = H.nb;
    const float* partial = H.partial;
    double t[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    int b = threadIdx.x;
    for (; b + 3 * 256 < nb; b += 4 * 256) {  // four rows' loads in flight
        float v[4][5];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < 5; ++k) v[u][k] = partial[(size_t)(b + u * 256) * 5 + k];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int k = 0; k < 5; ++k) t[k] += v[u][k];
    }
    for (; b < nb; b += 256) {
#pragma unroll
        for (int k = 0; k < 5; ++k) t[k] += partial[(size_t)b * 5 + k];
    }
    block_sum_n(t, red);
    if (threadIdx.x == 0) {
        H.ls_grad[0] = (float)t[3] - H.ent_coef;
        H.ls_grad[1] = (float)t[4] - H.ent_coef;
        *H.acc_pl += (float)(-t[0] / m);
        *H.acc_vl += (float)(t[1] / m);
        *H.acc_clip += (float)(t[2] / m);
        *H.acc_ent += (0.5f + HALF_LOG_2PI + H.log_std[0]) + (0.5f + HALF_LOG_2PI + H.log_std[1]);
    }
}
__global__ __launch_bounds__(256) void head_finish_kernel(HeadArgs H) { head_finish_body(H); }

// ------------------------------------------------------------------ per-sample MLP passes
// blockIdx.y = 0: the policy net (27-64-64 tanh -> 2), 1: the value net (-> 1); the activations are
// rows of [m][64] arrays.
struct MlpNet {
    const float* w1;  // [64][27]
    const float* b1;  // [64]
    const float* w2;  // [64][64]
    const float* b2;  // [64]
    const float* w3;  // [od][64]
    const float* b3;  // [od]
    float* h1;        // [m][64]
    float* h2;        // [m][64]
    float* out;       // [m][od]: the action mean (od = 2) or the value (od = 1)
    float* g1;        // [m][64] layer-1 output gradient (backward)
    float* g2;        // [m][64]
    float* gout;      // [m][od] d loss / d out
    int od;
};
struct MlpPair {
    MlpNet net[2];
};
constexpr int MLP_BLOCK = 256, OBS = 27, HID = 64;

// TPS threads per (sample, net): thread t of a workgroup serves sample t / TPS of the workgroup's
// MLP_SPB and owns output units [UNITS (t % TPS), UNITS (t % TPS + 1)) of every layer; the layer
// inputs of a sample (x, h1; g2 in the backward pass) are an LDS column all its threads read.
constexpr int TPS = 4, MLP_SPB = MLP_BLOCK / TPS, UNITS = HID / TPS;

// (A VALU forward, one thread per (sample, net) quarter with the weights staged in LDS, ran 42.5 us
// per 32 768-sample minibatch against 25 us for the matrix-core kernel below; removed in round 4.)

// The forward pass on the matrix cores (v_mfma_f32_32x32x2_f32): a workgroup takes FM_TILES = 2
// tiles of FM_SPB = 32 samples and both nets; wave w computes the 32 (samples) x 32 (units) tile
// [net w / 2, units 32 (w % 2) ..] of each hidden layer, D[i = sample][j = unit] = sum_k A[i][k] B[k][j]
// with A = the layer input (LDS, one sample per lane) and B = W^T, whose 46 operand values per lane
// (W's row j = a lane) are staged once through LDS into registers.  The tile's lane holds unit j and
// 16 samples, so h1 goes through LDS (as the next layer's A operand, and to global memory as row
// stores) and so does h2 (the output layers are 64-term dot products per (output row, sample), one
// thread each, weights in LDS).  Measured per 32768-sample minibatch (rocprofv3): 1 tile per
// workgroup 29.8 us, 2 tiles 25.4 us, 4 tiles 35.0 us (one workgroup per CU).
constexpr int FM_SPB = 32, FM_TILES = 2, XS = OBS + 2, HS = HID + 1;  // LDS row strides: bank spread
// tanh for the matrix-core forward: |x| < 0.25 an odd Taylor polynomial (next term
// < 3e-8 relative), else (1 - t) / (1 + t) with t = exp(-2 |x|) from v_exp_f32 and v_rcp_f32 (no
// cancellation: 1 - t >= 0.39): a few ulp, 15 instructions instead of the library's ~60, which made
// the hidden layers' activations the longest part of a forward workgroup.
__device__ __forceinline__ float ftanh(float x) {
    const float ax = fabsf(x), x2 = x * x;
    const float p = x * (1.0f + x2 * (-0.333333333f + x2 * (0.133333333f + x2 * (-0.0539682540f + x2 * 0.0218694885f))));
    const float t = __builtin_amdgcn_exp2f(ax * -2.88539008f);  // exp(-2 |x|)
    const float r = (1.0f - t) * __builtin_amdgcn_rcpf(1.0f + t);
    return ax < 0.25f ? p : copysignf(r, x);
}
// h1 or h2 of a 32-sample tile (both nets), LDS -> global as 16-byte row-contiguous stores: 4 per
// thread instead of 16 dword column stores per lane (the MFMA's C/D layout holds a unit's column),
// which made the forward store-issue-bound.
__device__ __forceinline__ void store_tile(const MlpPair& P, int s0, int m, const float (*hs)[FM_SPB][HS], int tid,
                                           bool second) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int c = q * 256 + tid, n = c >> 9, r = (c >> 4) & 31, k = (c & 15) * 4;
        if (s0 + r < m) {
            const float* src = &hs[n][r][k];
            float* dst = (second ? P.net[n].h2 : P.net[n].h1) + (size_t)(s0 + r) * HID + k;
            *reinterpret_cast<float4*>(dst) = make_float4(src[0], src[1], src[2], src[3]);
        }
    }
}
__device__ void rollout_epilogue(const d2d_ppo_rollout& R, int m, const float (*outs)[FM_TILES * FM_SPB]);
// diagnostic builds only (-DD2D_PPO_STAMPS, tools/ubench_ppo_fwd.py --stamps): s_memtime at the
// forward's phase boundaries, lane 0 of every wave, [workgroup][wave][8]
#ifdef D2D_PPO_STAMPS
__device__ uint64_t* d2d_ppo_stamp_buf;
#define PPO_STAMP(k)                                                                                  \
    do {                                                                                              \
        if (d2d_ppo_stamp_buf && (threadIdx.x & 63) == 0)                                             \
            d2d_ppo_stamp_buf[(((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + (threadIdx.x >> 6)) * 8 + (k)] = \
                __builtin_amdgcn_s_memtime();                                                         \
    } while (0)
#else
#define PPO_STAMP(k) \
    do {             \
    } while (0)
#endif
// RO: the rollout step (d2d_ppo_rollout_step): rows are the envs in order (idx == nullptr), h1 / h2
// stay on chip, the outputs go to LDS for the action / GAE epilogue instead of to P.net[].out
template <bool RO>
__device__ __forceinline__ void mlp_forward_mfma_body(const MlpPair& P, int m, const int64_t* __restrict__ idx,
                                                      const float* __restrict__ obs, float* __restrict__ xg,
                                                      const float* __restrict__ adv, double* __restrict__ ws,
                                                      const d2d_ppo_rollout* R) {
    // One LDS region, used first to stage both nets' W1 and W2 (read with coalesced loads: the
    // register operands below gathered straight from global memory touch 32 cache lines per
    // instruction, which made the kernel address-bound), then for the inputs and hidden tiles.
    constexpr int WST1 = HID * OBS, WSTN = WST1 + HID * HS;  // staged floats per net (W2 rows padded)
    static_assert(FM_TILES * FM_SPB * XS + 2 * FM_SPB * HS <= 2 * WSTN, "LDS union");
    __shared__ float ubuf[2 * WSTN];
    float(*xs)[XS] = reinterpret_cast<float(*)[XS]>(ubuf);
    float(*hs)[FM_SPB][HS] = reinterpret_cast<float(*)[FM_SPB][HS]>(ubuf + FM_TILES * FM_SPB * XS);
    __shared__ int64_t rows[FM_TILES * FM_SPB];
    __shared__ float w3s[4][HID + 1];  // output rows of both nets (od0 + od1 <= 4), bias in column HID
    const int sb = blockIdx.x * FM_TILES * FM_SPB, tid = threadIdx.x, od0 = P.net[0].od;
    const int w = tid >> 6, lane = tid & 63, ci = lane & 31, h = lane >> 5;
    const int net = w >> 1, j0 = (w & 1) * 32;
    const MlpNet& N = P.net[net];
    PPO_STAMP(0);
    {
        constexpr int NWE = 2 * WST1 + 2 * HID * HID, NWI = (NWE + 255) / 256;
        float wv[NWI];
#pragma unroll
        for (int c = 0; c < NWI; ++c) {
            const int e = c * 256 + tid;
            if (e < 2 * WST1) {
                const int n = e >= WST1;
                wv[c] = P.net[n].w1[e - n * WST1];
            } else if (e < NWE) {
                const int f = e - 2 * WST1, n = f >> 12;
                wv[c] = P.net[n].w2[f & 4095];
            }
        }
#pragma unroll
        for (int c = 0; c < NWI; ++c) {
            const int e = c * 256 + tid;
            if (e < 2 * WST1) {
                const int n = e >= WST1;
                ubuf[n * WSTN + e - n * WST1] = wv[c];
            } else if (e < NWE) {
                const int f = e - 2 * WST1, n = f >> 12, g = f & 4095;
                ubuf[n * WSTN + WST1 + (g >> 6) * HS + (g & 63)] = wv[c];
            }
        }
    }
    {
        const int orow = tid >> 6, j = tid & 63, on = orow >= od0, r = orow - on * od0;
        if (orow < od0 + P.net[1].od) {
            w3s[orow][j] = P.net[on].w3[r * HID + j];
            if (j == 0) w3s[orow][HID] = P.net[on].b3[r];
        }
    }
    if (tid < FM_TILES * FM_SPB) rows[tid] = sb + tid < m ? (RO ? (int64_t)(sb + tid) : idx[sb + tid]) : -1;
    __shared__ float outs[RO ? 3 : 1][FM_TILES * FM_SPB];  // RO: mean (2 rows) and value per sample
    const float b1 = N.b1[j0 + ci], b2 = N.b2[j0 + ci];
    __syncthreads();  // weights staged, rows
    PPO_STAMP(1);
    static_assert(FM_TILES * FM_SPB == D2D_PPO_HEAD_BLOCK, "one advantage partial per workgroup");
    if (adv != nullptr && tid < 64) {  // d2d_ppo_adv_stats' partials of this workgroup's 64 rows
        const int64_t r = rows[tid];
        const double x = r >= 0 ? (double)adv[r] : 0.0;
        const double s1 = wave_sum(x), s2 = wave_sum(x * x);
        if (tid == 0) {
            ws[2 * blockIdx.x] = s1;
            ws[2 * blockIdx.x + 1] = s2;
        }
    }
    constexpr int NX = FM_TILES * FM_SPB * OBS, NI = (NX + 255) / 256;
    float xv[NI];  // this thread's share of the minibatch's observation rows (gathered early)
#pragma unroll
    for (int c = 0; c < NI; ++c) {
        const int e = c * 256 + tid, sl = e / OBS, k = e % OBS;
        const int64_t r = e < NX ? rows[sl] : -1;
        xv[c] = r >= 0 ? obs[r * OBS + k] : 0.0f;
    }
    // the B operands stay in registers for the whole kernel: lane (ci, h) of wave w holds
    // W[j0 + ci][2 t + h] for every k step t of both layers (14 + 32 VGPRs)
    float w1r[(OBS + 1) / 2], w2r[HID / 2];
#pragma unroll
    for (int t = 0; t < (OBS + 1) / 2; ++t)
        w1r[t] = 2 * t + h < OBS ? ubuf[net * WSTN + (j0 + ci) * OBS + 2 * t + h] : 0.0f;
#pragma unroll
    for (int t = 0; t < HID / 2; ++t) w2r[t] = ubuf[net * WSTN + WST1 + (j0 + ci) * HS + 2 * t + h];
    __syncthreads();  // every wave holds its operands: the region becomes xs / hs
    PPO_STAMP(2);
    if (tid < FM_TILES * FM_SPB) xs[tid][OBS] = 0.0f;  // the k padding of the 28-deep layer-1 product
    {
#pragma unroll
        for (int c = 0; c < NI; ++c) {
            const int e = c * 256 + tid, sl = e / OBS, k = e % OBS;
            if (e < NX) {
                xs[sl][k] = xv[c];
                // the gathered minibatch observations, for the weight gradients
                if (xg != nullptr && sb + sl < m) xg[(size_t)sb * OBS + e] = xv[c];
            }
        }
    }
    for (int tile = 0; tile < FM_TILES; ++tile) {
        const int s0 = sb + tile * FM_SPB;
        __syncthreads();  // staging done / the previous tile's outputs have read hs
        PPO_STAMP(3 + tile);
        // layer 1 (k = 27 inputs, padded to 28)
        f32x16 acc = {};
#pragma unroll
        for (int t = 0; t < (OBS + 1) / 2; ++t)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xs[tile * FM_SPB + ci][2 * t + h], w1r[t], acc, 0, 0, 0);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int i = (v & 3) + 8 * (v >> 2) + 4 * h;  // sample of register v (C/D map)
            const float y = ftanh(acc[v] + b1);
            hs[net][i][j0 + ci] = y;
        }
        __syncthreads();
        if (!RO) store_tile(P, s0, m, hs, tid, false);
        // layer 2
        acc = f32x16{};
#pragma unroll
        for (int t = 0; t < HID / 2; ++t)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(hs[net][ci][2 * t + h], w2r[t], acc, 0, 0, 0);
        __syncthreads();  // every wave has read h1 before h2 overwrites it
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int i = (v & 3) + 8 * (v >> 2) + 4 * h;
            const float y = ftanh(acc[v] + b2);
            hs[net][i][j0 + ci] = y;
        }
        __syncthreads();
        if (!RO) store_tile(P, s0, m, hs, tid, true);
        // output layers: thread t -> (output row t / 32 of both nets' od0 + od1 rows, sample t % 32),
        // weights and biases from LDS
        if (tid < (od0 + P.net[1].od) * FM_SPB) {
            const int orow = tid / FM_SPB, sl = tid % FM_SPB, i = s0 + sl, on = orow >= od0;
            const int r = orow - on * od0;
            float o = w3s[orow][HID];
#pragma unroll 16
            for (int j = 0; j < HID; ++j) o += w3s[orow][j] * hs[on][sl][j];
            if (RO)
                outs[orow][tile * FM_SPB + sl] = o;
            else if (i < m)
                P.net[on].out[(size_t)i * P.net[on].od + r] = o;
        }
    }
    PPO_STAMP(5);
    if (RO) {
        __syncthreads();
        if (tid < FM_TILES * FM_SPB) rollout_epilogue(*R, m, outs);  // wave 0: one env per lane
    }
    PPO_STAMP(6);
}
__global__ __launch_bounds__(256) void mlp_forward_mfma_kernel(MlpPair P, int m, const int64_t* __restrict__ idx,
                                                               const float* __restrict__ obs,
                                                               float* __restrict__ xg,
                                                               const float* __restrict__ adv,
                                                               double* __restrict__ ws) {
    mlp_forward_mfma_body<false>(P, m, idx, obs, xg, adv, ws, nullptr);
}

// The rollout step's epilogue, lane l of wave 0 = env sb + l.  Operation order as the torch
// restatement (ppo.py _rollout_body / compute_gae), without contraction: the GAE recursion gives the
// bits torch computes from the same rewards, values and dones.
__device__ void rollout_epilogue(const d2d_ppo_rollout& R, int m, const float (*outs)[FM_TILES * FM_SPB]) {
#pragma clang fp contract(off)
    const int l = threadIdx.x, i = blockIdx.x * (FM_TILES * FM_SPB) + l, n = m, t = R.t, T = R.T;
    const bool ok = i < n;
    float rew_p = 0.0f;
    uint8_t d_p = 0;
    if (t > 0) {  // step t-1's env outputs
        double fin = 0.0, ret = 0.0;
        if (ok) {
            rew_p = R.prev_rew[i];
            d_p = (R.prev_term[i] | R.prev_trunc[i]) != 0;
            R.rew_buf[(size_t)(t - 1) * n + i] = rew_p;
            R.done_buf[(size_t)(t - 1) * n + i] = d_p;
            if (d_p) {
                fin = 1.0;
                if (R.prev_info != nullptr) ret = (double)R.prev_info[(size_t)i * R.info_dim + R.info_totrew];
            }
        }
        fin = wave_sum(fin);
        ret = wave_sum(ret);
        if (l == 0) {
            double* st = R.stats + ((size_t)(t - 1) * gridDim.x + blockIdx.x) * 2;
            st[0] = fin;
            st[1] = ret;
        }
    }
    if (!ok) return;
    const float v = outs[2][l];
    if (t < T) {
        const size_t row = (size_t)t * n + i;
        const float ls0 = R.log_std[0], ls1 = R.log_std[1];
        const float mu0 = outs[0][l], mu1 = outs[1][l];
        const float a0 = mu0 + expf(ls0) * R.noise[2 * i], a1 = mu1 + expf(ls1) * R.noise[2 * i + 1];
        const float z0 = (a0 - mu0) * expf(-ls0), z1 = (a1 - mu1) * expf(-ls1);
        const float lp = ((-0.5f * z0 * z0 - ls0) - HALF_LOG_2PI) + ((-0.5f * z1 * z1 - ls1) - HALF_LOG_2PI);
        R.act_buf[2 * row] = a0;
        R.act_buf[2 * row + 1] = a1;
        R.logp_buf[row] = lp;
        R.val_buf[row] = v;
        R.act_env[2 * i] = fminf(fmaxf(a0, -1.0f), 1.0f);
        R.act_env[2 * i + 1] = fminf(fmaxf(a1, -1.0f), 1.0f);
        return;
    }
    // t == T: GAE (RolloutBuffer.compute_returns_and_advantage); episode start of step s + 1 = done of s
    const float g = R.gamma, gl = R.gae_lambda_gamma;
    float last_gae = 0.0f, next_v = v;
    for (int s = T - 1; s >= 0; --s) {
        const size_t row = (size_t)s * n + i;
        const float vs = R.val_buf[row];
        const float rs = s == T - 1 ? rew_p : R.rew_buf[row];
        const float nnt = 1.0f - (float)(s == T - 1 ? d_p : R.done_buf[row]);
        const float delta = (rs + g * next_v * nnt) - vs;
        last_gae = delta + gl * nnt * last_gae;
        R.adv_buf[row] = last_gae;
        R.ret_buf[row] = last_gae + vs;
        next_v = vs;
    }
    R.start0[i] = d_p;
}
__global__ __launch_bounds__(256) void rollout_step_kernel(MlpPair P, int m, float* __restrict__ xg, d2d_ppo_rollout R) {
    mlp_forward_mfma_body<true>(P, m, nullptr, R.obs, xg, nullptr, nullptr, &R);
}

// ---------------------------------------------------------------- per-epoch minibatch shuffles
__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // the splitmix64 finaliser
    z ^= z >> 30;
    z *= 0xbf58476d1ce4e5b9ull;
    z ^= z >> 27;
    z *= 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
// x = (a << wb) | b on `bits` bits; a round maps (a, b) -> (b, a ^ F(b)) and swaps the widths, so
// every round (and the network) is a bijection of [0, 2^bits)
__device__ __forceinline__ uint64_t feistel(uint64_t x, int bits, const uint64_t (&key)[8]) {
    int wa = bits / 2, wb = bits - wa;
    uint64_t a = x >> wb, b = x & ((1ull << wb) - 1);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const uint64_t f = mix64(b ^ key[r]) & ((1ull << wa) - 1);
        const uint64_t na = b;
        b = a ^ f;
        a = na;
        const int tw = wa;
        wa = wb;
        wb = tw;
    }
    return (a << wb) | b;
}
__global__ __launch_bounds__(256) void permute_kernel(int64_t n, int bits, uint64_t seed,
                                                      const uint64_t* __restrict__ counter,
                                                      int64_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t e = counter[0] + blockIdx.y;
    uint64_t key[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) key[r] = mix64(seed ^ mix64(e * 8 + r + 0x5045524d00000000ull));  // "PERM"
    uint64_t x = (uint64_t)i;
    do {
        x = feistel(x, bits, key);
    } while (x >= (uint64_t)n);  // cycle walking: ends inside [0, n) (i's cycle holds i)
    out[(int64_t)blockIdx.y * n + i] = (int64_t)x;
}
__global__ void counter_add_kernel(uint64_t* c, uint64_t k) {
    if (threadIdx.x == 0) c[0] += k;
}

// the loss head (policy: the clipped surrogate's d/d mean; value: the squared error's d/d V) and the
// backward pass to the two hidden layers' output gradients; per-workgroup partial sums
// (sum min(s1, s2), sum (R - V)^2, #clipped, sum dL/dlogp (z0^2 - 1), sum dL/dlogp (z1^2 - 1)):
// policy blocks fill [b][0, 2, 3, 4], value blocks [nb + b][1].  nbs: adv_stats_kernel's blocks.
__global__ __launch_bounds__(MLP_BLOCK) void mlp_backward_kernel(MlpPair P, int m, const int64_t* __restrict__ idx,
                                                                 const float* __restrict__ act,
                                                                 const float* __restrict__ old_logp,
                                                                 const float* __restrict__ adv,
                                                                 const float* __restrict__ ret,
                                                                 const float* __restrict__ log_std,
                                                                 const double* __restrict__ ws, int nbs,
                                                                 int normalize, float clip, float vf_coef,
                                                                 float* __restrict__ partial) {
    __shared__ double red[5 * (MLP_BLOCK / 64)];
    __shared__ __attribute__((aligned(16))) float w2s[HID * HID];
    __shared__ float gcol[HID][MLP_SPB];
    const MlpNet& N = P.net[blockIdx.y];
    {  // W2 into LDS, all four loads per thread in flight before the stores
        static_assert(HID * HID == 4 * 4 * MLP_BLOCK, "W2 staging");
        float4 wv[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) wv[c] = reinterpret_cast<const float4*>(N.w2)[c * MLP_BLOCK + threadIdx.x];
#pragma unroll
        for (int c = 0; c < 4; ++c) reinterpret_cast<float4*>(w2s)[c * MLP_BLOCK + threadIdx.x] = wv[c];
    }
    // the sample's TPS threads own interleaved 4-unit groups (thread r: units 4 r + 4 TPS c ..), so a
    // wave's 16-byte row loads and stores cover 4 TPS contiguous floats per sample, not 4
    const int sl = threadIdx.x / TPS, r4 = (threadIdx.x % TPS) * 4;
    auto ub = [r4](int j) { return (j / 4) * 4 * TPS + r4; };  // first unit of this thread's group j / 4
    const int i = blockIdx.x * MLP_SPB + sl;
    const bool live = i < m;
    double q[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    float go0 = 0.0f, go1 = 0.0f;
    if (blockIdx.y == 0) {
        float adv_mean = 0.0f, adv_inv = 1.0f;
        if (normalize) {
            double s = 0.0, sq = 0.0;
            for (int b = threadIdx.x; b < nbs; b += blockDim.x) {
                s += ws[2 * b];
                sq += ws[2 * b + 1];
            }
            double sv[2] = {s, sq};
            block_sum_n(sv, red);
            s = sv[0];
            sq = sv[1];
            const double mu = s / m, var = (sq - s * mu) / (m > 1 ? m - 1 : 1);
            adv_mean = (float)mu;
            adv_inv = 1.0f / ((float)sqrt(var > 0.0 ? var : 0.0) + 1e-8f);
        }
        if (live) {  // both halves compute the head; the first one records it
            const int64_t j = idx[i];
            const float ls0 = log_std[0], ls1 = log_std[1];
            const float is0 = expf(-ls0), is1 = expf(-ls1);
            const float z0 = (act[2 * j] - N.out[2 * i]) * is0, z1 = (act[2 * j + 1] - N.out[2 * i + 1]) * is1;
            const float logp = (-0.5f * z0 * z0 - ls0 - HALF_LOG_2PI) + (-0.5f * z1 * z1 - ls1 - HALF_LOG_2PI);
            const float a = normalize ? (adv[j] - adv_mean) * adv_inv : adv[j];
            const float ratio = expf(logp - old_logp[j]);
            const float s1 = a * ratio, s2 = a * fminf(fmaxf(ratio, 1.0f - clip), 1.0f + clip);
            const float g_lp = (s1 <= s2) ? a * ratio * (-1.0f / m) : 0.0f;
            go0 = g_lp * z0 * is0;
            go1 = g_lp * z1 * is1;
            if (r4 == 0) {
                N.gout[2 * i] = go0;
                N.gout[2 * i + 1] = go1;
                q[0] = fminf(s1, s2);
                q[2] = fabsf(ratio - 1.0f) > clip ? 1.0 : 0.0;
                q[3] = (double)g_lp * (z0 * z0 - 1.0f);
                q[4] = (double)g_lp * (z1 * z1 - 1.0f);
            }
        }
    } else if (live) {
        const float err = ret[idx[i]] - N.out[i];
        go0 = err * (-2.0f * vf_coef / m);
        if (r4 == 0) {
            N.gout[i] = go0;
            q[1] = (double)err * err;
        }
    }
    block_sum_n(q, red);
    if (threadIdx.x == 0) {
        const double* t = q;
        float* o = partial + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 5;
#pragma unroll
        for (int k = 0; k < 5; ++k) o[k] = (float)t[k];
    }
    // g2 = (gout W3) * (1 - h2^2): this thread's 32 units, into the sample's LDS column
    if (live) {
        const float* h2 = N.h2 + (size_t)i * HID;
#pragma unroll
        for (int j = 0; j < UNITS; j += 4) {
            const float4 hv = *reinterpret_cast<const float4*>(h2 + ub(j));
            const float hh[4] = {hv.x, hv.y, hv.z, hv.w};
            float g[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float d = go0 * N.w3[ub(j) + u];
                if (N.od == 2) d += go1 * N.w3[HID + ub(j) + u];
                g[u] = d * (1.0f - hh[u] * hh[u]);
                gcol[ub(j) + u][sl] = g[u];
            }
            *reinterpret_cast<float4*>(N.g2 + (size_t)i * HID + ub(j)) = make_float4(g[0], g[1], g[2], g[3]);
        }
    }
    __syncthreads();  // W2 staged, both halves of g2 in the column
    if (!live) return;
    // g1[k] = (sum_j g2[j] W2[j][k]) (1 - h1[k]^2) for this thread's 32 units k
    float g1[UNITS];
#pragma unroll
    for (int k = 0; k < UNITS; ++k) g1[k] = 0.0f;
#pragma unroll 1
    for (int j = 0; j < HID; ++j) {
        const float gv = gcol[j][sl];
#pragma unroll
        for (int k4 = 0; k4 < UNITS / 4; ++k4) {
            const float4 wv = *reinterpret_cast<const float4*>(w2s + j * HID + ub(4 * k4));
            g1[4 * k4] += gv * wv.x;
            g1[4 * k4 + 1] += gv * wv.y;
            g1[4 * k4 + 2] += gv * wv.z;
            g1[4 * k4 + 3] += gv * wv.w;
        }
    }
    const float* h1 = N.h1 + (size_t)i * HID;
#pragma unroll
    for (int k = 0; k < UNITS; k += 4) {
        const float4 hv = *reinterpret_cast<const float4*>(h1 + ub(k));
        *reinterpret_cast<float4*>(N.g1 + (size_t)i * HID + ub(k)) =
            make_float4(g1[k] * (1.0f - hv.x * hv.x), g1[k + 1] * (1.0f - hv.y * hv.y),
                        g1[k + 2] * (1.0f - hv.z * hv.z), g1[k + 3] * (1.0f - hv.w * hv.w));
    }
}

// (g1 = g2 W2 on the matrix cores was bit-identical -- an f32 MFMA is an exact fmaf chain -- and
// measured 33.5 us against 23.4 us for this kernel: the 32 x 32 x 2 f32 MFMA runs at the f32 VALU rate
// and only adds tile hand-offs.  Removed in round 4.)

// ---------------------------------------------------------------------------- fused minibatch gradient
// One launch for what mlp_forward_mfma + mlp_backward + wgrad compute (D2D_PPO_FUSED, ABI v5): the
// workgroup (x, net) walks the minibatch's 64-sample chunks x, x + gridDim.x, ... and keeps the
// chunk's layer inputs, activations and output gradients in LDS, so nothing of the per-sample
// state goes through HBM.  Wave w takes the 32 x 32 tile (samples 32 (w / 2) .., units 32 (w % 2) ..)
// of both hidden layers and of g1 = g2 W2 on the matrix cores (W1 / W2 rows as register B operands
// for the forward, W2's columns for g1), then the chunk's contribution to dW2 = g2^T h1 (one 32 x 32
// tile per wave) and dW1 = g1^T x (waves 0, 1) accumulates on the matrix cores across chunks (the
// sample is the contraction index); waves 2, 3 sum the bias and output-layer gradients on the VALU.
// Each workgroup writes its sums into partial row x (the flat gradient's layout, its net's entries)
// and its loss-head sums into head row x (policy) / gridDim.x + x (value); d2d_ppo_grad_reduce
// finishes both.  Same formulas as the separate kernels, another summation order.
struct FusedNet {
    const float *w1, *b1, *w2, *b2, *w3, *b3;
    int off[6];  // offsets in the flat gradient of W1, b1, W2, b2, W3, b3
    int od;
};
struct FusedArgs {
    FusedNet net[2];
    int m;
    const int64_t* idx;
    const float *obs, *act, *old_logp, *adv, *ret, *log_std;
    const double* ws;  // d2d_ppo_adv_stats' partials of the minibatch
    int nbs, normalize;
    float clip, vf_coef;
    float* wpart;  // [gridDim.x][row_len]
    int row_len;
    float* hpart;  // [2 gridDim.x][5]
};
constexpr int FG_SPC = 64;
__global__ __launch_bounds__(256, 2) void mlp_fused_grad_kernel(FusedArgs A) {
    __shared__ float xs[FG_SPC][XS];
    __shared__ float h1s[FG_SPC][HS], h2s[FG_SPC][HS], g1s[FG_SPC][HS], g2s[FG_SPC][HS];
    __shared__ float gos[2][FG_SPC];
    __shared__ float w3s[2][HID + 1];  // output rows, bias in column HID
    __shared__ int64_t rows[FG_SPC];
    __shared__ double red[5 * 4];
    const int net = blockIdx.y;
    const FusedNet& N = A.net[net];
    const int od = N.od, m = A.m;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, ci = lane & 31, h = lane >> 5;
    const int st = w >> 1, u0 = (w & 1) * 32;  // this wave's sample tile and unit half
    const int jw = (w & 1) * 32, kw = (w >> 1) * 32;  // its dW2 tile
    // B operands, once per workgroup: W1 and W2 staged through LDS with coalesced loads (xs and g2s
    // as scratch: W1 rows in xs' stride, W2 rows in g2s' padded stride), then into registers (a
    // direct gather of W's rows touches 32 cache lines per load instruction)
    PPO_STAMP(0);
    {
        constexpr int NW1 = (HID * OBS + 255) / 256, NW2 = HID * HID / 256;
        float v1[NW1], v2[NW2];
#pragma unroll
        for (int c = 0; c < NW1; ++c) {
            const int e = c * 256 + tid;
            v1[c] = e < HID * OBS ? N.w1[e] : 0.0f;
        }
#pragma unroll
        for (int c = 0; c < NW2; ++c) v2[c] = N.w2[c * 256 + tid];
#pragma unroll
        for (int c = 0; c < NW1; ++c) {
            const int e = c * 256 + tid;
            if (e < HID * OBS) xs[e / OBS][e % OBS] = v1[c];
        }
#pragma unroll
        for (int c = 0; c < NW2; ++c) {
            const int e = c * 256 + tid;
            g2s[e >> 6][e & 63] = v2[c];
        }
    }
    __syncthreads();
    float w1r[(OBS + 1) / 2], w2r[HID / 2], w2b[HID / 2];
#pragma unroll
    for (int t = 0; t < (OBS + 1) / 2; ++t) w1r[t] = 2 * t + h < OBS ? xs[u0 + ci][2 * t + h] : 0.0f;
#pragma unroll
    for (int t = 0; t < HID / 2; ++t) {
        w2r[t] = g2s[u0 + ci][2 * t + h];
        w2b[t] = g2s[2 * t + h][u0 + ci];
    }
    const float b1v = N.b1[u0 + ci], b2v = N.b2[u0 + ci];
    for (int e = tid; e < 2 * (HID + 1); e += 256) {
        const int r = e / (HID + 1), j = e % (HID + 1);
        w3s[r][j] = r < od ? (j < HID ? N.w3[r * HID + j] : N.b3[r]) : 0.0f;
    }
    float adv_mean = 0.0f, adv_inv = 1.0f;
    if (net == 0 && A.normalize) {
        double sm = 0.0, sq = 0.0;
        for (int b = tid; b < A.nbs; b += 256) {
            sm += A.ws[2 * b];
            sq += A.ws[2 * b + 1];
        }
        double sv[2] = {sm, sq};
        block_sum_n(sv, red);
        const double mu = sv[0] / m, var = (sv[1] - sv[0] * mu) / (m > 1 ? m - 1 : 1);
        adv_mean = (float)mu;
        adv_inv = 1.0f / ((float)sqrt(var > 0.0 ? var : 0.0) + 1e-8f);
    }
    const float ls0 = A.log_std[0], ls1 = A.log_std[1], is0 = expf(-ls0), is1 = expf(-ls1);
    f32x16 dw2 = {}, dw1 = {};
    float db1 = 0.0f, db2 = 0.0f, dw3a = 0.0f, dw3b = 0.0f, db3a = 0.0f, db3b = 0.0f;
    double q[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    const int nch = (m + FG_SPC - 1) / FG_SPC;
    PPO_STAMP(1);
    for (int c = blockIdx.x; c < nch; c += gridDim.x) {
        const int s0 = c * FG_SPC;
        const bool first = c == (int)blockIdx.x;
        __syncthreads();  // the previous chunk's (or the operand staging's) LDS reads are done
        if (tid < FG_SPC) rows[tid] = s0 + tid < m ? A.idx[s0 + tid] : -1;
        __syncthreads();
        {  // the chunk's observation rows: every load issued before the first LDS store
            constexpr int NX = (FG_SPC * XS + 255) / 256;
            float xv[NX];
#pragma unroll
            for (int q = 0; q < NX; ++q) {
                const int e = q * 256 + tid, i = e / XS, k = e % XS;
                const int64_t r = e < FG_SPC * XS ? rows[i] : -1;
                xv[q] = (k < OBS && r >= 0) ? A.obs[r * OBS + k] : 0.0f;
            }
#pragma unroll
            for (int q = 0; q < NX; ++q) {
                const int e = q * 256 + tid;
                if (e < FG_SPC * XS) xs[e / XS][e % XS] = xv[q];
            }
        }
        __syncthreads();
        if (first) PPO_STAMP(2);
        f32x16 acc = {};
#pragma unroll
        for (int t = 0; t < (OBS + 1) / 2; ++t)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xs[st * 32 + ci][2 * t + h], w1r[t], acc, 0, 0, 0);
#pragma unroll
        for (int v = 0; v < 16; ++v) h1s[st * 32 + (v & 3) + 8 * (v >> 2) + 4 * h][u0 + ci] = ftanh(acc[v] + b1v);
        __syncthreads();
        acc = f32x16{};
#pragma unroll
        for (int t = 0; t < HID / 2; ++t)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(h1s[st * 32 + ci][2 * t + h], w2r[t], acc, 0, 0, 0);
#pragma unroll
        for (int v = 0; v < 16; ++v) h2s[st * 32 + (v & 3) + 8 * (v >> 2) + 4 * h][u0 + ci] = ftanh(acc[v] + b2v);
        __syncthreads();
        if (first) PPO_STAMP(3);
        {  // the outputs (four threads per sample, 16 units each) and the loss head (the first of the four)
            const int i = tid >> 2, pq = tid & 3, s = s0 + i;
            float o0 = 0.0f, o1 = 0.0f;
#pragma unroll
            for (int jj = 0; jj < HID / 4; ++jj) {
                const int j = pq * (HID / 4) + jj;
                const float hv = h2s[i][j];
                o0 += w3s[0][j] * hv;
                o1 += w3s[1][j] * hv;
            }
            o0 += __shfl_xor(o0, 1, 64);
            o1 += __shfl_xor(o1, 1, 64);
            o0 += __shfl_xor(o0, 2, 64);
            o1 += __shfl_xor(o1, 2, 64);
            o0 += w3s[0][HID];
            o1 += w3s[1][HID];
            if (pq == 0) {
                float g0 = 0.0f, g1v = 0.0f;
                if (s < m) {
                    const int64_t j = rows[i];
                    if (net == 0) {
                        const float z0 = (A.act[2 * j] - o0) * is0, z1 = (A.act[2 * j + 1] - o1) * is1;
                        const float logp =
                            (-0.5f * z0 * z0 - ls0 - HALF_LOG_2PI) + (-0.5f * z1 * z1 - ls1 - HALF_LOG_2PI);
                        const float a = A.normalize ? (A.adv[j] - adv_mean) * adv_inv : A.adv[j];
                        const float ratio = expf(logp - A.old_logp[j]);
                        const float s1 = a * ratio, s2 = a * fminf(fmaxf(ratio, 1.0f - A.clip), 1.0f + A.clip);
                        const float g_lp = (s1 <= s2) ? a * ratio * (-1.0f / m) : 0.0f;
                        g0 = g_lp * z0 * is0;
                        g1v = g_lp * z1 * is1;
                        q[0] += fminf(s1, s2);
                        q[2] += fabsf(ratio - 1.0f) > A.clip ? 1.0 : 0.0;
                        q[3] += (double)g_lp * (z0 * z0 - 1.0f);
                        q[4] += (double)g_lp * (z1 * z1 - 1.0f);
                    } else {
                        const float err = A.ret[j] - o0;
                        g0 = err * (-2.0f * A.vf_coef / m);
                        q[1] += (double)err * err;
                    }
                }
                gos[0][i] = g0;
                gos[1][i] = g1v;
                db3a += g0;
                db3b += g1v;
            }
        }
        __syncthreads();
        if (first) PPO_STAMP(4);
        // g2 = (gout W3) (1 - h2^2)
#pragma unroll 4
        for (int it = 0; it < FG_SPC * HID / 256; ++it) {
            const int e = it * 256 + tid, i = e >> 6, j = e & 63;
            const float d = gos[0][i] * w3s[0][j] + gos[1][i] * w3s[1][j];
            const float hv = h2s[i][j];
            g2s[i][j] = d * (1.0f - hv * hv);
        }
        __syncthreads();
        // g1 = (g2 W2) (1 - h1^2)
        acc = f32x16{};
#pragma unroll
        for (int t = 0; t < HID / 2; ++t)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(g2s[st * 32 + ci][2 * t + h], w2b[t], acc, 0, 0, 0);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int i = st * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
            const float hv = h1s[i][u0 + ci];
            g1s[i][u0 + ci] = acc[v] * (1.0f - hv * hv);
        }
        __syncthreads();
        if (first) PPO_STAMP(5);
        // this chunk's share of the weight gradients (padding samples carry zero gradients)
#pragma unroll
        for (int t = 0; t < FG_SPC / 2; ++t)
            dw2 = __builtin_amdgcn_mfma_f32_32x32x2f32(g2s[2 * t + h][jw + ci], h1s[2 * t + h][kw + ci], dw2, 0, 0, 0);
        if (w < 2) {
#pragma unroll
            for (int t = 0; t < FG_SPC / 2; ++t)
                dw1 = __builtin_amdgcn_mfma_f32_32x32x2f32(g1s[2 * t + h][jw + ci], ci < OBS ? xs[2 * t + h][ci] : 0.0f,
                                                           dw1, 0, 0, 0);
        } else {
            const int l = tid - 128, j = l & 63, hf = l >> 6;
#pragma unroll 8
            for (int k = 0; k < FG_SPC / 2; ++k) {
                const int i = hf * (FG_SPC / 2) + k;
                db1 += g1s[i][j];
                db2 += g2s[i][j];
                const float hv = h2s[i][j];
                dw3a += gos[0][i] * hv;
                dw3b += gos[1][i] * hv;
            }
        }
        if (first) PPO_STAMP(6);
    }
    // this workgroup's partial row
    float* P = A.wpart + (size_t)blockIdx.x * A.row_len;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int i = (v & 3) + 8 * (v >> 2) + 4 * h;
        P[N.off[2] + (jw + i) * HID + kw + ci] = dw2[v];
        if (w < 2 && ci < OBS) P[N.off[0] + (jw + i) * OBS + ci] = dw1[v];
    }
    __syncthreads();  // the chunk loop's LDS reads are done: g1s rows 0..3 become the half-sum scratch
    if (w >= 2 && ((tid - 128) >> 6) == 1) {
        const int j = (tid - 128) & 63;
        g1s[0][j] = db1;
        g1s[1][j] = db2;
        g1s[2][j] = dw3a;
        g1s[3][j] = dw3b;
    }
    __syncthreads();
    if (w >= 2) {
        const int l = tid - 128, j = l & 63, hf = l >> 6;
        if (hf == 0) {
            P[N.off[1] + j] = db1 + g1s[0][j];
            P[N.off[3] + j] = db2 + g1s[1][j];
            P[N.off[4] + j] = dw3a + g1s[2][j];
            if (od == 2) P[N.off[4] + HID + j] = dw3b + g1s[3][j];
        }
    }
    double b3[2] = {(double)db3a, (double)db3b};  // the head threads' output-bias sums
    block_sum_n(b3, red);
    if (tid == 0) {
        P[N.off[5]] = (float)b3[0];
        if (od == 2) P[N.off[5] + 1] = (float)b3[1];
    }
    block_sum_n(q, red);
    if (tid == 0) {
        float* o = A.hpart + ((size_t)net * gridDim.x + blockIdx.x) * 5;
#pragma unroll
        for (int k = 0; k < 5; ++k) o[k] = (float)q[k];
    }
    PPO_STAMP(7);
}

constexpr int ADAM_THREADS = 1024, ADAM_PER_THREAD = 16;  // n <= 16 384 parameters
__global__ __launch_bounds__(ADAM_THREADS) void adam_kernel(int n, float* __restrict__ p, float* __restrict__ g,
                                                            float* __restrict__ m1, float* __restrict__ m2,
                                                            float* __restrict__ t, float lr, float b1, float b2,
                                                            float eps, float max_norm) {
    __shared__ double red[ADAM_THREADS / 64];
    // the moments and parameters are loaded with the gradient, ahead of the norm's reduction, so
    // the update below waits on no memory
    float gv[ADAM_PER_THREAD], a0v[ADAM_PER_THREAD], v0v[ADAM_PER_THREAD], p0v[ADAM_PER_THREAD];
#pragma unroll
    for (int k = 0; k < ADAM_PER_THREAD; ++k) {
        const int i = threadIdx.x + k * ADAM_THREADS;
        const bool in = i < n;
        gv[k] = in ? g[i] : 0.0f;
        a0v[k] = in ? m1[i] : 0.0f;
        v0v[k] = in ? m2[i] : 0.0f;
        p0v[k] = in ? p[i] : 0.0f;
    }
    double q = 0.0;
#pragma unroll
    for (int k = 0; k < ADAM_PER_THREAD; ++k) q += (double)gv[k] * gv[k];
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
            const float a0 = a0v[k], v0 = v0v[k];
            const float a = a0 + (1.0f - b1) * (gi - a0);  // exp_avg.lerp_(grad, 1 - beta1)
            const float v = v0 * b2 + (1.0f - b2) * gi * gi;
            m1[i] = a;
            m2[i] = v;
            p[i] = p0v[k] - a * lr_t / (sqrtf(v) / bc2s + eps);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) t[0] = step;
}

// (A spread Adam -- ceil(n / 1024) workgroups, each computing the norm -- measured 8.1 us + 3.9 us for
// a one-thread step-counter launch against 10.8 us for this kernel; removed in round 4.)

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

// The products run on the matrix cores fed from this kernel's LDS tiles.  (Measured and removed in
// round 4: VALU 4 x 4 blocks from the same tiles, 36 us; matrix cores straight from memory, 55 us,
// load-latency bound.)
__global__ __launch_bounds__(256) void wgrad_kernel(WgradProblems P, int m, int row_len, float* __restrict__ partial) {
    __shared__ float ta[WG_TILE][64 + 4];
    __shared__ float tb[WG_TILE][64 + 4];
    const WgradProblem& pr = P.k[blockIdx.y];
    const int p = pr.p, q = pr.q;
    // this wave's 32 x 32 output tile
    const int mw = threadIdx.x >> 6, mci = threadIdx.x & 31, mh = (threadIdx.x >> 5) & 1;
    const int nqt = (q + 31) / 32, npt = (p + 31) / 32;
    const int mp0 = (mw / max(nqt, 1)) * 32, mq0 = (mw % max(nqt, 1)) * 32;
    f32x16 macc = {};
    float mbs = 0.0f;
    const int r0 = blockIdx.x * WG_ROWS, r1 = min(m, r0 + WG_ROWS);
    // element v of this thread's share of a tile: row (tid + 256 v) / 64, column (tid + 256 v) % 64;
    // the next tile is loaded into registers while the current one is multiplied
    constexpr int PER = WG_TILE * 64 / 256;
    float ra[PER], rb[PER];
    auto fetch = [&](int rt) {
#pragma unroll
        for (int v = 0; v < PER; ++v) {
            const int e = threadIdx.x + 256 * v, r = e >> 6, c = e & 63, row = rt + r;
            ra[v] = (row < r1 && c < p) ? pr.a[(size_t)row * pr.lda + c] : 0.0f;
            rb[v] = (row < r1 && c < q) ? pr.b[(size_t)row * pr.ldb + c] : 0.0f;
        }
    };
    fetch(r0);
    for (int rt = r0; rt < r1; rt += WG_TILE) {
        __syncthreads();  // the previous tile's products are done
#pragma unroll
        for (int v = 0; v < PER; ++v) {
            const int e = threadIdx.x + 256 * v;
            ta[e >> 6][e & 63] = ra[v];
            tb[e >> 6][e & 63] = rb[v];
        }
        __syncthreads();
        if (rt + WG_TILE < r1) fetch(rt + WG_TILE);
        // wave w: the 32 x 32 output tile (p0, q0); lane l: A[k = l / 32][i = l % 32] = a[row][p0 + i],
        // B[k][j = l % 32] = b[row][q0 + j], row = 2 t + l / 32
        if (mw < npt * nqt) {
#pragma unroll 8
            for (int t = 0; t < WG_TILE / 2; ++t) {
                const float av = ta[2 * t + mh][mp0 + mci];
                macc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, tb[2 * t + mh][mq0 + mci], macc, 0, 0, 0);
                mbs += av;
            }
        }
    }
    float* out = partial + (size_t)blockIdx.x * row_len;
    if (mw < npt * nqt) {
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int i = (v & 3) + 8 * (v >> 2) + 4 * mh;  // the C/D map of the 32 x 32 MFMA
            if (mp0 + i < p && mq0 + mci < q) out[pr.w_off + (mp0 + i) * q + mq0 + mci] = macc[v];
        }
        mbs += __shfl_xor(mbs, 32, 64);
        if (mq0 == 0 && mh == 0 && mp0 + mci < p) out[pr.b_off + mp0 + mci] = mbs;
    }
}

// g[e] = sum over the n_chunks rows of partial[.][e], e < row_len: 64 elements per workgroup, the
// chunks split over the workgroup's four waves
__device__ __forceinline__ void wgrad_reduce_body(int n_chunks, int row_len, const float* __restrict__ partial,
                                                  float* __restrict__ g, const HeadArgs& H) {
    const long ls_off = H.partial != nullptr ? (long)(H.ls_grad - g) : -8;
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + lane;
    float s = 0.0f;
    if (e < row_len) {  // chunks w, w + 4, ... in order, eight loads in flight at a time
        int c = w;
        for (; c + 28 < n_chunks; c += 32) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = partial[(size_t)(c + 4 * u) * row_len + e];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; c < n_chunks; c += 4) s += partial[(size_t)c * row_len + e];
    }
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && e < row_len && (e < ls_off || e >= ls_off + 2))
        g[e] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// (Clip + Adam as the last-finishing workgroup of this reduce, behind a device ticket and agent-scope
// fences, measured 0.0403 s per update against 0.0337 s for the separate launch; removed in round 4.)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(int n_chunks, int row_len, const float* __restrict__ partial,
                                                           float* __restrict__ g, HeadArgs H) {
    // with H.partial set, the last workgroup finishes the loss head (head_finish_kernel's work) and
    // writes log_std's two gradient slots, which the reduce then leaves alone
    if (H.partial != nullptr && blockIdx.x == gridDim.x - 1) {
        head_finish_body(H);
    } else {
        wgrad_reduce_body(n_chunks, row_len, partial, g, H);
    }
}

inline int32_t rc(hipError_t e) { return e == hipSuccess ? 0 : (int32_t)e; }

}  // namespace

extern "C" {

int32_t d2d_ppo_abi_version(void) { return D2D_PPO_ABI_VERSION; }
#ifdef D2D_PPO_STAMPS
int32_t d2d_ppo_debug_stamps(uint64_t* buf) {
    return rc(hipMemcpyToSymbol(HIP_SYMBOL(d2d_ppo_stamp_buf), &buf, sizeof(buf)));
}
#endif

int32_t d2d_ppo_adv_stats(int32_t m, const int64_t* idx, const float* adv, double* ws, void* stream) {
    if (m <= 0) return 0;
    const int nb = (m + D2D_PPO_HEAD_BLOCK - 1) / D2D_PPO_HEAD_BLOCK;
    hipLaunchKernelGGL(adv_stats_kernel, dim3(nb), dim3(D2D_PPO_HEAD_BLOCK), 0, (hipStream_t)stream, m, idx, adv, ws);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_head_finish(int32_t m, int32_t n_blocks, const float* partial, const float* log_std, float ent_coef,
                            float* log_std_grad, float* acc_pl, float* acc_vl, float* acc_ent, float* acc_clip,
                            void* stream) {
    if (m <= 0) return 0;
    const HeadArgs H{m, n_blocks, partial, log_std, ent_coef, log_std_grad, acc_pl, acc_vl, acc_ent, acc_clip};
    hipLaunchKernelGGL(head_finish_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, H);
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

static int32_t wgrad_launch(int32_t m, int32_t n_problems, const float* const* a, const int32_t* lda,
                            const float* const* b, const int32_t* ldb, const int32_t* p, const int32_t* q,
                            const int32_t* w_off, const int32_t* b_off, int32_t row_len, float* partial, float* g,
                            const HeadArgs& H, void* stream) {
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
    if (H.partial != nullptr && (H.ls_grad < g || H.ls_grad + 2 > g + row_len)) return (int32_t)hipErrorInvalidValue;
    const dim3 rgrid((row_len + 63) / 64 + (H.partial != nullptr));
    hipLaunchKernelGGL(wgrad_reduce_kernel, rgrid, dim3(256), 0, (hipStream_t)stream, nc, row_len, partial, g, H);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_wgrad(int32_t m, int32_t n_problems, const float* const* a, const int32_t* lda, const float* const* b,
                      const int32_t* ldb, const int32_t* p, const int32_t* q, const int32_t* w_off,
                      const int32_t* b_off, int32_t row_len, float* partial, float* g, void* stream) {
    return wgrad_launch(m, n_problems, a, lda, b, ldb, p, q, w_off, b_off, row_len, partial, g, HeadArgs{}, stream);
}

int32_t d2d_ppo_wgrad_head(int32_t m, int32_t n_problems, const float* const* a, const int32_t* lda,
                           const float* const* b, const int32_t* ldb, const int32_t* p, const int32_t* q,
                           const int32_t* w_off, const int32_t* b_off, int32_t row_len, float* partial, float* g,
                           int32_t n_blocks, const float* head_partial, const float* log_std, float ent_coef,
                           float* log_std_grad, float* acc_pl, float* acc_vl, float* acc_ent, float* acc_clip,
                           void* stream) {
    if (head_partial == nullptr) return (int32_t)hipErrorInvalidValue;
    const HeadArgs H{m, n_blocks, head_partial, log_std, ent_coef, log_std_grad, acc_pl, acc_vl, acc_ent, acc_clip};
    return wgrad_launch(m, n_problems, a, lda, b, ldb, p, q, w_off, b_off, row_len, partial, g, H, stream);
}

int32_t d2d_ppo_wgrad_chunks(int32_t m) { return (m + WG_ROWS - 1) / WG_ROWS; }

static MlpPair make_pair(const float* const* w, float* const* buf) {
    MlpPair P{};
    for (int n = 0; n < 2; ++n) {
        const float* const* W = w + 6 * n;
        float* const* B = buf + 5 * n;
        P.net[n] = MlpNet{W[0], W[1], W[2], W[3], W[4], W[5], B[0], B[1], B[2], B[3], B[4], nullptr, n == 0 ? 2 : 1};
    }
    return P;
}

int32_t d2d_ppo_mlp_forward_adv(int32_t m, const int64_t* idx, const float* obs, const float* adv,
                                const float* const* weights, float* const* bufs, float* xg, double* ws, void* stream) {
    if (m <= 0) return 0;
    if (adv != nullptr && ws == nullptr) return (int32_t)hipErrorInvalidValue;
    MlpPair P = make_pair(weights, bufs);
    hipLaunchKernelGGL(mlp_forward_mfma_kernel, dim3((m + FM_TILES * FM_SPB - 1) / (FM_TILES * FM_SPB)), dim3(256), 0,
                       (hipStream_t)stream, P, m, idx, obs, xg, adv, ws);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_mlp_forward(int32_t m, const int64_t* idx, const float* obs, const float* const* weights,
                            float* const* bufs, float* xg, void* stream) {
    return d2d_ppo_mlp_forward_adv(m, idx, obs, nullptr, weights, bufs, xg, nullptr, stream);
}

int32_t d2d_ppo_mlp_partial_rows(int32_t m) { return 2 * ((m + MLP_SPB - 1) / MLP_SPB); }

static int n_cus() {
    static int cached = 0;
    if (cached == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        cached = n;
    }
    return cached;
}

int32_t d2d_ppo_fused_rows(int32_t m) {
    if (m <= 0) return 0;
    const int nch = (m + FG_SPC - 1) / FG_SPC;
    return nch < n_cus() ? nch : n_cus();
}

int32_t d2d_ppo_fused_grad(int32_t m, const int64_t* idx, const float* obs, const float* act, const float* old_logp,
                           const float* adv, const float* ret, const float* log_std, const double* ws, int32_t normalize,
                           float clip, float vf_coef, const float* const* weights, const int32_t* offsets,
                           int32_t row_len, float* wpart, float* hpart, void* stream) {
    if (m <= 0) return 0;
    if (!idx || !obs || !act || !old_logp || !adv || !ret || !log_std || !weights || !offsets || !wpart || !hpart ||
        (normalize && !ws))
        return (int32_t)hipErrorInvalidValue;
    FusedArgs A{};
    for (int n = 0; n < 2; ++n) {
        const float* const* W = weights + 6 * n;
        A.net[n] = FusedNet{W[0], W[1], W[2], W[3], W[4], W[5], {0, 0, 0, 0, 0, 0}, n == 0 ? 2 : 1};
        for (int k = 0; k < 6; ++k) {
            const int o = offsets[6 * n + k];
            const int len = k == 0 ? HID * OBS : (k == 2 ? HID * HID : (k == 4 ? A.net[n].od * HID : (k == 5 ? A.net[n].od : HID)));
            if (o < 0 || o + len > row_len) return (int32_t)hipErrorInvalidValue;
            A.net[n].off[k] = o;
        }
    }
    A.m = m;
    A.idx = idx;
    A.obs = obs;
    A.act = act;
    A.old_logp = old_logp;
    A.adv = adv;
    A.ret = ret;
    A.log_std = log_std;
    A.ws = ws;
    A.nbs = (m + D2D_PPO_HEAD_BLOCK - 1) / D2D_PPO_HEAD_BLOCK;
    A.normalize = normalize;
    A.clip = clip;
    A.vf_coef = vf_coef;
    A.wpart = wpart;
    A.row_len = row_len;
    A.hpart = hpart;
    hipLaunchKernelGGL(mlp_fused_grad_kernel, dim3(d2d_ppo_fused_rows(m), 2), dim3(256), 0, (hipStream_t)stream, A);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_grad_reduce(int32_t n_rows, int32_t row_len, const float* partial, float* g, int32_t n_blocks,
                            const float* head_partial, int32_t m, const float* log_std, float ent_coef,
                            float* log_std_grad, float* acc_pl, float* acc_vl, float* acc_ent, float* acc_clip,
                            void* stream) {
    if (n_rows <= 0 || row_len <= 0) return 0;
    if (!partial || !g || !head_partial || !log_std || !log_std_grad || log_std_grad < g ||
        log_std_grad + 2 > g + row_len)
        return (int32_t)hipErrorInvalidValue;
    const HeadArgs H{m, n_blocks, head_partial, log_std, ent_coef, log_std_grad, acc_pl, acc_vl, acc_ent, acc_clip};
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((row_len + 63) / 64 + 1), dim3(256), 0, (hipStream_t)stream,
                       n_rows, row_len, partial, g, H);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_permute(int64_t n, int32_t n_perm, uint64_t seed, uint64_t* counter, int64_t* out, void* stream) {
    if (n <= 0 || n_perm <= 0) return 0;
    if (counter == nullptr || out == nullptr || n > ((int64_t)1 << 40) || n_perm > 65535)
        return (int32_t)hipErrorInvalidValue;
    int bits = 0;
    while (((int64_t)1 << bits) < n) ++bits;
    hipLaunchKernelGGL(permute_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)n_perm), dim3(256), 0,
                       (hipStream_t)stream, n, bits, seed, counter, out);
    hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, counter, (uint64_t)n_perm);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_rollout_step(const d2d_ppo_rollout* r, const float* const* weights, void* stream) {
    if (r == nullptr || weights == nullptr) return (int32_t)hipErrorInvalidValue;
    const d2d_ppo_rollout& R = *r;
    if (R.n <= 0) return 0;
    if (R.T <= 0 || R.t < 0 || R.t > R.T || R.obs == nullptr || R.log_std == nullptr || R.val_buf == nullptr)
        return (int32_t)hipErrorInvalidValue;
    if (R.t < R.T && (R.noise == nullptr || R.obs_buf == nullptr || R.act_buf == nullptr || R.logp_buf == nullptr ||
                      R.act_env == nullptr))
        return (int32_t)hipErrorInvalidValue;
    if (R.t > 0 && (R.prev_rew == nullptr || R.prev_term == nullptr || R.prev_trunc == nullptr ||
                    R.rew_buf == nullptr || R.done_buf == nullptr || R.stats == nullptr ||
                    (R.prev_info != nullptr && (R.info_totrew < 0 || R.info_totrew >= R.info_dim))))
        return (int32_t)hipErrorInvalidValue;
    if (R.t == R.T && (R.adv_buf == nullptr || R.ret_buf == nullptr || R.start0 == nullptr))
        return (int32_t)hipErrorInvalidValue;
    float* none[10] = {};
    MlpPair P = make_pair(weights, none);
    float* xg = R.t < R.T ? R.obs_buf + (size_t)R.t * R.n * OBS : nullptr;
    hipLaunchKernelGGL(rollout_step_kernel, dim3((R.n + FM_TILES * FM_SPB - 1) / (FM_TILES * FM_SPB)), dim3(256), 0,
                       (hipStream_t)stream, P, R.n, xg, R);
    return rc(hipGetLastError());
}

int32_t d2d_ppo_mlp_backward(int32_t m, const int64_t* idx, const float* act, const float* old_logp, const float* adv,
                             const float* ret, const float* log_std, const double* ws, int32_t normalize, float clip,
                             float vf_coef, const float* const* weights, float* const* bufs, float* const* gout,
                             float* partial, void* stream) {
    if (m <= 0) return 0;
    MlpPair P = make_pair(weights, bufs);
    P.net[0].gout = gout[0];
    P.net[1].gout = gout[1];
    const int nbs = (m + D2D_PPO_HEAD_BLOCK - 1) / D2D_PPO_HEAD_BLOCK;
    hipLaunchKernelGGL(mlp_backward_kernel, dim3((m + MLP_SPB - 1) / MLP_SPB, 2), dim3(MLP_BLOCK), 0,
                           (hipStream_t)stream, P, m, idx, act, old_logp, adv, ret, log_std, ws, nbs, normalize, clip,
                           vf_coef, partial);
    return rc(hipGetLastError());
}

}  // extern "C"
