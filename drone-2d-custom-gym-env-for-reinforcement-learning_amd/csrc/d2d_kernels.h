// d2d_kernels.h -- the three kernels of libdrone2d_hip.so (included by d2d_hip.hip).
//
// K1 d2d_step_kernel (cooperative, wave-specialised).  One 256-lane workgroup owns 64 envs (one
// per lane index); its four waves split one env step by role so that the long, independent fp64
// latency chains run concurrently instead of back to back:
//
//   phase 1  W0: load state, thrust, Chipmunk-equivalent 3-body/6-pivot step, collision, end
//                cause (collision / reach / AA / time-up are all known right after physics),
//                store post-physics state                         | W1: next-episode spawn draw
//   phase 2  W0: path role (Brent) on the current state           | W1: sensor role + CA reward
//            W2: path role on the spawn state of envs that ended  | W3: sensor role, same envs
//   phase 3  W0: reward, bookkeeping, auto-reset state writes     | all: store the obs tile
//
// Hand-offs go through LDS with two __syncthreads.  The obs rows of the workgroup are assembled in
// LDS and written as one contiguous 64x27 f32 span.  At 65 536 envs this is 1 024 workgroups =
// 4 per CU = 4 waves per SIMD (VGPR <= 128, LDS <= 40 KB), against 1 wave per SIMD for the
// one-lane-per-env fused kernel it replaces (see DESIGN.md "Kernel v2").
//
// K2 d2d_reset_kernel: masked reset, one lane per env.  K3 d2d_stats_kernel: fixed-order reduction.
#pragma once
#include "d2d_device.h"

namespace d2dk {
using namespace d2d;

constexpr int BLOCK = 256;      // K2 / K3 workgroup
constexpr int EPB = 64;         // K1: envs per workgroup
constexpr int K1_THREADS = 256; // K1: 4 waves
constexpr int MAX_LDS_SCN = 8;

struct StepArgs {
    int n;
    int n_scn;
    double* st;              // [NSTATE][n]
    int32_t* ist;            // [NISTATE][n]
    double* acc;             // [NSTATS][n]
    const d2d_scn* scn;      // [n_scn]
    const int32_t* env_scn;  // [n] or null (all scenario 0)
    d2d_cfg cfg;
    double damping_dt;       // pow(cfg.damping, dt), host glibc
    uint64_t seed;
    const float* act;
    float* obs;
    float* rew;
    uint8_t* term;
    uint8_t* trunc;
    float* info;
    float* tobs;
    const uint8_t* mask;     // reset kernel only
    uint64_t* stamps;        // diagnostic builds only (D2D_STAMPS): [waves][8] s_memtime stamps
};

// Diagnostic phase stamps (separate timing-only build, never in the product): lane 0 of each wave
// records s_memtime at the phase boundaries of K1.
#ifdef D2D_STAMPS
#define STAMP(k)                                                                                       \
    do {                                                                                               \
        if (a.stamps && (threadIdx.x & 63) == 0)                                                       \
            a.stamps[(size_t)(blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif

template <bool LDS, int NT>
__device__ __forceinline__ const d2d_scn* stage_scenarios(const StepArgs& a, d2d_scn* lds) {
    if (!LDS) return a.scn;
    const int words = a.n_scn * (int)(sizeof(d2d_scn) / 8);
    const double* src = reinterpret_cast<const double*>(a.scn);
    double* dst = reinterpret_cast<double*>(lds);
    for (int k = threadIdx.x; k < words; k += NT) dst[k] = src[k];
    return lds;
}

__device__ __forceinline__ size_t fidx(int f, int n, int i) { return (size_t)f * (size_t)n + (size_t)i; }
// SoA field access as (wave-uniform field base) + (per-lane 32-bit index): the base lives in SGPRs
// and the access uses saddr + voffset addressing, instead of one 64-bit VGPR address per field.
template <typename T>
__device__ __forceinline__ T& fld(T* base, int f, int n, int i) {
    T* fb = base + (size_t)__builtin_amdgcn_readfirstlane(f) * (size_t)__builtin_amdgcn_readfirstlane(n);
    return fb[i];
}

// ------------------------------------------------------------------------------------------ K1
struct K1Shared {
    double fr[6][EPB];        // post-physics frame: px, py, angle, vx, vy, w
    double sp[7][EPB];        // next-episode spawn: x, y, th, left (x, y), right (x, y)
    int cause[EPB];           // end cause of this step (0: running)
    int scn[EPB];             // scenario index per env
    uint32_t ep[EPB];         // episode counter (before this step's reset)
    uint32_t rflags[EPB];     // flags of the reset observation (LA lock)
    union {
        double jb[36][EPB];   // phase 1: W0's per-joint K^-1 (4) + bias (2), re-read every sweep
        struct {
            double ca[5][EPB];             // sensor -> reward: vel_ang, ca, lpa, lca, dclose
            float obs[EPB * D2D_OBS_DIM];  // the workgroup's obs rows
        } p;                  // phases 2-3
    } u;
};

template <bool LDS>
__global__ __launch_bounds__(K1_THREADS, 4) void d2d_step_kernel(StepArgs a) {
    // dynamic LDS: n_scn scenario tables (sized at launch, so a 1-scenario batch keeps 6 workgroups
    // per CU by LDS and a 7-scenario mixed batch still fits 4)
    extern __shared__ __attribute__((aligned(16))) d2d_scn s_scn[];
    __shared__ __attribute__((aligned(16))) K1Shared sh;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int e0 = blockIdx.x * EPB;
    const int i = e0 + lane;
    const bool valid = i < a.n;
    const int n = a.n;
    STAMP(0);
    const d2d_scn* scns = stage_scenarios<LDS, K1_THREADS>(a, s_scn);
    if (wave == 0) sh.scn[lane] = (valid && a.env_scn && a.n_scn > 1) ? a.env_scn[i] : 0;
    __syncthreads();
    STAMP(1);
    const d2d_scn& S = scns[sh.scn[lane]];

    // ---------------------------------------------------------------- phase 1
    double path_err = 0.0, tot_rew = 0.0;
    int t = 0;
    uint32_t flags = 0;
    int cause = 0;
    if (wave == 0) {
        if (valid) {
            Body B[3];
            double j[12];
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                B[b].px = fld(a.st, 6 * b + 0, n, i);
                B[b].py = fld(a.st, 6 * b + 1, n, i);
                B[b].a = fld(a.st, 6 * b + 2, n, i);
                B[b].vx = fld(a.st, 6 * b + 3, n, i);
                B[b].vy = fld(a.st, 6 * b + 4, n, i);
                B[b].w = fld(a.st, 6 * b + 5, n, i);
            }
#pragma unroll
            for (int k = 0; k < 12; ++k) j[k] = fld(a.st, D2D_S_J + k, n, i);
            path_err = fld(a.st, D2D_S_PATH_ERR, n, i);
            tot_rew = fld(a.st, D2D_S_TOT_REW, n, i);
            t = fld(a.ist, D2D_I_T, n, i);
            flags = (uint32_t)fld(a.ist, D2D_I_FLAGS, n, i);
            // thrust in float32 exactly as SB3's float32 action hits drone_2d_env.py:400-401
            const float2 act = reinterpret_cast<const float2*>(a.act)[i];
            const float fs = (float)a.cfg.force_scale;
            const float lf = __fmul_rn(__fadd_rn(act.x / 2.0f, 0.5f), fs);
            const float rf = __fmul_rn(__fadd_rn(act.y / 2.0f, 0.5f), fs);
            double cs[3], sn[3], fx, fy, tq;
            if (phys_positions(S, B, (double)lf, (double)rf, cs, sn, fx, fy, tq)) flags |= D2D_FLAG_COLLIDED;
            t += 1;
            cause = end_cause(a.cfg, S, B[0], (flags & D2D_FLAG_COLLIDED) != 0, t);
            // positions are final: retire them before the joint sweep (envs that end this step are
            // overwritten with their spawn state in phase 3)
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                fld(a.st, 6 * b + 0, n, i) = B[b].px;
                fld(a.st, 6 * b + 1, n, i) = B[b].py;
                fld(a.st, 6 * b + 2, n, i) = B[b].a;
            }
            sh.fr[0][lane] = B[0].px;
            sh.fr[1][lane] = B[0].py;
            sh.fr[2][lane] = B[0].a;
            const Arms A = make_arms(cs, sn);
            const double pos[6] = {B[0].px, B[0].py, B[1].px, B[1].py, B[2].px, B[2].py};
            double vel[9] = {B[0].vx, B[0].vy, B[0].w, B[1].vx, B[1].vy, B[1].w, B[2].vx, B[2].vy, B[2].w};
            phys_velocities<true>(A, pos, a.damping_dt, fx, fy, tq, vel, j, &sh.u.jb[0][lane], EPB);
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                fld(a.st, 6 * b + 3, n, i) = vel[3 * b + 0];
                fld(a.st, 6 * b + 4, n, i) = vel[3 * b + 1];
                fld(a.st, 6 * b + 5, n, i) = vel[3 * b + 2];
            }
#pragma unroll
            for (int k = 0; k < 12; ++k) fld(a.st, D2D_S_J + k, n, i) = j[k];
            sh.fr[3][lane] = vel[0];
            sh.fr[4][lane] = vel[1];
            sh.fr[5][lane] = vel[2];
        }
        sh.cause[lane] = cause;
    } else if (wave == 1 && valid) {
        // next-episode spawn (test-mode reset, drone_2d_env.py:218-311, Drone.py:20-52)
        const uint32_t ep = (uint32_t)fld(a.ist, D2D_I_EPISODE, n, i);
        double x, y, th;
        spawn_draw(S, a.seed, (uint32_t)a.cfg.env_id_base + (uint32_t)i, ep, x, y, th);
        double sl, cl, sr, cr;
        sincos_d(th + PI, sl, cl);
        sincos_d(th, sr, cr);
        sh.sp[0][lane] = x;
        sh.sp[1][lane] = y;
        sh.sp[2][lane] = th;
        sh.sp[3][lane] = cl * DRONE_R + x;
        sh.sp[4][lane] = sl * DRONE_R + y;
        sh.sp[5][lane] = cr * DRONE_R + x;
        sh.sp[6][lane] = sr * DRONE_R + y;
        sh.ep[lane] = ep;
    }
    STAMP(2);
    __syncthreads();
    STAMP(3);

    // ---------------------------------------------------------------- phase 2
    const int my_cause = sh.cause[lane];
    const bool done = valid && my_cause != 0;
    const bool auto_reset = a.cfg.auto_reset != 0;
    double po[8];
    float* orow = &sh.u.p.obs[lane * D2D_OBS_DIM];
    if (wave == 0 || wave == 2) {
        // path role: W0 current state, W2 spawn state of envs that ended (auto-reset)
        const bool rs = (wave == 2);
        if (valid && (!rs || (done && auto_reset))) {
            const double x = rs ? sh.sp[0][lane] : sh.fr[0][lane];
            const double y = rs ? sh.sp[1][lane] : sh.fr[1][lane];
            const double al = rs ? sh.sp[2][lane] : sh.fr[2][lane];
            uint32_t f = rs ? 0u : flags;
            path_obs(a.cfg, S, x, y, al, f, po);
            if (rs) sh.rflags[lane] = f;
            else flags = f;
            if (rs || !(done && auto_reset)) {
#pragma unroll
                for (int k = 0; k < 8; ++k) orow[19 + k] = (float)po[k];
            }
            if (!rs && done && a.tobs) {
#pragma unroll
                for (int k = 0; k < 8; ++k) a.tobs[(size_t)i * D2D_OBS_DIM + 19 + k] = (float)po[k];
            }
        }
    } else {
        // sensor role: W1 current state (+ the reward's CA part), W3 spawn state of ended envs
        const bool rs = (wave == 3);
        if (valid && (!rs || (done && auto_reset))) {
            Body F;
            if (rs) {
                F = Body{sh.sp[0][lane], sh.sp[1][lane], sh.sp[2][lane], 0.0, 0.0, 0.0};
            } else {
                F = Body{sh.fr[0][lane], sh.fr[1][lane], sh.fr[2][lane], sh.fr[3][lane], sh.fr[4][lane],
                         sh.fr[5][lane]};
            }
            double so[19];
            sensor_obs(a.cfg, S, F, so);
            if (!rs) {
                const CAPart P = reward_ca_part(a.cfg, S, so);
                sh.u.p.ca[0][lane] = P.vel_ang;
                sh.u.p.ca[1][lane] = P.ca;
                sh.u.p.ca[2][lane] = P.lpa;
                sh.u.p.ca[3][lane] = P.lca;
                sh.u.p.ca[4][lane] = P.dclose;
            }
            if (rs || !(done && auto_reset)) {
#pragma unroll
                for (int k = 0; k < 19; ++k) orow[k] = (float)so[k];
            }
            if (!rs && done && a.tobs) {
#pragma unroll
                for (int k = 0; k < 19; ++k) a.tobs[(size_t)i * D2D_OBS_DIM + k] = (float)so[k];
            }
        }
    }
    STAMP(4);
    __syncthreads();
    STAMP(5);

    // ---------------------------------------------------------------- phase 3
    // obs tile: rows [e0, e0+rows) are one contiguous span of global memory
    {
        const int rows = min(EPB, n - e0);
        const int words = rows * D2D_OBS_DIM;
        float* dst = a.obs + (size_t)e0 * D2D_OBS_DIM;
        for (int k = threadIdx.x; k < words; k += K1_THREADS) dst[k] = sh.u.p.obs[k];
    }
    if (wave == 0 && valid) {
        const Body F{sh.fr[0][lane], sh.fr[1][lane], sh.fr[2][lane], sh.fr[3][lane], sh.fr[4][lane], sh.fr[5][lane]};
        const CAPart P{sh.u.p.ca[0][lane], sh.u.p.ca[1][lane], sh.u.p.ca[2][lane], sh.u.p.ca[3][lane], sh.u.p.ca[4][lane]};
        const Reward R = reward_final(a.cfg, F, po, P, my_cause);
        path_err += R.dist_path;
        const double ape = path_err / (double)t;
        tot_rew += R.reward;
        bool trunc = false, term = done;
        if (a.cfg.timeup_truncates && done && my_cause == D2D_END_TIMEUP) {
            trunc = true;
            term = false;
        }
        a.rew[i] = (float)R.reward;
        a.term[i] = (uint8_t)term;
        a.trunc[i] = (uint8_t)trunc;
        if (a.info) {
            float* r = a.info + (size_t)i * D2D_INFO_DIM;
            r[D2D_INFO_CA] = (float)R.ca;
            r[D2D_INFO_PA] = (float)R.pa;
            r[D2D_INFO_PP] = (float)R.pp;
            r[D2D_INFO_COLL] = (float)R.coll;
            r[D2D_INFO_REACH] = (float)R.reach;
            r[D2D_INFO_AA] = (float)R.aa;
            r[D2D_INFO_DCLOSE] = (float)R.dclose;
            r[D2D_INFO_STEPS] = (float)t;
            r[D2D_INFO_CAUSE] = (float)my_cause;
            r[D2D_INFO_APE] = done ? (float)ape : 0.0f;
            r[D2D_INFO_TOTREW] = done ? (float)tot_rew : 0.0f;
            r[D2D_INFO_REWARD] = (float)R.reward;
        }
        if (done) {
            // finished-episode accumulators (info counters of drone_2d_env.py:593-613)
            const bool c1 = my_cause & D2D_END_COLLISION, c2 = my_cause & D2D_END_REACH;
            const bool c4 = my_cause & D2D_END_TIMEUP, c5 = my_cause & D2D_END_AA;
            fld(a.acc, D2D_ST_RETURN, n, i) += tot_rew;
            fld(a.acc, D2D_ST_EPISODES, n, i) += 1.0;
            fld(a.acc, D2D_ST_SUCCESS, n, i) += c2 ? 1.0 : 0.0;
            fld(a.acc, D2D_ST_FAIL, n, i) += (c1 || c4 || c5) ? 1.0 : 0.0;
            fld(a.acc, D2D_ST_COLLISION, n, i) += (c1 && !c2 && !c4 && !c5) ? 1.0 : 0.0;
            fld(a.acc, D2D_ST_APE, n, i) += ape;
            fld(a.acc, D2D_ST_LEN, n, i) += (double)t;
        }
        if (done && auto_reset) {
            const double x = sh.sp[0][lane], y = sh.sp[1][lane], th = sh.sp[2][lane];
            const double bodies[18] = {x, y, th, 0.0, 0.0, 0.0, sh.sp[3][lane], sh.sp[4][lane], th, 0.0, 0.0, 0.0,
                                       sh.sp[5][lane], sh.sp[6][lane], th, 0.0, 0.0, 0.0};
#pragma unroll
            for (int f = 0; f < 18; ++f) fld(a.st, f, n, i) = bodies[f];
#pragma unroll
            for (int k = 0; k < 12; ++k) fld(a.st, D2D_S_J + k, n, i) = 0.0;
            fld(a.st, D2D_S_PATH_ERR, n, i) = 0.0;
            fld(a.st, D2D_S_TOT_REW, n, i) = 0.0;
            fld(a.ist, D2D_I_T, n, i) = 0;
            fld(a.ist, D2D_I_FLAGS, n, i) = (int32_t)sh.rflags[lane];
            fld(a.ist, D2D_I_EPISODE, n, i) = (int32_t)(sh.ep[lane] + 1u);
        } else {
            fld(a.st, D2D_S_PATH_ERR, n, i) = path_err;
            fld(a.st, D2D_S_TOT_REW, n, i) = tot_rew;
            fld(a.ist, D2D_I_T, n, i) = t;
            fld(a.ist, D2D_I_FLAGS, n, i) = (int32_t)flags;
        }
    }
    STAMP(6);
}

// ------------------------------------------------------------------------------------------ K2
template <bool LDS>
__global__ __launch_bounds__(BLOCK) void d2d_reset_kernel(StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) d2d_scn s_scn[];
    const d2d_scn* scns = stage_scenarios<LDS, BLOCK>(a, s_scn);
    __syncthreads();
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= a.n) return;
    if (a.mask && !a.mask[i]) return;
    const int n = a.n;
    const d2d_scn& s = scns[(a.env_scn && a.n_scn > 1) ? a.env_scn[i] : 0];
    const uint32_t ep = (uint32_t)fld(a.ist, D2D_I_EPISODE, n, i);
    double x, y, th;
    spawn_draw(s, a.seed, (uint32_t)a.cfg.env_id_base + (uint32_t)i, ep, x, y, th);
    double sl, cl, sr, cr;
    sincos_d(th + PI, sl, cl);
    sincos_d(th, sr, cr);
    const double bodies[18] = {x, y, th, 0.0, 0.0, 0.0, cl * DRONE_R + x, sl * DRONE_R + y, th, 0.0, 0.0, 0.0,
                               cr * DRONE_R + x, sr * DRONE_R + y, th, 0.0, 0.0, 0.0};
    uint32_t flags = 0;
    double obs[D2D_OBS_DIM];
    observe(a.cfg, s, Body{x, y, th, 0.0, 0.0, 0.0}, flags, obs);
#pragma unroll
    for (int f = 0; f < 18; ++f) fld(a.st, f, n, i) = bodies[f];
#pragma unroll
    for (int k = 0; k < 12; ++k) fld(a.st, D2D_S_J + k, n, i) = 0.0;
    fld(a.st, D2D_S_PATH_ERR, n, i) = 0.0;
    fld(a.st, D2D_S_TOT_REW, n, i) = 0.0;
    fld(a.ist, D2D_I_T, n, i) = 0;
    fld(a.ist, D2D_I_FLAGS, n, i) = (int32_t)flags;
    fld(a.ist, D2D_I_EPISODE, n, i) = (int32_t)(ep + 1u);
    if (a.obs) {
#pragma unroll
        for (int k = 0; k < D2D_OBS_DIM; ++k) a.obs[(size_t)i * D2D_OBS_DIM + k] = (float)obs[k];
    }
}

// ------------------------------------------------------------------------------------------ K3
// one workgroup per statistic; fixed per-lane stride order + fixed LDS tree => bitwise reproducible
__global__ __launch_bounds__(BLOCK) void d2d_stats_kernel(const double* acc, int n, double* out, int clear,
                                                          double* acc_w) {
    __shared__ double red[BLOCK];
    const int k = blockIdx.x;
    const double* src = acc + (size_t)k * n;
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += BLOCK) s += src[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = BLOCK / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[k] = red[0];
    if (clear) {
        double* dst = acc_w + (size_t)k * n;
        for (int i = threadIdx.x; i < n; i += BLOCK) dst[i] = 0.0;
    }
}

}  // namespace d2dk
