// d2d_hip.hip -- kernels + C ABI of libdrone2d_hip.so (see include/drone2d.h).
//
// Kernels (gfx950, one lane per env, 256-lane workgroups):
//   K1 d2d_step_kernel   thrust -> Chipmunk-equivalent step -> collision -> k-nearest sensing ->
//                        Brent closest point -> 27-dim obs -> reward/termination -> SB3-style
//                        auto-reset; SoA fp64 state in HBM, scenario tables staged in LDS, obs rows
//                        transposed through LDS so the [N,27] fp32 store is one contiguous stream.
//   K2 d2d_reset_kernel  masked reset: Philox spawn draw + observation.
//   K3 d2d_stats_kernel  fixed-order reduction of the per-env finished-episode accumulators
//                        (feeds the single RCCL all-reduce of the multi-GPU path).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "d2d_device.h"

using namespace d2d;

namespace {

constexpr int BLOCK = 256;
constexpr int MAX_LDS_SCN = 8;

struct StepArgs {
    int n;
    int n_scn;
    double* st;            // [NSTATE][n]
    int32_t* ist;          // [NISTATE][n]
    double* acc;           // [NSTATS][n]
    const d2d_scn* scn;    // [n_scn]
    const int32_t* env_scn;  // [n] or null (all scenario 0)
    d2d_cfg cfg;
    double damping_dt;     // pow(cfg.damping, dt), host glibc
    uint64_t seed;
    const float* act;
    float* obs;
    float* rew;
    uint8_t* term;
    uint8_t* trunc;
    float* info;
    float* tobs;
    const uint8_t* mask;   // reset kernel only
};

template <bool LDS>
__device__ __forceinline__ const d2d_scn* stage_scenarios(const StepArgs& a, d2d_scn* lds) {
    if (!LDS) return a.scn;
    const int words = a.n_scn * (int)(sizeof(d2d_scn) / 8);
    const double* src = reinterpret_cast<const double*>(a.scn);
    double* dst = reinterpret_cast<double*>(lds);
    for (int k = threadIdx.x; k < words; k += BLOCK) dst[k] = src[k];
    __syncthreads();
    return lds;
}

__device__ __forceinline__ void load_state(const StepArgs& a, int i, Body B[3], double j[12]) {
    const size_t n = (size_t)a.n;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        B[b].px = a.st[(size_t)(6 * b + 0) * n + i];
        B[b].py = a.st[(size_t)(6 * b + 1) * n + i];
        B[b].a = a.st[(size_t)(6 * b + 2) * n + i];
        B[b].vx = a.st[(size_t)(6 * b + 3) * n + i];
        B[b].vy = a.st[(size_t)(6 * b + 4) * n + i];
        B[b].w = a.st[(size_t)(6 * b + 5) * n + i];
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) j[k] = a.st[(size_t)(D2D_S_J + k) * n + i];
}
__device__ __forceinline__ void store_state(const StepArgs& a, int i, const Body B[3], const double j[12],
                                            double path_err, double tot_rew) {
    const size_t n = (size_t)a.n;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        a.st[(size_t)(6 * b + 0) * n + i] = B[b].px;
        a.st[(size_t)(6 * b + 1) * n + i] = B[b].py;
        a.st[(size_t)(6 * b + 2) * n + i] = B[b].a;
        a.st[(size_t)(6 * b + 3) * n + i] = B[b].vx;
        a.st[(size_t)(6 * b + 4) * n + i] = B[b].vy;
        a.st[(size_t)(6 * b + 5) * n + i] = B[b].w;
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) a.st[(size_t)(D2D_S_J + k) * n + i] = j[k];
    a.st[(size_t)D2D_S_PATH_ERR * n + i] = path_err;
    a.st[(size_t)D2D_S_TOT_REW * n + i] = tot_rew;
}

// test-mode spawn (drone_2d_env.py:218-311, Drone.py:20-52): frame at (x, y, th), motors rigidly
// at +-40 along the body axis, zero velocities, zero joint impulses.
__device__ __forceinline__ void spawn(const StepArgs& a, const d2d_scn& s, int i, uint32_t episode, Body B[3],
                                      double j[12]) {
    uint32_t o[4];
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
    const uint32_t gid = (uint32_t)a.cfg.env_id_base + (uint32_t)i;
    philox(gid, episode, 0u, 0u, k0, k1, o);
    const double u0 = u53(o[0], o[1]), u1 = u53(o[2], o[3]);
    philox(gid, episode, 1u, 0u, k0, k1, o);
    const double u2 = u53(o[0], o[1]);
    const double x = s.spawn_xmin + (s.spawn_xmax - s.spawn_xmin) * u0;
    const double y = s.spawn_ymin + (s.spawn_ymax - s.spawn_ymin) * u1;
    const double th = s.spawn_amin + (s.spawn_amax - s.spawn_amin) * u2;
    B[0] = Body{x, y, th, 0.0, 0.0, 0.0};
    B[1] = Body{cos(th + PI) * DRONE_R + x, sin(th + PI) * DRONE_R + y, th, 0.0, 0.0, 0.0};
    B[2] = Body{cos(th) * DRONE_R + x, sin(th) * DRONE_R + y, th, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 12; ++k) j[k] = 0.0;
}

__device__ __forceinline__ void write_obs_row(float* dst, const double* obs) {
#pragma unroll
    for (int k = 0; k < D2D_OBS_DIM; ++k) dst[k] = (float)obs[k];
}

// ------------------------------------------------------------------------------------------ K1
template <bool LDS>
__global__ __launch_bounds__(BLOCK) void d2d_step_kernel(StepArgs a) {
    __shared__ d2d_scn s_scn[LDS ? MAX_LDS_SCN : 1];
    __shared__ float s_obs[BLOCK * D2D_OBS_DIM];
    const d2d_scn* scns = stage_scenarios<LDS>(a, s_scn);
    const int i0 = blockIdx.x * BLOCK;
    const int i = i0 + threadIdx.x;
    if (i < a.n) {
        const size_t n = (size_t)a.n;
        const d2d_scn& s = scns[(a.env_scn && a.n_scn > 1) ? a.env_scn[i] : 0];
        Body B[3];
        double j[12];
        load_state(a, i, B, j);
        double path_err = a.st[(size_t)D2D_S_PATH_ERR * n + i];
        double tot_rew = a.st[(size_t)D2D_S_TOT_REW * n + i];
        int t = a.ist[(size_t)D2D_I_T * n + i];
        uint32_t flags = (uint32_t)a.ist[(size_t)D2D_I_FLAGS * n + i];
        // thrust in float32 exactly as SB3's float32 action hits drone_2d_env.py:400-401
        const float2 act = reinterpret_cast<const float2*>(a.act)[i];
        const float fs = (float)a.cfg.force_scale;
        const float lf = __fmul_rn(__fadd_rn(act.x / 2.0f, 0.5f), fs);
        const float rf = __fmul_rn(__fadd_rn(act.y / 2.0f, 0.5f), fs);
        const bool hit = space_step(s, a.damping_dt, B, j, (double)lf, (double)rf);
        if (hit) flags |= D2D_FLAG_COLLIDED;
        t += 1;
        double obs[D2D_OBS_DIM];
        observe(a.cfg, s, B[0], flags, obs);
        const Reward R = reward_fn(a.cfg, s, obs, (flags & D2D_FLAG_COLLIDED) != 0, t);
        path_err += R.dist_path;
        const double ape = path_err / (double)t;
        tot_rew += R.reward;
        const bool done = R.cause != 0;
        bool trunc = false, term = done;
        if (a.cfg.timeup_truncates && done && R.cause == D2D_END_TIMEUP) {
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
            r[D2D_INFO_CAUSE] = (float)R.cause;
            r[D2D_INFO_APE] = done ? (float)ape : 0.0f;
            r[D2D_INFO_TOTREW] = done ? (float)tot_rew : 0.0f;
            r[D2D_INFO_REWARD] = (float)R.reward;
        }
        if (done) {
            // per-env finished-episode accumulators (info counters of drone_2d_env.py:593-613)
            const bool c1 = R.cause & D2D_END_COLLISION, c2 = R.cause & D2D_END_REACH;
            const bool c4 = R.cause & D2D_END_TIMEUP, c5 = R.cause & D2D_END_AA;
            a.acc[D2D_ST_RETURN * n + i] += tot_rew;
            a.acc[D2D_ST_EPISODES * n + i] += 1.0;
            a.acc[D2D_ST_SUCCESS * n + i] += c2 ? 1.0 : 0.0;
            a.acc[D2D_ST_FAIL * n + i] += (c1 || c4 || c5) ? 1.0 : 0.0;
            a.acc[D2D_ST_COLLISION * n + i] += (c1 && !c2 && !c4 && !c5) ? 1.0 : 0.0;
            a.acc[D2D_ST_APE * n + i] += ape;
            a.acc[D2D_ST_LEN * n + i] += (double)t;
            if (a.tobs) write_obs_row(a.tobs + (size_t)i * D2D_OBS_DIM, obs);
            if (a.cfg.auto_reset) {
                const uint32_t ep = (uint32_t)a.ist[(size_t)D2D_I_EPISODE * n + i];
                spawn(a, s, i, ep, B, j);
                flags = 0;
                t = 0;
                path_err = 0.0;
                tot_rew = 0.0;
                observe(a.cfg, s, B[0], flags, obs);
                a.ist[(size_t)D2D_I_EPISODE * n + i] = (int32_t)(ep + 1u);
            }
        }
        store_state(a, i, B, j, path_err, tot_rew);
        a.ist[(size_t)D2D_I_T * n + i] = t;
        a.ist[(size_t)D2D_I_FLAGS * n + i] = (int32_t)flags;
#pragma unroll
        for (int k = 0; k < D2D_OBS_DIM; ++k) s_obs[threadIdx.x * D2D_OBS_DIM + k] = (float)obs[k];
    }
    __syncthreads();
    // rows [i0, i0+rows) of obs are one contiguous span: store it with consecutive lanes
    const int rows = min(BLOCK, a.n - i0);
    const int words = rows * D2D_OBS_DIM;
    float* dst = a.obs + (size_t)i0 * D2D_OBS_DIM;
    for (int k = threadIdx.x; k < words; k += BLOCK) dst[k] = s_obs[k];
}

// ------------------------------------------------------------------------------------------ K2
template <bool LDS>
__global__ __launch_bounds__(BLOCK) void d2d_reset_kernel(StepArgs a) {
    __shared__ d2d_scn s_scn[LDS ? MAX_LDS_SCN : 1];
    const d2d_scn* scns = stage_scenarios<LDS>(a, s_scn);
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= a.n) return;
    if (a.mask && !a.mask[i]) return;
    const size_t n = (size_t)a.n;
    const d2d_scn& s = scns[(a.env_scn && a.n_scn > 1) ? a.env_scn[i] : 0];
    const uint32_t ep = (uint32_t)a.ist[(size_t)D2D_I_EPISODE * n + i];
    Body B[3];
    double j[12];
    spawn(a, s, i, ep, B, j);
    uint32_t flags = 0;
    double obs[D2D_OBS_DIM];
    observe(a.cfg, s, B[0], flags, obs);
    store_state(a, i, B, j, 0.0, 0.0);
    a.ist[(size_t)D2D_I_T * n + i] = 0;
    a.ist[(size_t)D2D_I_FLAGS * n + i] = (int32_t)flags;
    a.ist[(size_t)D2D_I_EPISODE * n + i] = (int32_t)(ep + 1u);
    if (a.obs) write_obs_row(a.obs + (size_t)i * D2D_OBS_DIM, obs);
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

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char* what) {
    return fail(D2D_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

struct d2d_handle {
    d2d_cfg cfg;
    int n = 0;
    int device = 0;
    int n_scn = 0;
    double* st = nullptr;
    int32_t* ist = nullptr;
    double* acc = nullptr;
    d2d_scn* scn = nullptr;
    int32_t* env_scn = nullptr;
    uint64_t seed = 0;
    bool reset_done = false;
};

namespace {

StepArgs make_args(const d2d_t* h) {
    StepArgs a{};
    a.n = h->n;
    a.n_scn = h->n_scn;
    a.st = h->st;
    a.ist = h->ist;
    a.acc = h->acc;
    a.scn = h->scn;
    a.env_scn = h->env_scn;
    a.cfg = h->cfg;
    a.damping_dt = std::pow(h->cfg.damping, 1.0 / 60.0);
    a.seed = h->seed;
    return a;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

extern "C" {

int32_t d2d_abi_version(void) { return D2D_ABI_VERSION; }
const char* d2d_last_error(void) { return g_err.c_str(); }

int32_t d2d_create(const d2d_cfg* cfg, int32_t n_envs, int32_t device, d2d_t** out) {
    if (!cfg || !out || n_envs <= 0) return fail(D2D_E_ARG, "d2d_create: null cfg/out or n_envs <= 0");
    if (cfg->n_steps <= 0) return fail(D2D_E_ARG, "d2d_create: n_steps must be > 0");
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    if (device < 0 || device >= ndev) return fail(D2D_E_ARG, "d2d_create: bad device index");
    DeviceGuard g(device);
    d2d_t* h = new (std::nothrow) d2d_t();
    if (!h) return fail(D2D_E_NOMEM, "d2d_create: host allocation failed");
    h->cfg = *cfg;
    h->n = n_envs;
    h->device = device;
    const size_t n = (size_t)n_envs;
    if ((e = hipMalloc(&h->st, sizeof(double) * D2D_NSTATE * n)) != hipSuccess ||
        (e = hipMalloc(&h->ist, sizeof(int32_t) * D2D_NISTATE * n)) != hipSuccess ||
        (e = hipMalloc(&h->acc, sizeof(double) * D2D_NSTATS * n)) != hipSuccess ||
        (e = hipMalloc(&h->env_scn, sizeof(int32_t) * n)) != hipSuccess) {
        d2d_destroy(h);
        return hip_fail(e, "d2d_create: hipMalloc");
    }
    (void)hipMemset(h->st, 0, sizeof(double) * D2D_NSTATE * n);
    (void)hipMemset(h->ist, 0, sizeof(int32_t) * D2D_NISTATE * n);
    (void)hipMemset(h->acc, 0, sizeof(double) * D2D_NSTATS * n);
    (void)hipMemset(h->env_scn, 0, sizeof(int32_t) * n);
    if ((e = hipDeviceSynchronize()) != hipSuccess) {
        d2d_destroy(h);
        return hip_fail(e, "d2d_create: memset");
    }
    *out = h;
    return D2D_OK;
}

void d2d_destroy(d2d_t* h) {
    if (!h) return;
    DeviceGuard g(h->device);
    if (h->st) (void)hipFree(h->st);
    if (h->ist) (void)hipFree(h->ist);
    if (h->acc) (void)hipFree(h->acc);
    if (h->scn) (void)hipFree(h->scn);
    if (h->env_scn) (void)hipFree(h->env_scn);
    delete h;
}

int32_t d2d_n_envs(const d2d_t* h) { return h ? h->n : -1; }

int32_t d2d_set_scenarios(d2d_t* h, const d2d_scn* scns, int32_t n_scn, const int32_t* env_scn_host) {
    if (!h || !scns || n_scn <= 0) return fail(D2D_E_ARG, "d2d_set_scenarios: null handle/scenarios or n_scn <= 0");
    for (int k = 0; k < n_scn; ++k) {
        const d2d_scn& s = scns[k];
        if (s.n_wps < 3 || s.n_wps > D2D_MAX_WPS)
            return fail(D2D_E_ARG, "d2d_set_scenarios: n_wps out of range [3, D2D_MAX_WPS]");
        if (s.n_circles < 0 || s.n_circles > D2D_MAX_CIRCLES)
            return fail(D2D_E_ARG, "d2d_set_scenarios: n_circles out of range [0, D2D_MAX_CIRCLES]");
    }
    if (env_scn_host) {
        for (int i = 0; i < h->n; ++i)
            if (env_scn_host[i] < 0 || env_scn_host[i] >= n_scn)
                return fail(D2D_E_ARG, "d2d_set_scenarios: env scenario index out of range");
    }
    DeviceGuard g(h->device);
    hipError_t e;
    if (h->scn) {
        (void)hipFree(h->scn);
        h->scn = nullptr;
    }
    if ((e = hipMalloc(&h->scn, sizeof(d2d_scn) * (size_t)n_scn)) != hipSuccess) return hip_fail(e, "hipMalloc scn");
    if ((e = hipMemcpy(h->scn, scns, sizeof(d2d_scn) * (size_t)n_scn, hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "hipMemcpy scn");
    if (env_scn_host) {
        if ((e = hipMemcpy(h->env_scn, env_scn_host, sizeof(int32_t) * (size_t)h->n, hipMemcpyHostToDevice)) !=
            hipSuccess)
            return hip_fail(e, "hipMemcpy env_scn");
    } else if ((e = hipMemset(h->env_scn, 0, sizeof(int32_t) * (size_t)h->n)) != hipSuccess) {
        return hip_fail(e, "hipMemset env_scn");
    }
    h->n_scn = n_scn;
    return D2D_OK;
}

int32_t d2d_reset(d2d_t* h, const uint8_t* mask_dev, uint64_t seed, float* obs_dev, void* stream) {
    if (!h) return fail(D2D_E_ARG, "d2d_reset: null handle");
    if (h->n_scn <= 0) return fail(D2D_E_STATE, "d2d_reset: call d2d_set_scenarios first");
    DeviceGuard g(h->device);
    h->seed = seed;
    StepArgs a = make_args(h);
    a.obs = obs_dev;
    a.mask = mask_dev;
    const dim3 grid((h->n + BLOCK - 1) / BLOCK);
    if (h->n_scn <= MAX_LDS_SCN)
        hipLaunchKernelGGL(d2d_reset_kernel<true>, grid, dim3(BLOCK), 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(d2d_reset_kernel<false>, grid, dim3(BLOCK), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "d2d_reset launch");
    h->reset_done = true;
    return D2D_OK;
}

int32_t d2d_step(d2d_t* h, const float* act_dev, float* obs_dev, float* rew_dev, uint8_t* term_dev,
                 uint8_t* trunc_dev, float* info_dev, float* term_obs_dev, void* stream) {
    if (!h || !act_dev || !obs_dev || !rew_dev || !term_dev || !trunc_dev)
        return fail(D2D_E_ARG, "d2d_step: null handle or required buffer");
    if (!h->reset_done) return fail(D2D_E_STATE, "d2d_step: call d2d_reset first");
    if (((uintptr_t)act_dev & 7u) != 0) return fail(D2D_E_ARG, "d2d_step: act_dev must be 8-byte aligned");
    DeviceGuard g(h->device);
    StepArgs a = make_args(h);
    a.act = act_dev;
    a.obs = obs_dev;
    a.rew = rew_dev;
    a.term = term_dev;
    a.trunc = trunc_dev;
    a.info = info_dev;
    a.tobs = term_obs_dev;
    const dim3 grid((h->n + BLOCK - 1) / BLOCK);
    if (h->n_scn <= MAX_LDS_SCN)
        hipLaunchKernelGGL(d2d_step_kernel<true>, grid, dim3(BLOCK), 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(d2d_step_kernel<false>, grid, dim3(BLOCK), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "d2d_step launch");
    return D2D_OK;
}

int32_t d2d_get_state(d2d_t* h, double* state_dev, int32_t* istate_dev, void* stream) {
    if (!h) return fail(D2D_E_ARG, "d2d_get_state: null handle");
    DeviceGuard g(h->device);
    hipError_t e;
    const size_t n = (size_t)h->n;
    if (state_dev &&
        (e = hipMemcpyAsync(state_dev, h->st, sizeof(double) * D2D_NSTATE * n, hipMemcpyDeviceToDevice,
                            (hipStream_t)stream)) != hipSuccess)
        return hip_fail(e, "d2d_get_state");
    if (istate_dev &&
        (e = hipMemcpyAsync(istate_dev, h->ist, sizeof(int32_t) * D2D_NISTATE * n, hipMemcpyDeviceToDevice,
                            (hipStream_t)stream)) != hipSuccess)
        return hip_fail(e, "d2d_get_state");
    return D2D_OK;
}

int32_t d2d_set_state(d2d_t* h, const double* state_dev, const int32_t* istate_dev, void* stream) {
    if (!h) return fail(D2D_E_ARG, "d2d_set_state: null handle");
    DeviceGuard g(h->device);
    hipError_t e;
    const size_t n = (size_t)h->n;
    if (state_dev &&
        (e = hipMemcpyAsync(h->st, state_dev, sizeof(double) * D2D_NSTATE * n, hipMemcpyDeviceToDevice,
                            (hipStream_t)stream)) != hipSuccess)
        return hip_fail(e, "d2d_set_state");
    if (istate_dev &&
        (e = hipMemcpyAsync(h->ist, istate_dev, sizeof(int32_t) * D2D_NISTATE * n, hipMemcpyDeviceToDevice,
                            (hipStream_t)stream)) != hipSuccess)
        return hip_fail(e, "d2d_set_state");
    h->reset_done = true;
    return D2D_OK;
}

int32_t d2d_episode_stats(d2d_t* h, double* out_dev, int32_t clear, void* stream) {
    if (!h || !out_dev) return fail(D2D_E_ARG, "d2d_episode_stats: null handle/out");
    DeviceGuard g(h->device);
    hipLaunchKernelGGL(d2d_stats_kernel, dim3(D2D_NSTATS), dim3(BLOCK), 0, (hipStream_t)stream, h->acc, h->n,
                       out_dev, clear, h->acc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "d2d_episode_stats launch");
    return D2D_OK;
}

}  // extern "C"
