// d2d_hip.hip -- kernels + C ABI of libdrone2d_hip.so (see include/drone2d.h).
//
// Kernels: see d2d_kernels.h (K1 cooperative step, K2 masked reset, K3 episode statistics, K4 reset
// observation cache fill).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "d2d_kernels.h"

using namespace d2dk;

#ifndef D2D_BRTAB
#define D2D_BRTAB 1  // 0: searches without the golden-march tables (diagnostic A/B builds only)
#endif

namespace {
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
    d2d::Scn* scn = nullptr;    // device table: ABI scenarios + derived fields
    d2d::BrTab* brt = nullptr;  // golden-march tables of the scenarios (d2d_brtab_kernel)
    int32_t* env_scn = nullptr;
    uint64_t seed = 0;
    bool reset_done = false;
    uint64_t* stamps = nullptr;  // diagnostic builds (D2D_STAMPS) only
    // auto-reset observation cache (d2d_kernels.h, "Auto-reset observation cache")
    float* rc_obs = nullptr;     // [n][27]
    int32_t* rc_rfl = nullptr;   // [n]
    int32_t* rc_tag = nullptr;   // [n]
    bool rc_dirty = true;        // scenarios changed since the cache was last dropped
    uint64_t n_steps = 0;        // d2d_step calls (fill cadence)
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
    a.brt = D2D_BRTAB ? h->brt : nullptr;
    a.env_scn = h->env_scn;
    a.cfg = h->cfg;
    a.damping_dt = std::pow(h->cfg.damping, 1.0 / 60.0);
    a.seed = h->seed;
    a.stamps = h->stamps;
    a.rc_obs = h->rc_obs;
    a.rc_rfl = h->rc_rfl;
    a.rc_tag = h->rc_tag;
    return a;
}

// K4: fill every cache entry that does not belong to its env's current episode, ordered on `stream`
hipError_t rc_fill(d2d_t* h, hipStream_t stream) {
    StepArgs a = make_args(h);
    const dim3 grid((h->n + BLOCK - 1) / BLOCK);
    if (sizeof(d2d::Scn) * (size_t)h->n_scn <= K2_LDS_BUDGET)
        hipLaunchKernelGGL(d2d_fill_kernel<true>, grid, dim3(BLOCK), sizeof(d2d::Scn) * h->n_scn, stream, a);
    else
        hipLaunchKernelGGL(d2d_fill_kernel<false>, grid, dim3(BLOCK), 0, stream, a);
    return hipGetLastError();
}
// drop every entry (new seed, counters or scenarios) and refill, ordered on `stream`
hipError_t rc_rebuild(d2d_t* h, hipStream_t stream) {
    hipError_t e = hipMemsetAsync(h->rc_tag, 0xFF, sizeof(int32_t) * (size_t)h->n, stream);
    if (e == hipSuccess && D2D_FILL_PERIOD > 0) e = rc_fill(h, stream);
    if (e == hipSuccess) h->rc_dirty = false;
    return e;
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
        (e = hipMalloc(&h->env_scn, sizeof(int32_t) * n)) != hipSuccess ||
        (e = hipMalloc(&h->rc_obs, sizeof(float) * D2D_OBS_DIM * n)) != hipSuccess ||
        (e = hipMalloc(&h->rc_rfl, sizeof(int32_t) * n)) != hipSuccess ||
        (e = hipMalloc(&h->rc_tag, sizeof(int32_t) * n)) != hipSuccess) {
        d2d_destroy(h);
        return hip_fail(e, "d2d_create: hipMalloc");
    }
    (void)hipMemset(h->st, 0, sizeof(double) * D2D_NSTATE * n);
    (void)hipMemset(h->ist, 0, sizeof(int32_t) * D2D_NISTATE * n);
    (void)hipMemset(h->acc, 0, sizeof(double) * D2D_NSTATS * n);
    (void)hipMemset(h->env_scn, 0, sizeof(int32_t) * n);
    (void)hipMemset(h->rc_tag, 0xFF, sizeof(int32_t) * n);
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
    if (h->brt) (void)hipFree(h->brt);
    if (h->env_scn) (void)hipFree(h->env_scn);
    if (h->rc_obs) (void)hipFree(h->rc_obs);
    if (h->rc_rfl) (void)hipFree(h->rc_rfl);
    if (h->rc_tag) (void)hipFree(h->rc_tag);
    delete h;
}

int32_t d2d_n_envs(const d2d_t* h) { return h ? h->n : -1; }

#ifdef D2D_STAMPS
// diagnostic builds only: K1 writes 8 s_memtime stamps per wave into buf ([n_blocks*4][8] u64)
int32_t d2d_debug_stamps(d2d_t* h, uint64_t* buf) {
    if (!h) return fail(D2D_E_ARG, "d2d_debug_stamps: null handle");
    h->stamps = buf;
    return D2D_OK;
}
#endif

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
    if (h->brt) {
        (void)hipFree(h->brt);
        h->brt = nullptr;
    }
    std::vector<d2d::Scn> tab((size_t)n_scn);
    for (int k = 0; k < n_scn; ++k) {
        if (!d2d::scn_build(scns[k], tab[k]))
            return fail(D2D_E_ARG, "d2d_set_scenarios: us[n_wps-2] - us[n_wps-3] must exceed 0.001");
    }
    const size_t bytes = sizeof(d2d::Scn) * (size_t)n_scn;
    if ((e = hipMalloc(&h->scn, bytes)) != hipSuccess) return hip_fail(e, "hipMalloc scn");
    if ((e = hipMemcpy(h->scn, tab.data(), bytes, hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "hipMemcpy scn");
    // golden-march tables: forced searches on the device (same arithmetic as the step kernels)
    const size_t tbytes = sizeof(d2d::BrTab) * (size_t)n_scn;
    if ((e = hipMalloc(&h->brt, tbytes)) != hipSuccess) return hip_fail(e, "hipMalloc brt");
    if ((e = hipMemset(h->brt, 0, tbytes)) != hipSuccess) return hip_fail(e, "hipMemset brt");
    hipLaunchKernelGGL(d2d_brtab_kernel, dim3((2 * n_scn + 63) / 64), dim3(64), 0, 0, h->scn, n_scn, h->brt);
    if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "d2d_brtab_kernel launch");
    if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "d2d_brtab_kernel");
    if (env_scn_host) {
        if ((e = hipMemcpy(h->env_scn, env_scn_host, sizeof(int32_t) * (size_t)h->n, hipMemcpyHostToDevice)) !=
            hipSuccess)
            return hip_fail(e, "hipMemcpy env_scn");
    } else if ((e = hipMemset(h->env_scn, 0, sizeof(int32_t) * (size_t)h->n)) != hipSuccess) {
        return hip_fail(e, "hipMemset env_scn");
    }
    h->n_scn = n_scn;
    h->rc_dirty = true;  // cached reset observations belong to the old scenarios
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
    if (sizeof(d2d::Scn) * (size_t)h->n_scn <= K2_LDS_BUDGET)
        hipLaunchKernelGGL(d2d_reset_kernel<true>, grid, dim3(BLOCK), sizeof(d2d::Scn) * h->n_scn, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(d2d_reset_kernel<false>, grid, dim3(BLOCK), 0, (hipStream_t)stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "d2d_reset launch");
    // cached next-reset observations depend on the seed and the episode counters: drop and refill
    if ((e = rc_rebuild(h, (hipStream_t)stream)) != hipSuccess) return hip_fail(e, "d2d_reset: cache rebuild");
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
    hipError_t e;
    if (h->rc_dirty && (e = rc_rebuild(h, (hipStream_t)stream)) != hipSuccess)
        return hip_fail(e, "d2d_step: cache rebuild");
    StepArgs a = make_args(h);
    a.act = act_dev;
    a.obs = obs_dev;
    a.rew = rew_dev;
    a.term = term_dev;
    a.trunc = trunc_dev;
    a.info = info_dev;
    a.tobs = term_obs_dev;
    const dim3 grid((h->n + EPB - 1) / EPB);
    const size_t lds_scn = sizeof(d2d::Scn) * (size_t)h->n_scn, lds_hot = sizeof(d2d::BtHot) * (size_t)h->n_scn;
    if (a.brt && lds_scn + lds_hot + sizeof(K1Shared) <= K1_LDS_BUDGET)
        hipLaunchKernelGGL((d2d_step_kernel<true, true>), grid, dim3(K1_THREADS), lds_scn + lds_hot, (hipStream_t)stream, a);
    else if (lds_scn + sizeof(K1Shared) <= K1_LDS_BUDGET)
        hipLaunchKernelGGL((d2d_step_kernel<true, false>), grid, dim3(K1_THREADS), lds_scn, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL((d2d_step_kernel<false, false>), grid, dim3(K1_THREADS), 0, (hipStream_t)stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "d2d_step launch");
    if (D2D_FILL_PERIOD > 0 && h->cfg.auto_reset && ++h->n_steps % D2D_FILL_PERIOD == 0 &&
        (e = rc_fill(h, (hipStream_t)stream)) != hipSuccess)
        return hip_fail(e, "d2d_step: cache fill");
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
    if ((e = rc_rebuild(h, (hipStream_t)stream)) != hipSuccess) return hip_fail(e, "d2d_set_state: cache rebuild");
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

int32_t d2d_selftest(int32_t which, int64_t n, uint64_t seed, uint64_t* mismatches) {
    if (!mismatches || n < 0 || which < 0 || which > 2) return fail(D2D_E_ARG, "d2d_selftest: bad arguments");
    unsigned long long* bad = nullptr;
    hipError_t e;
    if ((e = hipMalloc(&bad, sizeof(unsigned long long))) != hipSuccess) return hip_fail(e, "d2d_selftest alloc");
    (void)hipMemset(bad, 0, sizeof(unsigned long long));
    hipLaunchKernelGGL(d2d_selftest_kernel, dim3(2048), dim3(256), 0, 0, which, (long long)n, seed, bad);
    e = hipGetLastError();
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(bad);
    if (e != hipSuccess) return hip_fail(e, "d2d_selftest");
    *mismatches = (uint64_t)h;
    return D2D_OK;
}

}  // extern "C"
