// d2d_hip.hip -- kernels + C ABI of libdrone2d_hip.so (see include/drone2d.h).
//
// Kernels: see d2d_kernels.h (K1 cooperative step, K2 masked reset, K3 episode statistics, K4 reset
// observation cache fill).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "d2d_kernels.h"

using namespace d2dk;



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
    int ns = 0;   // state slots (columns of the internal [F][ns] arrays): n, or the grouped layout's
    int device = 0;
    int n_scn = 0;
    double* st = nullptr;
    int32_t* ist = nullptr;
    double* acc = nullptr;
    void* scn = nullptr;        // device table: ABI scenarios + derived fields, ScnF or ScnR (rm)
    bool rm = false;            // the table's layout: ScnR where K1 reads it from global memory
    d2d::BrTab* brt = nullptr;  // golden-march tables of the scenarios (d2d_brtab_kernel)
    int32_t* env_scn = nullptr;
    // pool mode: the scenario table has two halves of pool_n entries; resets draw from the half at
    // pool_base (host copy; the kernels read *pool_dev), d2d_refresh_pool fills and switches halves
    int pool_base = 0, pool_n = 0;
    int32_t* pool_dev = nullptr;
    int32_t* fill_ctl = nullptr;  // [2] K4's tick and finished-workgroup count
    uint64_t seed = 0;
    bool reset_done = false;
    uint64_t* stamps = nullptr;  // diagnostic builds (D2D_STAMPS) only
    // auto-reset observation cache (d2d_kernels.h, "Auto-reset observation cache")
    float* rc_obs = nullptr;     // [n][27]
    int32_t* rc_rfl = nullptr;   // [n]
    int32_t* rc_tag = nullptr;   // [n]
    bool rc_dirty = true;        // scenarios changed since the cache was last dropped
    // scenario-grouped slot layout (StepArgs::lane_env), built by d2d_set_scenarios
    int32_t* lane_env = nullptr;  // [ns] slot -> env (-1: padding)
    int32_t* wg_scn = nullptr;    // [ns / EPB] scenario of each slot group
    int32_t* env_slot = nullptr;  // [n] env -> slot
    int n_groups = 0;
    uint64_t n_steps = 0;        // d2d_step calls (fill cadence)
    // pool / fresh curriculum
    d2d_scn* abi = nullptr;      // [n_scn] ABI records of the table (pool and fresh modes: readback)
    int pool_valid = 0;          // pool mode: bit h = half h holds uploaded scenarios
    d2d_curriculum cur{};        // fresh mode: generator parameters
    int32_t* scn_tag = nullptr;  // fresh mode: [2 n] episode key of each slot
    int64_t* gclk = nullptr;     // fresh mode: [2 n] clock at generation
    int32_t* fresh_q = nullptr;  // fresh mode: [fresh_ring + FR_WORDS] K5's ring of slots to generate + its words
    size_t fresh_ring = 0;       // ring size: the power of two >= 2 n
    int64_t* clock = nullptr;    // [1] the step clock (K1 advances it)
    uint64_t fresh_seed = 0;
    bool fresh_seeded = false;
    int32_t generation = 0;      // bumped whenever captured graphs' pointers go stale
    int n_cu = 0;                      // compute units of the device
    std::vector<double> scn_cost;      // relative step cost per scenario (d2d_set_scenario_costs)
};

namespace {

StepArgs make_args(const d2d_t* h) {
    StepArgs a{};
    a.n = h->n;
    a.ns = h->ns;
    a.n_scn = h->n_scn;
    a.st = h->st;
    a.ist = h->ist;
    a.acc = h->acc;
    a.scn = h->scn;
    a.brt = h->brt;  // (null in fresh curriculum mode: docs/DESIGN_HISTORY.md "Round 4")
    a.env_scn = h->env_scn;
    a.pool_base = h->pool_dev;
    a.pool_n = h->pool_n;
    a.fill_ctl = h->fill_ctl;
    a.fill_every = FILL_EVERY;
    a.fill_force = 0;
    a.cfg = h->cfg;
    a.damping_dt = std::pow(h->cfg.damping, 1.0 / 60.0);
    a.seed = h->seed;
    a.stamps = h->stamps;
    a.rc_obs = h->rc_obs;
    a.rc_rfl = h->rc_rfl;
    a.rc_tag = h->rc_tag;
    a.lane_env = h->lane_env;
    a.wg_scn = h->wg_scn;
    a.scn_tag = h->scn_tag;
    a.clock = h->clock;
    if (h->cfg.scn_pool == 2 && h->fresh_q) {
        a.fq = h->fresh_q;
        a.fqc = reinterpret_cast<uint32_t*>(h->fresh_q + h->fresh_ring);
        a.fq_mask = (uint32_t)h->fresh_ring - 1u;
    }
    return a;
}

constexpr int GEN_GRID = 2048;  // K5b workgroups
// K5: the fresh curriculum's scenario slots (restore: every slot from its recipe), on `stream`
hipError_t fresh_regen(d2d_t* h, hipStream_t stream, bool restore = false, bool queued = false) {
    FreshArgs f{};
    f.n = h->n;
    f.ist = h->ist;
    f.env_scn = h->env_scn;
    f.cur = h->cur;
    f.W = h->cfg.screen_w;
    f.H = h->cfg.screen_h;
    f.seed = h->seed;
    f.env_id_base = (uint32_t)h->cfg.env_id_base;
    f.abi = h->abi;
    f.scn = static_cast<d2d::ScnR*>(h->scn);  // (fresh mode: h->rm)
    f.tag = h->scn_tag;
    f.gclk = h->gclk;
    f.clock = h->clock;
    f.queue = h->fresh_q;
    f.ring = reinterpret_cast<uint32_t*>(h->fresh_q + h->fresh_ring);
    f.mask = (uint32_t)h->fresh_ring - 1u;
    f.scan = queued ? 0 : 1;
    f.restore = restore ? 1 : 0;
#ifdef D2D_GEN_STAMPS
    f.stamps = h->stamps;
#endif
    const int items = restore ? 2 * h->n : h->n;
    if (!queued) hipLaunchKernelGGL(d2d_fresh_scan_kernel, dim3((items + 255) / 256), dim3(256), 0, stream, f);
    // one wave per queued slot: ~800 per step at 65 536 envs stepped with random actions (the items
    // of a step all run at once); a reset queues every env (the grid's workgroups then take several)
    hipLaunchKernelGGL(d2d_fresh_gen_kernel, dim3(std::min(items, GEN_GRID)), dim3(64), 0, stream, f);
    hipError_t e = hipGetLastError();
    // after a K1, K5b itself leaves the next tail (FreshRing: no launch; the round-4 clear kernel
    // after every K5b cost 5.5 us per step); after a scan, both tails to the head
    if (e != hipSuccess || queued) return e;
    hipLaunchKernelGGL(d2d_fresh_tail_kernel, dim3(1), dim3(64), 0, stream, f.ring);
    return hipGetLastError();
}
bool fresh_mode(const d2d_t* h) { return h->cfg.scn_pool == 2; }
size_t ring_size(size_t slots) {  // FreshRing: a power of two holding every slot
    size_t r = 64;
    while (r < slots) r <<= 1;
    return r;
}

// The scenario table's layout (d2d_device.h ScnF / ScnR): ScnR exactly when K1 will read it from
// global memory -- the fresh curriculum, and tables too big to stage (pools) unless the map is grouped
// (a grouped workgroup stages only its own scenarios).  d2d_step dispatches on the same rule.
bool table_rm(bool fresh, bool grouped, size_t n_total) {
    if (fresh) return true;
    if (grouped) return false;
    return sizeof(d2d::ScnF) * n_total + sizeof(K1Shared) > K1_LDS_BUDGET;
}
size_t scn_size(bool rm) { return rm ? sizeof(d2d::ScnR) : sizeof(d2d::ScnF); }
void* scn_at(const d2d_t* h, size_t k) { return static_cast<char*>(h->scn) + k * scn_size(h->rm); }
// host tables in either layout; entries with use(k) false stay zero.  False: a scenario scn_build refuses
template <class S>
bool build_tables_t(const d2d_scn* src, size_t n, std::vector<unsigned char>& out, const std::vector<bool>* use) {
    out.assign(n * sizeof(S), 0);
    for (size_t k = 0; k < n; ++k)
        if ((!use || (*use)[k]) && !d2d::scn_build(src[k], *reinterpret_cast<S*>(out.data() + k * sizeof(S))))
            return false;
    return true;
}
bool build_tables(bool rm, const d2d_scn* src, size_t n, std::vector<unsigned char>& out,
                  const std::vector<bool>* use = nullptr) {
    return rm ? build_tables_t<d2d::ScnR>(src, n, out, use) : build_tables_t<d2d::ScnF>(src, n, out, use);
}
void launch_brtab(bool rm, const void* scn, int n, d2d::BrTab* out) {
    const dim3 grid((2 * n + 63) / 64);
    if (rm) hipLaunchKernelGGL(d2d_brtab_kernel<d2d::ScnR>, grid, dim3(64), 0, 0, (const d2d::ScnR*)scn, n, out);
    else hipLaunchKernelGGL(d2d_brtab_kernel<d2d::ScnF>, grid, dim3(64), 0, 0, (const d2d::ScnF*)scn, n, out);
}

// K4: fill every cache entry that does not belong to its env's current episode, ordered on `stream`
hipError_t rc_fill(d2d_t* h, hipStream_t stream, bool force = false) {
    StepArgs a = make_args(h);
    a.fill_force = force ? 1 : 0;
    const dim3 grid((h->ns + FILL_SPB - 1) / FILL_SPB);
    // dynamic LDS padded to K1's per-workgroup LDS, so K4 is resident 4 per CU as K1 (d2d_fill_kernel)
    const size_t pad = sizeof(d2d::ScnF) + sizeof(d2d::BtHot) + sizeof(K1Shared) - 2048;
    const size_t lds = scn_size(h->rm) * (size_t)h->n_scn;
    if (lds <= K2_LDS_BUDGET) {
        if (h->rm) hipLaunchKernelGGL((d2d_fill_kernel<true, true>), grid, dim3(BLOCK), std::max(lds, pad), stream, a);
        else hipLaunchKernelGGL((d2d_fill_kernel<true, false>), grid, dim3(BLOCK), std::max(lds, pad), stream, a);
    } else {
        if (h->rm) hipLaunchKernelGGL((d2d_fill_kernel<false, true>), grid, dim3(BLOCK), pad, stream, a);
        else hipLaunchKernelGGL((d2d_fill_kernel<false, false>), grid, dim3(BLOCK), pad, stream, a);
    }
    return hipGetLastError();
}
// drop every entry (new seed, counters or scenarios) and refill, ordered on `stream`
hipError_t rc_rebuild(d2d_t* h, hipStream_t stream) {
    hipError_t e = hipMemsetAsync(h->rc_tag, 0xFF, sizeof(int32_t) * RC_SLOTS * (size_t)h->ns, stream);
    if (e == hipSuccess) e = rc_fill(h, stream, true);
    if (e == hipSuccess) h->rc_dirty = false;
    return e;
}

// Scenario-grouped slot layout for a static env -> scenario map with several scenarios: each K1
// workgroup then steps 64 envs of ONE scenario (no per-lane scenario divergence in the Brent
// search, one scenario + probe table staged in LDS) whose state is contiguous.  The envs, sorted
// by (scenario, id), are cut into ceil(n / 64) groups -- no padding between scenarios, so the grid
// is no larger than the identity layout's (at 65 536 envs: 1 024 workgroups = one resident round)
// and at most n_scn - 1 groups straddle scenarios: wg_scn = -(s + 2) for a group of scenarios s and
// s + 1 (K1 stages both scenarios in LDS; their probe tables are read through L1/L2), -1 for a group
// of three or more (everything through L1/L2).  Groups are then
// ordered by their first env id, so groups whose envs interleave (e.g. scenario = id mod 7) get
// consecutive numbers (xcd_group places consecutive numbers on one XCD).
constexpr double STRADDLE_W = 1.25;  // balance_groups: a straddling group's cost over its heavier scenario's
// host copy of the kernels' block -> group numbering (d2d_kernels.h xcd_group)
int xcd_group_host(int b, int nb) {
    const int per = nb / 8, rem = nb % 8, x = b % 8, k = b / 8;
    return (x < rem) ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
}
// Co-residency balance (mixed batches).  When every workgroup of K1 is resident at once (ng <= 4 x
// CUs), the dispatcher fills the CUs round by round in one fixed CU order, so blocks b, b + n_cu,
// b + 2 n_cu, ... share a CU (measured on MI355X: blocks congruent mod 256 share a CU, in every step
// of a replayed graph, tools/cu_map.py).  A step lasts as long as its slowest workgroup, and a heavy
// scenario's workgroup slows down when its CU also runs other heavy ones, so the groups of each XCD's
// chunk (xcd_group keeps a chunk of consecutive group numbers on one XCD) are dealt over the chunk's
// CUs by cost, heaviest first onto the least-loaded CU (straddling groups count 1.25 x their heavier
// scenario).  Renumbers the groups (lanes / ws) in place; the arithmetic is unchanged.
void balance_groups(int n_cu, const double* cost, int n_cost, std::vector<int32_t>& lanes, std::vector<int32_t>& ws) {
    const int ng = (int)ws.size();
    if (n_cu <= 0 || n_cu % 8 != 0 || ng > 4 * n_cu || ng < 2) return;
    double cmax = 0.0;
    for (int k = 0; k < n_cost; ++k) cmax = std::max(cmax, cost[k]);
    auto c = [&](int sc) { return (sc >= 0 && sc < n_cost) ? cost[sc] : cmax; };
    auto gcost = [&](int g) {
        const int w = ws[(size_t)g];
        return w >= 0 ? c(w) : (w <= -2 ? STRADDLE_W * std::max(c(-w - 2), c(-w - 1)) : 1.5 * cmax);
    };
    std::vector<int32_t> block_of((size_t)ng);  // group number -> the block that runs it
    for (int b = 0; b < ng; ++b) block_of[(size_t)xcd_group_host(b, ng)] = b;
    std::vector<int32_t> newnum((size_t)ng, -1);
    const int per = ng / 8, rem = ng % 8;
    for (int x = 0, first = 0; x < 8; ++x) {
        const int cnt = per + (x < rem ? 1 : 0);
        // the chunk's positions grouped by CU, each CU's positions in dispatch order
        std::vector<std::pair<int, int>> pos;  // (cu, position)
        for (int p = first; p < first + cnt; ++p) pos.emplace_back(block_of[(size_t)p] % n_cu, p);
        std::stable_sort(pos.begin(), pos.end(), [&](const std::pair<int, int>& u, const std::pair<int, int>& v) {
            return u.first != v.first ? u.first < v.first : block_of[(size_t)u.second] < block_of[(size_t)v.second];
        });
        std::vector<int> cus;
        std::vector<std::vector<int>> free_pos;
        for (const auto& q : pos) {
            if (cus.empty() || cus.back() != q.first) {
                cus.push_back(q.first);
                free_pos.emplace_back();
            }
            free_pos.back().push_back(q.second);
        }
        std::vector<double> load(cus.size(), 0.0);
        std::vector<size_t> used(cus.size(), 0);
        std::vector<int> gs;
        for (int g = first; g < first + cnt; ++g) gs.push_back(g);
        std::stable_sort(gs.begin(), gs.end(), [&](int u, int v) { return gcost(u) > gcost(v); });
        for (int g : gs) {
            size_t best = cus.size();
            for (size_t k = 0; k < cus.size(); ++k)
                if (used[k] < free_pos[k].size() && (best == cus.size() || load[k] < load[best])) best = k;
            newnum[(size_t)g] = free_pos[best][used[best]++];
            load[best] += gcost(g);
        }
        first += cnt;
    }
    std::vector<int32_t> l2(lanes.size(), -1), w2((size_t)ng, 0);
    for (int g = 0; g < ng; ++g) {
        const size_t d = (size_t)newnum[(size_t)g];
        w2[d] = ws[(size_t)g];
        for (int l = 0; l < EPB; ++l) l2[d * EPB + (size_t)l] = lanes[(size_t)g * EPB + (size_t)l];
    }
    lanes.swap(l2);
    ws.swap(w2);
}

void make_groups(int n, const int32_t* env_scn, int n_scn, std::vector<int32_t>& lanes, std::vector<int32_t>& ws) {
    std::vector<int32_t> order((size_t)n);
    for (int i = 0; i < n; ++i) order[(size_t)i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return env_scn[x] < env_scn[y]; });
    const size_t ng = ((size_t)n + EPB - 1) / EPB;
    std::vector<size_t> gi(ng);
    for (size_t g = 0; g < ng; ++g) gi[g] = g;
    std::sort(gi.begin(), gi.end(), [&](size_t x, size_t y) { return order[x * EPB] < order[y * EPB]; });
    lanes.assign(ng * EPB, -1);
    ws.assign(ng, 0);
    for (size_t g = 0; g < ng; ++g) {
        const size_t o = gi[g] * EPB;
        const int32_t lo = env_scn[order[o]];
        int32_t hi = lo;
        for (size_t l = 0; l < EPB && o + l < (size_t)n; ++l) {
            lanes[g * EPB + l] = order[o + l];
            hi = std::max(hi, env_scn[order[o + l]]);
        }
        // pure: the scenario; straddling exactly two consecutive scenarios: -(lo + 2); more: -1
        ws[g] = hi == lo ? lo : (hi == lo + 1 ? -(lo + 2) : -1);
    }
}

// Internal arrays of one slot layout.
struct Layout {
    int ns = 0;
    double* st = nullptr;
    int32_t* ist = nullptr;
    double* acc = nullptr;
    float* rc_obs = nullptr;
    int32_t* rc_rfl = nullptr;
    int32_t* rc_tag = nullptr;
    int32_t* lane_env = nullptr;
    int32_t* wg_scn = nullptr;
    int32_t* env_slot = nullptr;
};
void free_layout(Layout& L) {
    for (void* p : {(void*)L.st, (void*)L.ist, (void*)L.acc, (void*)L.rc_obs, (void*)L.rc_rfl, (void*)L.rc_tag,
                    (void*)L.lane_env, (void*)L.wg_scn, (void*)L.env_slot})
        if (p) (void)hipFree(p);
    L = Layout{};
}
// allocate a layout of n envs: identity (lanes empty) or grouped (lanes: slot -> env, ws: scenario
// per group); state zeroed, reset cache empty
hipError_t alloc_layout(Layout& L, int n, const std::vector<int32_t>& lanes, const std::vector<int32_t>& ws) {
    L = Layout{};
    L.ns = lanes.empty() ? n : (int)lanes.size();
    const size_t ns = (size_t)L.ns;
    hipError_t e;
    if ((e = hipMalloc(&L.st, sizeof(double) * D2D_NSTATE * ns)) != hipSuccess ||
        (e = hipMalloc(&L.ist, sizeof(int32_t) * D2D_NISTATE * ns)) != hipSuccess ||
        (e = hipMalloc(&L.acc, sizeof(double) * D2D_NSTATS * ns)) != hipSuccess ||
        (e = hipMalloc(&L.rc_obs, sizeof(float) * D2D_OBS_DIM * RC_SLOTS * ns)) != hipSuccess ||
        (e = hipMalloc(&L.rc_rfl, sizeof(int32_t) * RC_SLOTS * ns)) != hipSuccess ||
        (e = hipMalloc(&L.rc_tag, sizeof(int32_t) * RC_SLOTS * ns)) != hipSuccess ||
        (e = hipMemset(L.st, 0, sizeof(double) * D2D_NSTATE * ns)) != hipSuccess ||
        (e = hipMemset(L.ist, 0, sizeof(int32_t) * D2D_NISTATE * ns)) != hipSuccess ||
        (e = hipMemset(L.acc, 0, sizeof(double) * D2D_NSTATS * ns)) != hipSuccess ||
        (e = hipMemset(L.rc_tag, 0xFF, sizeof(int32_t) * RC_SLOTS * ns)) != hipSuccess) {
        free_layout(L);
        return e;
    }
    if (!lanes.empty()) {
        std::vector<int32_t> es((size_t)n, 0);
        for (size_t k = 0; k < lanes.size(); ++k)
            if (lanes[k] >= 0) es[(size_t)lanes[k]] = (int32_t)k;
        if ((e = hipMalloc(&L.lane_env, sizeof(int32_t) * ns)) != hipSuccess ||
            (e = hipMalloc(&L.wg_scn, sizeof(int32_t) * ws.size())) != hipSuccess ||
            (e = hipMalloc(&L.env_slot, sizeof(int32_t) * (size_t)n)) != hipSuccess ||
            (e = hipMemcpy(L.lane_env, lanes.data(), sizeof(int32_t) * ns, hipMemcpyHostToDevice)) != hipSuccess ||
            (e = hipMemcpy(L.wg_scn, ws.data(), sizeof(int32_t) * ws.size(), hipMemcpyHostToDevice)) != hipSuccess ||
            (e = hipMemcpy(L.env_slot, es.data(), sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice)) != hipSuccess) {
            free_layout(L);
            return e;
        }
    }
    return hipSuccess;
}
Layout take_layout(d2d_t* h) {
    Layout L;
    L.ns = h->ns;
    L.st = h->st;
    L.ist = h->ist;
    L.acc = h->acc;
    L.rc_obs = h->rc_obs;
    L.rc_rfl = h->rc_rfl;
    L.rc_tag = h->rc_tag;
    L.lane_env = h->lane_env;
    L.wg_scn = h->wg_scn;
    L.env_slot = h->env_slot;
    return L;
}
void put_layout(d2d_t* h, const Layout& L) {
    h->ns = L.ns;
    h->st = L.st;
    h->ist = L.ist;
    h->acc = L.acc;
    h->rc_obs = L.rc_obs;
    h->rc_rfl = L.rc_rfl;
    h->rc_tag = L.rc_tag;
    h->lane_env = L.lane_env;
    h->wg_scn = L.wg_scn;
    h->env_slot = L.env_slot;
    h->n_groups = L.lane_env ? L.ns / EPB : 0;
}
// every env's state, flags and accumulators from layout `from` to layout `to` (stream-ordered)
template <typename T>
hipError_t permute(const T* src, int sstride, const int32_t* sslot, T* dst, int dstride, const int32_t* dslot, int nf,
                   int n, hipStream_t stream) {
    hipLaunchKernelGGL(d2d_permute_kernel<T>, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, stream, src, sstride, sslot,
                       dst, dstride, dslot, nf, n);
    return hipGetLastError();
}
hipError_t move_state(const Layout& from, const Layout& to, int n) {
    hipError_t e;
    if ((e = permute(from.st, from.ns, from.env_slot, to.st, to.ns, to.env_slot, D2D_NSTATE, n, 0)) != hipSuccess ||
        (e = permute(from.ist, from.ns, from.env_slot, to.ist, to.ns, to.env_slot, D2D_NISTATE, n, 0)) != hipSuccess ||
        (e = permute(from.acc, from.ns, from.env_slot, to.acc, to.ns, to.env_slot, D2D_NSTATS, n, 0)) != hipSuccess)
        return e;
    return hipDeviceSynchronize();
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
    if (hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) h->n_cu = 256;
    const size_t n = (size_t)n_envs;
    Layout L;
    if ((e = hipMalloc(&h->env_scn, sizeof(int32_t) * n)) != hipSuccess ||
        (e = hipMalloc(&h->pool_dev, sizeof(int32_t))) != hipSuccess ||
        (e = hipMemset(h->pool_dev, 0, sizeof(int32_t))) != hipSuccess ||
        (e = hipMalloc(&h->fill_ctl, 2 * sizeof(int32_t))) != hipSuccess ||
        (e = hipMemset(h->fill_ctl, 0, 2 * sizeof(int32_t))) != hipSuccess ||
        (e = hipMalloc(&h->clock, sizeof(int64_t))) != hipSuccess ||
        (e = hipMemset(h->clock, 0, sizeof(int64_t))) != hipSuccess ||
        (e = alloc_layout(L, n_envs, {}, {})) != hipSuccess) {
        d2d_destroy(h);
        return hip_fail(e, "d2d_create: hipMalloc");
    }
    put_layout(h, L);
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
    Layout L = take_layout(h);
    free_layout(L);
    if (h->scn) (void)hipFree(h->scn);
    if (h->brt) (void)hipFree(h->brt);
    if (h->env_scn) (void)hipFree(h->env_scn);
    if (h->pool_dev) (void)hipFree(h->pool_dev);
    if (h->fill_ctl) (void)hipFree(h->fill_ctl);
    if (h->clock) (void)hipFree(h->clock);
    if (h->abi) (void)hipFree(h->abi);
    if (h->scn_tag) (void)hipFree(h->scn_tag);
    if (h->gclk) (void)hipFree(h->gclk);
    if (h->fresh_q) (void)hipFree(h->fresh_q);
    delete h;
}

int32_t d2d_n_envs(const d2d_t* h) { return h ? h->n : -1; }

#if defined(D2D_STAMPS) || defined(D2D_GEN_STAMPS)
// diagnostic builds only: K1 writes 8 s_memtime stamps per wave into buf ([n_blocks*4][8] u64)
int32_t d2d_debug_stamps(d2d_t* h, uint64_t* buf) {
    if (!h) return fail(D2D_E_ARG, "d2d_debug_stamps: null handle");
    h->stamps = buf;
    return D2D_OK;
}
#endif
#ifdef D2D_BSTAMP
// diagnostic builds only: the Brent-step stamps (d2d_device.h, D2D_BSTAMP): clear = 1 zeroes them,
// else copies [1024][64][8] u64 into out
int32_t d2d_debug_bstamps(uint64_t* out, int32_t clear) {
    void* p = nullptr;
    hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(d2d_bst));
    if (e == hipSuccess) e = clear ? hipMemset(p, 0, sizeof(uint64_t) * BST_N)
                                   : hipMemcpy(out, p, sizeof(uint64_t) * BST_N, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return e == hipSuccess ? D2D_OK : hip_fail(e, "d2d_debug_bstamps");
}
#endif

int32_t d2d_set_scenarios(d2d_t* h, const d2d_scn* scns, int32_t n_scn, const int32_t* env_scn_host) {
    if (!h || !scns || n_scn <= 0) return fail(D2D_E_ARG, "d2d_set_scenarios: null handle/scenarios or n_scn <= 0");
    if (fresh_mode(h)) return fail(D2D_E_ARG, "d2d_set_scenarios: fresh curriculum mode (cfg.scn_pool = 2) uses d2d_set_curriculum");
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
    // validate and build everything before touching the handle: a bad scenario leaves it as it was
    // pool mode: room for a second pool half (d2d_refresh_pool), zero until the first refresh
    const size_t T = (size_t)n_scn * (h->cfg.scn_pool ? 2 : 1);
    const bool grouped = env_scn_host && n_scn > 1 && !h->cfg.scn_pool;
    const bool rm = table_rm(false, grouped, T);
    std::vector<unsigned char> tab;
    if (!build_tables(rm, scns, (size_t)n_scn, tab))
        return fail(D2D_E_ARG, "d2d_set_scenarios: us[n_wps-2] - us[n_wps-3] must exceed 0.001");
    DeviceGuard g(h->device);
    hipError_t e;
    void* scn = nullptr;
    d2d::BrTab* brt = nullptr;
    d2d_scn* abi = nullptr;
    auto drop = [&](hipError_t err, const char* what) {
        if (scn) (void)hipFree(scn);
        if (brt) (void)hipFree(brt);
        if (abi) (void)hipFree(abi);
        return hip_fail(err, what);
    };
    const size_t sz = scn_size(rm);
    if ((e = hipMalloc(&scn, sz * T)) != hipSuccess) return drop(e, "hipMalloc scn");
    if ((e = hipMemset(scn, 0, sz * T)) != hipSuccess) return drop(e, "hipMemset scn");
    if ((e = hipMemcpy(scn, tab.data(), tab.size(), hipMemcpyHostToDevice)) != hipSuccess) return drop(e, "hipMemcpy scn");
    if (h->cfg.scn_pool) {  // pool mode keeps the ABI records for checkpoints / readback
        if ((e = hipMalloc(&abi, sizeof(d2d_scn) * T)) != hipSuccess) return drop(e, "hipMalloc abi");
        if ((e = hipMemset(abi, 0, sizeof(d2d_scn) * T)) != hipSuccess) return drop(e, "hipMemset abi");
        if ((e = hipMemcpy(abi, scns, sizeof(d2d_scn) * (size_t)n_scn, hipMemcpyHostToDevice)) != hipSuccess)
            return drop(e, "hipMemcpy abi");
    }
    // golden-march tables: forced searches on the device (same arithmetic as the step kernels)
    if ((e = hipMalloc(&brt, sizeof(d2d::BrTab) * T)) != hipSuccess) return drop(e, "hipMalloc brt");
    if ((e = hipMemset(brt, 0, sizeof(d2d::BrTab) * T)) != hipSuccess) return drop(e, "hipMemset brt");
    launch_brtab(rm, scn, n_scn, brt);
    if ((e = hipGetLastError()) != hipSuccess) return drop(e, "d2d_brtab_kernel launch");
    if ((e = hipMemset(h->pool_dev, 0, sizeof(int32_t))) != hipSuccess) return drop(e, "hipMemset pool");
    if ((e = hipDeviceSynchronize()) != hipSuccess) return drop(e, "d2d_brtab_kernel");
    // slot layout: grouped for a static mixed map (pool mode redraws scenarios at every reset);
    // the current state moves into the new layout
    std::vector<int32_t> lanes, ws;
    if (grouped) {
        make_groups(h->n, env_scn_host, n_scn, lanes, ws);
        if ((int)h->scn_cost.size() == n_scn) balance_groups(h->n_cu, h->scn_cost.data(), n_scn, lanes, ws);
    }
    Layout to;
    const bool relayout = !lanes.empty() || h->lane_env;
    if (relayout) {
        if ((e = alloc_layout(to, h->n, lanes, ws)) != hipSuccess) return drop(e, "d2d_set_scenarios: layout");
        if ((e = move_state(take_layout(h), to, h->n)) != hipSuccess) {
            free_layout(to);
            return drop(e, "d2d_set_scenarios: layout move");
        }
    }
    // commit: from here on the handle holds the new scenarios
    if (relayout) {
        Layout from = take_layout(h);
        put_layout(h, to);
        free_layout(from);
    }
    if (h->scn) (void)hipFree(h->scn);
    if (h->brt) (void)hipFree(h->brt);
    if (h->abi) (void)hipFree(h->abi);
    h->scn = scn;
    h->rm = rm;
    h->brt = brt;
    h->abi = abi;
    h->n_scn = (int)T;
    h->pool_base = 0;
    h->pool_n = n_scn;
    h->pool_valid = 1;
    h->generation += 1;  // the old tables are freed: captured graphs point at them
    h->rc_dirty = true;  // cached reset observations belong to the old scenarios
    if ((int)h->scn_cost.size() != n_scn) h->scn_cost.assign((size_t)n_scn, 1.0);
    e = env_scn_host ? hipMemcpy(h->env_scn, env_scn_host, sizeof(int32_t) * (size_t)h->n, hipMemcpyHostToDevice)
                     : hipMemset(h->env_scn, 0, sizeof(int32_t) * (size_t)h->n);
    if (e != hipSuccess) {
        // the env -> scenario map is unknown: no step or reset until the next d2d_set_scenarios
        h->n_scn = 0;
        h->reset_done = false;
        return hip_fail(e, "d2d_set_scenarios: env_scn upload");
    }
    return D2D_OK;
}

int32_t d2d_set_scenario_costs(d2d_t* h, const double* cost, int32_t n_scn) {
    if (!h || !cost) return fail(D2D_E_ARG, "d2d_set_scenario_costs: null argument");
    if (h->cfg.scn_pool || n_scn != h->n_scn) return fail(D2D_E_ARG, "d2d_set_scenario_costs: one cost per scenario (test mode)");
    for (int k = 0; k < n_scn; ++k)
        if (!(cost[k] >= 0.0)) return fail(D2D_E_ARG, "d2d_set_scenario_costs: costs must be >= 0");
    DeviceGuard g(h->device);
    hipError_t e;
    if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "d2d_set_scenario_costs: sync");
    h->scn_cost.assign(cost, cost + n_scn);
    if (h->lane_env) {
        // grouped layout: deal the groups over the CUs by the new costs (balance_groups); the state
        // moves into the renumbered layout, the reset cache refills
        std::vector<int32_t> es((size_t)h->n);
        if ((e = hipMemcpy(es.data(), h->env_scn, sizeof(int32_t) * (size_t)h->n, hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(e, "d2d_set_scenario_costs: env_scn");
        std::vector<int32_t> lanes, ws;
        make_groups(h->n, es.data(), n_scn, lanes, ws);
        balance_groups(h->n_cu, h->scn_cost.data(), n_scn, lanes, ws);
        Layout to;
        if ((e = alloc_layout(to, h->n, lanes, ws)) != hipSuccess) return hip_fail(e, "d2d_set_scenario_costs: layout");
        if ((e = move_state(take_layout(h), to, h->n)) != hipSuccess) {
            free_layout(to);
            return hip_fail(e, "d2d_set_scenario_costs: layout move");
        }
        Layout from = take_layout(h);
        put_layout(h, to);
        free_layout(from);
        h->generation += 1;  // captured graphs hold the old layout's buffers
        h->rc_dirty = true;
    }
    return D2D_OK;
}

int32_t d2d_get_group_layout(d2d_t* h, int32_t* slot_env, int32_t* group_scn) {
    if (!h) return fail(D2D_E_ARG, "d2d_get_group_layout: null handle"), -1;
    if (!h->lane_env) return 0;
    if (!slot_env || !group_scn) return fail(D2D_E_ARG, "d2d_get_group_layout: null output"), -1;
    DeviceGuard g(h->device);
    hipError_t e;
    if ((e = hipDeviceSynchronize()) != hipSuccess ||
        (e = hipMemcpy(slot_env, h->lane_env, sizeof(int32_t) * (size_t)h->ns, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(group_scn, h->wg_scn, sizeof(int32_t) * (size_t)h->n_groups, hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(e, "d2d_get_group_layout"), -1;
    return h->n_groups;
}

int32_t d2d_reset(d2d_t* h, const uint8_t* mask_dev, uint64_t seed, float* obs_dev, void* stream) {
    if (!h) return fail(D2D_E_ARG, "d2d_reset: null handle");
    if (h->n_scn <= 0) return fail(D2D_E_STATE, "d2d_reset: call d2d_set_scenarios first");
    DeviceGuard g(h->device);
    hipError_t e;
    if (fresh_mode(h) && mask_dev && (!h->fresh_seeded || h->fresh_seed != seed))
        return fail(D2D_E_ARG, "d2d_reset: fresh curriculum -- a masked reset must keep the seed of the "
                               "previous full reset");
    h->seed = seed;
    if (fresh_mode(h)) {
        // scenarios are keyed by the seed: a new seed drops every slot; then the slots of the
        // episodes this reset starts.  (A masked reset cannot change the seed, checked above: the
        // envs it leaves running would keep old-seed scenarios no recipe (key, clock) regenerates.)
        if (!h->fresh_seeded || h->fresh_seed != seed) {
            if ((e = hipMemsetAsync(h->scn_tag, 0xFF, sizeof(int32_t) * 2 * (size_t)h->n, (hipStream_t)stream)) !=
                hipSuccess)
                return hip_fail(e, "d2d_reset: fresh slots");
            h->fresh_seed = seed;
            h->fresh_seeded = true;
        }
        if ((e = fresh_regen(h, (hipStream_t)stream)) != hipSuccess) return hip_fail(e, "d2d_reset: fresh scenarios");
    }
    StepArgs a = make_args(h);
    a.obs = obs_dev;
    a.mask = mask_dev;
    const dim3 grid((h->ns + BLOCK - 1) / BLOCK);
    const size_t lds = scn_size(h->rm) * (size_t)h->n_scn;
    const hipStream_t rs = (hipStream_t)stream;
    if (lds <= K2_LDS_BUDGET) {
        if (h->rm) hipLaunchKernelGGL((d2d_reset_kernel<true, true>), grid, dim3(BLOCK), lds, rs, a);
        else hipLaunchKernelGGL((d2d_reset_kernel<true, false>), grid, dim3(BLOCK), lds, rs, a);
    } else {
        if (h->rm) hipLaunchKernelGGL((d2d_reset_kernel<false, true>), grid, dim3(BLOCK), 0, rs, a);
        else hipLaunchKernelGGL((d2d_reset_kernel<false, false>), grid, dim3(BLOCK), 0, rs, a);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "d2d_reset launch");
    if (fresh_mode(h) && (e = fresh_regen(h, (hipStream_t)stream)) != hipSuccess)
        return hip_fail(e, "d2d_reset: fresh scenarios");
    // cached next-reset observations depend on the seed and the episode counters: drop and refill
    if ((e = rc_rebuild(h, (hipStream_t)stream)) != hipSuccess) return hip_fail(e, "d2d_reset: cache rebuild");
    h->reset_done = true;
    return D2D_OK;
}

int32_t d2d_step(d2d_t* h, const float* act_dev, float* obs_dev, float* rew_dev, uint8_t* term_dev,
                 uint8_t* trunc_dev, float* info_dev, float* term_obs_dev, void* stream) {
    if (!h || !act_dev || !obs_dev || !rew_dev || !term_dev || !trunc_dev)
        return fail(D2D_E_ARG, "d2d_step: null handle or required buffer");
    if (h->n_scn <= 0 || !h->reset_done) return fail(D2D_E_STATE, "d2d_step: call d2d_set_scenarios and d2d_reset first");
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
    const size_t lds_scn = sizeof(d2d::ScnF) * (size_t)h->n_scn, lds_hot = sizeof(d2d::BtHot) * (size_t)h->n_scn;
    static_assert(sizeof(d2d::ScnF) + sizeof(d2d::BtHot) + sizeof(K1Shared) <= K1_LDS_BUDGET, "grouped K1 LDS");
    {
        // the three-way table re-check pays when the SIMDs have idle issue slots (at most one K1
        // workgroup per CU: 4 096 / 16 384 envs -4 %), not at full load (65 536 envs +3.6 %)
        const int nwg = h->lane_env ? h->n_groups : (int)grid.x;
        const bool s3 = nwg <= std::max(h->n_cu, 1);
        auto launch = [&](auto kern, dim3 g, size_t lds) {
            hipLaunchKernelGGL(kern, g, dim3(K1_THREADS), lds, (hipStream_t)stream, a);
        };
        if (h->lane_env) {
            const size_t lds = sizeof(d2d::ScnF) + sizeof(d2d::BtHot);
            if (s3) launch(d2d_step_grouped_kernel<true>, dim3(h->n_groups), lds);
            else launch(d2d_step_grouped_kernel<false>, dim3(h->n_groups), lds);
        } else if (!h->rm && a.brt && lds_scn + lds_hot + sizeof(K1Shared) <= K1_LDS_BUDGET) {
            if (s3) launch(d2d_step_kernel<true, true, true>, grid, lds_scn + lds_hot);
            else launch(d2d_step_kernel<true, true, false>, grid, lds_scn + lds_hot);
        } else if (!h->rm) {  // (table_rm: a ScnF table fits K1's LDS)
            if (s3) launch(d2d_step_kernel<true, false, true>, grid, lds_scn);
            else launch(d2d_step_kernel<true, false, false>, grid, lds_scn);
        } else {
            // the plain search's staged knots only without golden-march tables (fresh curriculum);
            // a pool's tables (a.brt) take the table path, which never reads them
            const size_t kn = a.brt ? 0 : K1_KN_BYTES;
            static_assert(sizeof(K1Shared) + K1_KN_BYTES <= K1_LDS_BUDGET, "K1 LDS with the staged knots");
            if (s3) launch(d2d_step_kernel<false, false, true>, grid, kn);
            else launch(d2d_step_kernel<false, false, false>, grid, kn);
        }
    }
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "d2d_step launch");
    if (fresh_mode(h) && (e = fresh_regen(h, (hipStream_t)stream, false, h->cfg.auto_reset != 0)) !=
                             hipSuccess)
        return hip_fail(e, "d2d_step: fresh scenarios");
    if (h->cfg.auto_reset && ++h->n_steps % FILL_PERIOD == 0) {
        // K4's cadence.  A step being captured into a graph launches K4 every FILL_PERIOD steps and
        // lets the device tick pick every FILL_EVERY-th launch to fill, so replays keep the cadence
        // whatever the graph's length; an eager step launches only the filling launches (every
        // FILL_PERIOD x FILL_EVERY steps), saving the two launches per period that would find the tick
        // says "skip" (~4 us each).  Either way an entry is an optimisation: a reset whose entry is
        // missing computes the same observation in K1.
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if ((e = hipStreamIsCapturing((hipStream_t)stream, &cs)) != hipSuccess)
            return hip_fail(e, "d2d_step: capture query");
        if (cs != hipStreamCaptureStatusNone) {
            if ((e = rc_fill(h, (hipStream_t)stream)) != hipSuccess) return hip_fail(e, "d2d_step: cache fill");
        } else if (h->n_steps % (FILL_PERIOD * FILL_EVERY) == 0) {
            if ((e = rc_fill(h, (hipStream_t)stream, true)) != hipSuccess) return hip_fail(e, "d2d_step: cache fill");
        }
    }
    return D2D_OK;
}

int32_t d2d_get_state(d2d_t* h, double* state_dev, int32_t* istate_dev, void* stream) {
    if (!h) return fail(D2D_E_ARG, "d2d_get_state: null handle");
    DeviceGuard g(h->device);
    hipError_t e;
    const size_t n = (size_t)h->n;
    const hipStream_t s = (hipStream_t)stream;
    if (h->lane_env) {  // grouped slot layout -> env order
        if (state_dev && (e = permute(h->st, h->ns, h->env_slot, state_dev, h->n, (const int32_t*)nullptr, D2D_NSTATE,
                                      h->n, s)) != hipSuccess)
            return hip_fail(e, "d2d_get_state");
        if (istate_dev && (e = permute(h->ist, h->ns, h->env_slot, istate_dev, h->n, (const int32_t*)nullptr,
                                       D2D_NISTATE, h->n, s)) != hipSuccess)
            return hip_fail(e, "d2d_get_state");
        return D2D_OK;
    }
    if (state_dev &&
        (e = hipMemcpyAsync(state_dev, h->st, sizeof(double) * D2D_NSTATE * n, hipMemcpyDeviceToDevice, s)) !=
            hipSuccess)
        return hip_fail(e, "d2d_get_state");
    if (istate_dev &&
        (e = hipMemcpyAsync(istate_dev, h->ist, sizeof(int32_t) * D2D_NISTATE * n, hipMemcpyDeviceToDevice, s)) !=
            hipSuccess)
        return hip_fail(e, "d2d_get_state");
    return D2D_OK;
}

int32_t d2d_set_state(d2d_t* h, const double* state_dev, const int32_t* istate_dev, void* stream) {
    if (!h) return fail(D2D_E_ARG, "d2d_set_state: null handle");
    if (h->n_scn <= 0) return fail(D2D_E_STATE, "d2d_set_state: call d2d_set_scenarios first");
    DeviceGuard g(h->device);
    hipError_t e;
    const size_t n = (size_t)h->n;
    const hipStream_t s = (hipStream_t)stream;
    if (h->lane_env) {  // env order -> grouped slot layout
        if (state_dev && (e = permute(state_dev, h->n, (const int32_t*)nullptr, h->st, h->ns, h->env_slot, D2D_NSTATE,
                                      h->n, s)) != hipSuccess)
            return hip_fail(e, "d2d_set_state");
        if (istate_dev && (e = permute(istate_dev, h->n, (const int32_t*)nullptr, h->ist, h->ns, h->env_slot,
                                       D2D_NISTATE, h->n, s)) != hipSuccess)
            return hip_fail(e, "d2d_set_state");
    } else {
        if (state_dev &&
            (e = hipMemcpyAsync(h->st, state_dev, sizeof(double) * D2D_NSTATE * n, hipMemcpyDeviceToDevice, s)) !=
                hipSuccess)
            return hip_fail(e, "d2d_set_state");
        if (istate_dev &&
            (e = hipMemcpyAsync(h->ist, istate_dev, sizeof(int32_t) * D2D_NISTATE * n, hipMemcpyDeviceToDevice, s)) !=
                hipSuccess)
            return hip_fail(e, "d2d_set_state");
    }
    if (fresh_mode(h) && (e = fresh_regen(h, (hipStream_t)stream)) != hipSuccess)
        return hip_fail(e, "d2d_set_state: fresh scenarios");
    if ((e = rc_rebuild(h, (hipStream_t)stream)) != hipSuccess) return hip_fail(e, "d2d_set_state: cache rebuild");
    h->reset_done = true;
    return D2D_OK;
}

int32_t d2d_refresh_pool(d2d_t* h, const d2d_scn* scns, int32_t n_scn) {
    if (!h || !scns) return fail(D2D_E_ARG, "d2d_refresh_pool: null handle/scenarios");
    if (h->cfg.scn_pool != 1) return fail(D2D_E_ARG, "d2d_refresh_pool: pool mode only (cfg.scn_pool = 1)");
    if (h->n_scn <= 0) return fail(D2D_E_STATE, "d2d_refresh_pool: call d2d_set_scenarios first");
    if (n_scn != h->pool_n) return fail(D2D_E_ARG, "d2d_refresh_pool: n_scn must equal the pool size");
    for (int k = 0; k < n_scn; ++k) {
        const d2d_scn& s = scns[k];
        if (s.n_wps < 3 || s.n_wps > D2D_MAX_WPS || s.n_circles < 0 || s.n_circles > D2D_MAX_CIRCLES)
            return fail(D2D_E_ARG, "d2d_refresh_pool: invalid scenario");
    }
    std::vector<unsigned char> tab;
    if (!build_tables(h->rm, scns, (size_t)n_scn, tab)) return fail(D2D_E_ARG, "d2d_refresh_pool: invalid scenario");
    DeviceGuard g(h->device);
    hipError_t e;
    const size_t P = (size_t)n_scn;
    const int half = h->pool_base == 0 ? n_scn : 0;
    // the half about to be overwritten must not hold a running episode (one that started before the
    // previous refresh): episodes last at most cfg.n_steps steps, so refreshes further apart are safe
    std::vector<int32_t> es((size_t)h->n);
    if ((e = hipDeviceSynchronize()) != hipSuccess ||  // in-flight steps may still draw from the old half
        (e = hipMemcpy(es.data(), h->env_scn, sizeof(int32_t) * es.size(), hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(e, "d2d_refresh_pool: read env_scn");
    int busy = 0;
    for (int32_t v : es) busy += (v >= half && v < half + n_scn);
    if (busy)
        return fail(D2D_E_STATE, "d2d_refresh_pool: " + std::to_string(busy) +
                                     " envs still run episodes from the pool before the previous refresh");
    if ((e = hipMemcpy(scn_at(h, half), tab.data(), tab.size(), hipMemcpyHostToDevice)) != hipSuccess ||
        (h->abi && (e = hipMemcpy(h->abi + half, scns, P * sizeof(d2d_scn), hipMemcpyHostToDevice)) != hipSuccess) ||
        (e = hipMemset(h->brt + half, 0, P * sizeof(d2d::BrTab))) != hipSuccess)
        return hip_fail(e, "d2d_refresh_pool: upload");
    launch_brtab(h->rm, scn_at(h, half), n_scn, h->brt + half);
    if ((e = hipGetLastError()) != hipSuccess || (e = hipDeviceSynchronize()) != hipSuccess)
        return hip_fail(e, "d2d_refresh_pool: d2d_brtab_kernel");
    if ((e = hipMemcpy(h->pool_dev, &half, sizeof(int32_t), hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "d2d_refresh_pool: switch");
    h->pool_base = half;
    h->pool_valid |= (half == 0) ? 1 : 2;
    // cached next-episode observations were drawn from the old half: drop and refill now (a
    // captured graph replays d2d_step's kernels without the host-side rebuild check)
    if ((e = rc_rebuild(h, nullptr)) != hipSuccess || (e = hipDeviceSynchronize()) != hipSuccess)
        return hip_fail(e, "d2d_refresh_pool: cache rebuild");
    return D2D_OK;
}

int32_t d2d_get_env_scenarios(d2d_t* h, int32_t* env_scn_dev, void* stream) {
    if (!h || !env_scn_dev) return fail(D2D_E_ARG, "d2d_get_env_scenarios: null handle/out");
    DeviceGuard g(h->device);
    hipError_t e = hipMemcpyAsync(env_scn_dev, h->env_scn, sizeof(int32_t) * (size_t)h->n, hipMemcpyDeviceToDevice,
                                  (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "d2d_get_env_scenarios");
    return D2D_OK;
}

int32_t d2d_set_env_scenarios(d2d_t* h, const int32_t* env_scn_dev, void* stream) {
    if (!h || !env_scn_dev) return fail(D2D_E_ARG, "d2d_set_env_scenarios: null handle/map");
    if (h->cfg.scn_pool != 1)
        return fail(D2D_E_ARG, "d2d_set_env_scenarios: pool mode only (a static map changes with d2d_set_scenarios; "
                               "fresh curriculum slots are restored by d2d_fresh_recipes)");
    if (h->n_scn <= 0) return fail(D2D_E_STATE, "d2d_set_env_scenarios: call d2d_set_scenarios first");
    DeviceGuard g(h->device);
    const hipStream_t s = (hipStream_t)stream;
    std::vector<int32_t> m((size_t)h->n);
    hipError_t e = hipMemcpyAsync(m.data(), env_scn_dev, sizeof(int32_t) * m.size(), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "d2d_set_env_scenarios: read map");
    for (int32_t v : m) {
        if (v < 0 || v >= h->n_scn) return fail(D2D_E_ARG, "d2d_set_env_scenarios: scenario index out of range");
        if (!(h->pool_valid & (v >= h->pool_n ? 2 : 1)))
            return fail(D2D_E_ARG, "d2d_set_env_scenarios: index into a pool half that holds no scenarios");
    }
    if ((e = hipMemcpyAsync(h->env_scn, m.data(), sizeof(int32_t) * m.size(), hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return hip_fail(e, "d2d_set_env_scenarios");
    return D2D_OK;
}

int32_t d2d_pool_state(d2d_t* h, int32_t* active_base, int32_t* valid_mask) {
    if (!h || !active_base || !valid_mask) return fail(D2D_E_ARG, "d2d_pool_state: null argument");
    if (h->cfg.scn_pool != 1 || h->n_scn <= 0) return fail(D2D_E_STATE, "d2d_pool_state: pool mode with scenarios only");
    *active_base = h->pool_base;
    *valid_mask = h->pool_valid;
    return D2D_OK;
}

int32_t d2d_restore_pool(d2d_t* h, const d2d_scn* scns, int32_t n_total, int32_t active_base, int32_t valid_mask) {
    if (!h || !scns) return fail(D2D_E_ARG, "d2d_restore_pool: null argument");
    if (h->cfg.scn_pool != 1 || h->n_scn <= 0) return fail(D2D_E_STATE, "d2d_restore_pool: pool mode with scenarios only");
    const int P = h->pool_n;
    if (n_total != 2 * P) return fail(D2D_E_ARG, "d2d_restore_pool: n_total must be twice the pool size");
    if (active_base != 0 && active_base != P) return fail(D2D_E_ARG, "d2d_restore_pool: active_base must be 0 or pool_n");
    if (!(valid_mask & (active_base ? 2 : 1)) || (valid_mask & ~3))
        return fail(D2D_E_ARG, "d2d_restore_pool: the active half must be valid");
    std::vector<bool> use((size_t)n_total);
    for (int k = 0; k < n_total; ++k) {
        use[k] = (valid_mask & (k >= P ? 2 : 1)) != 0;
        if (!use[k]) continue;
        const d2d_scn& sc = scns[k];
        if (sc.n_wps < 3 || sc.n_wps > D2D_MAX_WPS || sc.n_circles < 0 || sc.n_circles > D2D_MAX_CIRCLES)
            return fail(D2D_E_ARG, "d2d_restore_pool: invalid scenario");
    }
    std::vector<unsigned char> tab;
    if (!build_tables(h->rm, scns, (size_t)n_total, tab, &use)) return fail(D2D_E_ARG, "d2d_restore_pool: invalid scenario");
    const size_t sz = scn_size(h->rm);
    DeviceGuard g(h->device);
    hipError_t e;
    if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "d2d_restore_pool: sync");
    for (int half = 0; half < 2; ++half) {
        const size_t o = (size_t)half * P;
        if (!(valid_mask & (1 << half))) {
            if ((e = hipMemset(scn_at(h, o), 0, P * sz)) != hipSuccess ||
                (e = hipMemset(h->abi + o, 0, P * sizeof(d2d_scn))) != hipSuccess ||
                (e = hipMemset(h->brt + o, 0, P * sizeof(d2d::BrTab))) != hipSuccess)
                return hip_fail(e, "d2d_restore_pool: clear");
            continue;
        }
        if ((e = hipMemcpy(scn_at(h, o), tab.data() + o * sz, P * sz, hipMemcpyHostToDevice)) != hipSuccess ||
            (e = hipMemcpy(h->abi + o, scns + o, P * sizeof(d2d_scn), hipMemcpyHostToDevice)) != hipSuccess ||
            (e = hipMemset(h->brt + o, 0, P * sizeof(d2d::BrTab))) != hipSuccess)
            return hip_fail(e, "d2d_restore_pool: upload");
        launch_brtab(h->rm, scn_at(h, o), P, h->brt + o);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "d2d_restore_pool: d2d_brtab_kernel");
    }
    if ((e = hipMemcpy(h->pool_dev, &active_base, sizeof(int32_t), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipDeviceSynchronize()) != hipSuccess)
        return hip_fail(e, "d2d_restore_pool: switch");
    h->pool_base = active_base;
    h->pool_valid = valid_mask;
    h->rc_dirty = true;
    return D2D_OK;
}

int32_t d2d_set_curriculum(d2d_t* h, const d2d_curriculum* c) {
    if (!h || !c) return fail(D2D_E_ARG, "d2d_set_curriculum: null argument");
    if (!fresh_mode(h)) return fail(D2D_E_ARG, "d2d_set_curriculum: needs cfg.scn_pool = 2 (fresh curriculum)");
    if (c->n_wps < 4 || c->n_wps > D2D_MAX_WPS) return fail(D2D_E_ARG, "d2d_set_curriculum: n_wps out of range [4, D2D_MAX_WPS]");
    if (!(c->segment_length > 0.001)) return fail(D2D_E_ARG, "d2d_set_curriculum: segment_length must exceed 0.001");
    if (c->stage < 0 || c->stage > 5) return fail(D2D_E_ARG, "d2d_set_curriculum: stage must be 0 (schedule) or 1..5");
    if (c->random_path_spawn && (c->corner_lo < 1 || c->corner_hi > 4 || c->corner_lo > c->corner_hi))
        return fail(D2D_E_ARG, "d2d_set_curriculum: spawn corners must satisfy 1 <= lo <= hi <= 4");
    if (!(c->envs_total >= 1.0)) return fail(D2D_E_ARG, "d2d_set_curriculum: envs_total must be >= 1");
    DeviceGuard g(h->device);
    hipError_t e;
    const size_t S = 2 * (size_t)h->n;
    if (h->n_scn != (int)S || !h->scn_tag) {
        if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "d2d_set_curriculum: sync");
        for (void* p : {(void*)h->scn, (void*)h->brt, (void*)h->abi, (void*)h->scn_tag, (void*)h->gclk,
                        (void*)h->fresh_q})  // (fresh mode keeps no golden-march tables: brt stays null)
            if (p) (void)hipFree(p);
        h->scn = nullptr;
        h->brt = nullptr;
        h->abi = nullptr;
        h->scn_tag = nullptr;
        h->gclk = nullptr;
        h->fresh_q = nullptr;
        h->fresh_ring = ring_size(S);
        h->n_scn = 0;
        h->rm = true;  // (the fresh curriculum's tables are read per lane from global memory)
        if ((e = hipMalloc(&h->scn, sizeof(d2d::ScnR) * S)) != hipSuccess ||
            (e = hipMalloc(&h->abi, sizeof(d2d_scn) * S)) != hipSuccess ||
            (e = hipMalloc(&h->scn_tag, sizeof(int32_t) * S)) != hipSuccess ||
            (e = hipMalloc(&h->gclk, sizeof(int64_t) * S)) != hipSuccess ||
            (e = hipMalloc(&h->fresh_q, sizeof(int32_t) * (ring_size(S) + FR_WORDS))) != hipSuccess ||
            (e = hipMemset(h->fresh_q, 0, sizeof(int32_t) * (ring_size(S) + FR_WORDS))) != hipSuccess ||
            (e = hipMemset(h->scn, 0, sizeof(d2d::ScnR) * S)) != hipSuccess ||
            (e = hipMemset(h->abi, 0, sizeof(d2d_scn) * S)) != hipSuccess ||
            (e = hipMemset(h->gclk, 0, sizeof(int64_t) * S)) != hipSuccess)
            return hip_fail(e, "d2d_set_curriculum: hipMalloc");
    }
    // the schedule restarts at c->sim_num0: sim_num = sim_num0 + clock * envs_total counts the steps
    // taken on THIS curriculum, not those since the handle was created
    if ((e = hipMemset(h->scn_tag, 0xFF, sizeof(int32_t) * S)) != hipSuccess ||
        (e = hipMemset(h->clock, 0, sizeof(int64_t))) != hipSuccess ||
        (e = hipMemset(h->fresh_q + h->fresh_ring, 0, sizeof(int32_t) * FR_WORDS)) != hipSuccess ||  // (FreshRing)
        (e = hipDeviceSynchronize()) != hipSuccess)
        return hip_fail(e, "d2d_set_curriculum: slots");
    h->cur = *c;
    h->n_scn = (int)S;
    h->pool_n = 0;
    h->fresh_seeded = false;
    h->reset_done = false;  // every env starts over on the new curriculum (d2d_reset)
    h->rc_dirty = true;
    h->generation += 1;
    return D2D_OK;
}

int32_t d2d_fresh_recipes(d2d_t* h, int32_t* keys, int64_t* clocks, int64_t* clock, int32_t set) {
    if (!h || !keys || !clocks || !clock) return fail(D2D_E_ARG, "d2d_fresh_recipes: null argument");
    if (!fresh_mode(h) || !h->scn_tag) return fail(D2D_E_STATE, "d2d_fresh_recipes: call d2d_set_curriculum first");
    DeviceGuard g(h->device);
    hipError_t e;
    const size_t S = 2 * (size_t)h->n;
    if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "d2d_fresh_recipes: sync");
    if (!set) {
        if ((e = hipMemcpy(keys, h->scn_tag, sizeof(int32_t) * S, hipMemcpyDeviceToHost)) != hipSuccess ||
            (e = hipMemcpy(clocks, h->gclk, sizeof(int64_t) * S, hipMemcpyDeviceToHost)) != hipSuccess ||
            (e = hipMemcpy(clock, h->clock, sizeof(int64_t), hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(e, "d2d_fresh_recipes: read");
        return D2D_OK;
    }
    if (!h->fresh_seeded) return fail(D2D_E_STATE, "d2d_fresh_recipes: call d2d_reset (the seed) before restoring");
    if ((e = hipMemcpy(h->scn_tag, keys, sizeof(int32_t) * S, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(h->gclk, clocks, sizeof(int64_t) * S, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(h->clock, clock, sizeof(int64_t), hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "d2d_fresh_recipes: write");
    if ((e = fresh_regen(h, nullptr, true)) != hipSuccess || (e = hipDeviceSynchronize()) != hipSuccess)
        return hip_fail(e, "d2d_fresh_recipes: regenerate");
    h->rc_dirty = true;
    return D2D_OK;
}

int32_t d2d_get_scenario_table(d2d_t* h, int32_t first, int32_t count, d2d_scn* out) {
    if (!h || !out || first < 0 || count < 0) return fail(D2D_E_ARG, "d2d_get_scenario_table: bad arguments");
    if (!h->abi) return fail(D2D_E_STATE, "d2d_get_scenario_table: pool or fresh curriculum mode with scenarios only");
    if (first + count > h->n_scn) return fail(D2D_E_ARG, "d2d_get_scenario_table: range beyond the table");
    DeviceGuard g(h->device);
    hipError_t e;
    if ((e = hipDeviceSynchronize()) != hipSuccess ||
        (e = hipMemcpy(out, h->abi + first, sizeof(d2d_scn) * (size_t)count, hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(e, "d2d_get_scenario_table");
    return D2D_OK;
}

int32_t d2d_generation(const d2d_t* h) { return h ? h->generation : -1; }

int32_t d2d_episode_stats(d2d_t* h, double* out_dev, int32_t clear, void* stream) {
    if (!h || !out_dev) return fail(D2D_E_ARG, "d2d_episode_stats: null handle/out");
    DeviceGuard g(h->device);
    hipLaunchKernelGGL(d2d_stats_kernel, dim3(D2D_NSTATS), dim3(BLOCK), 0, (hipStream_t)stream, h->acc, h->ns,
                       out_dev, clear, h->acc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "d2d_episode_stats launch");
    return D2D_OK;
}

int32_t d2d_group_layout(int32_t n, const int32_t* env_scn, int32_t n_scn, int32_t* slot_env, int32_t* group_scn) {
    if (n <= 0 || n_scn <= 0 || !env_scn || !slot_env || !group_scn)
        return fail(D2D_E_ARG, "d2d_group_layout: n, n_scn must be > 0 and pointers non-null"), -1;
    for (int i = 0; i < n; ++i)
        if (env_scn[i] < 0 || env_scn[i] >= n_scn)
            return fail(D2D_E_ARG, "d2d_group_layout: env scenario index out of range"), -1;
    std::vector<int32_t> lanes, ws;
    make_groups(n, env_scn, n_scn, lanes, ws);
    std::copy(lanes.begin(), lanes.end(), slot_env);
    std::copy(ws.begin(), ws.end(), group_scn);
    return (int32_t)ws.size();
}

int32_t d2d_balanced_group_layout(int32_t n, const int32_t* env_scn, int32_t n_scn, const double* cost, int32_t n_cu,
                                  int32_t* slot_env, int32_t* group_scn) {
    if (n <= 0 || n_scn <= 0 || !env_scn || !cost || !slot_env || !group_scn || n_cu < 0)
        return fail(D2D_E_ARG, "d2d_balanced_group_layout: bad arguments"), -1;
    for (int i = 0; i < n; ++i)
        if (env_scn[i] < 0 || env_scn[i] >= n_scn)
            return fail(D2D_E_ARG, "d2d_balanced_group_layout: env scenario index out of range"), -1;
    std::vector<int32_t> lanes, ws;
    make_groups(n, env_scn, n_scn, lanes, ws);
    balance_groups(n_cu, cost, n_scn, lanes, ws);
    std::copy(lanes.begin(), lanes.end(), slot_env);
    std::copy(ws.begin(), ws.end(), group_scn);
    return (int32_t)ws.size();
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
