// d2d_kernels.h -- the kernels of libdrone2d_hip.so (included by d2d_hip.hip).
//
// K1 d2d_step_kernel (cooperative, wave-specialised).  One 256-lane workgroup owns 64 envs (one
// per lane index); its four waves split one env step by role so that the long, independent fp64
// latency chains run concurrently instead of back to back.  The frame's post-step position depends
// only on its pre-step position and velocity (forces act on velocities), so every wave derives it
// from the state in HBM and no wave waits for another before its own chain:
//
//   W0  load state, thrust, 3-body position update, collision, end cause (published to the other
//       waves at once), 6-pivot joint sweep,
//       store the state; velocity part of the observation (obs 0-2, 17-18) and of the reward
//   W1  sensor part (obs 3..16, CA inputs); for envs that end: the spawn-state sensor part
//   W2  path role: Brent closest point through the golden-march tables (steps [1, bt_split) of the
//       table re-check), obs 19..26, the position / path terms of the reward while the physics wave
//       finishes (W0 takes the sum)
//   W3  steps [bt_split, len) of W2's table re-check; then, for envs that end, the
//       spawn state and the spawn-state path part
//   (W1 and W3 take the spawn-state parts from the auto-reset observation cache when it is ready)
//   epilogue (no barrier: an LDS count of the waves whose rows are written): W1-W3 store the 64x27
//   f32 obs tile as one contiguous span; W0 writes reward / flags / info / bookkeeping.
//
// W2's Brent search runs at the highest wave priority.  At 65 536 envs this is 1 024 workgroups = 4
// per CU = 4 waves per SIMD, one of each role (VGPR <= 128, LDS <= 40 KB); every SIMD then issues
// VALU work ~87 % of the time (DESIGN.md "What bounds K1").  The scenario (+ probe table) is staged
// into LDS by LDS-DMA while the waves' first state loads are in flight.  d2d_step_grouped_kernel is
// the same body over the scenario-grouped slot layout (StepArgs::lane_env).
//
// K2 d2d_reset_kernel: masked reset, one lane per env.  K3 d2d_stats_kernel: fixed-order reduction.
// K4 d2d_fill_kernel: fills the auto-reset observation cache (the envs that need it compacted,
// four waves per 64 of them: fill_split).
#pragma once
#include <type_traits>

#include "d2d_curriculum.h"
#include "d2d_device.h"

namespace d2dk {
using namespace d2d;

constexpr int BLOCK = 256;      // K2 / K3 workgroup
constexpr int EPB = 64;         // K1: envs per workgroup
constexpr int K1_THREADS = 256; // K1: 4 waves
// scenario tables go to LDS when they fit next to K1's own LDS within the 4-workgroups-per-CU
// budget (160 KB / 4); larger sets are read from global memory (L1/L2 resident)
constexpr size_t K1_LDS_BUDGET = 40 * 1024;
constexpr size_t K2_LDS_BUDGET = 64 * 1024;
// Wave priorities per role (s_setprio, 0..3): the Brent waves win issue arbitration on their SIMD,
// the physics waves come next (their 10-sweep joint chain must end before the search does); once
// its search is done the path wave drops to 0, since the physics wave is then the critical one.
// A/B (tools/variants.py, µs per step at 65 536 envs, corridor / S_corridor / large / mixed):
// W0..W3 = 2,0,3,2 29.46 / 37.97 / 35.73 / 40.11; 2,1,3,1 28.86 / 37.99 / 35.78 / 40.00; with W2 -> 0
// after the search 28.55 / 37.61 / 35.78 / 40.11 (kept); all equal (0) 39.9, W0 = W2 = 3 35.2.
// W3 re-checks its part of W2's golden-march table at W2's priority, then drops to PRIO_W3; W2 drops
// to PRIO_W2_POST once its search is done (the reward terms and waits).
constexpr int PRIO_W0 = 2, PRIO_W1 = 1, PRIO_W2 = 3, PRIO_W3 = 1, PRIO_W2_POST = 0;
// (A four-group 1 024-thread "quad" workgroup with host-chosen role -> SIMD placement was measured
// 2-13 % slower than four 256-thread workgroups and removed in round 4: docs/DESIGN_HISTORY.md.)

struct StepArgs {
    int n;                   // envs
    int ns;                  // state slots: the column count of every [F][ns] internal array (= n
                             // unless the grouped lane map pads scenario groups, see lane_env)
    int n_scn;
    double* st;              // [NSTATE][n]
    int32_t* ist;            // [NISTATE][n]
    double* acc;             // [NSTATS][n]
    const void* scn;         // [n_scn] ScnF or ScnR (d2d_t::rm), see scn_tab
    const BrTab* brt;        // [n_scn] golden-march tables (d2d_brtab_kernel), or null
    int32_t* env_scn;        // [n] or null (all scenario 0); rewritten at resets in pool mode
    int32_t* fill_ctl;         // K4's device tick [0] and finished-workgroup count [1]
    int fill_every;            // K4 fills on every fill_every-th launch (the tick), others exit
    int fill_force;            // K4 fills regardless of the tick (rebuilds)
    const int32_t* pool_base;  // pool mode: resets draw from scenarios [*pool_base, *pool_base + pool_n);
    int pool_n;                // d2d_refresh_pool switches *pool_base between the two table halves
                               // (device memory, so captured graphs follow a refresh)
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
    // auto-reset observation cache (handle-internal; see "Auto-reset observation cache" below)
    float* rc_obs;           // [RC_SLOTS][n][27] reset observations (rc_entry: the slot of a key)
    int32_t* rc_rfl;         // [RC_SLOTS][n] their flags (LA lock)
    int32_t* rc_tag;         // [RC_SLOTS][n] episode counter an entry belongs to (-1: none)
    // Scenario-grouped slot layout (null unless the env -> scenario map is static and mixed).
    // Internal state lives in slots: slot s holds env lane_env[s] (-1: padding), and slots
    // [64 g, 64 g + 64) all hold envs of scenario wg_scn[g], so K1 workgroup g (after the XCD-aware
    // renumbering, xcd_group) reads its state coalesced and stages one scenario.  The caller's
    // buffers (actions, obs, reward, flags, info, terminal obs), the scenario map and the spawn RNG
    // stay indexed by env id.  Without the map slot == env.
    const int32_t* lane_env;  // [ns] slot -> env
    const int32_t* wg_scn;    // [ns / 64]  (-(s + 2): scenarios s and s + 1; -1: three or more)
    // fresh curriculum (cfg.scn_pool == 2): the episode key each scenario slot holds (K4 fills a
    // reset observation only once its scenario exists) and the step clock K1 advances
    const int32_t* scn_tag;   // [2 n]
    int64_t* clock;           // [1]
    // ... and K5's queue: K1 appends the slot of the episode after next of every env it resets
    // (null: K5a scans for them; auto-reset off)
    int32_t* fq;              // [fq_mask + 1] slots (a ring, see FreshRing)
    uint32_t* fqc;            // FreshRing words ([FR_HEAD]: appends so far)
    uint32_t fq_mask;         // ring size - 1 (a power of two >= 2 n)
};

// the scenario table in the layout the launch was instantiated for (ScnF: the handle stages its
// scenarios in LDS; ScnR: K1 reads them from global memory, d2d_hip.hip table_rm)
template <class S>
__device__ __forceinline__ const S* scn_tab(const StepArgs& a) { return static_cast<const S*>(a.scn); }

// Auto-reset observation cache.  The observation an env gets when it auto-resets depends only on
// (seed, env id, episode counter, scenario), so it is computed ahead of time, while the env is still
// running, by the fill kernel K4 that d2d_step launches after every FILL_PERIOD-th step (and
// d2d_reset / d2d_set_state after theirs): one lane per env, every env whose entry is not tagged
// with its current episode counter computes the spawn-state observation of its next episode.  K1
// takes an entry only when its tag matches; otherwise (an episode shorter than the fill period) it
// computes the observation synchronously.  Running the fill as its own kernel keeps it off K1's
// issue slots: inside K1 it would run a whole wave for the ~0.5 of 64 envs that reset per step.
// Reset-cache entries per env: the next reset's observation and the one after (slot = episode
// counter mod 2), so K4 may fill every 48 steps instead of 16 without more envs falling back to the
// synchronous reset.  K4 is launched after every FILL_PERIOD steps (a captured 16-step graph holds one
// launch) and every FILL_EVERY-th launch fills (a device tick).
constexpr int RC_SLOTS = 2;
constexpr int FILL_PERIOD = 16;
constexpr int FILL_EVERY = 3;
// K4: slots per block -- about one 64-item round per block between fills (~35 per 48 steps of 64 slots)
constexpr int FILL_SPB = 64;


// Diagnostic phase stamps (separate timing-only build, never in the product): lane 0 of each wave
// records s_memtime at the phase boundaries of K1 (slots 4, 5: role-specific hand-off points).
#ifdef D2D_STAMPS
#define STAMP(k)                                                                                       \
    do {                                                                                               \
        if (a.stamps && (threadIdx.x & 63) == 0)                                                       \
            a.stamps[(size_t)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
        if (a.stamps && (threadIdx.x & 63) == 0 && (k) == 0)                                           \
            a.stamps[(size_t)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + 7] =                          \
                ((uint64_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32) |                          \
                (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) | ((uint64_t)(wave & 3) << 36) |   \
                ((uint64_t)(uint32_t)(wg + 1) << 40);                                                  \
    } while (0)
// K4: the same per wave, at offset D2D_FSTAMP_BASE of the buffer (0 start, 1 staged + compacted,
// 2 spawn state, 3 the wave's first part, 4 first barrier, 5 continuation, 6 path part, 7 end)
#define D2D_FSTAMP_BASE 65536
#define FSTAMP(k)                                                                                      \
    do {                                                                                               \
        if (a.stamps && (threadIdx.x & 63) == 0)                                                       \
            a.stamps[D2D_FSTAMP_BASE + (size_t)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (k)] =      \
                __builtin_amdgcn_s_memtime();                                                          \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#define FSTAMP(k) \
    do {          \
    } while (0)
#endif

__device__ __forceinline__ const BrTab* brtab(const StepArgs& a, int si) { return a.brt ? a.brt + si : nullptr; }
// the reset-cache entry of slot i for key ep (the observation of the reset that ends episode ep):
// slot ep % RC_SLOTS, so the entries of two consecutive episodes coexist
__device__ __forceinline__ size_t rc_entry(const StepArgs& a, int i, uint32_t ep) {
    return (size_t)(ep & 1u) * (size_t)a.ns + (size_t)i;
}

// Scenarios [first, first + count) into LDS; the returned table is indexed by the global scenario
// index (a grouped K1 workgroup stages only its own scenario: the base is offset by -first, LDS
// addresses are 32-bit and wrap back into the staged block for the indices it holds).
template <bool LDS, int NT, class S>
__device__ __forceinline__ const S* stage_scenarios(const StepArgs& a, S* lds, int first = 0, int count = -1) {
    if (!LDS) return scn_tab<S>(a);
    if (count < 0) count = a.n_scn;
    const int words = count * (int)(sizeof(S) / 8);
    const double* src = reinterpret_cast<const double*>(scn_tab<S>(a) + first);
    double* dst = reinterpret_cast<double*>(lds);
    for (int k = threadIdx.x; k < words; k += NT) dst[k] = src[k];
    return lds - first;
}
// the probe tables of the golden-march tables (BrTab::hot), staged after the scenarios
template <int NT>
__device__ __forceinline__ const BtHot* stage_hot(const StepArgs& a, BtHot* lds, int first = 0, int count = -1) {
    if (count < 0) count = a.n_scn;
    const int per = (int)(sizeof(BtHot) / 16);
    for (int k = threadIdx.x; k < count * per; k += NT) {
        const double2* src = reinterpret_cast<const double2*>(&a.brt[first + k / per].hot) + (k % per);
        reinterpret_cast<double2*>(lds)[k] = *src;
    }
    return lds - first;
}
// Contiguous global -> LDS copy with LDS-DMA (global_load_lds_dwordx4: no VGPRs, asynchronous until
// the next vmcnt wait; the __syncthreads() that follows drains it).  Each wave instruction moves
// 1 KB (64 lanes x 16 B, LDS written at the wave-uniform base + lane x 16); bytes % 16 == 0.
template <int NWAVES>
__device__ __forceinline__ void glds_copy(void* lds_dst, const void* gsrc, int bytes) {
    using LP = __attribute__((address_space(3))) void;
    using GP = __attribute__((address_space(1))) void;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    for (int c = wave; c * 1024 < bytes; c += NWAVES) {
        const int off = c * 1024 + lane * 16;
        if (off < bytes)
            __builtin_amdgcn_global_load_lds((GP*)((const char*)gsrc + off), (LP*)((char*)lds_dst + c * 1024), 16, 0, 0);
    }
}

// Workgroup renumbering for the grouped lane map: blocks b and b + 8 share an XCD (and its L2)
// when the grid is dealt round-robin over the 8 XCDs, so consecutive group numbers -- groups whose
// envs share cache lines -- go to blocks on one XCD.  Placement only affects speed.
// XCD x = b % 8 holds per + (x < rem) blocks; its k-th block (k = b / 8) takes group number
// (groups of XCDs before x) + k, a bijection on [0, nb).
__device__ __forceinline__ int xcd_group(int b, int nb) {
    const int per = nb / 8, rem = nb % 8, x = b % 8, k = b / 8;
    return (x < rem) ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
}

__device__ __forceinline__ size_t fidx(int f, int n, int i) { return (size_t)f * (size_t)n + (size_t)i; }
// SoA field access as (wave-uniform field base) + (per-lane 32-bit index): the base lives in SGPRs
// and the access uses saddr + voffset addressing, instead of one 64-bit VGPR address per field.
template <typename T>
__device__ __forceinline__ T& fld(T* base, int f, int n, int i) {
    T* fb = base + (size_t)__builtin_amdgcn_readfirstlane(f) * (size_t)__builtin_amdgcn_readfirstlane(n);
    return fb[i];
}

// frame state as stored (pre-step)
__device__ __forceinline__ Body load_frame(const StepArgs& a, int i) {
    const int n = a.ns;
    return Body{fld(a.st, 0, n, i), fld(a.st, 1, n, i), fld(a.st, 2, n, i),
                fld(a.st, 3, n, i), fld(a.st, 4, n, i), fld(a.st, 5, n, i)};
}
// next-episode spawn (test-mode reset, drone_2d_env.py:218-311, Drone.py:20-52)
template <class SC>
__device__ __forceinline__ void spawn_state(const StepArgs& a, const SC& S, int i, uint32_t ep, double sp[7]) {
    double x, y, th;
    spawn_draw(S, a.seed, (uint32_t)a.cfg.env_id_base + (uint32_t)i, ep, x, y, th);
    double sl, cl, sr, cr;
    sincos_d(th + PI, sl, cl);
    sincos_d(th, sr, cr);
    sp[0] = x;
    sp[1] = y;
    sp[2] = th;
    sp[3] = cl * DRONE_R + x;
    sp[4] = sl * DRONE_R + y;
    sp[5] = cr * DRONE_R + x;
    sp[6] = sr * DRONE_R + y;
}

// wave-uniform read of an LDS flag written by another wave of the workgroup
// (explicit LDS address space: a generic volatile access would become a flat load)
using LdsU32 = __attribute__((address_space(3))) uint32_t;
__device__ __forceinline__ bool flag_seen(const uint32_t& f) {
    return __builtin_amdgcn_readfirstlane(*(const volatile LdsU32*)&f) != 0u;
}
// scenario of the episode that follows episode counter `ep` of env j (curriculum pool: a fresh draw)
__device__ __forceinline__ int pool_scenario(const StepArgs& a, int j, uint32_t ep) {
    return *a.pool_base + (a.pool_n > 1 ? pool_pick(a.seed, (uint32_t)a.cfg.env_id_base + (uint32_t)j, ep, a.pool_n) : 0);
}
// fresh curriculum: env j's two scenario slots alternate by episode key (d2d_fresh_kernel writes
// the slot of key ep -- the episode the next reset starts -- one step ahead)
__device__ __forceinline__ int fresh_slot(int j, uint32_t ep) { return 2 * j + (int)(ep & 1u); }
// FreshRing: the fresh curriculum's slots to generate, in a ring nobody clears.  FR_HEAD counts the
// appends (K1 at its auto-resets, or K5a), modulo 2^32; K5b drains [tail, head) and leaves the new
// tail in the word of the next clock parity -- the one the K5b after the next K1 reads -- so no
// workgroup of a launch writes a word another reads (the step clock, advanced by K1, is stable
// during K5b).  After a scan (K5a) the tail is the later of the two words, and a one-thread launch
// sets both to the head.
enum { FR_HEAD = 0, FR_TAIL0 = 1, FR_TAIL1 = 2, FR_WORDS = 4 };
__device__ __forceinline__ int next_scenario(const StepArgs& a, int j, uint32_t ep) {
    if (a.cfg.scn_pool == 2) return fresh_slot(j, ep);
    if (a.cfg.scn_pool) return pool_scenario(a, j, ep);
    if (a.n_scn <= 1) return 0;
    return a.env_scn[j];
}

// ------------------------------------------------------------------------------------------ K1
// Intra-workgroup hand-offs are LDS flags (raised after a release fence, polled with s_sleep), so
// no wave waits at a barrier for work it does not depend on.  Dependencies (all acyclic):
//   f_done  W0 -> W1,W2,W3  which envs end this step, cache readiness (right after the positions)
//   f_ca    W1 -> W0,W2     CA inputs from obs 8..10 (CAStatic)
//   f_gs    W0 -> W1,W2,W3  joint sweep finished: the jb region becomes the obs tile
//   f_rp    W2 -> W0        the position / path terms of the reward (W0 sums the reward: the physics
//                           wave ends last at full load, so the sum waits for no other wave)
//   f_ver   W3 -> W2        first differing step in the second half of the table re-check
//   f_acc   W3 -> W0        the finished episodes' accumulators and the running path error / return
//                           are in LDS (W0's epilogue)
//   n_tile  W0..W3 -> W1..W3  count of waves whose obs-tile rows are written: W1-W3 store the tile
//                           once all four are, while W0 finishes the reward and its bookkeeping
//                           (no workgroup barrier: the tile store does not wait for the reward sum)
struct K1Shared {
    double cas[6][EPB];       // W1 -> W0, W2: CAStatic (d, os, oc, lpa, lca, rr)
    int scn[EPB];             // scenario index per env
    uint8_t cause[EPB];       // W0 -> W1, W2, W3: end cause (0: the env keeps running)
    uint8_t cvalid[EPB];      // W0 -> W1, W3: the env's reset-cache entry is ready
    uint32_t pflags[EPB];     // W3 -> W2: first differing step of the second half of the table re-check;
                              // then W2 -> W0: LA-lock bit after the path role
    uint32_t ep[EPB];         // W0 -> W1, W3: episode counter (the state's copy changes at a reset)
    double sina[EPB];         // W0 -> W2: sin of the post-step frame angle (AA reward)
    uint32_t w0t[EPB], w0fl[EPB];  // W0 -> W0: the step counter t and the flags, for after the joint sweep
    uint32_t f_done, f_ca, f_gs, f_rp, f_ver, f_ver1, f_acc, n_tile;
    double pe[2][EPB];        // W3 -> W0: path_err, total_reward (prefetched for the epilogue)
    double acc[D2D_NSTATS][EPB];  // W3 -> W0: episode accumulators of envs that end (prefetched)
    union {
        struct {
            double jb[6 * JB_PER_JOINT][EPB];  // W0's joint sweep: per-joint K^-1 + bias
            double arms[ARMS_N][EPB];          // ... and the rotated anchor arms
        } g;
        struct {
            double post[7][EPB];           // W2 -> W0: LA bearing (sin, cos), pa, dist, aa, coll, reach
            alignas(16) float obs[EPB * D2D_OBS_DIM];  // the workgroup's obs rows (16-B aligned: float4 stores)
        } p;                               // after f_gs
    } u;
};

// the lane index by instructions the compiler cannot merge with threadIdx.x, so that a wave can
// drop the index across a register-bound region and recompute it after
__device__ __forceinline__ int lane_fresh() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
__device__ __forceinline__ void flag_raise(uint32_t& f) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63) == 0) *(volatile LdsU32*)&f = 1u;
}
__device__ __forceinline__ void flag_wait(const uint32_t& f) {
    while (!flag_seen(f)) __builtin_amdgcn_s_sleep(1)  /* 64 cycles between polls */;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// the obs-tile count: a wave's rows are written (release), and the wait for all `n` waves (acquire)
__device__ __forceinline__ void tile_arrive(uint32_t& c) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63) == 0) atomicAdd(&c, 1u);
}
__device__ __forceinline__ void tile_wait(const uint32_t& c, uint32_t n) {
    while (__builtin_amdgcn_readfirstlane(*(const volatile LdsU32*)&c) < n) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Scenario staging of a 256-thread K1 workgroup (group wg).  LDS: scenario tables in LDS; LTAB: the
// golden-march probe tables too (after the scenarios); GRP: grouped slot layout (a.lane_env) -- with
// LDS, the group is pure and stages only its own scenario.  s_scn: the dynamic LDS (scenario tables
// [+ probe tables], sized at launch).  Returns the tables indexed by global scenario id and the
// group's (first) scenario s0.
template <bool LDS, bool LTAB, bool GRP, class S>
__device__ __forceinline__ void k1_stage(const StepArgs& a, S* s_scn, int wg, const S*& scns,
                                         const BtHot*& hots, int& s0) {
    const int ws = (GRP && LDS) ? a.wg_scn[wg] : 0;
    s0 = ws >= 0 ? ws : -ws - 2;          // a straddling group: its two scenarios s0, s0 + 1
    const int ncopy = (GRP && LDS) ? (ws >= 0 ? 1 : 2) : a.n_scn;
    hots = nullptr;
    if (LDS && (ncopy == 1 || !LTAB)) {
        // one scenario (+ its probe table) or scenarios only: contiguous sources, LDS-DMA
        glds_copy<K1_THREADS / 64>(s_scn, scn_tab<S>(a) + s0, (int)sizeof(S) * ncopy);
        if (LTAB) glds_copy<K1_THREADS / 64>(s_scn + 1, &a.brt[s0].hot, (int)sizeof(BtHot));
        scns = s_scn - s0;
        if (LTAB) hots = reinterpret_cast<const BtHot*>(s_scn + 1) - s0;
    } else {
        scns = stage_scenarios<LDS, K1_THREADS>(a, s_scn, s0, ncopy);
        if (LTAB) hots = stage_hot<K1_THREADS>(a, reinterpret_cast<BtHot*>(s_scn + ncopy), s0, ncopy);
    }
}

// the dynamic LDS of every kernel (scenarios [+ probe tables]; global-memory tables: the path wave's
// staged knots, K1_KN_BYTES), sized at launch
extern __shared__ __attribute__((aligned(16))) uint4 d2d_dyn_lds[];
constexpr int K1_KN_BYTES = D2D_MAX_WPS * 64 * 8;
// One env step for the 64 envs of group wg (slots [64 wg, 64 wg + 64)) by the calling wave in role `role` (0..3, wave-uniform); qt =
// 64 role + lane, the thread's index among the group's 256.  scns / hots: the scenario and probe
// tables indexed by global scenario id (LDS when staged: LDS / LTAB), s0 the group's scenario.
// All 256 threads of the group call it once; the staging barrier is block-wide, so every wave of
// the block runs k1_body exactly once.
template <bool LDS, bool LTAB, bool GRP, bool S3, class SC>
__device__ __forceinline__ void k1_body(const StepArgs& a, const SC* scns, const BtHot* hots, int s0, K1Shared& sh,
                                        int wg, int role, int qt) {
    const int wave = role;
    const int lane = threadIdx.x & 63;
    const bool gvalid = wg >= 0;
    const int e0 = gvalid ? wg * EPB : 0;
    const int i = e0 + lane;                     // slot: internal arrays, reset cache
    const int ie = (GRP && gvalid) ? a.lane_env[i] : i;  // env: caller's buffers, scenario map, spawn RNG
    const bool valid = gvalid && (GRP ? ie >= 0 : i < a.n);
    const int n = a.ns;
    const bool auto_reset = a.cfg.auto_reset != 0;
    STAMP(0);
    if (wg == 0 && qt == 0 && a.fill_ctl)  // K4's tick: publish its next value
        __hip_atomic_store(&a.fill_ctl[0], __hip_atomic_load(&a.fill_ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wg == 0 && qt == 0 && a.clock)  // the step clock (fresh curriculum stage schedule)
        __hip_atomic_fetch_add(a.clock, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wave == 0) sh.scn[lane] = (valid && a.env_scn && a.n_scn > 1) ? a.env_scn[ie] : s0;
    if (S3 && wave == 0) sh.pflags[lane] = 0x7fffffffu;  // W1 and W3 min their table parts in
    // W1..W3 load the pre-step frame before the staging barrier, so its HBM latency overlaps the
    // staging (and every read precedes W0's stores of the new positions).  W0 loads its state after
    // the barrier: issuing those ~30 loads earlier spilled registers (42 vs 32 us, docs/DESIGN_HISTORY.md).
    Body PF{};
    if (valid && wave != 0) PF = load_frame(a, i);
    if (qt == 0) {
        sh.f_done = 0u;
        sh.f_ca = 0u;
        sh.f_gs = 0u;
        sh.f_rp = 0u;
        sh.f_ver = 0u;
        sh.f_ver1 = 0u;
        sh.f_acc = 0u;
        sh.n_tile = 0u;
    }
    __syncthreads();
    STAMP(1);
    const SC& S = scns[sh.scn[lane]];
    float* const trow = a.tobs ? a.tobs + (size_t)ie * D2D_OBS_DIM : nullptr;
    float* const orow = &sh.u.p.obs[lane * D2D_OBS_DIM];

    // W0 results kept for the epilogue
    Body F0{};
    double path_err = 0.0, tot_rew = 0.0;
    int t = 0, cause = 0;
    uint32_t flags = 0;
    RewardVel RV{};
    double dclose = 0.0, rew_sum = 0.0, rew_pp = 0.0, pdist = 0.0;
    uint32_t plal = 0;                  // W2's LA-lock bit
    bool done = false;
    if (wave == 0) {
        // ---------------------------------------------------------------- physics
        __builtin_amdgcn_s_setprio(PRIO_W0);
        double ov[19];
        Body B[3];
        double j[12], cs[3], sn[3], fx = 0.0, fy = 0.0, tq = 0.0;
        if (valid) {
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
            t = fld(a.ist, D2D_I_T, n, i);
            flags = (uint32_t)fld(a.ist, D2D_I_FLAGS, n, i);
            // thrust in float32 exactly as SB3's float32 action hits drone_2d_env.py:400-401
            const float2 act = reinterpret_cast<const float2*>(a.act)[ie];
            const float fs = (float)a.cfg.force_scale;
            const float lf = __fmul_rn(__fadd_rn(act.x / 2.0f, 0.5f), fs);
            const float rf = __fmul_rn(__fadd_rn(act.y / 2.0f, 0.5f), fs);
            if (phys_positions(S, B, (double)lf, (double)rf, cs, sn, fx, fy, tq)) flags |= D2D_FLAG_COLLIDED;
            t += 1;
            cause = end_cause(a.cfg, S, B[0], (flags & D2D_FLAG_COLLIDED) != 0, t);
            done = cause != 0;
            // which envs end (for W1, W2, W3) and whether their reset observation is cached
            const int32_t ep = fld(a.ist, D2D_I_EPISODE, n, i);
            const bool cv = done && auto_reset && a.rc_tag[rc_entry(a, i, (uint32_t)ep)] == ep;
            sh.ep[lane] = (uint32_t)ep;
            sh.cause[lane] = (uint8_t)cause;
            sh.sina[lane] = sn[0];
            sh.cvalid[lane] = cv ? 1u : 0u;
            sh.w0t[lane] = (uint32_t)t;
            sh.w0fl[lane] = flags;
            // positions and angles are final now (the sweep changes velocities only); envs that
            // auto-reset get their spawn state from W3 instead
            if (!(done && auto_reset)) {
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    fld(a.st, 6 * b + 0, n, i) = B[b].px;
                    fld(a.st, 6 * b + 1, n, i) = B[b].py;
                    fld(a.st, 6 * b + 2, n, i) = B[b].a;
                }
            }
        }
        flag_raise(sh.f_done);
        if (valid) {
            const Arms A = make_arms(cs, sn);
            const double pos[6] = {B[0].px, B[0].py, B[1].px, B[1].py, B[2].px, B[2].py};
            double vel[9] = {B[0].vx, B[0].vy, B[0].w, B[1].vx, B[1].vy, B[1].w, B[2].vx, B[2].vy, B[2].w};
            phys_velocities<true>(A, pos, a.damping_dt, fx, fy, tq, vel, j, &sh.u.g.jb[0][lane], EPB,
                                  &sh.u.g.arms[0][lane]);
            // the lane index, t, flags and the end cause are re-read from LDS or recomputed from here
            // on (kept live across the sweep they were spilled to scratch: 40 B per lane each way)
            asm volatile("" ::: "memory");
            const int ln = lane_fresh(), iw = e0 + ln;
            const uint32_t cw = sh.cause[ln];
            cause = (int)cw;
            done = cw != 0u;
            t = (int)sh.w0t[ln];
            flags = sh.w0fl[ln];
            if (!(done && auto_reset)) {
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                fld(a.st, 6 * b + 3, n, iw) = vel[3 * b + 0];
                fld(a.st, 6 * b + 4, n, iw) = vel[3 * b + 1];
                fld(a.st, 6 * b + 5, n, iw) = vel[3 * b + 2];
            }
#pragma unroll
            for (int k = 0; k < 12; ++k) fld(a.st, D2D_S_J + k, n, iw) = j[k];
            }
            F0 = Body{0.0, 0.0, B[0].a, vel[0], vel[1], vel[2]};
        }
        flag_raise(sh.f_gs);
        STAMP(4);
        const int ln = lane_fresh(), iw = e0 + ln, iew = GRP ? ie : iw;
        const bool vw = gvalid && (GRP ? iew >= 0 : iw < a.n);
        // velocity part of the observation (obs 0-2, 17-18) into the tile / terminal obs
        if (vw) {
            float* const orw = &sh.u.p.obs[ln * D2D_OBS_DIM];
            float* const trw = a.tobs ? a.tobs + (size_t)iew * D2D_OBS_DIM : nullptr;
            sensor_vel(F0, sh.sina[ln], cs[0], ov);
            if (!(done && auto_reset)) {
                orw[0] = (float)ov[0];
                orw[1] = (float)ov[1];
                orw[2] = (float)ov[2];
                orw[17] = (float)ov[17];
                orw[18] = (float)ov[18];
            }
            if (done && trw) {
                trw[0] = (float)ov[0];
                trw[1] = (float)ov[1];
                trw[2] = (float)ov[2];
                trw[17] = (float)ov[17];
                trw[18] = (float)ov[18];
            }
        }
        tile_arrive(sh.n_tile);
        // velocity part of the reward (speed, velocity angle, CA total), for W2
        flag_wait(sh.f_ca);
        STAMP(5);
        if (vw) {
            CAStatic C;
            C.d = sh.cas[0][ln];
            C.os = sh.cas[1][ln];
            C.oc = sh.cas[2][ln];
            C.lpa = sh.cas[3][ln];
            C.lca = sh.cas[4][ln];
            C.rr = sh.cas[5][ln];
            RV = reward_vel(a.cfg, ov, C);
            dclose = C.d;
        }
        // at full load: W3's prefetched path error / return (long ready) read before the wait on
        // W2, so the epilogue after it starts from registers (corridor 26.68 -> 26.49 us per step;
        // with one workgroup per CU, where W3 first takes a third of the table re-check, the
        // epilogue reads them: 20.29 vs 20.73 us at 4 096 envs)
        if (!S3) {
            flag_wait(sh.f_acc);
            const int lp = lane_fresh();
            path_err = sh.pe[0][lp];
            tot_rew = sh.pe[1][lp];
        }
        // the reward: W2's position / path terms (usually long ready: the physics chain ends last)
        flag_wait(sh.f_rp);
        if (vw) {
            RewardPos RP{};
            RP.aa = sh.u.p.post[4][ln];
            RP.coll = sh.u.p.post[5][ln];
            RP.reach = sh.u.p.post[6][ln];
            RewardPath RQ{};
            RQ.ls = sh.u.p.post[0][ln];
            RQ.lc = sh.u.p.post[1][ln];
            RQ.pa = sh.u.p.post[2][ln];
            if (!GRP) {  // (read with the other terms; the grouped kernel measured 1.5 % slower so)
                pdist = sh.u.p.post[3][ln];
                plal = sh.pflags[ln];
            }
            const RewardSum Q = reward_sum(a.cfg, RP, RV, RQ);
            rew_sum = Q.reward;
            rew_pp = Q.pp;
        }
    } else if (wave == 1) {
        // ---------------------------------------------------------------- sensing
        float row[19];
        bool need = false;
        if (S3) {
            // the middle third of W2's golden-march re-check first, at W2's priority (its critical path)
            __builtin_amdgcn_s_setprio(PRIO_W2);
            if (valid && a.brt) {
                const BrTab& T = a.brt[sh.scn[lane]];
                const BtHot* hot = LTAB ? hots + sh.scn[lane] : &T.hot;
                Body F = PF;
                advance_position(F);
                BtLane L = bt_start<LTAB>(T, hot, F.px, F.py);
                const int k0 = bt_third(T, 1), k1 = bt_third(T, 2);
                if (k0 < min(k1, L.len)) {
                    if (k0 >= 4) bt_window<LTAB>(hot, L, k0, F.px, F.py);
                else bt_window_snap<LTAB>(T, hot, L, k0, F.px, F.py);
                    bt_verify<LTAB>(hot, L, k0, k1, F.px, F.py);
                }
                atomicMin(&sh.pflags[lane], (uint32_t)L.dev);
            }
            flag_raise(sh.f_ver1);
        }
        __builtin_amdgcn_s_setprio(PRIO_W1);
        if (valid) {
            Body F = PF;
            advance_position(F);
            double so[19];
            sensor_pos(a.cfg, S, F.px, F.py, F.a, so);
            const CAStatic C = ca_static(a.cfg, S, so);
            sh.cas[0][lane] = C.d;
            sh.cas[1][lane] = C.os;
            sh.cas[2][lane] = C.oc;
            sh.cas[3][lane] = C.lpa;
            sh.cas[4][lane] = C.lca;
            sh.cas[5][lane] = C.rr;
#pragma unroll
            for (int k = 0; k < 19; ++k) row[k] = (float)so[k];
        }
        flag_raise(sh.f_ca);
        // envs that end (W0): terminal rows, and the spawn-state sensor part (cached when ready)
        flag_wait(sh.f_done);
        if (valid) {
            done = sh.cause[lane] != 0u;
            need = done && auto_reset;
            if (done && trow) {
#pragma unroll
                for (int k = 3; k < 17; ++k) trow[k] = row[k];
            }
        }
        if (__ballot(need) != 0ull) {
            if (need) {
                if (sh.cvalid[lane] != 0u) {
                    const float* c = a.rc_obs + rc_entry(a, i, sh.ep[lane]) * D2D_OBS_DIM;
#pragma unroll
                    for (int k = 0; k < 19; ++k) row[k] = c[k];
                } else {
                    const uint32_t ep = sh.ep[lane];
                    const SC& SN = scns[next_scenario(a, ie, ep)];
                    double sp[7], so[19];
                    spawn_state(a, SN, ie, ep, sp);
                    sensor_obs(a.cfg, SN, Body{sp[0], sp[1], sp[2], 0.0, 0.0, 0.0}, so);
#pragma unroll
                    for (int k = 0; k < 19; ++k) row[k] = (float)so[k];
                }
            }
        }
        STAMP(4);
        flag_wait(sh.f_gs);
        STAMP(5);
        if (valid) {
            // a reset row holds the whole spawn-state sensor part, otherwise obs 3..16
            if (need) {
#pragma unroll
                for (int k = 0; k < 19; ++k) orow[k] = row[k];
            } else {
#pragma unroll
                for (int k = 3; k < 17; ++k) orow[k] = row[k];
            }
        }
        tile_arrive(sh.n_tile);
    } else if (wave == 2) {
        // ---------------------------------------------------------------- path search (critical)
        // the critical path, so it wins issue arbitration on its SIMD
        __builtin_amdgcn_s_setprio(PRIO_W2);
        double po[8];
        Body F{};
        if (valid) {
            F = PF;
            advance_position(F);
            uint32_t f = (uint32_t)fld(a.ist, D2D_I_FLAGS, n, i);
            const BrTab* T = brtab(a, sh.scn[lane]);
            if (T) {
                // golden-march re-check of steps [1, split); W3 checks [split, len) meanwhile
                const BtHot* hot = LTAB ? hots + sh.scn[lane] : &T->hot;
                BtLane L = bt_start<LTAB>(*T, hot, F.px, F.py);
                // (tables in global memory: W2 re-checks the whole table, W3 none)
                bt_verify<LTAB>(hot, L, 1, !LDS ? BT_K : S3 ? bt_third(*T, 1) : bt_split(*T), F.px, F.py);
                flag_wait(sh.f_ver);
                if (S3) flag_wait(sh.f_ver1);
                L.dev = min(L.dev, (int)sh.pflags[lane]);
                int iu;
                const double u = bt_finish<LTAB>(S, *T, hot, L.kind, L.dev, F.px, F.py, iu);
                path_obs_u(a.cfg, S, F.px, F.py, F.a, u, f, po, iu);
            } else {
                // (global-memory tables: the plain search scans the lane's knots staged in LDS)
                path_obs<LTAB, SC::RM>(a.cfg, S, T, F.px, F.py, F.a, f, po, LTAB ? hots + sh.scn[lane] : nullptr,
                                       SC::RM ? reinterpret_cast<double*>(d2d_dyn_lds) : nullptr);
            }
            sh.pflags[lane] = f & D2D_FLAG_LA_LOCK;
        }
        STAMP(4);
        __builtin_amdgcn_s_setprio(PRIO_W2_POST);
        // the reward terms that do not need the joint sweep, while the physics wave finishes
        flag_wait(sh.f_done);
        flag_wait(sh.f_ca);
        RewardPos RP{};
        RewardPath RQ{};
        bool d = false;
        if (valid) {
            const int cause = (int)sh.cause[lane];
            d = cause != 0;
            CAStatic C;
            C.lpa = sh.cas[3][lane];
            RP = reward_pos(a.cfg, F, cause, sh.sina[lane]);
            RQ = reward_path(a.cfg, RP, C, po);
        }
        flag_wait(sh.f_gs);
        if (valid) {
            if (!(d && auto_reset)) {
#pragma unroll
                for (int k = 0; k < 8; ++k) orow[19 + k] = (float)po[k];
            }
            if (d && trow) {
#pragma unroll
                for (int k = 0; k < 8; ++k) trow[19 + k] = (float)po[k];
            }
        }
        if (valid) {
            // the position / path terms for W0's sum (u.p is the obs-tile region: after f_gs)
            sh.u.p.post[0][lane] = RQ.ls;
            sh.u.p.post[1][lane] = RQ.lc;
            sh.u.p.post[2][lane] = RQ.pa;
            sh.u.p.post[3][lane] = RQ.dist;
            sh.u.p.post[4][lane] = RP.aa;
            sh.u.p.post[5][lane] = RP.coll;
            sh.u.p.post[6][lane] = RP.reach;
        }
        flag_raise(sh.f_rp);
        tile_arrive(sh.n_tile);
        STAMP(5);
    } else {
        // ---------------------------------------------------------------- auto-reset observation
        __builtin_amdgcn_s_setprio(PRIO_W2);  // the re-check below is on W2's critical path
        double po[8];
        if (!LDS) {
            sh.pflags[lane] = 0x7fffffffu;
        } else if (valid && a.brt) {
            // second half of W2's golden-march re-check (its first wave-priority work)
            const BrTab& T = a.brt[sh.scn[lane]];
            const BtHot* hot = LTAB ? hots + sh.scn[lane] : &T.hot;
            Body F = PF;
            advance_position(F);
            BtLane L = bt_start<LTAB>(T, hot, F.px, F.py);
            const int k0 = S3 ? bt_third(T, 2) : bt_split(T);
            if (k0 < L.len) {
                if (k0 >= 4) bt_window<LTAB>(hot, L, k0, F.px, F.py);
                else bt_window_snap<LTAB>(T, hot, L, k0, F.px, F.py);
                bt_verify<LTAB>(hot, L, k0, BT_K, F.px, F.py);
            }
            if (S3) atomicMin(&sh.pflags[lane], (uint32_t)L.dev);
            else sh.pflags[lane] = (uint32_t)L.dev;
        }
        flag_raise(sh.f_ver);
        __builtin_amdgcn_s_setprio(PRIO_W3);
        if (valid) {
            // running path error / return for W0's epilogue
            sh.pe[0][lane] = fld(a.st, D2D_S_PATH_ERR, n, i);
            sh.pe[1][lane] = fld(a.st, D2D_S_TOT_REW, n, i);
        }
        flag_wait(sh.f_done);
        const bool cv = valid && sh.cvalid[lane] != 0u;
        if (valid) done = sh.cause[lane] != 0u;
        if (valid && done) {
            // finished-episode accumulators, read now so the epilogue does not wait on them
#pragma unroll
            for (int k = 0; k < D2D_NSTATS; ++k) sh.acc[k][lane] = fld(a.acc, k, n, i);
        }
        flag_raise(sh.f_acc);
        if (valid && done && auto_reset) {
            // the next episode: spawn state, reset observation (cached or computed), new state
            const uint32_t ep = sh.ep[lane];
            const int nscn = next_scenario(a, ie, ep);
            const SC& SN = scns[nscn];
            double sp[7];
            spawn_state(a, SN, ie, ep, sp);
            uint32_t rfl = 0;
            if (cv) {
                const size_t ce = rc_entry(a, i, ep);
                const float* c = a.rc_obs + ce * D2D_OBS_DIM + 19;
#pragma unroll
                for (int k = 0; k < 8; ++k) po[k] = (double)c[k];
                rfl = (uint32_t)a.rc_rfl[ce];
            } else {
                path_obs(a.cfg, SN, brtab(a, nscn), sp[0], sp[1], sp[2], rfl, po);
            }
            const double th = sp[2];
            const double bodies[18] = {sp[0], sp[1], th, 0.0, 0.0, 0.0, sp[3], sp[4], th, 0.0, 0.0, 0.0,
                                       sp[5], sp[6], th, 0.0, 0.0, 0.0};
#pragma unroll
            for (int f = 0; f < 18; ++f) fld(a.st, f, n, i) = bodies[f];
#pragma unroll
            for (int k = 0; k < 12; ++k) fld(a.st, D2D_S_J + k, n, i) = 0.0;
            fld(a.st, D2D_S_PATH_ERR, n, i) = 0.0;
            fld(a.st, D2D_S_TOT_REW, n, i) = 0.0;
            fld(a.ist, D2D_I_T, n, i) = 0;
            fld(a.ist, D2D_I_FLAGS, n, i) = (int32_t)rfl;
            fld(a.ist, D2D_I_EPISODE, n, i) = (int32_t)(ep + 1u);
            if (a.cfg.scn_pool && a.env_scn) a.env_scn[ie] = nscn;
        }
        if (!LDS && a.fq) {  // (fresh mode reads its tables from global memory: the LDS
                                             // instantiations carry no queue code, +0.9 us at 4 096 envs)
            // fresh curriculum: the slot the finished episode ran on now takes the episode after
            // next (key ep + 2 - 1 = the new counter), generated by K5 after this launch
            const bool need = valid && done && auto_reset;
            const uint64_t m = __ballot(need);
            if (m != 0ull) {
                const int first = __ffsll((unsigned long long)m) - 1;
                uint32_t base = 0;
                if (lane == first) base = atomicAdd(&a.fqc[FR_HEAD], (uint32_t)__popcll(m));
                base = __shfl(base, first);
                const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (need) a.fq[pos & a.fq_mask] = fresh_slot(ie, sh.ep[lane] + 1u);
            }
        }
        STAMP(4);
        flag_wait(sh.f_gs);
        STAMP(5);
        if (valid && done && auto_reset) {
#pragma unroll
            for (int k = 0; k < 8; ++k) orow[19 + k] = (float)po[k];
        }
        tile_arrive(sh.n_tile);
    }
    STAMP(2);

    // ---------------------------------------------------------------- epilogue
    // W1-W3 store the obs tile once every wave's rows are in it; W0 meanwhile takes the reward sum
    // (above) and writes the bookkeeping (below).  Rows [e0, e0+rows) are one contiguous span of
    // global memory (grouped: one contiguous 108-byte row per env).
    if (wave != 0) {
        tile_wait(sh.n_tile, 4u);
        STAMP(3);
        constexpr int TT = K1_THREADS - 64;  // the storing threads
        const int tq = qt - 64;
        if (GRP) {
            for (int k = tq; gvalid && k < EPB * D2D_OBS_DIM; k += TT) {
                const int r = k / D2D_OBS_DIM;
                const int e = a.lane_env[e0 + r];
                if (e >= 0) a.obs[(size_t)e * D2D_OBS_DIM + (k - r * D2D_OBS_DIM)] = sh.u.p.obs[k];
            }
        } else {
            const int rows = gvalid ? max(0, min(EPB, a.n - e0)) : 0;
            const int words = rows * D2D_OBS_DIM;
            float* dst = a.obs + (size_t)e0 * D2D_OBS_DIM;
            // a full tile is 64 x 27 floats = 432 float4 at a 16-B aligned offset (e0 * 108 B, e0 % 64
            // == 0; the caller's obs buffer is a torch allocation): 16-byte stores
            int k0 = 0;
            if (rows == EPB && ((uintptr_t)a.obs & 15u) == 0) {
                float4* d4 = reinterpret_cast<float4*>(dst);
                const float4* s4 = reinterpret_cast<const float4*>(sh.u.p.obs);
                for (int k = tq; k < words / 4; k += TT) d4[k] = s4[k];
                k0 = words;
            }
            for (int k = k0 + tq; k < words; k += TT) dst[k] = sh.u.p.obs[k];
        }
    } else {
        if (S3) flag_wait(sh.f_acc);  // (at full load W0 waited for it before the reward)
        STAMP(3);
    }
    const int lne = lane_fresh(), ile = e0 + lne, iee = GRP ? ie : ile;
    const bool vle = gvalid && (GRP ? iee >= 0 : ile < a.n);
    if (wave == 0 && vle) {
        const int lane = lne, i = ile, ie = iee;
        if (S3) {
            path_err = sh.pe[0][lane];
            tot_rew = sh.pe[1][lane];
        }
        flags = (flags & ~D2D_FLAG_LA_LOCK) | (GRP ? sh.pflags[lane] : plal);
        const double reward = rew_sum;
        path_err += GRP ? sh.u.p.post[3][lane] : pdist;
        // (the grouped kernel divides here; the env-ordered one only for the envs that end)
        const double ape_g = GRP ? path_err / (double)t : 0.0;
        tot_rew += reward;
        bool trunc = false, term = done;
        if (a.cfg.timeup_truncates && done && cause == D2D_END_TIMEUP) {
            trunc = true;
            term = false;
        }
        const int io = ie;
        a.rew[io] = (float)reward;
        a.term[io] = (uint8_t)term;
        a.trunc[io] = (uint8_t)trunc;
        if (a.info) {
            float* r = a.info + (size_t)ie * D2D_INFO_DIM;
            r[D2D_INFO_CA] = (float)RV.cal;
            r[D2D_INFO_PA] = (float)sh.u.p.post[2][lane];
            r[D2D_INFO_PP] = (float)rew_pp;
            r[D2D_INFO_COLL] = (float)sh.u.p.post[5][lane];
            r[D2D_INFO_REACH] = (float)sh.u.p.post[6][lane];
            r[D2D_INFO_AA] = (float)sh.u.p.post[4][lane];
            r[D2D_INFO_DCLOSE] = (float)dclose;
            r[D2D_INFO_STEPS] = (float)t;
            r[D2D_INFO_CAUSE] = (float)cause;
            r[D2D_INFO_APE] = done ? (float)(GRP ? ape_g : path_err / (double)t) : 0.0f;
            r[D2D_INFO_TOTREW] = done ? (float)tot_rew : 0.0f;
            r[D2D_INFO_REWARD] = (float)reward;
        }
        if (done) {
            // finished-episode accumulators (info counters of drone_2d_env.py:593-613)
            double pacc[D2D_NSTATS];
#pragma unroll
            for (int k = 0; k < D2D_NSTATS; ++k) pacc[k] = sh.acc[k][lane];
            const double ape = GRP ? ape_g : path_err / (double)t;
            const bool c1 = cause & D2D_END_COLLISION, c2 = cause & D2D_END_REACH;
            const bool c4 = cause & D2D_END_TIMEUP, c5 = cause & D2D_END_AA;
            fld(a.acc, D2D_ST_RETURN, n, i) = pacc[D2D_ST_RETURN] + tot_rew;
            fld(a.acc, D2D_ST_EPISODES, n, i) = pacc[D2D_ST_EPISODES] + 1.0;
            fld(a.acc, D2D_ST_SUCCESS, n, i) = pacc[D2D_ST_SUCCESS] + (c2 ? 1.0 : 0.0);
            fld(a.acc, D2D_ST_FAIL, n, i) = pacc[D2D_ST_FAIL] + ((c1 || c4 || c5) ? 1.0 : 0.0);
            fld(a.acc, D2D_ST_COLLISION, n, i) = pacc[D2D_ST_COLLISION] + ((c1 && !c2 && !c4 && !c5) ? 1.0 : 0.0);
            fld(a.acc, D2D_ST_APE, n, i) = pacc[D2D_ST_APE] + ape;
            fld(a.acc, D2D_ST_LEN, n, i) = pacc[D2D_ST_LEN] + (double)t;
        }
        if (!(done && auto_reset)) {
            fld(a.st, D2D_S_PATH_ERR, n, i) = path_err;
            fld(a.st, D2D_S_TOT_REW, n, i) = tot_rew;
            fld(a.ist, D2D_I_T, n, i) = t;
            fld(a.ist, D2D_I_FLAGS, n, i) = (int32_t)flags;
        }
    }
    STAMP(6);
}

template <bool LDS, bool LTAB, bool GRP, bool S3, class S>
__device__ __forceinline__ void k1_group(const StepArgs& a, S* s_scn, K1Shared& sh, int wg) {
    const S* scns;
    const BtHot* hots;
    int s0;
    k1_stage<LDS, LTAB, GRP, S>(a, s_scn, wg, scns, hots, s0);
    k1_body<LDS, LTAB, GRP, S3, S>(a, scns, hots, s0, sh, wg, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                                   (int)threadIdx.x);
}
// S3: the three-way table re-check (W2, W1 and W3 one third each of the golden-march table), chosen at
// launch when K1 has at most one workgroup per CU (4 096 / 16 384 envs -4 %; at full load +3.6 %)
// (LDS: the handle's tables are ScnF, staged; otherwise ScnR, read per lane from global memory)
template <bool LDS, bool LTAB, bool S3>
__global__ __launch_bounds__(K1_THREADS, 4) void d2d_step_kernel(StepArgs a) {
    using S = std::conditional_t<LDS, ScnF, ScnR>;
    __shared__ __attribute__((aligned(16))) K1Shared sh;
    k1_group<LDS, LTAB, false, S3, S>(a, reinterpret_cast<S*>(d2d_dyn_lds), sh, blockIdx.x);
}
// grouped slot layout: a pure group stages its scenario and probe table in LDS; a group that
// straddles two scenarios (at most n_scn - 1 of them: the layout has no padding between scenarios)
// stages both scenarios (2 x Scn fits in the Scn + BtHot allocation) and reads the probe tables
// through L1/L2; a group of three or more scenarios reads everything through L1/L2
template <bool S3>
__global__ __launch_bounds__(K1_THREADS, 4) void d2d_step_grouped_kernel(StepArgs a) {
    ScnF* s_scn = reinterpret_cast<ScnF*>(d2d_dyn_lds);  // (a grouped map's tables are ScnF)
    __shared__ __attribute__((aligned(16))) K1Shared sh;
    static_assert(2 * sizeof(ScnF) <= sizeof(ScnF) + sizeof(BtHot), "two staged scenarios");
    const int wg = xcd_group(blockIdx.x, gridDim.x);
    const int ws = a.wg_scn[wg];
    if (a.brt && ws >= 0)
        k1_group<true, true, true, S3, ScnF>(a, s_scn, sh, wg);
    else if (ws <= -2)
        k1_group<true, false, true, S3, ScnF>(a, s_scn, sh, wg);
    else
        k1_group<false, false, true, S3, ScnF>(a, s_scn, sh, wg);
}

// ------------------------------------------------------------------------------------------ K2
// LDS: stage every scenario; RM: the handle's layout (ScnR / ScnF)
template <bool LDS, bool RM>
__global__ __launch_bounds__(BLOCK) void d2d_reset_kernel(StepArgs a) {
    using S = std::conditional_t<RM, ScnR, ScnF>;
    const S* scns = stage_scenarios<LDS, BLOCK>(a, reinterpret_cast<S*>(d2d_dyn_lds));
    __syncthreads();
    const int i = blockIdx.x * BLOCK + threadIdx.x;  // slot
    if (i >= a.ns) return;
    const int ie = a.lane_env ? a.lane_env[i] : i;  // env
    if (ie < 0) return;
    if (a.mask && !a.mask[ie]) return;
    const int n = a.ns;
    int si = (a.env_scn && a.n_scn > 1) ? a.env_scn[ie] : 0;
    if (a.cfg.scn_pool) {
        si = next_scenario(a, ie, (uint32_t)fld(a.ist, D2D_I_EPISODE, n, i));
        a.env_scn[ie] = si;
    }
    const S& s = scns[si];
    double sp[7];
    spawn_state(a, s, ie, (uint32_t)fld(a.ist, D2D_I_EPISODE, n, i), sp);
    const double th = sp[2];
    const double bodies[18] = {sp[0], sp[1], th, 0.0, 0.0, 0.0, sp[3], sp[4], th, 0.0, 0.0, 0.0,
                               sp[5], sp[6], th, 0.0, 0.0, 0.0};
    uint32_t flags = 0;
    double obs[D2D_OBS_DIM];
    observe(a.cfg, s, brtab(a, si), Body{sp[0], sp[1], th, 0.0, 0.0, 0.0}, flags, obs);
#pragma unroll
    for (int f = 0; f < 18; ++f) fld(a.st, f, n, i) = bodies[f];
#pragma unroll
    for (int k = 0; k < 12; ++k) fld(a.st, D2D_S_J + k, n, i) = 0.0;
    fld(a.st, D2D_S_PATH_ERR, n, i) = 0.0;
    fld(a.st, D2D_S_TOT_REW, n, i) = 0.0;
    fld(a.ist, D2D_I_T, n, i) = 0;
    fld(a.ist, D2D_I_FLAGS, n, i) = (int32_t)flags;
    fld(a.ist, D2D_I_EPISODE, n, i) += 1;
    if (a.obs) {
#pragma unroll
        for (int k = 0; k < D2D_OBS_DIM; ++k) a.obs[(size_t)ie * D2D_OBS_DIM + k] = (float)obs[k];
    }
}

// ------------------------------------------------------------------------------ slot permutation
// dst[f][dslot(e)] = src[f][sslot(e)] for every env e and field f < nf (a null map: slot == env):
// get_state / set_state through the grouped slot layout, and re-layouts in d2d_set_scenarios
template <typename T>
__global__ __launch_bounds__(BLOCK) void d2d_permute_kernel(const T* src, int sstride, const int32_t* sslot, T* dst,
                                                            int dstride, const int32_t* dslot, int nf, int n) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    const int si = sslot ? sslot[e] : e, di = dslot ? dslot[e] : e;
    for (int f = 0; f < nf; ++f) dst[(size_t)f * dstride + di] = src[(size_t)f * sstride + si];
}

// ------------------------------------------------------------------------------ cache fill (K4)
// K4 with the four waves of a block working on the same 64 compacted envs at a time (K4 runs
// alone on a mostly idle GPU, so its duration is one env's latency chain): wave 0 the spawn-state
// sensor part, waves 1-3 one third each of the golden-march re-check, then wave 1 the Brent
// continuation and the path part.  Same operations as the one-lane-per-env path.
template <class SC>
__device__ __forceinline__ void fill_split(const StepArgs& a, const SC* scns, const int* list, int total) {
    __shared__ int devp[3][64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int n = a.ns;
    for (int r0 = 0; r0 < total; r0 += 64) {
        const bool act = r0 + lane < total;
        const int item = list[act ? r0 + lane : r0];  // inactive lanes repeat the round's first item
        const int i = item >> 1;                      // slot; key = the env's episode counter + (item & 1)
        const int32_t ep = fld(a.ist, D2D_I_EPISODE, n, i) + (item & 1);
        const size_t ce = rc_entry(a, i, (uint32_t)ep);
        const int ie = a.lane_env ? a.lane_env[i] : i;
        const int si = next_scenario(a, ie, (uint32_t)ep);
        const SC& S = scns[si];
        const BrTab* T = brtab(a, si);
        double sp[7];
        spawn_state(a, S, ie, (uint32_t)ep, sp);
        if (r0 == 0) FSTAMP(2);
        float* c = a.rc_obs + ce * D2D_OBS_DIM;
        if (wave != 0 && T) {
            const int w = wave - 1;
            BtLane L = bt_start<false>(*T, &T->hot, sp[0], sp[1]);
            // steps [1, b1), [b1, b2), [b2, BT_K)
            const int third = (T->len[0] + 2) / 3;
            const int b1 = 1 + third, b2 = 1 + 2 * third;
            if (w == 0) {
                bt_verify<false>(&T->hot, L, 1, b1, sp[0], sp[1]);
            } else {
                const int k0 = (w == 1) ? b1 : b2, k1 = (w == 1) ? b2 : BT_K;
                if (k0 < min(k1, L.len)) {
                    // the window before step k0 (table-following so far): the snapshot's probes
                    const BtSnap& W = T->snap[L.kind][k0];
                    L.fa = bt_dist<false>(&T->hot, L.kind, W.j_fulc, sp[0], sp[1]);
                    L.fb = bt_dist<false>(&T->hot, L.kind, W.j_nfc, sp[0], sp[1]);
                    L.fc = bt_dist<false>(&T->hot, L.kind, W.j_xf, sp[0], sp[1]);
                    bt_verify<false>(&T->hot, L, k0, k1, sp[0], sp[1]);
                }
            }
            devp[w][lane] = L.dev;
        }
        if (r0 == 0) FSTAMP(3);
        __syncthreads();
        if (r0 == 0) FSTAMP(4);
        if (wave == 0) {
            // the sensor part is independent of the path search: off the barrier's critical path
            double so[19];
            sensor_obs(a.cfg, S, Body{sp[0], sp[1], sp[2], 0.0, 0.0, 0.0}, so);
            if (act) {
#pragma unroll
                for (int k = 0; k < 19; ++k) c[k] = (float)so[k];
            }
        }
        if (wave == 1) {
            double o[8];
            uint32_t f = 0;
            if (T) {
                const int kind = bt_start<false>(*T, &T->hot, sp[0], sp[1]).kind;
                const int dev = min(devp[0][lane], min(devp[1][lane], devp[2][lane]));
                int iu;
                const double u = bt_finish<false>(S, *T, &T->hot, kind, dev, sp[0], sp[1], iu);
                if (r0 == 0) FSTAMP(5);
                path_obs_u(a.cfg, S, sp[0], sp[1], sp[2], u, f, o, iu);
                if (r0 == 0) FSTAMP(6);
            } else {
                path_obs(a.cfg, S, nullptr, sp[0], sp[1], sp[2], f, o);
            }
            if (act) {
#pragma unroll
                for (int k = 0; k < 8; ++k) c[19 + k] = (float)o[k];
                a.rc_rfl[ce] = (int32_t)f;
            }
        }
        __syncthreads();  // the sensor part is stored before the tag; devp is reused next round
        if (wave == 1 && act) a.rc_tag[ce] = ep;
    }
}

// an env whose entry does not belong to its current episode computes the observation its next
// auto-reset will return (test-mode spawn of the next episode's scenario).  Only the envs reset
// since the last fill need it (~1/5 of them at fill period 16): each workgroup compacts its
// envs that do into the leading lanes (ballot + popcount), so the long search runs in as few
// waves as possible instead of one wave per 64 envs with a few active lanes.
template <bool LDS, class S>
__device__ __forceinline__ void fill_work(const StepArgs& a) {
    __shared__ int list[BLOCK];
    __shared__ int cnt[BLOCK / 64];
    FSTAMP(0);
    const S* scns = stage_scenarios<LDS, BLOCK>(a, reinterpret_cast<S*>(d2d_dyn_lds));
    const int n = a.ns;
    // work items: (slot, which) -- the entry for the env's current episode counter (which = 0) and
    // for the next one (which = 1); thread t takes slot t % FILL_SPB, which t / FILL_SPB
    static_assert(RC_SLOTS == 2 && 2 * FILL_SPB <= BLOCK, "two items per slot");
    const int which = (int)threadIdx.x / FILL_SPB;
    const int i0 = blockIdx.x * FILL_SPB + (int)threadIdx.x % FILL_SPB;  // slot
    const bool need = ((int)threadIdx.x < RC_SLOTS * FILL_SPB) && (i0 < n) && (!a.lane_env || a.lane_env[i0] >= 0) && [&] {
        const int32_t key = fld(a.ist, D2D_I_EPISODE, n, i0) + which;
        // fresh curriculum: only once the scenario of that episode exists
        return a.rc_tag[rc_entry(a, i0, (uint32_t)key)] != key &&
               (a.cfg.scn_pool != 2 || a.scn_tag[fresh_slot(i0, (uint32_t)key)] == key);
    }();
    const uint64_t m = __ballot(need);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) cnt[wave] = __popcll(m);
    __syncthreads();
    int off = 0, total = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) {
        off += (w < wave) ? cnt[w] : 0;
        total += cnt[w];
    }
    if (need) list[off + __popcll(m & ((1ull << lane) - 1ull))] = 2 * i0 + which;
    __syncthreads();
    if (total == 0) return;  // block-uniform
    FSTAMP(1);
    fill_split(a, scns, list, total);
    FSTAMP(7);
#ifdef D2D_STAMPS
    if (a.stamps && threadIdx.x == 0)  // the block's number of fills after the stamps
        a.stamps[D2D_FSTAMP_BASE + (size_t)gridDim.x * 32 + blockIdx.x] = (uint64_t)total;
#endif
}

// The launch cadence is fixed on the host (every FILL_PERIOD steps, so a captured graph of 16
// steps holds one launch); only every FILL_EVERY-th launch fills, decided
// by a device tick (so a replayed graph alternates too): every workgroup reads ctl[0], workgroup 0
// writes the next value to ctl[1], and the next K1 launch copies it to ctl[0] -- no workgroup
// writes what another may still read, and no atomics contend on one address.
// K4 runs with K1's residency (4 waves per SIMD, K1's LDS per workgroup: exactly 4 workgroups per
// CU, one round).  K4 (1 024 workgroups at 65 536 envs) otherwise ran 3 per CU and left the CUs'
// wave-placement rotation uneven, and the next K1 then put two path waves of one CU on one SIMD on
// a few CUs (+7 us on that step, tools/ubench_after_stamps.py).
template <bool LDS, bool RM>
__global__ __launch_bounds__(BLOCK, 4) void d2d_fill_kernel(StepArgs a) {
    const bool ticked = !a.fill_force && a.fill_every > 1;
    bool run = true;
    if (ticked) {
        const int tick = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&a.fill_ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        run = tick % a.fill_every == a.fill_every - 1;
        if (blockIdx.x == 0 && threadIdx.x == 0)
            __hip_atomic_store(&a.fill_ctl[1], tick + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (run) fill_work<LDS, std::conditional_t<RM, ScnR, ScnF>>(a);
}

// ------------------------------------------------------------------------ fresh curriculum (K5)
// Scenario generation for the fresh curriculum (d2d_curriculum.h).  The scenario of the episode env
// i's next reset starts (key = its episode counter) goes into slot 2 i + (key & 1) unless that slot
// already holds it; the other slot holds the running episode's.  Launched after every K1 (the slot is
// needed one step later at the earliest), before and after K2, and after d2d_set_state; restore = 1
// regenerates every slot from its recipe (key, clock) instead.  Two launches:
//   K5a d2d_fresh_scan_kernel  one thread per env (slot when restoring): the slots to generate are
//                              appended to a device queue (one atomic per wave)
//   K5b d2d_fresh_gen_kernel   one wave per queued slot: gen_curriculum_wave builds the scenario in
//                              LDS with all 64 lanes, then the golden-march tables (lanes 0 and 1, one
//                              forced run each) and coalesced copies of the ABI record and the device
//                              table.  ~90 slots per step at 65 536 envs: they run side by side, so the
//                              launch lasts about one slot's latency.
// (Round 3's K5 built each scenario serially on one lane, with the device table in global memory:
// 320 us mean, 3.8 ms max per launch.)
struct FreshArgs {
    int n;                   // envs (pool modes keep the identity slot layout: slot == env)
    const int32_t* ist;      // [NISTATE][n] (episode counters)
    int32_t* env_scn;        // [n] the running episode's slot, 2 i + ((ep - 1) & 1)
    d2d_curriculum cur;
    double W, H;
    uint64_t seed;
    uint32_t env_id_base;
    d2d_scn* abi;            // [2 n] ABI records (read back for the oracle)
    ScnR* scn;               // [2 n] (the fresh curriculum's tables are ScnR)
    int32_t* tag;            // [2 n] episode key of each slot (-1: empty)
    int64_t* gclk;           // [2 n] clock at generation
    const int64_t* clock;    // the step clock (K1 advances it)
    int32_t* queue;          // [mask + 1] slots to generate (K1 / K5a -> K5b), a ring (FreshRing)
    uint32_t* ring;          // FreshRing words: head, the two tails
    uint32_t mask;           // ring size - 1
    int scan;                // 1: K5a appended (the tail is the later of the two words)
    uint64_t* stamps;        // diagnostic builds only (D2D_GEN_STAMPS): [queue position][8]
    int restore;
};
__global__ __launch_bounds__(256) void d2d_fresh_scan_kernel(FreshArgs f) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    bool need = false;
    int slot = 0;
    if (f.restore) {
        if (t < 2 * f.n) {
            slot = t;
            need = f.tag[slot] >= 0;
        }
    } else if (t < f.n) {
        const int32_t ep = f.ist[(size_t)D2D_I_EPISODE * f.n + t];
        f.env_scn[t] = fresh_slot(t, (uint32_t)(ep - 1));
        slot = fresh_slot(t, (uint32_t)ep);
        need = f.tag[slot] != ep;
    }
    const uint64_t m = __ballot(need);
    if (m == 0ull) return;
    const int lane = threadIdx.x & 63, first = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(&f.ring[FR_HEAD], (uint32_t)__popcll(m));
    base = __shfl(base, first);
    const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (need) f.queue[pos & f.mask] = slot;
}
// K5b: one wave per queued slot generates the scenario in LDS (d2d_curriculum.h) and writes the device
// table and the ABI record.  (No golden-march tables in fresh mode: built per scenario they cost K5b
// more than they save K1, docs/DESIGN_HISTORY.md "Round 4".)  It drains the ring from the tail to the head
// (FreshRing) and, after a K1, leaves the head as the next tail.
__global__ __launch_bounds__(64) void d2d_fresh_gen_kernel(FreshArgs f) {
    __shared__ __attribute__((aligned(16))) GenLds G;
    const int lane = threadIdx.x;
    const uint32_t head = f.ring[FR_HEAD];  // (K1 / K5a have finished: stable)
    uint32_t tail;
    if (f.scan) {  // the later of the two tails (both are at or behind the head, modulo 2^32)
        tail = head - min(head - f.ring[FR_TAIL0], head - f.ring[FR_TAIL1]);
    } else {  // after K1: its clock parity picks the word; the other one is the next K5b's
        const int64_t clk = *f.clock;
        tail = f.ring[FR_TAIL0 + (int)(clk & 1)];
        if (blockIdx.x == 0 && lane == 0) f.ring[FR_TAIL0 + (int)((clk + 1) & 1)] = head;
    }
    // (at most 2 n slots exist, and the ring holds them; never read more than the ring)
    const int count = (int)min(head - tail, f.mask + 1u);
    for (int it = blockIdx.x; it < count; it += gridDim.x) {
        const int slot = f.queue[(tail + (uint32_t)it) & f.mask];
        const int i = slot >> 1;
        int key;
        int64_t clk;
        if (f.restore) {
            key = f.tag[slot];
            clk = f.gclk[slot];
        } else {
            key = f.ist[(size_t)D2D_I_EPISODE * f.n + i];
            clk = *f.clock;
        }
        uint64_t* st = nullptr;
#ifdef D2D_GEN_STAMPS
        if (f.stamps && it < 2 * f.n) st = f.stamps + (size_t)it * 8;
#endif
        const double sim = f.cur.sim_num0 + (double)clk * f.cur.envs_total;
        const uint32_t gid = f.env_id_base + (uint32_t)i;
        const int pos = gen_path_wave(f.cur, f.W, f.H, f.seed, gid, (uint32_t)key, G, lane, st);
        gen_rest_wave(f.cur, f.W, f.H, f.seed, gid, (uint32_t)key, sim, pos, G, lane, st);
        // the device table and the ABI record, 8-byte words across the wave
        const double* src = reinterpret_cast<const double*>(&G.s);
        double* dst = reinterpret_cast<double*>(f.scn + slot);
        for (int k = lane; k < (int)(sizeof(ScnR) / 8); k += 64) dst[k] = src[k];
        static_assert(sizeof(d2d_scn) % 8 == 0, "d2d_scn size");
        const double* sa = reinterpret_cast<const double*>(&G.a);
        double* da = reinterpret_cast<double*>(f.abi + slot);
        for (int k = lane; k < (int)(sizeof(d2d_scn) / 8); k += 64) da[k] = sa[k];
        GSTAMP(st, 6);
        if (lane == 0) {
            f.gclk[slot] = clk;
            f.tag[slot] = key;
        }
        __syncthreads();  // G is reused by the next item
    }
}

// after a scan's K5b: both tails to the head (FreshRing; a kernel node, ordered like every other
// launch of a graph)
__global__ __launch_bounds__(64) void d2d_fresh_tail_kernel(uint32_t* ring) {
    if (threadIdx.x == 0) ring[FR_TAIL0] = ring[FR_TAIL1] = ring[FR_HEAD];
}

// ------------------------------------------------------------------------- golden-march tables
// one thread per (scenario, kind): the forced runs of brtab_build (d2d_device.h)
template <class S>
__global__ __launch_bounds__(64) void d2d_brtab_kernel(const S* scn, int n_scn, BrTab* out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 2 * n_scn) return;
    brtab_build(scn[t >> 1], t & 1, out[t >> 1]);
}

// ------------------------------------------------------------------------------------ self-test
// random fp64 with a biased exponent in [emin, emax] and 52 random mantissa bits
__device__ __forceinline__ double st_rand(uint32_t hi, uint32_t lo, int emin, int emax, uint32_t sign) {
    const uint32_t span = (uint32_t)(emax - emin + 1);
    const uint64_t ex = (uint64_t)(emin + (int)((hi >> 20) % span));
    const uint64_t bits = ((uint64_t)(sign & 1u) << 63) | (ex << 52) | ((uint64_t)(hi & 0xFFFFFu) << 32) | lo;
    return __longlong_as_double((long long)bits);
}
__global__ __launch_bounds__(256) void d2d_selftest_kernel(int which, long long n, uint64_t seed,
                                                           unsigned long long* bad) {
    unsigned long long cnt = 0;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
        uint32_t o[4], p[4];
        philox((uint32_t)k, (uint32_t)(k >> 32), 0x5E1F7E57u, (uint32_t)which, k0, k1, o);
        philox((uint32_t)k, (uint32_t)(k >> 32), 0x5E1F7E58u, (uint32_t)which, k0, k1, p);
        double got, want;
        if (which == D2D_SELFTEST_SQRT) {
            const uint32_t sel = p[0] & 63u;  // 1/64 zeros, 1/64 +inf, the rest in [2^-767, max]
            const double x = (sel == 0u) ? 0.0 : ((sel == 1u) ? __builtin_inf() : st_rand(o[0], o[1], 1023 - 767, 2046, 0u));
            // odd indices through sqrt_dist (the wave-uniform fix-up branch: waves with a zero or an
            // infinity among their lanes take it), even ones through sqrt_nz
            got = (k & 1) ? sqrt_dist(x) : sqrt_nz(x);
            want = sqrt(x);
        } else {
            const double a = st_rand(o[0], o[1], 1023 - 400, 1023 + 400, o[2]);
            const double b = st_rand(p[0], p[1], 1023 - 400, 1023 + 400, p[2]);
            want = a / b;
            got = (which == D2D_SELFTEST_DIV) ? div_normal(a, b) : div_by_recip(a, b, 1.0 / b);
        }
        cnt += (__double_as_longlong(got) != __double_as_longlong(want)) ? 1ull : 0ull;
    }
    if (cnt) atomicAdd(bad, cnt);
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
