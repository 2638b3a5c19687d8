// d2d_device.h -- device functions of the batched Drone2dEnv step (gfx950, fp64).
//
// Evaluation order follows the reference's NumPy order term by term (oracle/d2d_oracle.c is the
// plain restatement, tests/golden the pinned vectors); compiled with -ffp-contract=off, the only
// fused ops are where NumPy/OpenBLAS itself fuses (np.linalg.norm, 2x2 np.matmul).
//
// The step is split into two "roles" that the cooperative kernel runs on different waves:
//   path role    Brent closest point -> closest/lookahead point, LA lock, LA/CP angles (obs 19..26)
//   sensor role  kinematics, 3-nearest circles, velocity angle (obs 0..18) + the reward's CA part
// Their latency chains are independent, so running them on different waves of one workgroup turns
// sum(latency) into max(latency).  All branches inside a role are written as selects so a wave's
// lanes never serialise over divergent paths.
//
// Reference anchors (drone_2d_custom_gym_env/):
//   thrust            drone_2d_env.py:400-404
//   physics           Chipmunk2D cpSpaceStep for Drone.py:9-95
//   collision         drone_2d_env.py:17-19, 190-191, 543-547 (frame box vs circles)
//   sensing           drone_2d_env.py:617-629, 660-720, 948-961
//   observation       drone_2d_env.py:631-773
//   path / Brent      predef_path.py:53-142, 226-266 ; scipy fminbound
//   reward / done     drone_2d_env.py:423-615
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/drone2d.h"
#include "d2d_pmath.h"

// bool conditions are combined with & / | on purpose (selects instead of short-circuit branches)
#pragma clang diagnostic ignored "-Wbitwise-instead-of-logical"

// D2D_BSTAMP (diagnostic builds only, tools/bstamps.py): s_memtime stamps inside the golden-march
// continuation's Brent steps, per path wave -- [workgroup][step < 64][8] in d2d_bst: entry, candidate
// computed, interval found, probe evaluated, state updated, the step's B.num, whether the wave took
// the knot scan, the active lanes.
#ifdef D2D_BSTAMP
#define BST_N (1024 * 64 * 8)
__device__ uint64_t d2d_bst[BST_N];
#define BST_ARG , uint64_t* bst = nullptr
// (the stamp waits for `dep`, and volatile asm keeps the stamps in program order)
#define BST(k, dep)                                                                                      \
    do {                                                                                                 \
        if (bst) {                                                                                       \
            uint64_t bst_v;                                                                              \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(bst_v) : "v"(dep));            \
            bst_t[k] = bst_v;                                                                            \
        }                                                                                                \
    } while (0)
#else
#define BST_ARG
#define BST(k, dep) \
    do {       \
    } while (0)
#endif

namespace d2d {

constexpr double PI = 3.141592653589793;      // np.pi
constexpr double TWO_PI = 6.283185307179586;  // 2*np.pi
constexpr double DT = 1.0 / 60.0;             // drone_2d_env.py:406
constexpr double GRAV_Y = -1000.0;            // drone_2d_env.py:185
constexpr double DRONE_R = 40.0;              // Drone.py:11 (100/2 - 20/2)
constexpr double FRAME_HX = 50.0, FRAME_HY = 5.0;   // Drone.py:16 box (100, 10)
constexpr double VEL_MAX = 1330.0;            // drone_2d_env.py:635

// Device-side scenario, built once from the ABI table (d2d_scn) by scn_build in d2d_set_scenarios.
//   us[k >= n_wps] = +inf: unused knots never count in u_index.
//   rec[.][n] = everything QPMI2D.__call__ needs once u's knot interval n is known, read from one
//   per-lane base (field-major, so lanes in different intervals hit different LDS banks) instead
//   of the scattered coefficient gathers: the "B" quadratic min(n, nseg-1), the "A" quadratic of
//   the blend (n-1, or the last one for n = 0: Python's x_params[-1]), us[n], us[n+1] and
//   RN(1 / (us[n+1] - us[n])), and the blend threshold T: in interval n QPMI2D.__call__ blends the
//   two quadratics exactly when u < T[n] (below).
enum { REC_XB = 0, REC_XA = 6, REC_U0 = 12, REC_U1 = 13, REC_IDU = 14, REC_T = 15, REC_N = 16 };
// Two layouts of the same table, one per way K1 reads it (both in the one library, chosen per
// handle by where K1 reads the scenarios from; the kernels are templated on the type):
//   ScnF  field-major rec[f][n] + the knots us[k]: tables K1 stages in LDS (test scenarios, mixed
//         maps).  Lanes in different knot intervals read different banks.
//   ScnR  record-major with a one-double pad (interval n's 16 fields contiguous, 136 bytes apart):
//         tables K1 reads from global memory, one lane per scenario (pools, the fresh curriculum):
//         one QPMI2D evaluation touches two cache lines per lane instead of 16.
// Measured (profiles/r04/layout/): ScnR for every path costs the LDS paths 0.6 % (corridor), 3 %
// (mixed) and 5.6 % (4 096 envs); ScnF for the fresh curriculum's step kernel 179 vs 105 us.
constexpr int REC_W = REC_N + 1;  // ScnR's pad word: a 136-byte record stride
#define D2D_SCN_TAIL                                                                                      \
    double cx[D2D_MAX_CIRCLES], cy[D2D_MAX_CIRCLES], cr[D2D_MAX_CIRCLES];                               \
    double wp_last_x, wp_last_y;                                                                          \
    double spawn_xmin, spawn_xmax, spawn_ymin, spawn_ymax, spawn_amin, spawn_amax;                        \
    /* the common radius when every circle has the same one (all test scenarios), else NaN (also keeps */ \
    /* the size a multiple of 16: the probe tables staged after it stay aligned) */                       \
    double r_uniform;
struct ScnF {
    static constexpr bool RM = false;
    int32_t n_wps, n_circles;
    double us_[D2D_MAX_WPS];
    double rec_[REC_N][D2D_MAX_WPS];
    D2D_SCN_TAIL
    __host__ __device__ __forceinline__ double& rec(int f, int n) { return rec_[f][n]; }
    __host__ __device__ __forceinline__ const double& rec(int f, int n) const { return rec_[f][n]; }
};
struct ScnR {
    static constexpr bool RM = true;
    int32_t n_wps, n_circles;
    double us_[D2D_MAX_WPS];
    double rec_[D2D_MAX_WPS][REC_W];
    D2D_SCN_TAIL
    __host__ __device__ __forceinline__ double& rec(int f, int n) { return rec_[n][f]; }
    __host__ __device__ __forceinline__ const double& rec(int f, int n) const { return rec_[n][f]; }
};
static_assert(sizeof(ScnF) % 16 == 0 && sizeof(ScnR) % 16 == 0, "Scn size");
#define SREC(s, f, n) ((s).rec((f), (n)))
#define SUS(s, k) ((s).us_[(k)])

// Returns false if the table is outside what the record form reproduces exactly: the last-segment
// window us[nw-2] - 0.001 must not reach back past us[nw-3] (always true for real waypoints).
template <class S>
__host__ __device__ inline bool scn_build(const d2d_scn& a, S& s) {
    const int nw = a.n_wps, nseg = nw - 2;
    if (nw >= 4 && !(a.us[nw - 2] - 0.001 > a.us[nw - 3])) return false;
    s.n_wps = nw;
    s.n_circles = a.n_circles;
    double us[D2D_MAX_WPS];
    for (int k = 0; k < D2D_MAX_WPS; ++k) us[k] = (k < nw) ? a.us[k] : __builtin_inf();
    for (int k = 0; k < D2D_MAX_WPS; ++k) s.us_[k] = us[k];
    if constexpr (S::RM) {
        for (int n = 0; n < D2D_MAX_WPS && REC_W > REC_N; ++n) s.rec_[n][REC_W - 1] = 0.0;  // the pad
    }
    for (int n = 0; n < D2D_MAX_WPS; ++n) {
        const int b = (n < nseg - 1) ? n : nseg - 1;
        const int q = (n == 0) ? nseg - 1 : ((n - 1 < nseg - 1) ? n - 1 : nseg - 1);
        const double v[REC_N] = {a.xa[b], a.xb[b], a.xc[b], a.ya[b], a.yb[b], a.yc[b],
                                 a.xa[q], a.xb[q], a.xc[q], a.ya[q], a.yb[q], a.yc[q], 0.0, 0.0, 0.0};
        for (int f = 0; f < REC_N; ++f) SREC(s, f, n) = v[f];
        const int n1 = (n + 1 < D2D_MAX_WPS) ? n + 1 : D2D_MAX_WPS - 1;
        SREC(s, REC_U0, n) = us[n];
        SREC(s, REC_U1, n) = us[n1];
        SREC(s, REC_IDU, n) = 1.0 / (us[n1] - us[n]);
        // predef_path.py:88-142 per interval n = u_index(u): "first" (u in [us[0], us[1]], B only),
        // "last" (u in [us[-2] - 0.001, us[-1]] or n == nw-1, B only), else the blend.  For n < nw-1
        // u <= us[n+1] <= L, so last <=> u >= last_lo; for n = 0, first <=> u >= us[0].  Hence blend
        // <=> u < T[n] with T[0] = min(us[0], last_lo), T[0 < n < nw-1] = last_lo, T[nw-1] = -inf
        // (also for NaN u, which u_index maps to nw-1).  scn_build's check above keeps last_lo
        // inside interval nw-3.
        const double last_lo = us[nw - 2] - 0.001;
        SREC(s, REC_T, n) = (n == 0) ? (us[0] < last_lo ? us[0] : last_lo)
                                   : (n < nw - 1 ? last_lo : -__builtin_inf());
    }
    for (int k = 0; k < D2D_MAX_CIRCLES; ++k) {
        s.cx[k] = a.cx[k];
        s.cy[k] = a.cy[k];
        s.cr[k] = a.cr[k];
    }
    s.wp_last_x = a.wp_last_x;
    s.wp_last_y = a.wp_last_y;
    s.spawn_xmin = a.spawn_xmin;
    s.spawn_xmax = a.spawn_xmax;
    s.spawn_ymin = a.spawn_ymin;
    s.spawn_ymax = a.spawn_ymax;
    s.spawn_amin = a.spawn_amin;
    s.spawn_amax = a.spawn_amax;
    s.r_uniform = __builtin_nan("");
    if (a.n_circles > 0) {
        bool same = true;
        for (int k = 1; k < a.n_circles; ++k) same = same && (a.cr[k] == a.cr[0]);
        if (same) s.r_uniform = a.cr[0];
    }
    return true;
}
// a / b correctly rounded from y = RN(1/b) (Markstein): q = RN(a*y) is within 1 ulp of a/b, the
// residual a - q*b is exact under fma, and RN(q + r*y) == RN(a/b) for normal operands.  Three
// dependent ops instead of the ~10 of the IEEE division sequence.
__device__ __forceinline__ double div_by_recip(double a, double b, double y) {
    const double q = a * y;
    const double r = fma(-q, b, a);
    return fma(r, y, q);
}
// Correctly rounded sqrt for x = +-0, +inf, NaN or x >= 2^-767: the device library's sequence
// (rsq estimate + Goldschmidt/Newton refinement) without its range-scaling steps, which only act
// below 2^-767.  Squared distances between fp64 points are 0 or far above that.  Checked bitwise
// against sqrt() by d2d_selftest.
__device__ __forceinline__ double sqrt_refine(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = 0.5 * y;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    return fma(d, h, g);
}
__device__ __forceinline__ double sqrt_nz(double x) {
    // +-0 and +inf return themselves (the refinement would give NaN for inf), NaN propagates
    return __builtin_amdgcn_class(x, 0x260) ? x : sqrt_refine(x);
}
// distances: the range-limited sqrt (squared fp64 distances are 0 or >= 2^-767).  The +-0 / inf /
// NaN fix-up is a wave-uniform branch taken only when some lane needs it (a probe exactly on the
// drone's position): one compare per distance instead of a compare and two selects.  The same
// results as sqrt_nz bit for bit (d2d_selftest checks it against sqrt()).
// (the fix-up by selects in every distance measured +2.8 % corridor / +4.2 % small batch,
// profiles/r05/stash/)
__device__ __forceinline__ double sqrt_dist(double x) {
    double g = sqrt_refine(x);
    if (__builtin_expect(__ballot(__builtin_amdgcn_class(x, 0x260)) != 0ull, 0)) {
        asm volatile("" ::: "memory");  // keeps the branch (no if-conversion into selects)
        g = __builtin_amdgcn_class(x, 0x260) ? x : g;
    }
    return g;
}
// max(|r|, t) for finite r and t > 0: one v_max_f64 with the abs modifier (fmax first quiets both
// operands for its NaN rule, two more v_max_f64, and no operand here can be NaN)
__device__ __forceinline__ double max_abs_fin(double r, double t) {
    double m;
    asm("v_max_f64 %0, |%1|, %2" : "=v"(m) : "v"(r), "v"(t));
    return m;
}
// min / max of two non-NaN doubles, one instruction each (fmin / fmax first quiet their operands for
// the NaN rule: two more v_max_f64 per call)
__device__ __forceinline__ double min_fin(double a, double b) {
    double m;
    asm("v_min_f64 %0, %1, %2" : "=v"(m) : "v"(a), "v"(b));
    return m;
}
__device__ __forceinline__ double max_fin(double a, double b) {
    double m;
    asm("v_max_f64 %0, %1, %2" : "=v"(m) : "v"(a), "v"(b));
    return m;
}
// Correctly rounded a / b for normal operands with a normal quotient (no div_scale / div_fixup
// range handling: results for zero / inf / NaN / extreme-exponent operands are unspecified).
// Checked bitwise against '/' by d2d_selftest.
__device__ __forceinline__ double div_normal(double a, double b) {
    double y = __builtin_amdgcn_rcp(b);
    double e = fma(-b, y, 1.0);
    y = fma(y, e, y);
    e = fma(-b, y, 1.0);
    y = fma(y, e, y);
    const double q = a * y;
    const double r = fma(-b, q, a);
    return fma(r, y, q);
}

// ------------------------------------------------------------------------------ scalar helpers
// fmod(a, 2*pi), bit-exact, without ocml's fmod loop (239 cycles dependent latency on gfx950 vs
// ~50 here).  fmod's result a - q*b (q = trunc(a/b)) is exactly representable, so once q is the
// true quotient fma(-q, b, a) is exact; the estimate from a * (1/b) is off by at most one, which the
// sign / range test below detects and corrects.  |a| >= 2^40 (and NaN/inf) falls back to fmod.
__device__ __forceinline__ double fmod_2pi(double a) {
    constexpr double INV = 0.15915494309189535;  // 1/(2*pi), rounded
    if (!(fabs(a) < 1099511627776.0)) return fmod(a, TWO_PI);
    double q = trunc(a * INV);
    double r = fma(-q, TWO_PI, a);
    if (a >= 0.0) {
        const double dq = (r < 0.0) ? -1.0 : ((r >= TWO_PI) ? 1.0 : 0.0);
        if (dq != 0.0) r = fma(-(q + dq), TWO_PI, a);
    } else {
        const double dq = (r > 0.0) ? 1.0 : ((r <= -TWO_PI) ? -1.0 : 0.0);
        if (dq != 0.0) r = fma(-(q + dq), TWO_PI, a);
    }
    return r;
}
// Python/NumPy float modulo by 2*pi (npy_remainder: fmod, then move into the divisor's sign)
__device__ __forceinline__ double pymod_2pi(double a) {
    double m = fmod_2pi(a);
    return (m != 0.0) ? ((m < 0.0) ? m + TWO_PI : m) : 0.0;
}
// transformations.py:6-7
__device__ __forceinline__ double ssa(double a) { return pymod_2pi(a + PI) - PI; }
// drone_2d_env.py:972-978
__device__ __forceinline__ double m1to1(double v, double lo, double hi) { return 2.0 * (v - lo) / (hi - lo) - 1.0; }
__device__ __forceinline__ double invm1to1(double v, double lo, double hi) { return (v + 1.0) * (hi - lo) / 2.0 + lo; }
__device__ __forceinline__ double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
// np.linalg.norm of a 2-vector == sqrt(OpenBLAS ddot) == sqrt(fma(dy, dy, dx*dx))
__device__ __forceinline__ double norm2(double dx, double dy) { return sqrt_dist(fma(dy, dy, dx * dx)); }
// np.sign(x) + (x == 0): 1 for x > 0 and +-0, -1 for x < 0, NaN for NaN (two selects)
__device__ __forceinline__ double sgn_nz(double x) {
    const double s = (x < 0.0) ? -1.0 : 1.0;
    return (x != x) ? x : s;
}
// D2D_EXACT_TRIG (a second build of the library, libdrone2d_hip_exact.so, exact_trig=True in the
// Python facade): every sine / cosine / arctangent the state or the observation depends on is
// d2d_pmath.h's fdlibm restatement, which the CPU oracle's exact build (libd2d_oracle_exact.so)
// uses too, and the bearings take the reference sequence (atan2 -> ssa -> sincos) instead of the
// rotated unit vectors: state and observation are then bit-identical to that oracle's, so a closed
// loop (a policy acting on the observations) stays identical to it, episode for episode
// (tests/test_harness.py).  The default build uses the device library and the cheaper sequences
// (a few ulp apart; DESIGN.md "Arithmetic").
#ifndef D2D_EXACT_TRIG
#define D2D_EXACT_TRIG 0
#endif
__device__ __forceinline__ void sincos_d(double x, double& s, double& c) {
#if D2D_EXACT_TRIG
    d2d_pm_sincos(x, &s, &c);
#else
    sincos(x, &s, &c);
#endif
}
__device__ __forceinline__ double atan2_d(double y, double x) {
#if D2D_EXACT_TRIG
    return d2d_pm_atan2(y, x);
#else
    return atan2(y, x);
#endif
}

// ------------------------------------------------------------------------------ Philox4x32-10
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                       uint32_t k1, uint32_t out[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}
// test-mode spawn draw (drone_2d_env.py:229-232): x, y, theta for (seed, global env id, episode)
// curriculum pool (d2d_cfg.scn_pool): scenario of the episode that starts at this reset
__device__ __forceinline__ int pool_pick(uint64_t seed, uint32_t gid, uint32_t episode, int n_scn) {
    uint32_t o[4];
    philox(gid, episode, 2u, 0u, (uint32_t)seed, (uint32_t)(seed >> 32), o);
    return (int)(o[0] % (uint32_t)n_scn);
}
template <class S>
__device__ __forceinline__ void spawn_draw(const S& s, uint64_t seed, uint32_t gid, uint32_t episode,
                                           double& x, double& y, double& th) {
    uint32_t o[4];
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    philox(gid, episode, 0u, 0u, k0, k1, o);
    const double u0 = u53(o[0], o[1]), u1 = u53(o[2], o[3]);
    philox(gid, episode, 1u, 0u, k0, k1, o);
    const double u2 = u53(o[0], o[1]);
    x = s.spawn_xmin + (s.spawn_xmax - s.spawn_xmin) * u0;
    y = s.spawn_ymin + (s.spawn_ymax - s.spawn_ymin) * u1;
    th = s.spawn_amin + (s.spawn_amax - s.spawn_amin) * u2;
}

// ------------------------------------------------------------------------------ QPMI2D path
// get_u_index (predef_path.py:53-63): first n with u <= us[n+1]; for non-decreasing knots this is
// the number of knots k >= 1 with !(u <= us[k]) (NaN -> n_wps-1, as the Python loop).
// (Counting the sign bits of us[k] - u instead of compares gives the same counts and was measured
// slower in the full kernel.)
template <class S>
__device__ __forceinline__ int u_index(const S& s, double u) {
    uint32_t c = 0;
#pragma unroll
    for (int k = 1; k < D2D_MAX_WPS; ++k) c += !(u <= SUS(s, k)) ? 1u : 0u;
    const int nw1 = s.n_wps - 1;
    return (u != u) ? nw1 : min((int)c, nw1);
}
// the same with the knots read at an opaque offset z (= 0): keeps the table's address space (LDS
// loads for a staged table) while stopping the compiler from keeping the knots in registers
template <class S>
__device__ __forceinline__ int u_index_at(const S& s, double u, int z) {
    uint32_t c = 0;
#pragma unroll
    for (int k = 1; k < D2D_MAX_WPS; ++k) c += !(u <= SUS(s, k + z)) ? 1u : 0u;
    const int nw1 = s.n_wps - 1;
    return (u != u) ? nw1 : min((int)c, nw1);
}
// the same over a lane's knots staged in LDS, knot k at kn[64 k + lane] (conflict-free), read at an
// opaque offset z (= 0) so the compiler keeps them in LDS
__device__ __forceinline__ int u_index_kn(const double* kn, int nw, double u, int z) {
    const int lane = (int)(threadIdx.x & 63) + z;
    uint32_t c = 0;
#pragma unroll
    for (int k = 1; k < D2D_MAX_WPS; ++k) c += !(u <= kn[64 * k + lane]) ? 1u : 0u;
    const int nw1 = nw - 1;
    return (u != u) ? nw1 : min((int)c, nw1);
}
// loop invariants of path_eval (hoisted out of the Brent loop)
struct PathK {
    double us0, last_lo, L;
    int nw;
};
template <class S>
__device__ __forceinline__ PathK path_k(const S& s) {
    const int nw = s.n_wps;
    return PathK{SUS(s, 0), SUS(s, nw - 2) - 0.001, SUS(s, nw - 1), nw};
}
// QPMI2D.__call__ (predef_path.py:88-142), branch-free: both candidate quadratics are evaluated
// and the reference's case analysis picks the result with selects (same arithmetic per case).
// first <=> n == 0 && u >= us[0];  last <=> u in [us[nw-2] - 0.001, L] or n == nw-1, and in every
// first / last case the record's "B" quadratic is the one the reference uses (scn_build).
__device__ __forceinline__ void path_eval_rec(const double r[REC_N], const PathK& K, double u, int n, double& x,
                                              double& y, double& u1_out) {
    // the reference's first / last / blend case analysis as one compare (scn_build, REC_T)
    const bool blend = u < r[REC_T];
    const double uu = u * u;
    const double xB = r[REC_XB + 0] * uu + r[REC_XB + 1] * u + r[REC_XB + 2];
    const double yB = r[REC_XB + 3] * uu + r[REC_XB + 4] * u + r[REC_XB + 5];
    const double xA = r[REC_XA + 0] * uu + r[REC_XA + 1] * u + r[REC_XA + 2];
    const double yA = r[REC_XA + 3] * uu + r[REC_XA + 4] * u + r[REC_XA + 5];
    const double u0 = r[REC_U0], u1 = r[REC_U1], idu = r[REC_IDU];
    const double du = u1 - u0;
    const double mu_r = div_by_recip(u - u0, du, idu);   // (u - u0) / (u1 - u0)
    const double mu_f = div_by_recip(u1 - u, du, idu);   // (u1 - u) / (u1 - u0)
    const double xb = mu_r * xB + mu_f * xA, yb = mu_r * yB + mu_f * yA;
    x = blend ? xb : xB;
    y = blend ? yb : yB;
    u1_out = u1;
}
template <class S>
__device__ __forceinline__ void path_eval_n(const S& s, const PathK& K, double u, int n, double& x, double& y,
                                            double& u1_out) {
    double r[REC_N];
#pragma unroll
    for (int f = 0; f < REC_N; ++f) r[f] = SREC(s, f, n);
    path_eval_rec(r, K, u, n, x, y, u1_out);
}
template <class S>
__device__ __forceinline__ void path_eval(const S& s, const PathK& K, double u, double& x, double& y) {
    double u1;
    path_eval_n(s, K, u, u_index(s, u), x, y, u1);
}
template <class S>
__device__ __forceinline__ void path_eval(const S& s, double u, double& x, double& y) {
    path_eval(s, path_k(s), u, x, y);
}
template <class S>
__device__ __forceinline__ double path_dist_n(const S& s, const PathK& K, double u, int n, double px, double py,
                                              double& u1) {
    double x, y;
    path_eval_n(s, K, u, n, x, y, u1);
    // (sqrt_nz measured slower here than the library sequence: tools/ubench_step.hip)
    return norm2(x - px, y - py);
}
// get_closest_u (predef_path.py:226-248) = scipy fminbound(x1=-10, x2=L+10, xtol=1e-6, maxfun=500),
// restated from scipy 1.15.3 _minimize_scalar_bounded (_optimize.py:2251-2398) probe for probe; the
// golden/parabolic case analysis is evaluated with selects (identical arithmetic per case).
// The search state is explicit so that a search can be suspended and resumed bit-exactly (the
// auto-reset observation cache runs it in slices across steps); xm / tol1 / tol2 are functions of
// the state, recomputed exactly as scipy recomputes them at the end of each iteration.
// Knot-interval tracking: u_index is monotone in u, so a probe u in [a, b] has
// idx(a) <= idx(u) <= idx(b).  The state carries ia = idx(a), ib = idx(b), ixf = idx(xf) and the
// knots ka = us[ia + 1], kxf = us[ixf + 1] (each taken from the record of the probe that set it);
// once the bracket spans at most two intervals (ib <= ia + 1) a probe's index is
// min(ia + !(u <= ka), nw - 1) -- one compare instead of the knot scan.  Exact: it is the same count.
struct Brent {
    double a, b, fulc, ffulc, nfc, fnfc, xf, fx, rat, e;
    double ka, kxf;
    int num, ia, ib, ixf;
};
constexpr double BR_SQRT_EPS = 1.4832396974191326e-08;  // sqrt(2.2e-16)
constexpr double BR_GOLDEN = 0.3819660112501051;        // 0.5*(3.0 - sqrt(5.0))
constexpr double BR_XATOL3 = 1e-6 / 3.0;
constexpr int BT_K_MAX = 48;  // = BT_K (golden-march table steps): a snapshot's num is at most BT_K + 1
template <class S>
__device__ __forceinline__ void brent_init(const S& s, const PathK& K, double px, double py, Brent& B) {
    B.a = 0.0 - 10.0;
    B.b = K.L + 10.0;
    B.fulc = B.a + BR_GOLDEN * (B.b - B.a);
    B.nfc = B.fulc;
    B.xf = B.fulc;
    B.rat = 0.0;
    B.e = 0.0;
    B.ia = u_index(s, B.a);
    B.ib = u_index(s, B.b);
    B.ka = SREC(s, REC_U1, B.ia);
    B.ixf = u_index(s, B.xf);
    B.fx = path_dist_n(s, K, B.xf, B.ixf, px, py, B.kxf);
    B.num = 1;
    B.ffulc = B.fx;
    B.fnfc = B.fx;
}
// scipy's loop condition without maxfun: |xf - xm| > tol2 - (b - a) / 2
__device__ __forceinline__ bool brent_open(const Brent& B) {
    const double xm = 0.5 * (B.a + B.b);
    const double tol1 = BR_SQRT_EPS * fabs(B.xf) + BR_XATOL3;
    const double tol2 = 2.0 * tol1;
    return fabs(B.xf - xm) > (tol2 - 0.5 * (B.b - B.a));
}
__device__ __forceinline__ bool brent_active(const Brent& B) { return brent_open(B) & (B.num < 500); }
// One scipy iteration in its two halves: brent_cand = the candidate probe of the next step (it sets
// B.e and B.rat exactly as scipy's iteration does before the evaluation), brent_update = the decision
// on the evaluated probe.  brent_step = cand + evaluation + update.  (A speculative search built on
// the split -- a second probe per pass, the next step's under the last decision -- was bit-exact but
// slower everywhere it was tried: DESIGN.md "Curriculum".)
struct BrCand {
    double x;
    int ix;
};
template <bool KN, class S>
__device__ __forceinline__ int brent_interval(const S& s, const PathK& K, const Brent& B, double x, double ka,
                                              double* kn);
// KN: the knot scan reads the lane's knots staged in LDS at kn (global-memory tables, closest_u)
template <bool KN = false, class S>
__device__ __forceinline__ BrCand brent_cand(const S& s, const PathK& K, Brent& B, double* kn = nullptr) {
    const double a = B.a, b = B.b, xf = B.xf, fx = B.fx, nfc = B.nfc, fulc = B.fulc;
    // the upper knot of a's interval, for the one-compare interval test: re-read from a staged (LDS)
    // table; carried in the state (B.ka, B.kxf, from the records the probes already read) when the
    // table is read per lane from global memory (ScnR), where that load sat on every step's chain.
    // (Prefetching a's whole record before the candidate is known, or xf's, measured no faster.)
    const double ka = S::RM ? B.ka : SREC(s, REC_U1, B.ia);
    const double xm = 0.5 * (a + b);
    const double tol1 = BR_SQRT_EPS * fabs(xf) + BR_XATOL3;
    const double tol2 = 2.0 * tol1;
    // parabolic candidate (used only when |e| > tol1 and it is acceptable)
    const double r = (xf - nfc) * (fx - B.ffulc);
    double q = (xf - fulc) * (fx - B.fnfc);
    double p = (xf - fulc) * q - (xf - nfc) * r;
    q = 2.0 * (q - r);
    p = (q > 0.0) ? -p : p;
    q = fabs(q);
    const bool par = (fabs(B.e) > tol1) & (fabs(p) < fabs(0.5 * q * B.e)) & (p > q * (a - xf)) & (p < q * (b - xf));
    // only used when `par` holds: then q > 0 and |p / q| < |e| / 2, a normal quotient.  Skipped
    // when no lane of the wave takes the parabolic step (the golden tails of long searches; the
    // division on every step without this branch measured +2 %, profiles/r05/stash/)
    double rat_p = 0.0;
    if (__ballot(par) != 0ull) {
        rat_p = div_normal(p + 0.0, q);
        const double xp = xf + rat_p;
        // tol1 * (np.sign(d) + (d == 0)) for d = xm - xf: a, b and xf are finite (the initial
        // bracket and finite steps), so d is not NaN and the product is -tol1 for d < 0, else +tol1
        const double d = xm - xf;
        rat_p = (((xp - a) < tol2) | ((b - xp) < tol2)) ? ((d < 0.0) ? -tol1 : tol1) : rat_p;
    }
    // golden-section candidate
    const double e_g = (xf >= xm) ? a - xf : b - xf;
    const double rat_g = BR_GOLDEN * e_g;
    B.e = par ? B.rat : e_g;
    const double rat = par ? rat_p : rat_g;
    B.rat = rat;
    // x = xf + (sign(rat) + (rat == 0)) * max(|rat|, tol1).  rat is finite (a, b, xf are, and the
    // parabolic step is taken only when |p/q| < |e|/2), so np.max's NaN rule never applies and the
    // product is exactly -mx for rat < 0 and +mx otherwise
    const double mx = max_abs_fin(rat, tol1);
    // (rat is never -0: e_g = a - xf or b - xf is +0 at worst, the parabolic step is p + 0.0 over
    // |q| or tol1 times a nonzero sign, so copysign gives the same -mx / +mx)
    const double x = xf + copysign(mx, rat);
    return BrCand{x, brent_interval<KN>(s, K, B, x, ka, kn)};
}
// the knot interval of a probe x in [B.a, B.b] (ka = us[B.ia + 1])
template <bool KN, class S>
__device__ __forceinline__ int brent_interval(const S& s, const PathK& K, const Brent& B, double x, double ka,
                                              double* kn) {
    // knot interval of x: one compare once the bracket spans <= 2 intervals (wave-uniform choice).
    // x is always in [a, b], so the choice depends on the bracket alone -- known at the step's start,
    // which takes the branch off the step's dependency chain (a branch on a just-computed condition
    // costs ~50 cycles, on a ready one ~9: tools/ubench_lat.hip; small batch -2.4 %).  Why x is in
    // [a, b]: the loop runs only while b - a > tol2 = 2 tol1; a golden step moves from xf toward the
    // farther end by 0.38 of a distance >= (b - a) / 2 (or by tol1 < (b - a) / 2); an accepted
    // parabolic step either lands at least tol2 inside the bracket or is replaced by a tol1 step from
    // xf toward the midpoint, and max(|rat|, tol1) then moves it by less than tol1 more.  The margins
    // (tol1 >= 3.3e-7) dwarf the roundings.
    const bool fast = B.ib <= B.ia + 1;
    int ix;
    if (__ballot(!fast) == 0ull) {
        ix = min(B.ia + ((x <= ka) ? 0 : 1), K.nw - 1);
    } else {
        // the knot scan re-reads the knots each time (an opaque pointer or offset stops the compiler
        // from keeping all 15 in registers across the loop: the fast path does not need them).  With
        // the table in global memory (ScnR) an opaque offset keeps global loads where the opaque
        // pointer made flat ones (fresh curriculum K1 88.9 -> 85.4 us); for a staged (LDS) table the
        // offset form measured 1.3 % slower at 4 096 envs (profiles/r04/ring/), so the flat loads stay.
        if constexpr (S::RM) {
            int z = 0;
            asm volatile("" : "+v"(z));
            if constexpr (KN) {
                ix = u_index_kn(kn, K.nw, x, z);
            } else {
                ix = u_index_at(s, x, z);
            }
        } else {
            const S* sp = &s;
            asm volatile("" : "+v"(sp));
            ix = u_index(*sp, x);
        }
    }
    return ix;
}
// the decision on probe c (value fu, kx = us[c.ix + 1] from its record); returns le (the probe is not
// worse than xf)
template <class S>
__device__ __forceinline__ bool brent_update(Brent& B, const BrCand& c, double fu, double kx) {
    const double a = B.a, b = B.b, xf = B.xf, fx = B.fx, nfc = B.nfc, fulc = B.fulc;
    const double x = c.x;
    const int ix = c.ix;
    // (num, scipy's maxfun count, is not advanced here: brent_run derives it from its pass count)
    const bool le = fu <= fx;
    const bool c1 = !le & ((fu <= B.fnfc) | (nfc == xf));
    const bool c2 = !le & !c1 & ((fu <= B.ffulc) | (fulc == xf) | (fulc == nfc));
    // a <- (le ? xf : x) when le == (x >= xf), b <- the same value when le != (x >= xf): scipy's
    // four cases (x, xf are finite, so x >= xf and x < xf are complements)
    const bool ge = x >= xf;
    const bool to_a = le == ge;
    const double t = le ? xf : x;
    const int ti = le ? B.ixf : ix;
    B.a = to_a ? t : a;
    B.b = to_a ? b : t;
    B.ia = to_a ? ti : B.ia;
    B.ib = to_a ? B.ib : ti;
    B.ixf = le ? ix : B.ixf;
    if constexpr (S::RM) {  // (the same bookkeeping brtab_build does for its snapshots)
        const double tk = le ? B.kxf : kx;
        B.ka = to_a ? tk : B.ka;
        B.kxf = le ? kx : B.kxf;
    }
    const double nfulc = (le | c1) ? nfc : (c2 ? x : fulc);
    const double nffulc = (le | c1) ? B.fnfc : (c2 ? fu : B.ffulc);
    const double nnfc = le ? xf : (c1 ? x : nfc);
    const double nfnfc = le ? fx : (c1 ? fu : B.fnfc);
    B.fulc = nfulc;
    B.ffulc = nffulc;
    B.nfc = nnfc;
    B.fnfc = nfnfc;
    B.xf = le ? x : xf;
    B.fx = min_fin(fu, fx);  // == le ? fu : fx (le = fu <= fx; equal values are the same number; the
                             // distances are NaN only all together, for a NaN point)
    return le;
}
template <bool KN = false, class S>
__device__ __forceinline__ void brent_step(const S& s, const PathK& K, double px, double py, Brent& B,
                                           double* kn = nullptr BST_ARG) {
#ifdef D2D_BSTAMP
    uint64_t bst_t[5];
#endif
    BST(0, B.xf);
    const bool fast = B.ib <= B.ia + 1;
    const BrCand c = brent_cand<KN>(s, K, B, kn);
    BST(1, c.x);
    BST(2, c.ix);
    // (a per-lane LDS cache of the probe's interval record for global-memory tables measured slower:
    // fresh K1 80.5 vs 77.7 us, profiles/r05/a/ -- some lane of the wave misses on most early steps)
    double kx;
    const double fu = path_dist_n(s, K, c.x, c.ix, px, py, kx);
    BST(3, fu);
    brent_update<S>(B, c, fu, kx);
#ifdef D2D_BSTAMP
    BST(4, B.fx);
    const uint64_t act = __ballot(1);
    if (bst && (int)(threadIdx.x & 63) == __ffsll((unsigned long long)act) - 1) {
        for (int k = 0; k < 5; ++k) bst[k] = bst_t[k];
        bst[5] = 0;
        bst[6] = (uint64_t)(__ballot(!fast) != 0ull);
        bst[7] = (uint64_t)__popcll(act);
    }
#else
    (void)fast;
#endif
}
// scipy's `while` loop (maxfun = 500 included).  A lane takes one step per pass of the wave's loop
// until it is inactive (a finished search stays finished), so at pass `it` an active lane's num is
// its entry num + it; entry nums are at most BT_K + 1 (a golden-march snapshot), so num < 500 holds
// for every active lane while it + BT_K + 1 < 500 and the per-lane count is only tested past that
// (never reached by a search over a finite bracket: the golden steps alone shrink it below xtol in
// ~60 passes).  brent_step does not advance num; B.num stays the entry count.
template <bool KN = false, class S>
__device__ __forceinline__ void brent_run(const S& s, const PathK& K, double px, double py, Brent& B,
                                          double* kn = nullptr) {
    constexpr int IT_FREE = 500 - (BT_K_MAX + 1);
    for (int it = 0;; ++it) {
        bool act = brent_open(B);
        if (__builtin_expect(it >= IT_FREE, 0)) {
            asm volatile("" ::: "memory");  // a scalar branch, not a per-pass compare
            act = act & (B.num + it < 500);
        }
        if (!act) break;
#ifdef D2D_BSTAMP
        uint64_t* bst = nullptr;
        if ((threadIdx.x >> 6) == 2 && blockIdx.x < 1024 && it < 64) bst = d2d_bst + ((size_t)blockIdx.x * 64 + it) * 8;
        brent_step<KN>(s, K, px, py, B, kn, bst);
#else
        brent_step<KN>(s, K, px, py, B, kn);
#endif
    }
}
// (iu: the knot interval of the result, u_index(s, result), tracked by the search)
// kn (global-memory tables only, K1's path wave): LDS for the lane's knots, which the knot scans
// then read instead of global memory (16 x 64 doubles)
template <bool KN = false, class S>
__device__ __forceinline__ double closest_u(const S& s, double px, double py, int& iu, double* kn = nullptr) {
    static_assert(!KN || S::RM, "staged knots / record cache: global-memory tables only");
    const PathK K = path_k(s);
    if constexpr (KN) {
#pragma unroll
        for (int k = 0; k < D2D_MAX_WPS; ++k) kn[64 * k + (threadIdx.x & 63)] = SUS(s, k);
    }
    Brent B;
    brent_init(s, K, px, py, B);
    brent_run<KN>(s, K, px, py, B, kn);
    iu = B.ixf;
    return B.xf;
}

// ------------------------------------------------------------------ Brent golden-march tables
// Two probe sequences of fminbound do not depend on the point at all as long as its decisions are
// "golden step, the new probe is not worse" (after the first step):
//   kind 0 (golden-left):  step 0 worse, then every step better -> converges to u = -10
//                          (points behind the path start; 66 % of the bench's searches)
//   kind 1 (golden-right): every step better                 -> converges to u = L + 10
// In that regime a, b, the probes, e, rat and tol1 are functions of the step number only; the
// distances enter only the decisions.  So for each scenario a forced run (d2d_brtab_kernel, the
// same device arithmetic as brent_step) records per step k: the probe's path point (X, Y) and the
// f-independent operands of the parabolic-acceptance test, plus the whole search state before
// the step (the snapshot).  A search then (closest_u_tab):
//   1. evaluates the distances at the recorded probes and re-checks every decision with its own
//      distances: `par` (the parabolic acceptance test, same operations as brent_step) must be
//      false and `fu <= fx` true -- ~35 instructions per step, no path evaluation, no selects;
//   2. at the first step d whose decision differs (if any), restores the snapshot before step d
//      (its fx / fnfc / ffulc are the distances at recorded probes) and continues with brent_step.
// Both stages perform exactly the operations brent_step performs on the same operands, so the
// result is bit-identical to closest_u for every point (tests/test_gpu_parity.py grid test).
constexpr int BT_K = BT_K_MAX;  // recorded steps per kind (longer marches continue in brent_step)
constexpr int BT_HOT = BT_K + 3;  // probe entries per kind: 0..BT_K, plus zero entries the 3-step
                                  // unrolled check may read past a table's end
struct BtIt {             // probe j (0: the initial point; k + 1: the probe of step k) + step k's operands
    double X, Y;          // path(probe)
    double dxn, dxf;      // xf - nfc, xf - fulc before step k
    double e;             // e before step k if |e| > tol1 (parabolic step tried), else 0 (never accepted)
    double am, bm;        // a - xf, b - xf before step k
    double pad;
};
struct BtSnap {           // search state before step k (the f values are distances at probes j_*)
    double a, b, fulc, nfc, xf, rat, e, ka, kxf;
    int32_t num, ia, ib, ixf;
    int32_t j_fulc, j_nfc, j_xf, pad;
};
struct BtHot {
    BtIt it[2][BT_HOT];   // [kind][probe]
};
static_assert(sizeof(BtIt) == 64, "BtIt size");
struct BrTab {
    BtHot hot;            // first member: staged into LDS as one block
    BtSnap snap[2][BT_K + 1];
    int32_t len[2];       // recorded steps of each kind (the march's length, at most BT_K)
    int32_t pad[2];
};

// forced run of kind `kind` (one thread per scenario and kind; table generation, not on the step path)
template <class SC>
__device__ __forceinline__ void brtab_build(const SC& s, int kind, BrTab& T) {
    const PathK K = path_k(s);
    Brent B;
    B.a = 0.0 - 10.0;
    B.b = K.L + 10.0;
    B.fulc = B.a + BR_GOLDEN * (B.b - B.a);
    B.nfc = B.fulc;
    B.xf = B.fulc;
    B.rat = 0.0;
    B.e = 0.0;
    B.ia = u_index(s, B.a);
    B.ib = u_index(s, B.b);
    B.ka = SREC(s, REC_U1, B.ia);
    B.ixf = u_index(s, B.xf);
    B.num = 1;
    B.fx = B.ffulc = B.fnfc = 0.0;
    BtIt& h0 = T.hot.it[kind][0];
    path_eval_n(s, K, B.xf, B.ixf, h0.X, h0.Y, B.kxf);
    h0.dxn = h0.dxf = h0.e = h0.am = h0.bm = h0.pad = 0.0;
    int jf = 0, jn = 0, jx = 0;  // probe indices of fulc, nfc, xf
    int k = 0;
    for (; k < BT_K && brent_active(B); ++k) {
        BtSnap& S = T.snap[kind][k];
        S = BtSnap{B.a, B.b, B.fulc, B.nfc, B.xf, B.rat, B.e, B.ka, B.kxf, B.num, B.ia, B.ib, B.ixf, jf, jn, jx, 0};
        const double a = B.a, b = B.b, xf = B.xf, nfc = B.nfc, fulc = B.fulc;
        const double xm = 0.5 * (a + b);
        const double tol1 = BR_SQRT_EPS * fabs(xf) + BR_XATOL3;
        BtIt& h = T.hot.it[kind][k + 1];
        h.dxn = xf - nfc;
        h.dxf = xf - fulc;
        h.e = (fabs(B.e) > tol1) ? B.e : 0.0;
        h.am = a - xf;
        h.bm = b - xf;
        h.pad = 0.0;
        // golden step (brent_step with par == false)
        const double e_g = (xf >= xm) ? a - xf : b - xf;
        const double rat = BR_GOLDEN * e_g;
        B.e = e_g;
        B.rat = rat;
        const double mx = max_abs_fin(rat, tol1);
        const double x = xf + ((rat < 0.0) ? -mx : mx);
        const int ix = u_index(s, x);
        double kx;
        path_eval_n(s, K, x, ix, h.X, h.Y, kx);
        B.num += 1;
        // forced decision: kind 0 step 0 is worse (c1 holds: nfc == xf), every other step better
        const bool le = !(kind == 0 && k == 0);
        const bool c1 = !le;
        const bool ge = x >= xf;
        const bool to_a = le == ge;
        const double t = le ? xf : x;
        const int ti = le ? B.ixf : ix;
        const double tk = le ? B.kxf : kx;
        B.a = to_a ? t : a;
        B.b = to_a ? b : t;
        B.ia = to_a ? ti : B.ia;
        B.ka = to_a ? tk : B.ka;
        B.ib = to_a ? B.ib : ti;
        B.ixf = le ? ix : B.ixf;
        B.kxf = le ? kx : B.kxf;
        const int j = k + 1;
        const double nfulc = (le | c1) ? nfc : fulc;
        const int njf = (le | c1) ? jn : jf;
        const double nnfc = le ? xf : (c1 ? x : nfc);
        const int njn = le ? jx : (c1 ? j : jn);
        B.fulc = nfulc;
        B.nfc = nnfc;
        B.xf = le ? x : xf;
        jf = njf;
        jn = njn;
        jx = le ? j : jx;
    }
    T.snap[kind][k] = BtSnap{B.a, B.b, B.fulc, B.nfc, B.xf, B.rat, B.e, B.ka, B.kxf, B.num, B.ia, B.ib, B.ixf,
                             jf, jn, jx, 0};
    T.len[kind] = k;
}

// one recorded step re-checked with this point's distances (the operations of brent_step on the
// same operands): returns the probe's distance; dev <- k if the decision differs.  The window
// (ffulc, fnfc, fx) is the distances at fulc, nfc, xf before the step.
__device__ __forceinline__ double bt_check(const BtIt& h, int k, double px, double py, double ffulc, double fnfc,
                                           double fx, int& dev) {
    const double fu = norm2(h.X - px, h.Y - py);
    const double r = h.dxn * (fx - ffulc);
    double q = h.dxf * (fx - fnfc);
    double p = h.dxf * q - h.dxn * r;
    q = 2.0 * (q - r);
    p = (q > 0.0) ? -p : p;
    q = fabs(q);
    const bool par = (fabs(p) < fabs(0.5 * q * h.e)) & (p > q * h.am) & (p < q * h.bm);
    const bool ok = !par & (fu <= fx);
    dev = min(dev, ok ? BT_HOT : k);
    return fu;
}

// get_closest_u through the golden-march tables (bit-identical to closest_u, see above), in three
// pieces so that two waves can split the re-checks: bt_start (step 0, the kind), bt_verify (steps
// [k0, k1)), bt_finish (resume brent_step at the first differing step).
// `hot` is the scenario's probe table: LDS (address space 3) when LT, else global memory.
template <bool LT>
__device__ __forceinline__ BtIt bt_hot(const BtHot* hot, int kind, int j) {
    if (!LT) return hot->it[kind][j];
    using HL = __attribute__((address_space(3))) const double;
    const HL* q = (const HL*)&hot->it[kind][j];
    return BtIt{q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]};
}
template <bool LT>
__device__ __forceinline__ double bt_dist(const BtHot* hot, int kind, int j, double px, double py) {
    const BtIt h = bt_hot<LT>(hot, kind, j);
    return norm2(h.X - px, h.Y - py);
}
struct BtLane {
    int kind, len, dev;   // dev: first step whose decision differs from the table (len: none)
    double fa, fb, fc;    // distances at fulc, nfc, xf before the next step to check
};
// step 0: the initial point and step 0's probe are the same in both kinds; its decision picks the kind
template <bool LT>
__device__ __forceinline__ BtLane bt_start(const BrTab& T, const BtHot* hot, double px, double py) {
    const double f0 = bt_dist<LT>(hot, 0, 0, px, py);
    const double f1 = bt_dist<LT>(hot, 0, 1, px, py);
    BtLane L;
    L.kind = (f1 <= f0) ? 1 : 0;
    L.len = T.len[L.kind];
    L.dev = L.len;
    L.fa = f0;
    L.fb = L.kind ? f0 : f1;
    L.fc = L.kind ? f1 : f0;
    return L;
}
// the window before step k >= 4 when steps 1 .. k-1 followed the table: fulc, nfc, xf are the probes
// of steps k-3, k-2, k-1 (probe indices k-2, k-1, k).  (Before step 3 of a kind-0 march fulc is
// still the initial point, index 0: the snapshot's j_* indices hold the general case.)
template <bool LT>
__device__ __forceinline__ void bt_window(const BtHot* hot, BtLane& L, int k, double px, double py) {
    L.fa = bt_dist<LT>(hot, L.kind, k - 2, px, py);
    L.fb = bt_dist<LT>(hot, L.kind, k - 1, px, py);
    L.fc = bt_dist<LT>(hot, L.kind, k, px, py);
}
// re-check steps [k0, min(k1, len)) (three per pass: independent distance evaluations, the window
// rotates by name); L.dev <- the first differing step among them
template <bool LT>
__device__ __forceinline__ void bt_verify(const BtHot* hot, BtLane& L, int k0, int k1, double px, double py) {
    double fa = L.fa, fb = L.fb, fc = L.fc;
    int dev = L.dev;
    const int kind = L.kind;
    for (int k = k0; __ballot(k < min(dev, k1)) != 0ull; k += 3) {
        // tables in global memory (a lane's own scenario): a lane that is done loads nothing, so a
        // wave's long marches do not drag every lane's table lines in from HBM
        BtIt ha{}, hb{}, hc{};
        if (LT || k < min(dev, k1)) {
            ha = bt_hot<LT>(hot, kind, k + 1);
            hb = bt_hot<LT>(hot, kind, k + 2);
            hc = bt_hot<LT>(hot, kind, k + 3);
        }
        const double fd = bt_check(ha, k, px, py, fa, fb, fc, dev);
        const double fe = bt_check(hb, k + 1, px, py, fb, fc, fd, dev);
        const double ff = bt_check(hc, k + 2, px, py, fc, fd, fe, dev);
        fa = fd;
        fb = fe;
        fc = ff;
    }
    L.dev = min(dev, L.len);
    L.fa = fa;
    L.fb = fb;
    L.fc = fc;
}
// resume brent_step from the snapshot before step dev (a search that followed the table restores
// its final state, which is inactive unless the march is longer than BT_K); iu = result's interval
template <bool LT, class SC>
__device__ __forceinline__ double bt_finish(const SC& s, const BrTab& T, const BtHot* hot, int kind, int dev,
                                            double px, double py, int& iu) {
    const BtSnap& S = T.snap[kind][dev];
    Brent B;
    B.a = S.a;
    B.b = S.b;
    B.fulc = S.fulc;
    B.nfc = S.nfc;
    B.xf = S.xf;
    B.rat = S.rat;
    B.e = S.e;
    B.ka = S.ka;
    B.kxf = S.kxf;
    B.num = S.num;
    B.ia = S.ia;
    B.ib = S.ib;
    B.ixf = S.ixf;
    if (__ballot(brent_active(B)) != 0ull) {
        const PathK K = path_k(s);
        B.ffulc = bt_dist<LT>(hot, kind, S.j_fulc, px, py);
        B.fnfc = bt_dist<LT>(hot, kind, S.j_nfc, px, py);
        B.fx = bt_dist<LT>(hot, kind, S.j_xf, px, py);
        brent_run(s, K, px, py, B);
    }
    iu = B.ixf;
    return B.xf;
}
template <bool LT, class S>
__device__ __forceinline__ double closest_u_tab(const S& s, const BrTab& T, const BtHot* hot, double px,
                                                double py, int& iu) {
    BtLane L = bt_start<LT>(T, hot, px, py);
    bt_verify<LT>(hot, L, 1, BT_K, px, py);
    return bt_finish<LT>(s, T, hot, L.kind, L.dev, px, py, iu);
}
// split point of the two-wave re-check: the first wave checks steps [1, bt_split), the second
// [bt_split, len) (from its own window, bt_window)
__device__ __forceinline__ int bt_split(const BrTab& T) { return max(4, (T.len[0] + 3) / 2); }
// three-way split: part p in {0, 1, 2} checks steps [bt_third(p), bt_third(p + 1)) (bt_third(0) = 1,
// bt_third(3) = BT_K), as the fill kernel splits it
__device__ __forceinline__ int bt_third(const BrTab& T, int p) {
    const int third = (T.len[0] + 2) / 3;
    return p == 0 ? 1 : (p >= 3 ? BT_K : 1 + p * third);
}
// the window before step k0 for a search that followed the table so far, from the snapshot's probe
// indices (valid for every k0, also before step 4 of a kind-0 march)
template <bool LT>
__device__ __forceinline__ void bt_window_snap(const BrTab& T, const BtHot* hot, BtLane& L, int k0, double px,
                                               double py) {
    const BtSnap& W = T.snap[L.kind][k0];
    L.fa = bt_dist<LT>(hot, L.kind, W.j_fulc, px, py);
    L.fb = bt_dist<LT>(hot, L.kind, W.j_nfc, px, py);
    L.fc = bt_dist<LT>(hot, L.kind, W.j_xf, px, py);
}

// ------------------------------------------------------------------------------ bodies / physics
// One cpSpaceStep(1/60) of the Drone.py body/joint configuration, split in
// two stages so that a caller can retire the positions before the Gauss-Seidel sweep:
//   phys_positions   forces on the frame (drone_2d_env.py:403-404), cpBodyUpdatePosition of the
//                    3 bodies, frame-box vs circle contact (the sticky begin() flag, :17-19)
//   phys_velocities  PivotJoint preStep (K^-1, bias = -delta/dt), cpBodyUpdateVelocity, cached
//                    impulses (dt_coef = 1; after a reset jAcc = 0 so dt_coef = 0 is identical),
//                    10 Gauss-Seidel sweeps over the joints in space.add order.
// With JBUF = true the per-joint (K^-1, bias) live in a per-lane LDS buffer (`jb[f * stride]`,
// 6 x JB_PER_JOINT doubles) and are re-read every sweep (volatile): that keeps the sweep at ~90 VGPRs.
struct Body {
    double px, py, a, vx, vy, w;
};

constexpr double M_F = 0.2, M_M = 0.4;   // drone_2d_env.py:233 -> Drone.py:19,36,50

// cpMomentForPoly(m, cpBoxShapeNew2 verts) in Chipmunk's evaluation order
__host__ __device__ constexpr double moment_box(double m, double w, double h) {
    double hw = w / 2.0, hh = h / 2.0;
    double vx[4] = {hw, hw, -hw, -hw}, vy[4] = {-hh, hh, hh, -hh};
    double s1 = 0.0, s2 = 0.0;
    for (int i = 0; i < 4; ++i) {
        double v1x = vx[i] + 0.0, v1y = vy[i] + 0.0;
        double v2x = vx[(i + 1) % 4] + 0.0, v2y = vy[(i + 1) % 4] + 0.0;
        double aa = v2x * v1y - v2y * v1x;
        double bb = (v1x * v1x + v1y * v1y) + (v1x * v2x + v1y * v2y) + (v2x * v2x + v2y * v2y);
        s1 += aa * bb;
        s2 += aa;
    }
    return (m * s1) / (6.0 * s2);
}
constexpr double MI_F = 1.0 / M_F, MI_M = 1.0 / M_M;
constexpr double II_F = 1.0 / moment_box(M_F, 100.0, 10.0);
constexpr double II_M = 1.0 / moment_box(M_M, 20.0, 20.0);

// Joint anchors (Drone.py:61-95): motor side JA = (-7, 0, 7) for both motors, frame side JB.
// r = R(theta) * (a, 0) = (c*a + (-s)*0, s*a + c*0) == (c*a, s*a) (adding a signed zero never
// changes the value), and c*(-a) == -(c*a) bitwise, so each body needs only its c*|a|, s*|a|.
struct Arms {
    double m7c[2], m7s[2];          // motor (left, right): c*7, s*7
    double f47c, f47s, f40c, f40s, f33c, f33s;  // frame: c*47, s*47, c*40, s*40, c*33, s*33
};
__device__ __forceinline__ void arm(const Arms& A, int k, double& r1x, double& r1y, double& r2x, double& r2y) {
    const int m = k < 3 ? 0 : 1;
    const int q = k % 3;  // JA = -7, 0, 7
    r1x = (q == 0) ? -A.m7c[m] : ((q == 1) ? 0.0 : A.m7c[m]);
    r1y = (q == 0) ? -A.m7s[m] : ((q == 1) ? 0.0 : A.m7s[m]);
    // JB = -47, -40, -33, 33, 40, 47
    const double c = (k == 0 || k == 5) ? A.f47c : ((k == 1 || k == 4) ? A.f40c : A.f33c);
    const double s = (k == 0 || k == 5) ? A.f47s : ((k == 1 || k == 4) ? A.f40s : A.f33s);
    r2x = (k < 3) ? -c : c;
    r2y = (k < 3) ? -s : s;
}

// the same arms re-read from an LDS copy (JBUF mode: keeps the 14 values out of registers across the
// 10-sweep loop); field order of Arms: m7c[2], m7s[2], f47c, f47s, f40c, f40s, f33c, f33s
constexpr int ARMS_N = 10;
__device__ __forceinline__ void arms_store(const Arms& A, double* ab, int stride) {
    const double v[ARMS_N] = {A.m7c[0], A.m7c[1], A.m7s[0], A.m7s[1], A.f47c, A.f47s,
                              A.f40c, A.f40s, A.f33c, A.f33s};
#pragma unroll
    for (int q = 0; q < 10; ++q) ab[q * stride] = v[q];
}
__device__ __forceinline__ void arm_lds(const double* ab, int stride, int k, double& r1x, double& r1y, double& r2x,
                                        double& r2y) {
    using LdsD = __attribute__((address_space(3))) double;
    const volatile LdsD* v = (const volatile LdsD*)ab;
    const int m = k < 3 ? 0 : 1;
    const int q = k % 3;
    const double mc = (q == 1) ? 0.0 : v[(0 + m) * stride], ms = (q == 1) ? 0.0 : v[(2 + m) * stride];
    r1x = (q == 0) ? -mc : ((q == 1) ? 0.0 : mc);
    r1y = (q == 0) ? -ms : ((q == 1) ? 0.0 : ms);
    const int f = (k == 0 || k == 5) ? 4 : ((k == 1 || k == 4) ? 6 : 8);
    const double c = v[f * stride], sn = v[(f + 1) * stride];
    r2x = (k < 3) ? -c : c;
    r2y = (k < 3) ? -sn : sn;
}

// The Chipmunk arithmetic (this stage and phys_velocities) is contracted: every a + b * c of
// cpBodyUpdatePosition / UpdateVelocity, the PivotJoint preStep and applyImpulse is one fma, in the
// operand order oracle/d2d_oracle.c spells out with C fma() (the physics is parity-unpinned, SURVEY.md
// §8c; the unfused Python restatement tests/golden/ref_shims.py stays within the state tolerance).
__device__ __forceinline__ void advance_position(Body& b) {
    b.px = fma(b.vx + 0.0, DT, b.px);
    b.py = fma(b.vy + 0.0, DT, b.py);
    b.a = fma(b.w + 0.0, DT, b.a);
}
template <class S>
__device__ __forceinline__ bool frame_hits(const S& s, const Body& F, double cs, double sn) {
    bool hit = false;
    for (int k = 0; k < s.n_circles; ++k) {
        const double dx = s.cx[k] - F.px, dy = s.cy[k] - F.py;
        {
            // skip the circle for the whole wave when it is out of every lane's reach: every point of
            // the box is within sqrt(50^2 + 5^2) = 50.25 of its center, so a center offset of at
            // least r + 51.25 on either axis puts the circle beyond r of the box: the exact test
            // below would say "no contact" for this lane.  Steady state: ~8 % of the (wave, circle)
            // pairs of corridor, ~5 % of S_corridor's, have a lane in reach.
            const double reach = s.cr[k] + 51.25;
            const bool near = (fabs(dx) < reach) & (fabs(dy) < reach);
            if (__ballot(near) == 0ull) continue;
        }
        const double lx = dx * cs + dy * sn;
        const double ly = -dx * sn + dy * cs;
        // clamp by max / min: equal to clipd for every input (a NaN lx or ly gives a NaN e: no hit)
        const double ex = lx - fmin(fmax(lx, -FRAME_HX), FRAME_HX), ey = ly - fmin(fmax(ly, -FRAME_HY), FRAME_HY);
        const double r = s.cr[k];
        hit |= (ex * ex + ey * ey <= r * r);
    }
    return hit;
}
template <class S>
__device__ __forceinline__ bool phys_positions(const S& s, Body B[3], double fL, double fR, double cs[3],
                                               double sn[3], double& fx, double& fy, double& tq) {
    // forces on the frame at local (-40,0) then (40,0): cpBodyApplyForceAtLocalPoint
    double c0, s0;
    sincos_d(B[0].a, s0, c0);
    {
        const double tx = B[0].px - (0.0 * c0 - 0.0 * s0), ty = B[0].py - (0.0 * s0 + 0.0 * c0);
        const double cgx = c0 * 0.0 + (-s0) * 0.0 + tx, cgy = s0 * 0.0 + c0 * 0.0 + ty;
        double fwx = c0 * 0.0 + (-s0) * fL, fwy = s0 * 0.0 + c0 * fL;
        double rx = (c0 * -DRONE_R + (-s0) * 0.0 + tx) - cgx, ry = (s0 * -DRONE_R + c0 * 0.0 + ty) - cgy;
        fx = 0.0 + fwx;
        fy = 0.0 + fwy;
        tq = 0.0 + (rx * fwy - ry * fwx);
        fwx = c0 * 0.0 + (-s0) * fR;
        fwy = s0 * 0.0 + c0 * fR;
        rx = (c0 * DRONE_R + (-s0) * 0.0 + tx) - cgx;
        ry = (s0 * DRONE_R + c0 * 0.0 + ty) - cgy;
        fx = fx + fwx;
        fy = fy + fwy;
        tq += rx * fwy - ry * fwx;
    }
    // 1. cpBodyUpdatePosition (v_bias = 0)
#pragma unroll
    for (int i = 0; i < 3; ++i) advance_position(B[i]);
    sincos_d(B[0].a, sn[0], cs[0]);
    // the motors' rotations (cpBodySetAngle -> cos, sin) from the frame's: the pivot triples keep
    // d = angle - frame angle tiny, so sin / cos(frame + d) by the addition formula with d's series
    // (truncation < 1e-20 for |d| < 1e-2; a few ulp from sincos); larger d calls sincos
#pragma unroll
    for (int i = 1; i < 3; ++i) {
        const double d = B[i].a - B[0].a;
        if (!D2D_EXACT_TRIG && fabs(d) < 1e-2) {
            const double d2 = d * d;
            const double sd = d * fma(d2, fma(d2, fma(d2, -1.0 / 5040.0, 1.0 / 120.0), -1.0 / 6.0), 1.0);
            const double cdm1 = d2 * fma(d2, fma(d2, fma(d2, 1.0 / 40320.0, -1.0 / 720.0), 1.0 / 24.0), -0.5);
            sn[i] = fma(sn[0], cdm1, fma(cs[0], sd, sn[0]));   // sin0 * cos d + cos0 * sin d
            cs[i] = fma(cs[0], cdm1, fma(-sn[0], sd, cs[0]));  // cos0 * cos d - sin0 * sin d
        } else {
            sincos_d(B[i].a, sn[i], cs[i]);
        }
    }
    // 2. collision: CircleToPoly(circle, frame box) contact iff dist(center, box) <= r
    return frame_hits(s, B[0], cs[0], sn[0]);
}
// The frame's post-step position and contact flag from its pre-step state alone (forces only act
// on velocities): lets the observation waves start without waiting for the physics wave.
template <class S>
__device__ __forceinline__ bool frame_advance(const S& s, Body& F) {
    advance_position(F);
    double sn, cs;
    sincos_d(F.a, sn, cs);
    return frame_hits(s, F, cs, sn);
}

__device__ __forceinline__ Arms make_arms(const double cs[3], const double sn[3]) {
    Arms A;
    A.m7c[0] = cs[1] * 7.0; A.m7s[0] = sn[1] * 7.0;
    A.m7c[1] = cs[2] * 7.0; A.m7s[1] = sn[2] * 7.0;
    A.f47c = cs[0] * 47.0; A.f47s = sn[0] * 47.0;
    A.f40c = cs[0] * 40.0; A.f40s = sn[0] * 40.0;
    A.f33c = cs[0] * 33.0; A.f33s = sn[0] * 33.0;
    return A;
}

// stage 2.  pos = {frame px, py, left px, py, right px, py} (post position update); vel[9] =
// (vx, vy, w) of frame, left, right; j[12] the accumulated pivot impulses.
constexpr int JB_PER_JOINT = 5;  // K^-1 (a, b = c, d) + bias (x, y)
template <bool JBUF>
__device__ __forceinline__ void phys_velocities(const Arms& A, const double pos[6], double damping_dt, double fx,
                                                double fy, double tq, double vel[9], double j[12], double* jb,
                                                int stride, double* ab = nullptr) {
    if (JBUF) arms_store(A, ab, stride);
    const double bias_coef = -(1.0 - 0.0) / DT;  // error_bias = 0 -> bias_coef(0, dt) = 1 - 0^dt = 1
    double kk[JBUF ? 1 : 6][5];
    // preStep
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int m = k < 3 ? 1 : 2;
        double r1x, r1y, r2x, r2y;
        arm(A, k, r1x, r1y, r2x, r2y);
        const double m_sum = MI_M + MI_F;
        // k_mat: K = m_sum I + I_a^-1 [r1y^2, -r1x r1y; ., r1x^2] + I_F^-1 [...r2...]; k12 == k21
        double k11 = fma(r1y * r1y, II_M, m_sum), k22 = fma(r1x * r1x, II_M, m_sum);
        double k12 = fma(-r1x * r1y, II_M, 0.0);
        k11 = fma(r2y * r2y, II_F, k11);
        k12 = fma(-r2x * r2y, II_F, k12);
        k22 = fma(r2x * r2x, II_F, k22);
        const double det = fma(k11, k22, -(k12 * k12));
        const double det_inv = 1.0 / det;
        const double dx = (pos[0] + r2x) - (pos[2 * m] + r1x);
        const double dy = (pos[1] + r2y) - (pos[2 * m + 1] + r1y);
        // K^-1 = [[k22, -k12], [-k21, k11]] * det_inv; k12 and k21 are the same sums, so the two
        // off-diagonal entries are bitwise equal and one is kept
        const double v[5] = {k22 * det_inv, -k12 * det_inv, k11 * det_inv, dx * bias_coef, dy * bias_coef};
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            if (JBUF) jb[(JB_PER_JOINT * k + q) * stride] = v[q];
            else kk[JBUF ? 0 : k][q] = v[q];
        }
    }
    // cpBodyUpdateVelocity: gravity (0, -1000), damping^dt, forces on the frame only
    vel[0] = fma(vel[0], damping_dt, (0.0 + fx * MI_F) * DT);
    vel[1] = fma(vel[1], damping_dt, fma(fy, MI_F, GRAV_Y) * DT);
    vel[2] = fma(vel[2], damping_dt, tq * II_F * DT);
#pragma unroll
    for (int b = 1; b < 3; ++b) {
        vel[3 * b + 0] = fma(vel[3 * b + 0], damping_dt, (0.0 + 0.0 * MI_M) * DT);
        vel[3 * b + 1] = fma(vel[3 * b + 1], damping_dt, fma(0.0, MI_M, GRAV_Y) * DT);
        vel[3 * b + 2] = fma(vel[3 * b + 2], damping_dt, 0.0 * II_M * DT);
    }
    // applyCachedImpulse with dt_coef = 1
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int m = k < 3 ? 1 : 2;
        double r1x, r1y, r2x, r2y;
        arm(A, k, r1x, r1y, r2x, r2y);
        const double jx = j[2 * k] * 1.0, jy = j[2 * k + 1] * 1.0;
        vel[3 * m + 0] = fma(-jx, MI_M, vel[3 * m + 0]);
        vel[3 * m + 1] = fma(-jy, MI_M, vel[3 * m + 1]);
        vel[3 * m + 2] = fma(II_M, fma(r1x, -jy, -(r1y * (-jx))), vel[3 * m + 2]);
        vel[0] = fma(jx, MI_F, vel[0]);
        vel[1] = fma(jy, MI_F, vel[1]);
        vel[2] = fma(II_F, fma(r2x, jy, -(r2y * jx)), vel[2]);
    }
    // 10 sequential-impulse sweeps (Space.iterations default)
#pragma unroll 1  // (unrolled twice: 28 B of spills, no gain)
    for (int it = 0; it < 10; ++it) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int m = k < 3 ? 1 : 2;
            double r1x, r1y, r2x, r2y;
            if (JBUF) arm_lds(ab, stride, k, r1x, r1y, r2x, r2y);
            else arm(A, k, r1x, r1y, r2x, r2y);
            double ka, kb, kd, bx, by;
            if (JBUF) {
                // an explicit LDS (address_space 3) pointer: generic volatile loads would become flat
                // loads with one 64-bit address per slot
                using LdsD = __attribute__((address_space(3))) double;
                const volatile LdsD* kv = (const volatile LdsD*)jb;
                ka = kv[(JB_PER_JOINT * k + 0) * stride]; kb = kv[(JB_PER_JOINT * k + 1) * stride];
                kd = kv[(JB_PER_JOINT * k + 2) * stride];
                bx = kv[(JB_PER_JOINT * k + 3) * stride]; by = kv[(JB_PER_JOINT * k + 4) * stride];
            } else {
                const int kq = JBUF ? 0 : k;
                ka = kk[kq][0]; kb = kk[kq][1]; kd = kk[kq][2]; bx = kk[kq][3]; by = kk[kq][4];
            }
            const double kc = kb;
            // the middle pivots (k = 1, 4) sit at the motor's centre: r1 = (+0, +0), so the motor's
            // perp(r1) * w terms and its angular impulse are signed zeros.  Adding a signed zero
            // leaves a velocity unchanged unless it is -0, and velocities are never -0 here (the
            // gravity / force update adds +0 or a nonzero term, sums of nonzero terms round to +0,
            // never -0); they are dropped for finite states
            const bool za = (k % 3 == 1);
            const double v1x = za ? vel[3 * m + 0] : fma(-r1y, vel[3 * m + 2], vel[3 * m + 0]);
            const double v1y = za ? vel[3 * m + 1] : fma(r1x, vel[3 * m + 2], vel[3 * m + 1]);
            const double v2x = fma(-r2y, vel[2], vel[0]), v2y = fma(r2x, vel[2], vel[1]);
            const double ux = bx - (v2x - v1x), uy = by - (v2y - v1y);
            const double jx = fma(ux, ka, uy * kb);
            const double jy = fma(ux, kc, uy * kd);
            // jAcc += j.  Chipmunk clamps the sum to max_force * dt and applies the difference
            // jAcc_new - jAcc_old; max_force = inf makes the clamp the identity, so that difference is
            // j up to the rounding of the round trip, and j itself is applied (the oracle likewise)
            j[2 * k] = j[2 * k] + jx;
            j[2 * k + 1] = j[2 * k + 1] + jy;
            vel[3 * m + 0] = fma(-jx, MI_M, vel[3 * m + 0]);
            vel[3 * m + 1] = fma(-jy, MI_M, vel[3 * m + 1]);
            if (!za) vel[3 * m + 2] = fma(II_M, fma(r1x, -jy, -(r1y * (-jx))), vel[3 * m + 2]);
            vel[0] = fma(jx, MI_F, vel[0]);
            vel[1] = fma(jy, MI_F, vel[1]);
            vel[2] = fma(II_F, fma(r2x, jy, -(r2y * jx)), vel[2]);
        }
    }
}

// whole step, registers only (reference / diagnostics)
template <class S>
__device__ __forceinline__ bool space_step(const S& s, double damping_dt, Body B[3], double j[12], double fL,
                                           double fR) {
    double cs[3], sn[3], fx, fy, tq;
    const bool hit = phys_positions(s, B, fL, fR, cs, sn, fx, fy, tq);
    const Arms A = make_arms(cs, sn);
    const double pos[6] = {B[0].px, B[0].py, B[1].px, B[1].py, B[2].px, B[2].py};
    double vel[9] = {B[0].vx, B[0].vy, B[0].w, B[1].vx, B[1].vy, B[1].w, B[2].vx, B[2].vy, B[2].w};
    phys_velocities<false>(A, pos, damping_dt, fx, fy, tq, vel, j, nullptr, 0);
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        B[b].vx = vel[3 * b];
        B[b].vy = vel[3 * b + 1];
        B[b].w = vel[3 * b + 2];
    }
    return hit;
}

// ------------------------------------------------------------------------------ observation roles
// sensor role: obs[0..18] of get_observation (drone_2d_env.py:633-727) for frame state F.
// k = 3 nearest circles by min over the UNROTATED frame vertices (+-50, +-5) of |v+p-c| - r;
// sqrt is monotone and correctly rounded, so sqrt(min d^2) - r == min(sqrt(d^2) - r) bitwise.
// Split in the velocity-dependent entries (0, 1, 2, 17, 18: need the joint sweep's output) and the
// position-dependent ones (3..16: known right after the position update).
//
// Bearing observations.  The reference turns a direction vector (x, y) into an angle, subtracts
// the frame angle, wraps it (ssa) and stores its sin / cos (obs 9-16, 17-18, 23-26).  For a
// nonzero finite vector that is the unit vector rotated by -al; rel_dir computes it with one sqrt
// and one division instead of atan2 + fmod + sincos (~200 fp64 instructions each).  It differs from
// the reference sequence by a few ulp (|diff| <~ 1e-15 before the float32 rounding of the
// observation); zero / tiny / non-finite vectors, where atan2's signed-zero cases decide, take the
// reference sequence itself.  `ref` is that sequence (called only on the rare fallback lanes).
template <typename Ref>
__device__ __forceinline__ void rel_dir(double y, double x, double sa, double ca, double& s, double& c,
                                        const Ref& ref) {
    const double r2 = fma(y, y, x * x);
    if (!D2D_EXACT_TRIG && (r2 > 1e-200) & (r2 < 1e300)) {
        const double ir = 1.0 / sqrt_nz(r2);
        const double ux = x * ir, uy = y * ir;
        s = uy * ca - ux * sa;  // sin(phi - al)
        c = ux * ca + uy * sa;  // cos(phi - al)
    } else {
        ref(s, c);
    }
}
// velocity part of obs (0-2, 17-18) for frame state F; sa, ca = sin / cos of F.a
__device__ __forceinline__ void sensor_vel(const Body& F, double sa, double ca, double o[19]) {
    o[0] = m1to1(F.vx, -VEL_MAX, VEL_MAX);
    o[1] = m1to1(F.vy, -VEL_MAX, VEL_MAX);
    o[2] = clipd(F.w / 11.7, -1.0, 1.0);
    rel_dir(F.vy, F.vx, sa, ca, o[17], o[18], [&](double& s, double& c) {
        const double vab = ssa(atan2_d(F.vy, F.vx) - F.a);
        sincos_d(vab, s, c);
    });
}
__device__ __forceinline__ void sensor_vel(const Body& F, double o[19]) {
    double sa, ca;
    sincos_d(F.a, sa, ca);
    sensor_vel(F, sa, ca, o);
}
template <class S>
__device__ __forceinline__ void sensor_pos(const d2d_cfg& cfg, const S& s, double x, double y, double al,
                                           double o[19]) {
    const double W = cfg.screen_w, H = cfg.screen_h;
    o[3] = al / PI;
    o[4] = m1to1(s.wp_last_x - x, 0.0, W);
    o[5] = m1to1(s.wp_last_y - y, 0.0, H);
    o[6] = m1to1(x, 0.0, W);
    o[7] = m1to1(y, 0.0, H);
    double bd0 = __builtin_inf(), bd1 = __builtin_inf(), bd2 = __builtin_inf();
    int bi0 = -1, bi1 = -1, bi2 = -1;
    const int nc = s.n_circles;
    bool full = true;
    if (s.r_uniform == s.r_uniform) {
        // every circle has radius r: d = sqrt(q) - r is non-decreasing in the squared distance q,
        // so the stable top-3 by d is the stable top-3 by q unless two of the candidates round to
        // the same d (then the reference's index order among them can differ from q's order).
        // Keep the top 4 by q, take the 4 square roots, and fall back to the reference loop below
        // on any equal d among them -- otherwise every circle outside has d >= d4 > d3.
        const double r = s.r_uniform;
        double q0 = __builtin_inf(), q1 = __builtin_inf(), q2 = __builtin_inf(), q3 = __builtin_inf();
        int i0 = -1, i1 = -1, i2 = -1, i3 = -1;
        for (int i = 0; i < nc; ++i) {
            const double cx = s.cx[i], cy = s.cy[i];
            const double ax = (50.0 + x) - cx, bxx = (-50.0 + x) - cx;
            const double ay = (-5.0 + y) - cy, byy = (5.0 + y) - cy;
            const double mx = fmin(fabs(ax), fabs(bxx)), my = fmin(fabs(ay), fabs(byy));
            const double q = mx * mx + my * my;
            const bool l3 = (i3 < 0) || q < q3;
            // a circle no lane's top 4 takes changes nothing below (every l is false): skip the
            // insertion for the whole wave (most circles once the top 4 hold near ones)
            if (__ballot(l3) == 0ull) continue;
            const bool l0 = (i0 < 0) || q < q0, l1 = (i1 < 0) || q < q1, l2 = (i2 < 0) || q < q2;
            // the indices by the stable insertion's selects; the sorted keys by min / max (the
            // same values: inserting q into q0 <= q1 <= q2 <= q3 gives min(q_k, max(q_k-1, q)) in
            // slot k, empty slots hold +inf; one fp64 op per slot instead of two 32-bit selects per
            // nesting level -- a NaN q only arises for a NaN position, whose result the fallback
            // below recomputes, so the NaN-free min / max apply)
            i3 = l2 ? i2 : (l3 ? i : i3);
            i2 = l1 ? i1 : (l2 ? i : i2);
            i1 = l0 ? i0 : (l1 ? i : i1);
            i0 = l0 ? i : i0;
            q3 = min_fin(q3, max_fin(q2, q));
            q2 = min_fin(q2, max_fin(q1, q));
            q1 = min_fin(q1, max_fin(q0, q));
            q0 = min_fin(q0, q);
        }
        const double d0 = sqrt_dist(q0) - r, d1 = sqrt_dist(q1) - r, d2 = sqrt_dist(q2) - r,
                     d3 = sqrt_dist(q3) - r;
        const bool tie = ((i1 >= 0) & (d1 == d0)) | ((i2 >= 0) & (d2 == d1)) | ((i3 >= 0) & (d3 == d2)) |
                         (x != x) | (y != y);
        full = tie;
        bd0 = i0 >= 0 ? d0 : bd0;
        bd1 = i1 >= 0 ? d1 : bd1;
        bd2 = i2 >= 0 ? d2 : bd2;
        bi0 = i0;
        bi1 = i1;
        bi2 = i2;
    }
    if (full) {
        bd0 = bd1 = bd2 = __builtin_inf();
        bi0 = bi1 = bi2 = -1;
    }
    for (int i = 0; i < (full ? nc : 0); ++i) {
        const double cx = s.cx[i], cy = s.cy[i];
        const double ax = (50.0 + x) - cx, bxx = (-50.0 + x) - cx;
        const double ay = (-5.0 + y) - cy, byy = (5.0 + y) - cy;
        // min over the vertices (±50, ±5) of RN(dx² + dy²) == RN(min dx² + min dy²): squaring and
        // rounding are monotone, so the x and y parts minimise independently (bit-identical to
        // the four sums; NaN coordinates give NaN either way)
        const double mx = fmin(fabs(ax), fabs(bxx)), my = fmin(fabs(ay), fabs(byy));
        const double q = mx * mx + my * my;
        const double d = sqrt_dist(q) - s.cr[i];
        // stable ascending insertion into the top-3 (equal keys keep index order)
        const bool l0 = (bi0 < 0) || d < bd0, l1 = (bi1 < 0) || d < bd1, l2 = (bi2 < 0) || d < bd2;
        bd2 = l1 ? bd1 : (l2 ? d : bd2);
        bi2 = l1 ? bi1 : (l2 ? i : bi2);
        bd1 = l0 ? bd0 : (l1 ? d : bd1);
        bi1 = l0 ? bi0 : (l1 ? i : bi1);
        bd0 = l0 ? d : bd0;
        bi0 = l0 ? i : bi0;
    }
    const double diag = sqrt(W * W + H * H);
    const double bd[3] = {bd0, bd1, bd2};
    const int bi[3] = {bi0, bi1, bi2};
    double sal, cal;
    sincos_d(al, sal, cal);
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
        const int idx = bi[jj] < 0 ? 0 : bi[jj];
        const double dy = y - s.cy[idx], dx = x - s.cx[idx];
        double sa, ca;
        // ssa(atan2(dy, dx) - al - pi): the rotated unit vector, negated
        rel_dir(dy, dx, sal, cal, sa, ca, [&](double& rs, double& rc) {
            const double ang = ssa(atan2_d(dy, dx) - al - PI);
            sincos_d(ang, rs, rc);
            rs = -rs;
            rc = -rc;
        });
        sa = -sa;
        ca = -ca;
        const bool have = bi[jj] >= 0;
        o[8 + 3 * jj] = have ? m1to1(bd[jj], 0.0, diag) : 1.0;
        o[9 + 3 * jj] = have ? sa : 0.0;
        o[10 + 3 * jj] = have ? ca : 0.0;
    }
}
template <class S>
__device__ __forceinline__ void sensor_obs(const d2d_cfg& cfg, const S& s, const Body& F, double o[19]) {
    sensor_vel(F, o);
    sensor_pos(cfg, s, F.px, F.py, F.a, o);
}

// path role: obs[19..26] (drone_2d_env.py:729-763).  get_closest_u is evaluated once (the
// reference calls it twice with identical input, predef_path.py:255 and :261).  Updates the
// sticky LA lock in `flags`; returns the closest point (cpx, cpy) for the path-adherence reward.
// the part after the closest-point search, for a given u
// (iu: u's knot interval if known, else -1)
template <class S>
__device__ __forceinline__ void path_obs_u(const d2d_cfg& cfg, const S& s, double x, double y, double al,
                                           double u, uint32_t& flags, double o[8], int iu = -1) {
    const double W = cfg.screen_w, H = cfg.screen_h;
    double cpx, cpy, u1;
    path_eval_n(s, path_k(s), u, (iu >= 0) ? iu : u_index(s, u), cpx, cpy, u1);
    const double L = SUS(s, s.n_wps - 1);
    const double ula = (u + cfg.lookahead > L) ? L : u + cfg.lookahead;
    double lax, lay;
    path_eval(s, ula, lax, lay);
    if (fabs(lax - s.wp_last_x) < 10.0 && fabs(lay - s.wp_last_y) < 10.0) flags |= D2D_FLAG_LA_LOCK;
    const bool lock = (flags & D2D_FLAG_LA_LOCK) != 0;
    lax = lock ? s.wp_last_x : lax;
    lay = lock ? s.wp_last_y : lay;
    o[0] = m1to1(cpx, 0.0, W);
    o[1] = m1to1(cpy, 0.0, H);
    o[2] = m1to1(lax, 0.0, W);
    o[3] = m1to1(lay, 0.0, H);
    // ssa(atan2(R_w_b(alpha) d) - alpha): R_w_b rotates by +alpha, so this is the world bearing of
    // d itself (rel_dir with the identity rotation); the reference sequence on fallback lanes:
    // np.matmul(R_w_b(alpha), d): row r = fma(R[r][0], d0, R[r][1] * d1)
    const auto ref = [&](double dx, double dy, double& rs, double& rc) {
        double sa, ca;
        sincos_d(al, sa, ca);
        const double bx = fma(ca, dx, (-sa) * dy), by = fma(sa, dx, ca * dy);
        sincos_d(ssa(atan2_d(by, bx) - al), rs, rc);
    };
    const double ldx = lax - x, ldy = lay - y, cdx = cpx - x, cdy = cpy - y;
    rel_dir(ldy, ldx, 0.0, 1.0, o[4], o[5], [&](double& rs, double& rc) { ref(ldx, ldy, rs, rc); });
    rel_dir(cdy, cdx, 0.0, 1.0, o[6], o[7], [&](double& rs, double& rc) { ref(cdx, cdy, rs, rc); });
}
// T: the scenario's golden-march tables (null: plain search); hot: their probe table staged in LDS
// (LT) or null (read from T in global memory)
// KN: kn is LDS for the plain search's staged knots (closest_u; global-memory tables)
template <bool LT = false, bool KN = false, class S>
__device__ __forceinline__ void path_obs(const d2d_cfg& cfg, const S& s, const BrTab* T, double x, double y,
                                         double al, uint32_t& flags, double o[8], const BtHot* hot = nullptr,
                                         double* kn = nullptr) {
    int iu = -1;
    const double u = T ? (LT ? closest_u_tab<true>(s, *T, hot, x, y, iu) : closest_u_tab<false>(s, *T, &T->hot, x, y, iu))
                       : closest_u<KN>(s, x, y, iu, kn);
    path_obs_u(cfg, s, x, y, al, u, flags, o, iu);
}

// ------------------------------------------------------------------------------ reward
// The reward decodes from the fp64 observation exactly as the reference does (drone_2d_env.py:423-572).
// end conditions that need only the post-physics frame (drone_2d_env.py:543-571): collision,
// reach-end (decoded target distance), AA (decoded alpha), time-up.  Known before the observation,
// which lets the cooperative kernel start the auto-reset observation concurrently.
template <class S>
__device__ __forceinline__ int end_cause(const d2d_cfg& cfg, const S& s, const Body& F, bool collided, int t) {
    const double W = cfg.screen_w, H = cfg.screen_h;
    const double tdx = invm1to1(m1to1(s.wp_last_x - F.px, 0.0, W), 0.0, W);
    const double tdy = invm1to1(m1to1(s.wp_last_y - F.py, 0.0, H), 0.0, H);
    const double alpha = (F.a / PI) * PI;
    int cause = 0;
    if (collided) cause |= D2D_END_COLLISION;
    if (fabs(tdx) < cfg.reach_end_radius && fabs(tdy) < cfg.reach_end_radius) cause |= D2D_END_REACH;
    if (fabs(alpha) >= cfg.aa_angle) cause |= D2D_END_AA;
    if (t == cfg.n_steps) cause |= D2D_END_TIMEUP;
    return cause;
}
// reward_final split at its data dependencies, for the cooperative kernel (same arithmetic, same
// summation order):
//   CAStatic   obs 8..10 only (sensor role): closest distance, obstacle angle, lambdas, range term
//   RewardPos  the post-position frame + end cause (path role, while it waits for the physics)
//   RewardVel  the post-sweep velocity (physics role): speed term, velocity angle, CA total
//   reward_path / reward_sum   the path-observation terms, then the sum (path role)
// Angles the reward decodes from the observation (atan2 of a sin / cos pair, drone_2d_env.py:
// 438-445) enter it only through their differences: the PP term's cos(|wrap(LA - vel)|) is the dot
// product of the two (sin, cos) pairs, the CA term's |wrap(obst - vel)| the atan2 of their cross and
// dot products (one atan2 instead of two + two fmods; a few ulp from the reference sequence).
struct CAStatic {
    double d, os, oc, lpa, lca, rr;   // closest obstacle: distance, bearing (sin, cos) = obs 9, 10
};
template <class S>
__device__ __forceinline__ CAStatic ca_static(const d2d_cfg& cfg, const S& s, const double* o) {
    const double W = cfg.screen_w, H = cfg.screen_h;
    CAStatic C{__builtin_inf(), 0.0, 1.0, 1.0, 1.0, 0.0};
    if (s.n_circles > 0) {
        const double diag = sqrt(W * W + H * H);
        const double d = invm1to1(o[8], 0.0, diag);
        C.d = d;
        C.os = o[9];
        C.oc = o[10];
        const double Rr = cfg.danger_range, k = cfg.abs_inv_ca_min_rew;
        if (d < Rr && cfg.use_lambda) {
            const double l = (d / Rr) / 2.0;
            C.lpa = (l < 0.10) ? 0.10 : l;
            C.lca = 1.0 - C.lpa;
        }
        if (d < Rr) {
            const double rr = -(((Rr + k * Rr) / (d + k * Rr)) - 1.0);
            C.rr = (rr > 0.0) ? 0.0 : rr;
        }
    }
    return C;
}
struct RewardPos {
    double aa, coll, reach, pxd, pyd;
};
// sin_a: sin(F.a) (the physics wave's sincos of the frame angle); the reference takes sin(alpha) of
// alpha = (F.a / pi) * pi, within an ulp of F.a
__device__ __forceinline__ RewardPos reward_pos(const d2d_cfg& cfg, const Body& F, int cause, double sin_a) {
    const double W = cfg.screen_w, H = cfg.screen_h;
    RewardPos R;
    const double alpha = (F.a / PI) * PI;
    R.pxd = invm1to1(m1to1(F.px, 0.0, W), 0.0, W);
    R.pyd = invm1to1(m1to1(F.py, 0.0, H), 0.0, H);
    R.coll = (cause & D2D_END_COLLISION) ? cfg.rew_collision : 0.0;
    R.reach = (cause & D2D_END_REACH) ? cfg.rew_reach_end : 0.0;
    double aa = 0.0;
    if (alpha > cfg.aa_band) aa = -sin_a;
    if (alpha < -cfg.aa_band) aa = sin_a;
    if (cause & D2D_END_AA) aa = cfg.rew_aa;
    R.aa = aa;
    return R;
}
struct RewardVel {
    double sv, vs, vc, cal;   // speed term, velocity bearing (sin, cos) = obs 17, 18, CA total
};
// o = obs with entries 0, 1, 17, 18 filled (sensor_vel)
__device__ __forceinline__ RewardVel reward_vel(const d2d_cfg& cfg, const double* o, const CAStatic& C) {
    RewardVel R;
    const double vxd = invm1to1(o[0], -VEL_MAX, VEL_MAX);
    const double vyd = invm1to1(o[1], -VEL_MAX, VEL_MAX);
    R.sv = sqrt(vxd * vxd + vyd * vyd) * cfg.pp_vel_scale;
    R.vs = o[17];
    R.vc = o[18];
    double ca = 0.0;
    if (C.d < cfg.danger_range) {
        const double A = cfg.danger_angle, k = cfg.abs_inv_ca_min_rew;
        // |wrap(obstacle angle - velocity angle)| in degrees
        const double adiff = fabs(atan2_d(C.os * R.vc - C.oc * R.vs, C.oc * R.vc + C.os * R.vs) * (180.0 / PI));
        double ar = -(((A + k * A) / (adiff + k * A)) - 1.0);
        ar = (ar > 0.0) ? 0.0 : ar;
        ca = C.rr + ar;
    }
    R.cal = ca * C.lca;
    return R;
}
struct RewardPath {
    double ls, lc, dist, pa;   // LA bearing (sin, cos) = obs 23, 24
};
__device__ __forceinline__ RewardPath reward_path(const d2d_cfg& cfg, const RewardPos& P, const CAStatic& C,
                                                  const double* po) {
    const double W = cfg.screen_w, H = cfg.screen_h;
    RewardPath Q;
    const double cpx = invm1to1(po[0], 0.0, W), cpy = invm1to1(po[1], 0.0, H);
    Q.ls = po[4];
    Q.lc = po[5];
    Q.dist = norm2(cpx - P.pxd, cpy - P.pyd);
    const double pa = -(2.0 * (clipd(Q.dist, 0.0, cfg.pa_band_edge) / cfg.pa_band_edge) - 1.0) * cfg.pa_scale;
    Q.pa = pa * C.lpa;
    return Q;
}
struct RewardSum {
    double reward, pp;
};
__device__ __forceinline__ RewardSum reward_sum(const d2d_cfg& cfg, const RewardPos& P, const RewardVel& V,
                                                const RewardPath& Q) {
    RewardSum S;
    // cos(|wrap(LA angle - velocity angle)|)
    const double cvla = Q.lc * V.vc + Q.ls * V.vs;
    S.pp = clipd(cvla * V.sv, cfg.pp_rew_min, cfg.pp_rew_max);
    S.reward = P.aa + Q.pa + S.pp + P.coll + V.cal + P.reach;
    return S;
}

// full single-lane observation (reset kernel)
template <class S>
__device__ __forceinline__ void observe(const d2d_cfg& cfg, const S& s, const BrTab* T, const Body& F,
                                        uint32_t& flags, double obs[D2D_OBS_DIM]) {
    sensor_obs(cfg, s, F, obs);
    path_obs(cfg, s, T, F.px, F.py, F.a, flags, obs + 19);
}

}  // namespace d2d
