// d2d_curriculum.h -- the curriculum reset generator on the device (cfg.scn_pool = 2, "fresh").
//
// The reference's curriculum env draws a new scenario at every reset (drone_2d_env.py:199-215,
// 318-372): a corner (random.randint over spawn_corners), a random waypoint path
// (generate_random_waypoints_2d, predef_path.py:307-363) and its QPMI2D fit (:20-50), then by stage
// a spawn box (stage 2) or obstacles around / on the path (generate_obstacles_around_path,
// obstacles.py:58-89), the stage following the step count sim_num (:326-372).  Here the episode
// that env i starts with episode counter k gets G(seed, gid i, k, stage): the same draws in the
// same order from a Philox stream keyed by (seed, gid, k) instead of NumPy's / Python's global
// generators, so every episode's scenario is independent of the batch size and of the sharding.
// The stream, the fit and the arithmetic are restated by the CPU oracle (oracle/d2d_oracle.c,
// o_gen_curriculum); sin / cos / log come from d2d_pmath.h on both sides so the two draw
// bit-identical scenarios.  The host generator drone2d_amd/curriculum.py (bit-exact against the
// reference's own draws) is the distributional reference (tests/test_curriculum.py, GPU KS tests).
//
// Deviations from the reference, all distribution-preserving: the normal draws use the polar method
// (NumPy's legacy gauss) on Philox uniforms; np.random.binomial(1, p) is u < p; the direction angle
// of an obstacle offset is taken as the path gradient's unit normal, cos / sin(atan2(dy, dx) - pi/2)
// = (dy, -dx) / |(dx, dy)|; sim_num values that fall in the reference's schedule gaps (exactly
// 700 000, 1e6, 1.6e6, 2e6, where the reference creates no drone and fails) take the stage below.
#pragma once
#include "d2d_device.h"
#include "d2d_pmath.h"

namespace d2d {

constexpr uint32_t GEN_TAG = 0x43550000u;  // Philox counter word 2 of the generator's blocks

// sequential uniforms of one (seed, gid, key) stream: block b = Philox(gid, key, GEN_TAG + b, 0)
struct GenRng {
    uint32_t gid, key, k0, k1, blk, pos;
    uint32_t buf[4];
    __device__ void init(uint64_t seed, uint32_t g, uint32_t k) {
        gid = g;
        key = k;
        k0 = (uint32_t)seed;
        k1 = (uint32_t)(seed >> 32);
        blk = 0;
        pos = 4;
    }
    __device__ uint32_t next32() {
        if (pos == 4) {
            philox(gid, key, GEN_TAG + blk, 0u, k0, k1, buf);
            ++blk;
            pos = 0;
        }
        return buf[pos++];
    }
    __device__ double u01() {  // [0, 1), 53 bits
        const uint32_t a = next32(), b = next32();
        return u53(a, b);
    }
    // numpy / Python uniform(low, high) = low + (high - low) * random()
    __device__ double uniform(double lo, double hi) { return lo + (hi - lo) * u01(); }
    // random.randint(a, b): uniform over {a, ..., b}
    __device__ int randint(int a, int b) {
        const int k = (int)(u01() * (double)(b - a + 1));
        return a + (k < b - a ? k : b - a);
    }
    // np.random.normal(mean, std): the polar method (NumPy's legacy gauss), one value per pair
    __device__ double normal(double mean, double std) {
        double x1, x2, r2;
        int guard = 0;
        do {
            x1 = 2.0 * u01() - 1.0;
            x2 = 2.0 * u01() - 1.0;
            r2 = x1 * x1 + x2 * x2;
        } while ((r2 >= 1.0 || r2 == 0.0) && ++guard < 64);
        const double f = sqrt(-2.0 * d2d_pm_log(r2) / r2);
        return mean + std * (f * x2);
    }
};

// the reference's sim_num schedule (drone_2d_env.py:326-372); *chance: the obstacle spawn chance of
// stages 3 / 4 (linear ramps), from `stage` when the curriculum fixes one (stage_3: 0.6, stage_4: 1)
__host__ __device__ inline int gen_stage(const d2d_curriculum& c, double sim, double* chance) {
    *chance = 0.0;
    int st = c.stage;
    if (st < 1 || st > 5) {
        // (0 <= sim < 700 000: stage 1; the gaps 700 000 / 1e6 / 1.6e6 / 2e6 and negative counts,
        // where the reference creates no drone, take the stage below)
        if (sim <= 700000.0) st = 1;
        else if (sim <= 1000000.0) st = 2;
        else if (sim <= 1600000.0) st = 3;
        else if (sim <= 2000000.0) st = 4;
        else st = 5;
        if (st == 3) *chance = (sim - 1000000.0) * (0.6 - 0.2) / (1600000.0 - 1000000.0) + 0.2;
        if (st == 4) *chance = (sim - 1600000.0) * (1.0 - 0.6) / (2000000.0 - 1600000.0) + 0.6;
        return st;
    }
    if (st == 3) *chance = 0.6;
    if (st == 4) *chance = 1.0;
    return st;
}

// QPMI2D fit (predef_path.py:20-50): knots = cumulative segment lengths; one quadratic per interior
// waypoint n through (u_{n-1}, u_n, u_{n+1}), the 3x3 system solved by Gaussian elimination with
// partial pivoting (NumPy: inv(U_n).dot(wp); same solution to rounding)
__device__ inline void gen_solve3(double A[3][3], double b[3], double x[3]) {
    for (int c = 0; c < 3; ++c) {
        int p = c;
        for (int r = c + 1; r < 3; ++r)
            if (fabs(A[r][c]) > fabs(A[p][c])) p = r;
        if (p != c) {
            for (int k = 0; k < 3; ++k) {
                const double t = A[c][k];
                A[c][k] = A[p][k];
                A[p][k] = t;
            }
            const double t = b[c];
            b[c] = b[p];
            b[p] = t;
        }
        for (int r = c + 1; r < 3; ++r) {
            const double f = A[r][c] / A[c][c];
            for (int k = c + 1; k < 3; ++k) A[r][k] = A[r][k] - f * A[c][k];
            b[r] = b[r] - f * b[c];
        }
    }
    for (int r = 2; r >= 0; --r) {
        double s = b[r];
        for (int k = r + 1; k < 3; ++k) s = s - A[r][k] * x[k];
        x[r] = s / A[r][r];
    }
}
__device__ inline void gen_fit(const double* wx, const double* wy, int nw, d2d_scn& s) {
    s.n_wps = nw;
    double acc = 0.0;
    s.us[0] = 0.0;
    for (int i = 0; i + 1 < nw; ++i) {
        const double dx = wx[i + 1] - wx[i], dy = wy[i + 1] - wy[i];
        acc = acc + sqrt(dx * dx + dy * dy);
        s.us[i + 1] = acc;
    }
    for (int i = nw; i < D2D_MAX_WPS; ++i) s.us[i] = 0.0;
    for (int k = nw - 2; k < D2D_MAX_SEGS; ++k) s.xa[k] = s.xb[k] = s.xc[k] = s.ya[k] = s.yb[k] = s.yc[k] = 0.0;
    for (int n = 1; n + 1 < nw; ++n) {
        const double u[3] = {s.us[n - 1], s.us[n], s.us[n + 1]};
        double A[3][3], B[3][3], bx[3] = {wx[n - 1], wx[n], wx[n + 1]}, by[3] = {wy[n - 1], wy[n], wy[n + 1]}, px[3],
                                   py[3];
        for (int r = 0; r < 3; ++r) {
            A[r][0] = B[r][0] = u[r] * u[r];
            A[r][1] = B[r][1] = u[r];
            A[r][2] = B[r][2] = 1.0;
        }
        gen_solve3(A, bx, px);
        gen_solve3(B, by, py);
        s.xa[n - 1] = px[0];
        s.xb[n - 1] = px[1];
        s.xc[n - 1] = px[2];
        s.ya[n - 1] = py[0];
        s.yb[n - 1] = py[1];
        s.yc[n - 1] = py[2];
    }
}
// QPMI2D.calculate_gradient (predef_path.py:145-188; drone2d_amd/scenarios.py QPMIPath.gradient)
__device__ inline void gen_gradient(const d2d_scn& s, double u, double& gx, double& gy) {
    const int nw = s.n_wps, last = nw - 3;
    if (u >= s.us[0] && u <= s.us[1]) {
        gx = s.xa[0] * u * 2.0 + s.xb[0];
        gy = s.ya[0] * u * 2.0 + s.yb[0];
        return;
    }
    if (u >= s.us[nw - 2]) {
        gx = s.xa[last] * u * 2.0 + s.xb[last];
        gy = s.ya[last] * u * 2.0 + s.yb[last];
        return;
    }
    // (a branch-free count of the knots below u measured equal in K5: the loop stays)
    int n = 0;
    while (n < nw - 1 && !(u <= s.us[n + 1])) ++n;
    const double du = s.us[n + 1] - s.us[n];
    const double mr = (u - s.us[n]) / du, mf = (s.us[n + 1] - u) / du;
    const double dx1 = s.xa[n - 1] * u * 2.0 + s.xb[n - 1], dy1 = s.ya[n - 1] * u * 2.0 + s.yb[n - 1];
    const double dx2 = s.xa[n] * u * 2.0 + s.xb[n], dy2 = s.ya[n] * u * 2.0 + s.yb[n];
    gx = mr * dx2 + mf * dx1;
    gy = mr * dy2 + mf * dy1;
}

// generate_obstacles_around_path (obstacles.py:58-89): appends up to n circles (the reference's
// `while num_obstacles < n` with a real-valued n), rejection on |offset| <= size + 10 off the path
template <typename Rng>
__device__ inline void gen_obstacles(Rng& R, const ScnR& S, d2d_scn& s, double n, double mean, double std, bool on_path) {
    const double L = s.us[s.n_wps - 1];
    int num = 0, tries = 0;
    while ((double)num < n && s.n_circles < D2D_MAX_CIRCLES && tries < 4096) {
        ++tries;
        const double u = R.uniform(0.20 * L, 0.90 * L);
        double gx, gy;
        gen_gradient(s, u, gx, gy);
        const double dist = R.normal(mean, std);
        double x, y;
        path_eval(S, u, x, y);
        // (cos, sin)(atan2(gy, gx) - pi/2) = (gy, -gx) / |g|
        const double g = sqrt(gx * gx + gy * gy);
        const double ox = x + dist * (gy / g), oy = y + dist * (-gx / g);
        const double size = R.uniform(10.0, 50.0);
        const double dx = ox - x, dy = oy - y;
        const double off = sqrt(dx * dx + dy * dy);
        if (!on_path && off > size + 10.0) {
            s.cx[s.n_circles] = ox;
            s.cy[s.n_circles] = oy;
            s.cr[s.n_circles] = size;
            s.n_circles += 1;
            ++num;
        } else if (on_path) {
            s.cx[s.n_circles] = x;
            s.cy[s.n_circles] = y;
            s.cr[s.n_circles] = size;
            s.n_circles += 1;
            ++num;
        }
    }
}

// one curriculum reset: writes the ABI record `s` and its device form `S` (both in global memory)
__device__ inline void gen_curriculum(const d2d_curriculum& c, double W, double H, uint64_t seed, uint32_t gid,
                                      uint32_t key, double sim, d2d_scn& s, ScnR& S) {
    GenRng R;
    R.init(seed, gid, key);
    const int corner = c.random_path_spawn ? R.randint(c.corner_lo, c.corner_hi) : 2;  // 1 DL 2 DR 3 UL 4 UR
    const int nw = c.n_wps < 3 ? 3 : (c.n_wps > D2D_MAX_WPS ? D2D_MAX_WPS : c.n_wps);
    double wx[D2D_MAX_WPS], wy[D2D_MAX_WPS];
    double lo, hi;
    if (corner == 1) {
        wx[0] = R.uniform(100.0, 180.0);
        wy[0] = R.uniform(100.0, 180.0);
        lo = 0.0;
        hi = PI / 2.0;
    } else if (corner == 3) {
        wx[0] = R.uniform(100.0, 180.0);
        wy[0] = R.uniform(H - 180.0, H - 100.0);
        lo = 0.0;
        hi = -PI / 2.0;
    } else if (corner == 4) {
        wx[0] = R.uniform(W - 180.0, W - 100.0);
        wy[0] = R.uniform(H - 180.0, H - 100.0);
        lo = -PI / 2.0;
        hi = -PI;
    } else {
        wx[0] = R.uniform(W - 180.0, W - 100.0);
        wy[0] = R.uniform(100.0, 180.0);
        lo = PI / 2.0;
        hi = PI;
    }
    for (int i = 0; i + 1 < nw; ++i) {
        const double az = R.uniform(lo, hi);
        double sa, ca;
        d2d_pm_sincos(az, &sa, &ca);
        wx[i + 1] = wx[i] + c.segment_length * ca;
        wy[i + 1] = wy[i] + c.segment_length * sa;
    }
    gen_fit(wx, wy, nw, s);
    s.n_circles = 0;
    s.wp_last_x = wx[nw - 1];
    s.wp_last_y = wy[nw - 1];
    s.spawn_xmin = s.spawn_xmax = wx[0];
    s.spawn_ymin = s.spawn_ymax = wy[0];
    s.spawn_amin = -PI / 4.0;
    s.spawn_amax = PI / 4.0;
    double chance;
    const int stg = gen_stage(c, sim, &chance);
    if (stg == 2) {  // drone spawned uniformly on the screen, no obstacles (:333-337)
        s.spawn_xmin = 100.0;
        s.spawn_xmax = W - 100.0;
        s.spawn_ymin = 100.0;
        s.spawn_ymax = H - 100.0;
    }
    scn_build(s, S);  // the path, for the obstacle placement
    if (stg == 3) {
        if (R.u01() < chance) gen_obstacles(R, S, s, 1.0, 0.0, 100.0, false);
    } else if (stg == 4) {
        if (R.u01() < chance) gen_obstacles(R, S, s, 1.0, 0.0, 0.0, true);
    } else if (stg == 5) {
        double n_obs = R.normal(1.0, 4.0);
        if (n_obs < 0.0 && n_obs > -3.0) n_obs = 1.0;
        if (n_obs < -3.0) n_obs = 0.0;
        if (n_obs != 0.0) {
            gen_obstacles(R, S, s, n_obs, 0.0, 100.0, false);
            gen_obstacles(R, S, s, 1.0, 0.0, 0.0, true);
        }
    }
    for (int k = s.n_circles; k < D2D_MAX_CIRCLES; ++k) s.cx[k] = s.cy[k] = s.cr[k] = 0.0;
    scn_build(s, S);
}


// ------------------------------------------------------------------ wave-cooperative generation (K5)
// The same scenario as gen_curriculum, built by the 64 lanes of one wave in LDS: the stream's first
// GEN_WIN words (GEN_WIN_BLOCKS Philox blocks per lane), the azimuths' sincos, the segment lengths, the 20
// QPMI2D 3 x 3 solves and the 16 interval records in parallel; the few truly sequential parts (the
// waypoint and arc-length prefix sums, the obstacle rejection loop, which consumes a data-dependent
// number of draws) on lane 0 reading the stream from LDS.  Every value is produced by the same
// operations on the same operands as gen_curriculum (so the tables stay bit-identical to the CPU
// oracle's o_gen_curriculum); only the order in which independent values are computed changes.
constexpr int GEN_WIN_BLOCKS = 2;  // Philox blocks per lane in the window (round 4's 1: 256 words)
// stream words precomputed per item: corner + waypoints + the obstacle trials, which the wave evaluates
// at 64 starts 4 words apart (gen_obstacles_wave) -- 512 words keep the first evaluation's trials
// inside the window
constexpr int GEN_WIN = 256 * GEN_WIN_BLOCKS;

// LDS hand-off between the lanes of the one wave that runs the generator
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// serial reader of one (seed, gid, key) stream: words below GEN_WIN from the LDS window, later blocks
// computed on demand (the same block formula as GenRng)
struct GenStream {
    const uint32_t* win;
    uint32_t gid, key, k0, k1;
    int pos, bufblk;
    uint32_t buf[4];
    __device__ void init(const uint32_t* w, uint64_t seed, uint32_t g, uint32_t k, int p0) {
        win = w;
        gid = g;
        key = k;
        k0 = (uint32_t)seed;
        k1 = (uint32_t)(seed >> 32);
        pos = p0;
        bufblk = -1;
    }
    __device__ uint32_t next32() {
        const int p = pos++;
        if (p < GEN_WIN) return win[p];
        const int b = p >> 2;
        if (b != bufblk) {
            philox(gid, key, GEN_TAG + (uint32_t)b, 0u, k0, k1, buf);
            bufblk = b;
        }
        return buf[p & 3];
    }
    __device__ double u01() {
        const uint32_t a = next32(), b = next32();
        return u53(a, b);
    }
    __device__ double uniform(double lo, double hi) { return lo + (hi - lo) * u01(); }
    __device__ double normal(double mean, double std) {
        double x1, x2, r2;
        int guard = 0;
        do {
            x1 = 2.0 * u01() - 1.0;
            x2 = 2.0 * u01() - 1.0;
            r2 = x1 * x1 + x2 * x2;
        } while ((r2 >= 1.0 || r2 == 0.0) && ++guard < 64);
        const double f = sqrt(-2.0 * d2d_pm_log(r2) / r2);
        return mean + std * (f * x2);
    }
};
__device__ __forceinline__ double win_u01(const uint32_t* w, int p) { return u53(w[p], w[p + 1]); }

// scn_build with interval n on lane n (the path part: knots, interval records, n_wps) ...
__device__ inline void scn_build_path_lanes(const d2d_scn& a, ScnR& s, int lane) {
    const int nw = a.n_wps, nseg = nw - 2;
    if (lane < D2D_MAX_WPS) {
        const int n = lane;
        s.us_[n] = (n < nw) ? a.us[n] : __builtin_inf();
        if (REC_W > REC_N) s.rec_[n][REC_W - 1] = 0.0;
        const int b = (n < nseg - 1) ? n : nseg - 1;
        const int q = (n == 0) ? nseg - 1 : ((n - 1 < nseg - 1) ? n - 1 : nseg - 1);
        const double v[REC_N] = {a.xa[b], a.xb[b], a.xc[b], a.ya[b], a.yb[b], a.yc[b],
                                 a.xa[q], a.xb[q], a.xc[q], a.ya[q], a.yb[q], a.yc[q], 0.0, 0.0, 0.0};
        for (int f = 0; f < REC_N; ++f) SREC(s, f, n) = v[f];
        const int n1 = (n + 1 < D2D_MAX_WPS) ? n + 1 : D2D_MAX_WPS - 1;
        const double u0 = (n < nw) ? a.us[n] : __builtin_inf(), u1 = (n1 < nw) ? a.us[n1] : __builtin_inf();
        SREC(s, REC_U0, n) = u0;
        SREC(s, REC_U1, n) = u1;
        SREC(s, REC_IDU, n) = 1.0 / (u1 - u0);
        const double us0 = a.us[0];  // (nw >= 3: us[0] and us[nw - 2] are real knots)
        const double last_lo = a.us[nw - 2] - 0.001;
        SREC(s, REC_T, n) = (n == 0) ? (us0 < last_lo ? us0 : last_lo) : (n < nw - 1 ? last_lo : -__builtin_inf());
    }
    if (lane == 0) s.n_wps = nw;
}
// ... and the rest: circle k on lane k, the scalars and r_uniform on lane 0
__device__ inline void scn_build_rest_lanes(const d2d_scn& a, ScnR& s, int lane) {
    if (lane < D2D_MAX_CIRCLES) {
        s.cx[lane] = a.cx[lane];
        s.cy[lane] = a.cy[lane];
        s.cr[lane] = a.cr[lane];
    }
    if (lane == 0) {
        s.n_circles = a.n_circles;
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
    }
}

// Per-item LDS of the wave generator.
struct GenLds {
    d2d_scn a;                 // the ABI record being built
    ScnR s;                    // its device form (obstacle placement; the fresh curriculum's layout)
    uint32_t win[GEN_WIN];     // the stream's first GEN_WIN words
    double wx[D2D_MAX_WPS], wy[D2D_MAX_WPS], sa[D2D_MAX_WPS], ca[D2D_MAX_WPS], seg[D2D_MAX_WPS];
    int32_t wpos;            // the stream position after the obstacle calls
};

// generate_obstacles_around_path (gen_obstacles) with the wave: one rejection trial is a pure function
// of the stream word it starts at, and every trial consumes a multiple of 4 words (uniform 2 + the
// polar normal 4 per attempt + uniform 2), so the chain's trials start at w0, w0 + 4 k, ...: lane l
// evaluates the trial starting at word w0 + 4 l and the wave then walks the chain of trials the serial
// loop would run (w -> w + words consumed) in scalar registers, reading each visited trial from its
// lane, and appends the accepted circles in order; a chain that leaves the 64 evaluated starts
// continues from a new w0.  Same trials, same order, same arithmetic as gen_obstacles.  (Starts every
// 2 words, as in round 4, covered half the chain per evaluation: the stage-5 items with many
// obstacles needed 2-3 evaluations and set K5's duration.)
// then_on_path: the reference's next call, generate_obstacles_around_path(1, mean 0, std 0, on_path)
// (stage 5), is folded in.  Its trial at a word consumes the same draws as this call's trial there and
// is always accepted (on the path: the circle sits at the trial's path point), so once this call's
// chain ends at word w, the next call's one obstacle is the trial evaluated at w -- no second round of
// trials (unless w left the evaluated window).  Same trials, same order as the two separate calls.
// lane t's value as a wave-uniform scalar (v_readlane: t uniform)
__device__ __forceinline__ int gen_rl(int v, int t) { return __builtin_amdgcn_readlane(v, t); }
__device__ __forceinline__ double gen_rl(double v, int t) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), t),
                            __builtin_amdgcn_readlane(__double2loint(v), t));
}
__device__ inline void gen_obstacles_wave(GenLds& G, uint64_t seed, uint32_t gid, uint32_t key, double n, double mean,
                                          double std, bool on_path, int lane, bool then_on_path = false) {
    d2d_scn& s = G.a;
    const double L = s.us[s.n_wps - 1];
    // the walk's state is wave-uniform (scalar registers) and reads the trials' results from the lanes
    // that evaluated them (v_readlane): no LDS round trip per visited trial (round 4 kept the trials in
    // LDS and walked them on lane 0: ~2 dependent LDS reads per trial on the generator's serial chain)
    int num = 0, tries = 0, w = __builtin_amdgcn_readfirstlane(G.wpos);
    int nc = __builtin_amdgcn_readfirstlane(s.n_circles);
    int phase = 0;  // 0: this call's chain, 1: the folded on-path call, 2: done
    while (phase != 2) {
        double tox, toy, tpx, tpy, tsz;
        int tok, tcons;
        {
            GenStream R;
            R.init(G.win, seed, gid, key, w + 4 * lane);
            const double u = R.uniform(0.20 * L, 0.90 * L);
            double gx, gy;
            gen_gradient(s, u, gx, gy);
            const double dist = R.normal(mean, std);
            double x, y;
            path_eval(G.s, u, x, y);
            const double g = sqrt(gx * gx + gy * gy);
            const double ox = x + dist * (gy / g), oy = y + dist * (-gx / g);
            const double size = R.uniform(10.0, 50.0);
            const double dx = ox - x, dy = oy - y;
            const double off = sqrt(dx * dx + dy * dy);
            tok = (on_path || off > size + 10.0) ? 1 : 0;
            tox = on_path ? x : ox;
            toy = on_path ? y : oy;
            tpx = x;
            tpy = y;
            tsz = size;
            tcons = R.pos - (w + 4 * lane);
        }
        const int w0 = w;
        // A trial at word w was evaluated (on lane (w - w0) / 4) iff w - w0 is a multiple of 4 below
        // 256.  Every trial consumes a multiple of 4 words today (uniform 2, each polar-normal attempt
        // 4, uniform 2), so the walk stays on the evaluated starts; should a draw ever consume another
        // count, the walk leaves the window at that trial and the next pass evaluates from there
        // (slower, never a wrong trial).
        const auto evaluated = [&](int wv) { return (wv < w0 + 256) & (((wv - w0) & 3) == 0); };
        if (phase == 0) {
            while ((double)num < n && nc < D2D_MAX_CIRCLES && tries < 4096 && evaluated(w)) {
                const int t = (w - w0) >> 2;
                ++tries;
                if (gen_rl(tok, t)) {
                    const double cx = gen_rl(tox, t), cy = gen_rl(toy, t), cr = gen_rl(tsz, t);
                    if (lane == 0) {
                        s.cx[nc] = cx;
                        s.cy[nc] = cy;
                        s.cr[nc] = cr;
                    }
                    nc += 1;
                    ++num;
                }
                w += gen_rl(tcons, t);
            }
            if (!((double)num < n && nc < D2D_MAX_CIRCLES && tries < 4096)) {
                phase = then_on_path ? 1 : 2;
                num = 0;
                tries = 0;
            }
        }
        if (phase == 1) {
            // generate_obstacles_around_path(1.0, 0.0, 0.0, on_path=True): one trial, accepted
            if (nc >= D2D_MAX_CIRCLES) {
                phase = 2;
            } else if (evaluated(w)) {
                const int t = (w - w0) >> 2;
                const double cx = gen_rl(tpx, t), cy = gen_rl(tpy, t), cr = gen_rl(tsz, t);
                if (lane == 0) {
                    s.cx[nc] = cx;
                    s.cy[nc] = cy;
                    s.cr[nc] = cr;
                }
                nc += 1;
                w += gen_rl(tcons, t);
                phase = 2;
            }
        }
    }
    if (lane == 0) {
        s.n_circles = nc;
        G.wpos = w;
    }
    wave_sync();
}

// one curriculum reset by the calling wave (all 64 lanes, wave-uniform arguments) in two parts: the
// path (gen_path_wave: waypoints, fit, G.s's knots and interval records) and the rest (gen_rest_wave:
// stage fields, obstacles, G.s's circles and scalars).  The result is in G.a / G.s (LDS).  Same draws
// and arithmetic as gen_curriculum.
#ifdef D2D_GEN_STAMPS  // diagnostic builds only: s_memtime at K5b's phase boundaries, 8 per item
#define GSTAMP(st, k)                                                   \
    do {                                                                \
        if ((st) && lane == 0) (st)[k] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define GSTAMP(st, k) \
    do {              \
    } while (0)
#endif
// returns the stream position of the first draw after the azimuths
__device__ inline int gen_path_wave(const d2d_curriculum& c, double W, double H, uint64_t seed, uint32_t gid,
                                    uint32_t key, GenLds& G, int lane, uint64_t* st = nullptr) {
    (void)st;
    GSTAMP(st, 0);
#pragma unroll
    for (int blk = 0; blk < GEN_WIN_BLOCKS; ++blk) {
        uint32_t o[4];
        const uint32_t b = (uint32_t)(64 * blk + lane);
        philox(gid, key, GEN_TAG + b, 0u, (uint32_t)seed, (uint32_t)(seed >> 32), o);
        for (int k = 0; k < 4; ++k) G.win[4 * b + k] = o[k];
    }
    wave_sync();
    GSTAMP(st, 1);
    // stream positions (words) of the fixed-count draws: corner (random.randint), wx0, wy0, azimuths
    int p = 0;
    int corner = 2;
    if (c.random_path_spawn) {
        const int a0 = c.corner_lo, b0 = c.corner_hi;
        const int k = (int)(win_u01(G.win, p) * (double)(b0 - a0 + 1));
        corner = a0 + (k < b0 - a0 ? k : b0 - a0);
        p += 2;
    }
    const int nw = c.n_wps < 3 ? 3 : (c.n_wps > D2D_MAX_WPS ? D2D_MAX_WPS : c.n_wps);
    double lo, hi, x0lo, x0hi, y0lo, y0hi;
    if (corner == 1) {
        x0lo = 100.0; x0hi = 180.0; y0lo = 100.0; y0hi = 180.0; lo = 0.0; hi = PI / 2.0;
    } else if (corner == 3) {
        x0lo = 100.0; x0hi = 180.0; y0lo = H - 180.0; y0hi = H - 100.0; lo = 0.0; hi = -PI / 2.0;
    } else if (corner == 4) {
        x0lo = W - 180.0; x0hi = W - 100.0; y0lo = H - 180.0; y0hi = H - 100.0; lo = -PI / 2.0; hi = -PI;
    } else {
        x0lo = W - 180.0; x0hi = W - 100.0; y0lo = 100.0; y0hi = 180.0; lo = PI / 2.0; hi = PI;
    }
    const int paz = p + 4;  // azimuth i at paz + 2 i
    if (lane < nw - 1) {
        const double az = lo + (hi - lo) * win_u01(G.win, paz + 2 * lane);
        double sa, ca;
        d2d_pm_sincos(az, &sa, &ca);
        G.sa[lane] = sa;
        G.ca[lane] = ca;
    }
    wave_sync();
    if (lane == 0) {
        G.wx[0] = x0lo + (x0hi - x0lo) * win_u01(G.win, p);
        G.wy[0] = y0lo + (y0hi - y0lo) * win_u01(G.win, p + 2);
        for (int i = 0; i + 1 < nw; ++i) {
            G.wx[i + 1] = G.wx[i] + c.segment_length * G.ca[i];
            G.wy[i + 1] = G.wy[i] + c.segment_length * G.sa[i];
        }
    }
    wave_sync();
    // gen_fit: segment lengths (lanes), arc length prefix sum (lane 0), the fits (lanes)
    d2d_scn& s = G.a;
    if (lane + 1 < nw) {
        const double dx = G.wx[lane + 1] - G.wx[lane], dy = G.wy[lane + 1] - G.wy[lane];
        G.seg[lane] = sqrt(dx * dx + dy * dy);
    }
    if (lane < D2D_MAX_SEGS && lane >= nw - 2) s.xa[lane] = s.xb[lane] = s.xc[lane] = s.ya[lane] = s.yb[lane] = s.yc[lane] = 0.0;
    if (lane >= nw && lane < D2D_MAX_WPS) s.us[lane] = 0.0;
    wave_sync();
    if (lane == 0) {
        s.n_wps = nw;
        double acc = 0.0;
        s.us[0] = 0.0;
        for (int i = 0; i + 1 < nw; ++i) {
            acc = acc + G.seg[i];
            s.us[i + 1] = acc;
        }
    }
    wave_sync();
    {
        // lanes 0..nw-3: the x fit of interior waypoint n = lane + 1; lanes 32..32+nw-3: the y fit
        const int n = (lane & 31) + 1;
        if (n + 1 < nw && (lane & 31) < D2D_MAX_SEGS) {
            const bool yfit = lane >= 32;
            const double u[3] = {s.us[n - 1], s.us[n], s.us[n + 1]};
            double A[3][3], b[3], x[3];
            const double* w = yfit ? G.wy : G.wx;
            for (int r = 0; r < 3; ++r) {
                A[r][0] = u[r] * u[r];
                A[r][1] = u[r];
                A[r][2] = 1.0;
                b[r] = w[n - 1 + r];
            }
            gen_solve3(A, b, x);
            if (!yfit) {
                s.xa[n - 1] = x[0];
                s.xb[n - 1] = x[1];
                s.xc[n - 1] = x[2];
            } else {
                s.ya[n - 1] = x[0];
                s.yb[n - 1] = x[1];
                s.yc[n - 1] = x[2];
            }
        }
    }
    wave_sync();
    scn_build_path_lanes(s, G.s, lane);
    wave_sync();
    GSTAMP(st, 2);
    return paz + 2 * (nw - 1);
}
__device__ inline void gen_rest_wave(const d2d_curriculum& c, double W, double H, uint64_t seed, uint32_t gid,
                                     uint32_t key, double sim, int pos, GenLds& G, int lane, uint64_t* st = nullptr) {
    (void)st;
    d2d_scn& s = G.a;
    const int nw = s.n_wps;
    double chance;
    const int stg = gen_stage(c, sim, &chance);
    if (lane == 0) {
        s.n_circles = 0;
        s.wp_last_x = G.wx[nw - 1];
        s.wp_last_y = G.wy[nw - 1];
        s.spawn_xmin = s.spawn_xmax = G.wx[0];
        s.spawn_ymin = s.spawn_ymax = G.wy[0];
        s.spawn_amin = -PI / 4.0;
        s.spawn_amax = PI / 4.0;
        if (stg == 2) {  // drone spawned uniformly on the screen, no obstacles (:333-337)
            s.spawn_xmin = 100.0;
            s.spawn_xmax = W - 100.0;
            s.spawn_ymin = 100.0;
            s.spawn_ymax = H - 100.0;
        }
    }
    if (lane < D2D_MAX_CIRCLES) s.cx[lane] = s.cy[lane] = s.cr[lane] = 0.0;
    wave_sync();
    if (stg >= 3) {
        // the draws before the obstacle calls (lane 0), then the calls (gen_obstacles_wave; the path
        // in G.s is already built)
        __shared__ double s_nobs;
        if (lane == 0) {
            GenStream R;
            R.init(G.win, seed, gid, key, pos);
            double n_obs = 0.0;
            if (stg == 3 || stg == 4) {
                n_obs = (R.u01() < chance) ? 1.0 : 0.0;
            } else {
                n_obs = R.normal(1.0, 4.0);
                if (n_obs < 0.0 && n_obs > -3.0) n_obs = 1.0;
                if (n_obs < -3.0) n_obs = 0.0;
            }
            s_nobs = n_obs;
            G.wpos = R.pos;
        }
        wave_sync();
        const double n_obs = s_nobs;
        if (stg == 3) {
            if (n_obs != 0.0) gen_obstacles_wave(G, seed, gid, key, 1.0, 0.0, 100.0, false, lane);
        } else if (stg == 4) {
            if (n_obs != 0.0) gen_obstacles_wave(G, seed, gid, key, 1.0, 0.0, 0.0, true, lane);
        } else if (n_obs != 0.0) {
            // the two calls of stage 5 (obstacles around the path, then one on it) in one walk
            gen_obstacles_wave(G, seed, gid, key, n_obs, 0.0, 100.0, false, lane, true);
        }
    }
    GSTAMP(st, 4);
    scn_build_rest_lanes(s, G.s, lane);
    wave_sync();
    GSTAMP(st, 5);
}


}  // namespace d2d
