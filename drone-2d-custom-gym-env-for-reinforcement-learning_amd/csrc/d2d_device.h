// d2d_device.h -- per-env device functions of the batched Drone2dEnv step (gfx950, fp64).
//
// One lane = one env.  Everything here is straight-line fp64 on VGPRs; the scenario (path
// coefficients, knots, circles) is read from an LDS-staged copy shared by the workgroup.
// Evaluation order follows the reference's NumPy order term by term (see oracle/d2d_oracle.c for
// the plain restatement and tests/golden for the pinned vectors), compiled with
// -ffp-contract=off; the only fused ops are where NumPy/OpenBLAS itself fuses (norm, matmul).
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

// Diagnostic-only ablation mask (tools/ablate.py builds separate timing-only libraries with it;
// the product is always built with 0): 1 skip Brent, 2 skip sensing, 4 skip joint iterations,
// 8 skip collision test.
#ifndef D2D_ABLATE
#define D2D_ABLATE 0
#endif

namespace d2d {

constexpr double PI = 3.141592653589793;      // np.pi
constexpr double TWO_PI = 6.283185307179586;  // 2*np.pi
constexpr double DT = 1.0 / 60.0;             // drone_2d_env.py:406
constexpr double GRAV_Y = -1000.0;            // drone_2d_env.py:185
constexpr double DRONE_R = 40.0;              // Drone.py:11 (100/2 - 20/2)
constexpr double FRAME_HX = 50.0, FRAME_HY = 5.0;   // Drone.py:16 box (100, 10)

// ------------------------------------------------------------------------------ scalar helpers
// Python/NumPy float modulo (fmod, then move into the divisor's sign)
__device__ __forceinline__ double pymod(double a, double b) {
    double m = fmod(a, b);
    if (m != 0.0) {
        if ((b < 0.0) != (m < 0.0)) m += b;
    } else {
        m = copysign(0.0, b);
    }
    return m;
}
__device__ __forceinline__ double ssa(double a) { return pymod(a + PI, TWO_PI) - PI; }
__device__ __forceinline__ double m1to1(double v, double lo, double hi) { return 2.0 * (v - lo) / (hi - lo) - 1.0; }
__device__ __forceinline__ double invm1to1(double v, double lo, double hi) { return (v + 1.0) * (hi - lo) / 2.0 + lo; }
__device__ __forceinline__ double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
// np.linalg.norm of a 2-vector == sqrt(OpenBLAS ddot) == sqrt(fma(dy, dy, dx*dx))
__device__ __forceinline__ double norm2(double dx, double dy) { return sqrt(fma(dy, dy, dx * dx)); }
__device__ __forceinline__ double sgn_nz(double x) {
    double s = (x > 0.0) ? 1.0 : ((x < 0.0) ? -1.0 : (x == 0.0 ? 0.0 : x));
    return s + (x == 0.0 ? 1.0 : 0.0);
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

// ------------------------------------------------------------------------------ QPMI2D path
// get_u_index (predef_path.py:53-63): first n with u <= us[n+1]; for non-decreasing knots this is
// the number of knots k >= 1 with !(u <= us[k]) (NaN -> n_wps-1, as the Python loop).
__device__ __forceinline__ int u_index(const d2d_scn& s, double u) {
    int n = 0;
#pragma unroll
    for (int k = 1; k < D2D_MAX_WPS; ++k) n += (k < s.n_wps && !(u <= s.us[k])) ? 1 : 0;
    return n;
}
__device__ __forceinline__ void quad(const d2d_scn& s, int k, double u, double& x, double& y) {
    const double uu = u * u;
    x = s.xa[k] * uu + s.xb[k] * u + s.xc[k];
    y = s.ya[k] * uu + s.yb[k] * u + s.yc[k];
}
// QPMI2D.__call__ (predef_path.py:88-142)
__device__ __forceinline__ void path_eval(const d2d_scn& s, double u, double& x, double& y) {
    const int nw = s.n_wps, nseg = nw - 2;
    const int n = u_index(s, u);
    if (u >= s.us[0] && u <= s.us[1]) {
        quad(s, 0, u, x, y);
    } else if ((u >= s.us[nw - 2] - 0.001 && u <= s.us[nw - 1]) || n == nw - 1) {
        quad(s, nseg - 1, u, x, y);
    } else {
        const double u0 = s.us[n], u1 = s.us[n + 1];
        const double mu_r = (u - u0) / (u1 - u0);
        const double mu_f = (u1 - u) / (u1 - u0);
        const int k1 = (n == 0) ? nseg - 1 : n - 1;  // python x_params[n-1]
        double x1, y1, x2, y2;
        quad(s, k1, u, x1, y1);
        quad(s, n, u, x2, y2);
        x = mu_r * x2 + mu_f * x1;
        y = mu_r * y2 + mu_f * y1;
    }
}
__device__ __forceinline__ double path_dist(const d2d_scn& s, double u, double px, double py) {
    double x, y;
    path_eval(s, u, x, y);
    return norm2(x - px, y - py);
}
// get_closest_u (predef_path.py:226-248) = scipy fminbound(x1=-10, x2=L+10, xtol=1e-6, maxfun=500)
// restated from scipy 1.15.3 _minimize_scalar_bounded (_optimize.py:2251-2398), probe for probe.
__device__ double closest_u(const d2d_scn& s, double px, double py) {
    const double sqrt_eps = 1.4832396974191326e-08;   // sqrt(2.2e-16)
    const double golden_mean = 0.3819660112501051;    // 0.5*(3.0 - sqrt(5.0))
    const double xatol3 = 1e-6 / 3.0;
    double a = 0.0 - 10.0, b = s.us[s.n_wps - 1] + 10.0;
    double fulc = a + golden_mean * (b - a);
    double nfc = fulc, xf = fulc;
    double rat = 0.0, e = 0.0;
    double x = xf;
    double fx = path_dist(s, x, px, py);
    int num = 1;
    double ffulc = fx, fnfc = fx;
    double xm = 0.5 * (a + b);
    double tol1 = sqrt_eps * fabs(xf) + xatol3;
    double tol2 = 2.0 * tol1;
    while (fabs(xf - xm) > (tol2 - 0.5 * (b - a))) {
        bool golden = true;
        if (fabs(e) > tol1) {
            golden = false;
            double r = (xf - nfc) * (fx - ffulc);
            double q = (xf - fulc) * (fx - fnfc);
            double p = (xf - fulc) * q - (xf - nfc) * r;
            q = 2.0 * (q - r);
            if (q > 0.0) p = -p;
            q = fabs(q);
            r = e;
            e = rat;
            if ((fabs(p) < fabs(0.5 * q * r)) && (p > q * (a - xf)) && (p < q * (b - xf))) {
                rat = (p + 0.0) / q;
                x = xf + rat;
                if (((x - a) < tol2) || ((b - x) < tol2)) rat = tol1 * sgn_nz(xm - xf);
            } else {
                golden = true;
            }
        }
        if (golden) {
            e = (xf >= xm) ? a - xf : b - xf;
            rat = golden_mean * e;
        }
        const double ar = fabs(rat);
        const double mx = (ar != ar) ? ar : (ar > tol1 ? ar : tol1);
        x = xf + sgn_nz(rat) * mx;
        const double fu = path_dist(s, x, px, py);
        num += 1;
        if (fu <= fx) {
            if (x >= xf) a = xf; else b = xf;
            fulc = nfc; ffulc = fnfc;
            nfc = xf; fnfc = fx;
            xf = x; fx = fu;
        } else {
            if (x < xf) a = x; else b = x;
            if ((fu <= fnfc) || (nfc == xf)) {
                fulc = nfc; ffulc = fnfc;
                nfc = x; fnfc = fu;
            } else if ((fu <= ffulc) || (fulc == xf) || (fulc == nfc)) {
                fulc = x; ffulc = fu;
            }
        }
        xm = 0.5 * (a + b);
        tol1 = sqrt_eps * fabs(xf) + xatol3;
        tol2 = 2.0 * tol1;
        if (num >= 500) break;
    }
    return xf;
}

// ------------------------------------------------------------------------------ bodies / physics
struct Body {
    double px, py, a, vx, vy, w;
};

// cpMomentForPoly(m, cpBoxShapeNew2 verts) -- evaluated at compile time order, see oracle
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

// One cpSpaceStep(1/60) of the Drone.py body/joint configuration with the two thrusts already
// mapped (drone_2d_env.py:400-406).  B[0] frame, B[1] left motor, B[2] right motor; j[12] the six
// accumulated pivot impulses.  Returns true if the frame box touches any circle after the
// position update (the sticky begin() flag, drone_2d_env.py:17-19).
__device__ __forceinline__ bool space_step(const d2d_scn& s, double damping_dt, Body B[3], double j[12],
                                           double fL, double fR) {
    constexpr double M_F = 0.2, M_M = 0.4;
    constexpr double MI_F = 1.0 / M_F, MI_M = 1.0 / M_M;
    constexpr double II_F = 1.0 / moment_box(M_F, 100.0, 10.0);
    constexpr double II_M = 1.0 / moment_box(M_M, 20.0, 20.0);
    // ---- forces on the frame at local (-40,0) then (40,0): cpBodyApplyForceAtLocalPoint
    double c0 = cos(B[0].a), s0 = sin(B[0].a);
    double fx, fy, tq;
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
    // ---- 1. cpBodyUpdatePosition
    double cs[3], sn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        B[i].px = B[i].px + (B[i].vx + 0.0) * DT;
        B[i].py = B[i].py + (B[i].vy + 0.0) * DT;
        B[i].a = B[i].a + (B[i].w + 0.0) * DT;
        cs[i] = cos(B[i].a);
        sn[i] = sin(B[i].a);
    }
    // ---- 2. collision: CircleToPoly(circle, frame box) contact iff dist(center, box) <= r
    bool hit = false;
    for (int k = 0; k < ((D2D_ABLATE & 8) ? 0 : s.n_circles); ++k) {
        const double dx = s.cx[k] - B[0].px, dy = s.cy[k] - B[0].py;
        const double lx = dx * cs[0] + dy * sn[0];
        const double ly = -dx * sn[0] + dy * cs[0];
        const double ex = lx - clipd(lx, -FRAME_HX, FRAME_HX), ey = ly - clipd(ly, -FRAME_HY, FRAME_HY);
        const double r = s.cr[k];
        hit |= (ex * ex + ey * ey <= r * r);
    }
    // ---- 3. PivotJoint preStep: r1 (motor), r2 (frame), K^-1, bias = -delta/dt
    constexpr double JA[6] = {-7.0, 0.0, 7.0, -7.0, 0.0, 7.0};
    constexpr double JB[6] = {-47.0, -40.0, -33.0, 33.0, 40.0, 47.0};
    const double bias_coef = -(1.0 - 0.0) / DT;  // error_bias = 0 -> 1 - 0^dt = 1
    double r1x[6], r1y[6], r2x[6], r2y[6], ka[6], kb[6], kc[6], kd[6], bx[6], by[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int m = k < 3 ? 1 : 2;
        r1x[k] = cs[m] * JA[k] + (-sn[m]) * 0.0;
        r1y[k] = sn[m] * JA[k] + cs[m] * 0.0;
        r2x[k] = cs[0] * JB[k] + (-sn[0]) * 0.0;
        r2y[k] = sn[0] * JB[k] + cs[0] * 0.0;
        const double m_sum = MI_M + MI_F;
        double k11 = m_sum, k12 = 0.0, k21 = 0.0, k22 = m_sum;
        const double r1xsq = r1x[k] * r1x[k] * II_M, r1ysq = r1y[k] * r1y[k] * II_M;
        const double r1nxy = -r1x[k] * r1y[k] * II_M;
        k11 += r1ysq; k12 += r1nxy; k21 += r1nxy; k22 += r1xsq;
        const double r2xsq = r2x[k] * r2x[k] * II_F, r2ysq = r2y[k] * r2y[k] * II_F;
        const double r2nxy = -r2x[k] * r2y[k] * II_F;
        k11 += r2ysq; k12 += r2nxy; k21 += r2nxy; k22 += r2xsq;
        const double det = k11 * k22 - k12 * k21;
        const double det_inv = 1.0 / det;
        ka[k] = k22 * det_inv; kb[k] = -k12 * det_inv; kc[k] = -k21 * det_inv; kd[k] = k11 * det_inv;
        const double dx = (B[0].px + r2x[k]) - (B[m].px + r1x[k]);
        const double dy = (B[0].py + r2y[k]) - (B[m].py + r1y[k]);
        bx[k] = dx * bias_coef;
        by[k] = dy * bias_coef;
    }
    // ---- 4. cpBodyUpdateVelocity (gravity, damping^dt, forces on the frame only)
    B[0].vx = B[0].vx * damping_dt + (0.0 + fx * MI_F) * DT;
    B[0].vy = B[0].vy * damping_dt + (GRAV_Y + fy * MI_F) * DT;
    B[0].w = B[0].w * damping_dt + tq * II_F * DT;
#pragma unroll
    for (int i = 1; i < 3; ++i) {
        B[i].vx = B[i].vx * damping_dt + (0.0 + 0.0 * MI_M) * DT;
        B[i].vy = B[i].vy * damping_dt + (GRAV_Y + 0.0 * MI_M) * DT;
        B[i].w = B[i].w * damping_dt + 0.0 * II_M * DT;
    }
    // ---- 5. applyCachedImpulse (dt_coef = 1; after a reset jAcc = 0 so dt_coef = 0 is identical)
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int m = k < 3 ? 1 : 2;
        const double jx = j[2 * k] * 1.0, jy = j[2 * k + 1] * 1.0;
        B[m].vx = B[m].vx + (-jx) * MI_M;
        B[m].vy = B[m].vy + (-jy) * MI_M;
        B[m].w += II_M * (r1x[k] * (-jy) - r1y[k] * (-jx));
        B[0].vx = B[0].vx + jx * MI_F;
        B[0].vy = B[0].vy + jy * MI_F;
        B[0].w += II_F * (r2x[k] * jy - r2y[k] * jx);
    }
    // ---- 6. 10 Gauss-Seidel iterations over the joints in space.add order
    for (int it = 0; it < ((D2D_ABLATE & 4) ? 0 : 10); ++it) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int m = k < 3 ? 1 : 2;
            const double v1x = B[m].vx + (-r1y[k]) * B[m].w, v1y = B[m].vy + r1x[k] * B[m].w;
            const double v2x = B[0].vx + (-r2y[k]) * B[0].w, v2y = B[0].vy + r2x[k] * B[0].w;
            const double ux = bx[k] - (v2x - v1x), uy = by[k] - (v2y - v1y);
            double jx = ux * ka[k] + uy * kb[k];
            double jy = ux * kc[k] + uy * kd[k];
            const double ox = j[2 * k], oy = j[2 * k + 1];
            const double nx = ox + jx, ny = oy + jy;
            j[2 * k] = nx;
            j[2 * k + 1] = ny;
            jx = nx - ox;
            jy = ny - oy;
            B[m].vx = B[m].vx + (-jx) * MI_M;
            B[m].vy = B[m].vy + (-jy) * MI_M;
            B[m].w += II_M * (r1x[k] * (-jy) - r1y[k] * (-jx));
            B[0].vx = B[0].vx + jx * MI_F;
            B[0].vy = B[0].vy + jy * MI_F;
            B[0].w += II_F * (r2x[k] * jy - r2y[k] * jx);
        }
    }
    return hit;
}

// ------------------------------------------------------------------------------ observation
// get_observation (drone_2d_env.py:631-773) for frame body F; may set the sticky LA lock.
__device__ __forceinline__ void observe(const d2d_cfg& cfg, const d2d_scn& s, const Body& F, uint32_t& flags,
                                        double obs[D2D_OBS_DIM]) {
    const double W = cfg.screen_w, H = cfg.screen_h;
    const double x = F.px, y = F.py, al = F.a;
    obs[0] = m1to1(F.vx, -1330.0, 1330.0);
    obs[1] = m1to1(F.vy, -1330.0, 1330.0);
    obs[2] = clipd(F.w / 11.7, -1.0, 1.0);
    obs[3] = al / PI;
    obs[4] = m1to1(s.wp_last_x - x, 0.0, W);
    obs[5] = m1to1(s.wp_last_y - y, 0.0, H);
    obs[6] = m1to1(x, 0.0, W);
    obs[7] = m1to1(y, 0.0, H);
    // k = 3 nearest circles by min over the UNROTATED frame vertices (+-50, +-5) of |v+p-c| - r;
    // sqrt is monotone and correctly rounded, so sqrt(min d^2) - r == min(sqrt(d^2) - r) bitwise.
    double bd0 = 0.0, bd1 = 0.0, bd2 = 0.0;
    int bi0 = -1, bi1 = -1, bi2 = -1;
    const int nc = s.n_circles;
    for (int i = 0; i < ((D2D_ABLATE & 2) ? 0 : nc); ++i) {
        const double cx = s.cx[i], cy = s.cy[i];
        const double ax = (50.0 + x) - cx, bxx = (-50.0 + x) - cx;
        const double ay = (-5.0 + y) - cy, byy = (5.0 + y) - cy;
        const double ax2 = ax * ax, bx2 = bxx * bxx, ay2 = ay * ay, by2 = byy * byy;
        // vertex order (50,-5), (50,5), (-50,5), (-50,-5)
        const double q0 = ax2 + ay2, q1 = ax2 + by2, q2 = bx2 + by2, q3 = bx2 + ay2;
        double q = q0;
        q = (q1 < q) ? q1 : q;
        q = (q2 < q) ? q2 : q;
        q = (q3 < q) ? q3 : q;
        const double d = sqrt(q) - s.cr[i];
        // stable ascending insertion into the top-3
        if (bi0 < 0 || d < bd0) {
            bd2 = bd1; bi2 = bi1; bd1 = bd0; bi1 = bi0; bd0 = d; bi0 = i;
        } else if (bi1 < 0 || d < bd1) {
            bd2 = bd1; bi2 = bi1; bd1 = d; bi1 = i;
        } else if (bi2 < 0 || d < bd2) {
            bd2 = d; bi2 = i;
        }
    }
    const double diag = sqrt(W * W + H * H);
    {
        const double bd[3] = {bd0, bd1, bd2};
        const int bi[3] = {bi0, bi1, bi2};
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
            if (bi[jj] >= 0) {
                obs[8 + 3 * jj] = m1to1(bd[jj], 0.0, diag);
                const double ang = ssa(atan2(y - s.cy[bi[jj]], x - s.cx[bi[jj]]) - al - PI);
                obs[9 + 3 * jj] = sin(ang);
                obs[10 + 3 * jj] = cos(ang);
            } else {
                obs[8 + 3 * jj] = 1.0;
                obs[9 + 3 * jj] = 0.0;
                obs[10 + 3 * jj] = 0.0;
            }
        }
    }
    const double vab = ssa(atan2(F.vy, F.vx) - al);
    obs[17] = sin(vab);
    obs[18] = cos(vab);
    // closest point and lookahead: get_closest_u is evaluated once (the reference calls it twice
    // with identical input, predef_path.py:255 and :261)
    const double u = (D2D_ABLATE & 1) ? clipd(x - 100.0, -10.0, s.us[s.n_wps - 1]) : closest_u(s, x, y);
    double cpx, cpy;
    path_eval(s, u, cpx, cpy);
    obs[19] = m1to1(cpx, 0.0, W);
    obs[20] = m1to1(cpy, 0.0, H);
    const double L = s.us[s.n_wps - 1];
    const double ula = (u + cfg.lookahead > L) ? L : u + cfg.lookahead;
    double lax, lay;
    path_eval(s, ula, lax, lay);
    if (fabs(lax - s.wp_last_x) < 10.0 && fabs(lay - s.wp_last_y) < 10.0) flags |= D2D_FLAG_LA_LOCK;
    if (flags & D2D_FLAG_LA_LOCK) {
        lax = s.wp_last_x;
        lay = s.wp_last_y;
    }
    obs[21] = m1to1(lax, 0.0, W);
    obs[22] = m1to1(lay, 0.0, H);
    const double ca = cos(al), sa = sin(al);
    // np.matmul(R_w_b(alpha), d): row r = fma(R[r][0], d0, R[r][1] * d1)
    double dx = lax - x, dy = lay - y;
    double bxv = fma(ca, dx, (-sa) * dy), byv = fma(sa, dx, ca * dy);
    const double laa = ssa(atan2(byv, bxv) - al);
    obs[23] = sin(laa);
    obs[24] = cos(laa);
    dx = cpx - x;
    dy = cpy - y;
    bxv = fma(ca, dx, (-sa) * dy);
    byv = fma(sa, dx, ca * dy);
    const double cpa = ssa(atan2(byv, bxv) - al);
    obs[25] = sin(cpa);
    obs[26] = cos(cpa);
}

// ------------------------------------------------------------------------------ reward
struct Reward {
    double reward, ca, pa, pp, coll, reach, aa, dclose, dist_path;
    int cause;
};
// drone_2d_env.py:423-572 -- decodes from the (fp64) observation exactly as the reference does
__device__ __forceinline__ Reward reward_fn(const d2d_cfg& cfg, const d2d_scn& s, const double* obs,
                                            bool collided, int t) {
    const double W = cfg.screen_w, H = cfg.screen_h;
    Reward R;
    const double vxd = invm1to1(obs[0], -1330.0, 1330.0);
    const double vyd = invm1to1(obs[1], -1330.0, 1330.0);
    const double alpha = obs[3] * PI;
    const double tdx = invm1to1(obs[4], 0.0, W), tdy = invm1to1(obs[5], 0.0, H);
    const double pxd = invm1to1(obs[6], 0.0, W), pyd = invm1to1(obs[7], 0.0, H);
    const double vel_ang = pymod(atan2(obs[17] * PI, obs[18] * PI) + TWO_PI, TWO_PI);
    const double cpx = invm1to1(obs[19], 0.0, W), cpy = invm1to1(obs[20], 0.0, H);
    const double la_ang = pymod(atan2(obs[23], obs[24]) + TWO_PI, TWO_PI);
    double lpa = 1.0, lca = 1.0, ca = 0.0;
    R.dclose = __builtin_inf();
    if (s.n_circles > 0) {
        const double diag = sqrt(W * W + H * H);
        const double d = invm1to1(obs[8], 0.0, diag);
        R.dclose = d;
        const double oa = pymod(atan2(obs[9], obs[10]) + TWO_PI, TWO_PI);
        const double adiff = fabs((pymod(oa - vel_ang + PI, TWO_PI) - PI) * (180.0 / PI));
        const double Rr = cfg.danger_range, A = cfg.danger_angle, k = cfg.abs_inv_ca_min_rew;
        if (d < Rr && cfg.use_lambda) {
            lpa = (d / Rr) / 2.0;
            if (lpa < 0.10) lpa = 0.10;
            lca = 1.0 - lpa;
        }
        if (d < Rr) {
            double rr = -(((Rr + k * Rr) / (d + k * Rr)) - 1.0);
            double ar = -(((A + k * A) / (adiff + k * A)) - 1.0);
            if (ar > 0.0) ar = 0.0;
            if (rr > 0.0) rr = 0.0;
            ca = rr + ar;
        }
    }
    const double dist = norm2(cpx - pxd, cpy - pyd);
    R.dist_path = dist;
    const double pa = -(2.0 * (clipd(dist, 0.0, cfg.pa_band_edge) / cfg.pa_band_edge) - 1.0) * cfg.pa_scale;
    const double vel = sqrt(vxd * vxd + vyd * vyd);
    const double sv = vel * cfg.pp_vel_scale;
    const double vla = fabs(pymod(la_ang - vel_ang + PI, TWO_PI) - PI);
    const double pp = clipd(cos(vla) * sv, cfg.pp_rew_min, cfg.pp_rew_max);
    int cause = 0;
    double coll = 0.0;
    if (collided) {
        coll = cfg.rew_collision;
        cause |= D2D_END_COLLISION;
    }
    double reach = 0.0;
    if (fabs(tdx) < cfg.reach_end_radius && fabs(tdy) < cfg.reach_end_radius) {
        cause |= D2D_END_REACH;
        reach = cfg.rew_reach_end;
    }
    double aa = 0.0;
    if (alpha > cfg.aa_band) aa = -sin(alpha);
    if (alpha < -cfg.aa_band) aa = sin(alpha);
    if (fabs(alpha) >= cfg.aa_angle) {
        aa = cfg.rew_aa;
        cause |= D2D_END_AA;
    }
    if (t == cfg.n_steps) cause |= D2D_END_TIMEUP;
    R.reward = aa + pa * lpa + pp + coll + ca * lca + reach;
    R.ca = ca * lca;
    R.pa = pa * lpa;
    R.pp = pp;
    R.coll = coll;
    R.reach = reach;
    R.aa = aa;
    R.cause = cause;
    return R;
}

}  // namespace d2d
