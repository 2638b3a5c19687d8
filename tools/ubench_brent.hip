// Micro-benchmark (diagnostic, never shipped): cycles per Brent iteration of the path search at a
// controlled number of waves per SIMD, with compile-time knobs that remove pieces of the iteration
// to attribute its cost.  Driven by tools/ubench_brent.py.
//   UB_NOSQRT  distance without the sqrt      UB_NODIV   parabolic step without the division
//   UB_NOIDX   knot index fixed (no compares) UB_NOLDS   coefficients from registers, not LDS
#include "../drone-2d-custom-gym-env-for-reinforcement-learning_amd/csrc/d2d_device.h"

using namespace d2d;

#ifndef UB_NOSQRT
#define UB_NOSQRT 0
#endif
#ifndef UB_NODIV
#define UB_NODIV 0
#endif
#ifndef UB_NOIDX
#define UB_NOIDX 0
#endif

#ifndef UB_REC
#define UB_REC 0
#endif
// per-knot-interval record: B quad (6), A quad (6), u0, u1, 1/(u1-u0), pad
__shared__ double g_rec[D2D_MAX_WPS][16];
__device__ void build_rec(const Scn& s) {
    const int nw = s.n_wps, nseg = nw - 2;
    for (int n = threadIdx.x; n < D2D_MAX_WPS; n += 64) {
        const int b = n < nseg - 1 ? n : nseg - 1;
        const int a = (n == 0) ? nseg - 1 : (n - 1 < nseg - 1 ? n - 1 : nseg - 1);
        double* r = g_rec[n];
        r[0] = s.xa[b]; r[1] = s.xb[b]; r[2] = s.xc[b]; r[3] = s.ya[b]; r[4] = s.yb[b]; r[5] = s.yc[b];
        r[6] = s.xa[a]; r[7] = s.xb[a]; r[8] = s.xc[a]; r[9] = s.ya[a]; r[10] = s.yb[a]; r[11] = s.yc[a];
        const int n1 = n + 1 < D2D_MAX_WPS ? n + 1 : D2D_MAX_WPS - 1;
        r[12] = s.us[n]; r[13] = s.us[n1]; r[14] = s.inv_du[n]; r[15] = 0.0;
    }
}
__device__ __forceinline__ void path_eval_rec(const Scn& s, const PathK& K, double u, double& x, double& y) {
    const int nw = K.nw;
    const int n = u_index(s, u, K.kmax);
    const bool first = (n == 0) & (u >= K.us0);
    const bool last = !first & (((u >= K.last_lo) & (u <= K.L)) | (n == nw - 1));
    const bool blend = !first & !last;
    const double* r = g_rec[n];
    const double uu = u * u;
    const double xB = r[0] * uu + r[1] * u + r[2];
    const double yB = r[3] * uu + r[4] * u + r[5];
    const double xA = r[6] * uu + r[7] * u + r[8];
    const double yA = r[9] * uu + r[10] * u + r[11];
    const double u0 = r[12], u1 = r[13], idu = r[14];
    const double du = u1 - u0;
    const double mu_r = div_by_recip(u - u0, du, idu);
    const double mu_f = div_by_recip(u1 - u, du, idu);
    x = blend ? mu_r * xB + mu_f * xA : xB;
    y = blend ? mu_r * yB + mu_f * yA : yB;
}

__device__ __forceinline__ double ub_dist(const Scn& s, const PathK& K, double u, double px, double py) {
    double x, y;
    if (UB_REC) {
        path_eval_rec(s, K, u, x, y);
    } else if (UB_NOIDX) {
        const double uu = u * u;
        x = s.xa[1] * uu + s.xb[1] * u + s.xc[1];
        y = s.ya[1] * uu + s.yb[1] * u + s.yc[1];
    } else {
        path_eval(s, K, u, x, y);
    }
    const double dx = x - px, dy = y - py;
    return UB_NOSQRT ? fma(dy, dy, dx * dx) : sqrt(fma(dy, dy, dx * dx));
}

__global__ __launch_bounds__(64) void ub_kernel(const Scn* scn, const double* pxy, int n, double* out_u,
                                                long long* cyc, int* iters) {
    __shared__ Scn S;
    {
        const double* src = reinterpret_cast<const double*>(scn);
        double* dst = reinterpret_cast<double*>(&S);
        for (int k = threadIdx.x; k < (int)(sizeof(Scn) / 8); k += 64) dst[k] = src[k];
    }
    __syncthreads();
    if (UB_REC) build_rec(S);
    __syncthreads();
    const int i = (blockIdx.x * 64 + threadIdx.x) % n;
    const double px = pxy[2 * i], py = pxy[2 * i + 1];
    const PathK K = path_k(S);
    const long long t0 = clock64();
    Brent B;
    B.a = 0.0 - 10.0;
    B.b = K.L + 10.0;
    B.fulc = B.a + BR_GOLDEN * (B.b - B.a);
    B.nfc = B.fulc;
    B.xf = B.fulc;
    B.rat = 0.0;
    B.e = 0.0;
    B.fx = ub_dist(S, K, B.xf, px, py);
    B.num = 1;
    B.ffulc = B.fx;
    B.fnfc = B.fx;
    int it = 0;
    while (brent_active(B)) {
        const double a = B.a, b = B.b, xf = B.xf, fx = B.fx, nfc = B.nfc, fulc = B.fulc;
        const double xm = 0.5 * (a + b);
        const double tol1 = BR_SQRT_EPS * fabs(xf) + BR_XATOL3;
        const double tol2 = 2.0 * tol1;
        const double r = (xf - nfc) * (fx - B.ffulc);
        double q = (xf - fulc) * (fx - B.fnfc);
        double p = (xf - fulc) * q - (xf - nfc) * r;
        q = 2.0 * (q - r);
        p = (q > 0.0) ? -p : p;
        q = fabs(q);
        const bool par = (fabs(B.e) > tol1) & (fabs(p) < fabs(0.5 * q * B.e)) & (p > q * (a - xf)) & (p < q * (b - xf));
        double rat_p = UB_NODIV ? (p + 0.0) * q : (p + 0.0) / q;
        const double xp = xf + rat_p;
        rat_p = (((xp - a) < tol2) | ((b - xp) < tol2)) ? tol1 * sgn_nz(xm - xf) : rat_p;
        const double e_g = (xf >= xm) ? a - xf : b - xf;
        const double rat_g = BR_GOLDEN * e_g;
        B.e = par ? B.rat : e_g;
        const double rat = par ? rat_p : rat_g;
        B.rat = rat;
        const double ar = fabs(rat);
        const double mx = (ar != ar) ? ar : (ar > tol1 ? ar : tol1);
        const double x = xf + sgn_nz(rat) * mx;
        const double fu = ub_dist(S, K, x, px, py);
        B.num += 1;
        const bool le = fu <= fx;
        const bool c1 = !le & ((fu <= B.fnfc) | (nfc == xf));
        const bool c2 = !le & !c1 & ((fu <= B.ffulc) | (fulc == xf) | (fulc == nfc));
        B.a = le ? ((x >= xf) ? xf : a) : ((x < xf) ? x : a);
        B.b = le ? ((x >= xf) ? b : xf) : ((x < xf) ? b : x);
        const double nfulc = (le | c1) ? nfc : (c2 ? x : fulc);
        const double nffulc = (le | c1) ? B.fnfc : (c2 ? fu : B.ffulc);
        const double nnfc = le ? xf : (c1 ? x : nfc);
        const double nfnfc = le ? fx : (c1 ? fu : B.fnfc);
        B.fulc = nfulc;
        B.ffulc = nffulc;
        B.nfc = nnfc;
        B.fnfc = nfnfc;
        B.xf = le ? x : xf;
        B.fx = le ? fu : fx;
        ++it;
    }
    const long long t1 = clock64();
    out_u[blockIdx.x * 64 + threadIdx.x] = B.xf;
    // per wave: cycles and the wave's iteration count (max over lanes)
    int itmax = it;
    for (int off = 32; off > 0; off >>= 1) itmax = max(itmax, __shfl_xor(itmax, off));
    if (threadIdx.x == 0) {
        cyc[blockIdx.x] = t1 - t0;
        iters[blockIdx.x] = itmax;
    }
}

extern "C" int ub_run(const d2d_scn* scn_host, int nblocks, const double* pxy_host, int n, double* out_u_host,
                      long long* cyc_host, int* iters_host) {
    Scn s;
    static_cast<d2d_scn&>(s) = *scn_host;
    scn_derive(s);
    Scn* d_s;
    double *d_p, *d_u;
    long long* d_c;
    int* d_i;
    if (hipMalloc(&d_s, sizeof(Scn)) || hipMalloc(&d_p, sizeof(double) * 2 * n) ||
        hipMalloc(&d_u, sizeof(double) * 64 * nblocks) || hipMalloc(&d_c, sizeof(long long) * nblocks) ||
        hipMalloc(&d_i, sizeof(int) * nblocks))
        return 1;
    hipMemcpy(d_s, &s, sizeof(Scn), hipMemcpyHostToDevice);
    hipMemcpy(d_p, pxy_host, sizeof(double) * 2 * n, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(ub_kernel, dim3(nblocks), dim3(64), 0, 0, d_s, d_p, n, d_u, d_c, d_i);
    if (hipDeviceSynchronize()) return 2;
    hipMemcpy(out_u_host, d_u, sizeof(double) * 64 * nblocks, hipMemcpyDeviceToHost);
    hipMemcpy(cyc_host, d_c, sizeof(long long) * nblocks, hipMemcpyDeviceToHost);
    hipMemcpy(iters_host, d_i, sizeof(int) * nblocks, hipMemcpyDeviceToHost);
    hipFree(d_s); hipFree(d_p); hipFree(d_u); hipFree(d_c); hipFree(d_i);
    return 0;
}
