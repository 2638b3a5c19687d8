// Micro-benchmark (diagnostic, never shipped): cycles per iteration of the product's Brent path
// search (d2d_device.h brent_step / path_eval) at a controlled number of waves per SIMD.
// Driven by tools/ubench_brent.py; compile-time variants of the product code are passed as -D.
// (Earlier variants that located the cost -- LDS coefficient gathers and the knot-count compares
// -- are recorded in profiles/r01/v3_ubench_brent*.json.)
#include "../drone-2d-custom-gym-env-for-reinforcement-learning_amd/csrc/d2d_device.h"

using namespace d2d;

__global__ __launch_bounds__(64) void ub_kernel(const Scn* scn, const double* pxy, int n, double* out_u,
                                                long long* cyc, int* iters) {
    __shared__ Scn S;
    {
        const double* src = reinterpret_cast<const double*>(scn);
        double* dst = reinterpret_cast<double*>(&S);
        for (int k = threadIdx.x; k < (int)(sizeof(Scn) / 8); k += 64) dst[k] = src[k];
    }
    __syncthreads();
    const int i = (blockIdx.x * 64 + threadIdx.x) % n;
    const double px = pxy[2 * i], py = pxy[2 * i + 1];
    const PathK K = path_k(S);
    const long long t0 = clock64();
    Brent B;
    brent_init(S, K, px, py, B);
    int it = 0;
#ifdef UB_INLINE
    // same iteration as brent_step, written out in the kernel (compiler-scheduling comparison)
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
        double rat_p = div_normal(p + 0.0, q);
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
        const double fu = path_dist(S, K, x, px, py);
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
#endif
    while (brent_active(B)) {
        brent_step(S, K, px, py, B);
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
    if (!scn_build(*scn_host, s)) return 3;
    Scn* d_s;
    double *d_p, *d_u;
    long long* d_c;
    int* d_i;
    if (hipMalloc(&d_s, sizeof(Scn)) || hipMalloc(&d_p, sizeof(double) * 2 * n) ||
        hipMalloc(&d_u, sizeof(double) * 64 * nblocks) || hipMalloc(&d_c, sizeof(long long) * nblocks) ||
        hipMalloc(&d_i, sizeof(int) * nblocks))
        return 1;
    int bad = 0;
    bad |= hipMemcpy(d_s, &s, sizeof(Scn), hipMemcpyHostToDevice);
    bad |= hipMemcpy(d_p, pxy_host, sizeof(double) * 2 * n, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(ub_kernel, dim3(nblocks), dim3(64), 0, 0, d_s, d_p, n, d_u, d_c, d_i);
    bad |= hipDeviceSynchronize();
    bad |= hipMemcpy(out_u_host, d_u, sizeof(double) * 64 * nblocks, hipMemcpyDeviceToHost);
    bad |= hipMemcpy(cyc_host, d_c, sizeof(long long) * nblocks, hipMemcpyDeviceToHost);
    bad |= hipMemcpy(iters_host, d_i, sizeof(int) * nblocks, hipMemcpyDeviceToHost);
    bad |= hipFree(d_s) | hipFree(d_p) | hipFree(d_u) | hipFree(d_c) | hipFree(d_i);
    return bad ? 2 : 0;
}
