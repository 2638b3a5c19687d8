// Micro-benchmark (diagnostic, never shipped): cycles per Brent step of the product's plain
// closest-point search (d2d_device.h: brent_init + brent_run over a scenario staged in LDS) for one
// wave alone on its SIMD -- the latency the small batch's path wave runs its continuation at.
// Compile-time variants of the product code are passed as -D.  Driven by tools/ubench_step.py:
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared \
//         -I include -o tools/_abl/libub_step.so tools/ubench_step.hip
#include "../drone-2d-custom-gym-env-for-reinforcement-learning_amd/csrc/d2d_device.h"

using namespace d2d;

__global__ __launch_bounds__(64) void ub_search(const ScnF* scn, const double* pts, int n, double* out_u,
                                                unsigned long long* cyc, int* steps) {
    __shared__ ScnF S;
    {
        const double* src = reinterpret_cast<const double*>(scn);
        double* dst = reinterpret_cast<double*>(&S);
        for (int k = threadIdx.x; k < (int)(sizeof(ScnF) / 8); k += 64) dst[k] = src[k];
    }
    __syncthreads();
    const int i = (blockIdx.x * 64 + threadIdx.x) % n;
    const double px = pts[2 * i], py = pts[2 * i + 1];
    const PathK K = path_k(S);
    Brent B;
    brent_init(S, K, px, py, B);
    double xf0 = B.fx;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : "+v"(xf0));
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    brent_run(S, K, px, py, B);
    double xf = B.xf;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : "+v"(xf));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    // untimed: the lane's step count (the same loop, counting its passes)
    Brent C;
    brent_init(S, K, px, py, C);
    int it = 0;
    while (brent_open(C) && it < 500) {
        brent_step(S, K, px, py, C);
        ++it;
    }
    out_u[blockIdx.x * 64 + threadIdx.x] = xf + 0.0 * xf0;
    steps[blockIdx.x * 64 + threadIdx.x] = it;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

extern "C" int ub_run(const d2d_scn* src, const double* pts, int n, int waves, double* out_u,
                      unsigned long long* cyc, int* steps) {
    ScnF h;
    if (!scn_build(*src, h)) return -1;
    ScnF* d_s = nullptr;
    double *d_p = nullptr, *d_u = nullptr;
    unsigned long long* d_c = nullptr;
    int* d_n = nullptr;
    if (hipMalloc(&d_s, sizeof(ScnF)) != hipSuccess || hipMalloc(&d_p, sizeof(double) * 2 * n) != hipSuccess ||
        hipMalloc(&d_u, sizeof(double) * 64 * waves) != hipSuccess ||
        hipMalloc(&d_c, sizeof(unsigned long long) * waves) != hipSuccess ||
        hipMalloc(&d_n, sizeof(int) * 64 * waves) != hipSuccess)
        return -2;
    (void)hipMemcpy(d_s, &h, sizeof(ScnF), hipMemcpyHostToDevice);
    (void)hipMemcpy(d_p, pts, sizeof(double) * 2 * n, hipMemcpyHostToDevice);
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(ub_search, dim3(waves), dim3(64), 0, 0, d_s, d_p, n, d_u, d_c, d_n);
    if (hipDeviceSynchronize() != hipSuccess) return -3;
    (void)hipMemcpy(out_u, d_u, sizeof(double) * 64 * waves, hipMemcpyDeviceToHost);
    (void)hipMemcpy(cyc, d_c, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost);
    (void)hipMemcpy(steps, d_n, sizeof(int) * 64 * waves, hipMemcpyDeviceToHost);
    (void)hipFree(d_n);
    (void)hipFree(d_s);
    (void)hipFree(d_p);
    (void)hipFree(d_u);
    (void)hipFree(d_c);
    return 0;
}
