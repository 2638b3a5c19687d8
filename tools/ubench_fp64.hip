// Micro-benchmark (diagnostic): fp64 dependent-chain latency vs independent throughput at one
// wave per SIMD, LDS broadcast-read latency, and the shader clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_chain(double* out, long long* cyc, int iters, double x0, int mode) {
    double a = x0 + threadIdx.x, b = a * 1.5, c = a * 0.5, d = a + 2.0;
    long long t0 = clock64();
    long long r0 = wall_clock64();
    if (mode == 0) {          // one dependent chain of adds
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 16; ++k) a = a + 1e-9;
        }
    } else if (mode == 1) {   // four independent chains
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) { a = a + 1e-9; b = b + 1e-9; c = c + 1e-9; d = d + 1e-9; }
        }
    } else if (mode == 2) {   // dependent fma chain
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 16; ++k) a = fma(a, 1.0000001, 1e-9);
        }
    } else if (mode == 3) {   // dependent division chain
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) a = (a + 1.0) / (a + 0.5);
        }
    } else if (mode == 4) {   // dependent sqrt chain
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) a = sqrt(a + 1.0);
        }
    } else if (mode == 5) {   // dependent sin chain
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) a = sin(a) + 1.0;
        }
    } else if (mode == 6) {   // dependent atan2 chain
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) a = atan2(a, b) + 1.0;
        }
    } else if (mode == 7) {   // dependent fmod chain
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) a = fmod(a + 7.0, 6.283185307179586);
        }
    }
    long long t1 = clock64();
    long long r1 = wall_clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
    if (threadIdx.x == 0 && blockIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

int main() {
    double* out; long long* cyc;
    hipMalloc(&out, 256 * 1024 * sizeof(double));
    hipMalloc(&cyc, 2 * sizeof(long long));
    const char* names[] = {"add dep x16", "add 4 chains x4", "fma dep x16", "div dep x4", "sqrt dep x4",
                           "sin dep x4", "atan2 dep x4", "fmod dep x4"};
    const int per[] = {16, 16, 16, 4, 4, 4, 4, 4};
    int wclk = 0;
    hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0);
    for (int blocks : {256, 1024}) {
        for (int mode = 0; mode < 8; ++mode) {
            int iters = 2000;
            hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 1.0, mode);
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 1.0, mode);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            long long h[2]; hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
            double n_ops = (double)iters * per[mode];
            double ghz = (double)h[0] / ((double)h[1] / (wclk * 1e3)) / 1e9;
            printf("blocks=%4d %-16s cycles/op=%7.2f  clock=%.2f GHz  kernel=%.3f ms\n", blocks, names[mode],
                   h[0] / n_ops, ghz, ms);
        }
    }
    return 0;
}
