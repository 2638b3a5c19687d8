// Micro-benchmark (diagnostic, never shipped): what FETCH_SIZE / WRITE_SIZE report for the access
// widths d2d_step_kernel uses, against the bytes each kernel moves by construction.  VERDICT r04
// item 6: the traffic JSON doubles FETCH_SIZE (MI355X_MICROARCH.md, for 16-B/lane streaming reads);
// K1's state loads are 8 B per lane (fp64 SoA), its obs rows 4-B floats staged into 16-B stores,
// its flags 1 B per lane.  Each kernel below moves a known number of bytes at one of those widths;
// tools/ubench_traffic.sh runs it under one rocprofv3 --pmc pass per counter.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_traffic tools/ubench_traffic.hip
//   ./tools/ubench_traffic [envs]        (prints the algorithmic bytes of every launch)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// F fp64 fields of a [F][n] SoA array, 8 B per lane (K1's state loads); one fp64 written per lane
__global__ __launch_bounds__(256) void rd_f64_soa(const double* src, int F, int n, double* out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double s = 0.0;
    for (int f = 0; f < F; ++f) s += src[(size_t)f * n + i];
    out[i] = s;
}
// the same bytes as 16 B per lane (double2 over [F/2][n] pairs)
__global__ __launch_bounds__(256) void rd_f64x2(const double2* src, int F2, int n, double* out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double s = 0.0;
    for (int f = 0; f < F2; ++f) {
        const double2 v = src[(size_t)f * n + i];
        s += v.x + v.y;
    }
    out[i] = s;
}
// int32 fields SoA read (K1's t / flags / episode counter loads)
__global__ __launch_bounds__(256) void rd_i32_soa(const int* src, int F, int n, int* out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int s = 0;
    for (int f = 0; f < F; ++f) s += src[(size_t)f * n + i];
    out[i] = s;
}
// F fp64 fields written SoA (K1's state stores)
__global__ __launch_bounds__(256) void wr_f64_soa(double* dst, int F, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    for (int f = 0; f < F; ++f) dst[(size_t)f * n + i] = (double)(f + i);
}
// int32 fields SoA (t, flags)
__global__ __launch_bounds__(256) void wr_i32_soa(int* dst, int F, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    for (int f = 0; f < F; ++f) dst[(size_t)f * n + i] = f + i;
}
// one f32 per lane (reward)
__global__ __launch_bounds__(256) void wr_f32(float* dst, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = (float)i;
}
// one byte per lane (terminated / truncated)
__global__ __launch_bounds__(256) void wr_u8(unsigned char* dst, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) dst[i] = (unsigned char)(i & 1);
}
// 64 rows x 27 f32 per 64 lanes as contiguous float4 stores (K1's obs tile epilogue)
__global__ __launch_bounds__(256) void wr_obs_tile(float4* dst, int n) {
    const int words4 = 64 * 27 / 4;  // 432 float4 per 64-env tile
    const int tile = blockIdx.x, tiles = n / 64;
    if (tile >= tiles) return;
    for (int k = threadIdx.x; k < words4; k += 256)
        dst[(size_t)tile * words4 + k] = make_float4((float)k, (float)tile, 0.f, 1.f);
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 65536;
    const int F = 32;  // K1's state: 32 fp64 fields
    double *st, *out;
    int* ist;
    float *rew, *obs;
    unsigned char* u8;
    CK(hipMalloc(&st, sizeof(double) * F * n));
    CK(hipMalloc(&out, sizeof(double) * n));
    CK(hipMalloc(&ist, sizeof(int) * 2 * n));
    CK(hipMalloc(&rew, sizeof(float) * n));
    CK(hipMalloc(&obs, sizeof(float) * 27 * n));
    CK(hipMalloc(&u8, n));
    int *ist3, *iout;
    CK(hipMalloc(&ist3, sizeof(int) * 3 * n));
    CK(hipMalloc(&iout, sizeof(int) * n));
    CK(hipMemset(ist3, 0, sizeof(int) * 3 * n));
    CK(hipMemset(st, 0, sizeof(double) * F * n));
    const dim3 g((n + 255) / 256), b(256);
    for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(rd_f64_soa, g, b, 0, 0, st, F, n, out);
        hipLaunchKernelGGL(rd_f64x2, g, b, 0, 0, (const double2*)st, F / 2, n, out);
        hipLaunchKernelGGL(wr_f64_soa, g, b, 0, 0, st, F, n);
        hipLaunchKernelGGL(wr_i32_soa, g, b, 0, 0, ist, 2, n);
        hipLaunchKernelGGL(rd_i32_soa, g, b, 0, 0, ist3, 3, n, iout);
        hipLaunchKernelGGL(wr_f32, g, b, 0, 0, rew, n);
        hipLaunchKernelGGL(wr_u8, g, b, 0, 0, u8, n);
        hipLaunchKernelGGL(wr_obs_tile, dim3(n / 64), b, 0, 0, (float4*)obs, n);
    }
    CK(hipDeviceSynchronize());
    printf("{\"envs\": %d, \"rd_f64_soa\": {\"read\": %zu, \"write\": %zu}, \"rd_f64x2\": {\"read\": %zu, \"write\": %zu}, "
           "\"wr_f64_soa\": {\"write\": %zu}, \"wr_i32_soa\": {\"write\": %zu}, \"wr_f32\": {\"write\": %zu}, "
           "\"wr_u8\": {\"write\": %zu}, \"wr_obs_tile\": {\"write\": %zu}, "
           "\"rd_i32_soa\": {\"read\": %zu, \"write\": %zu}}\n",
           n, sizeof(double) * F * n, sizeof(double) * n, sizeof(double) * F * n, sizeof(double) * n,
           sizeof(double) * F * n, sizeof(int) * 2 * (size_t)n, sizeof(float) * (size_t)n, (size_t)n,
           sizeof(float) * 27 * (size_t)n, sizeof(int) * 3 * (size_t)n, sizeof(int) * (size_t)n);
    return 0;
}
