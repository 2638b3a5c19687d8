// Placement probe (diagnostic, never shipped): where the 8 waves of a 512-thread workgroup land when
// two such workgroups share a CU (the LDS footprint allows two per CU), read from HW_ID / XCC_ID.
// Question for a two-group K1 workgroup with per-SIMD role assignment: does each workgroup put
// exactly two waves on every SIMD, and do the two workgroups of a CU see different TG_ID parities?
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_place2 tools/ubench_place2.hip && ./tools/ubench_place2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

__global__ __launch_bounds__(512) void probe(unsigned* out, int spin) {
    __shared__ double pad[9000];  // 72 KB: two workgroups per CU
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID, 32 bits
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);   // HW_REG_XCC_ID, 4 bits
    if ((threadIdx.x & 63) == 0) {
        const unsigned w = threadIdx.x >> 6;
        out[(blockIdx.x * 8 + w) * 2 + 0] = hw;
        out[(blockIdx.x * 8 + w) * 2 + 1] = xcc;
    }
    pad[threadIdx.x] = (double)threadIdx.x;
    // keep every workgroup resident long enough that the whole grid is co-resident
    long long t0 = clock64();
    while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(10);
    __syncthreads();
    if (pad[(threadIdx.x + 1) % 512] < -1.0) out[0] = 0;
}

int main(int argc, char** argv) {
    const int nb = argc > 1 ? atoi(argv[1]) : 512;
    unsigned* d;
    hipMalloc(&d, sizeof(unsigned) * nb * 16);
    hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 0, 0, d, 200000);
    hipDeviceSynchronize();
    std::vector<unsigned> h(nb * 16);
    hipMemcpy(h.data(), d, sizeof(unsigned) * nb * 16, hipMemcpyDeviceToHost);
    // HW_ID (gfx9): wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13, tg 19:16
    int two_per_simd = 0, tg_par_differ = 0, cu_pairs = 0;
    std::map<unsigned, std::vector<int>> cu_blocks;
    for (int b = 0; b < nb; ++b) {
        int cnt[4] = {0, 0, 0, 0};
        for (int w = 0; w < 8; ++w) cnt[(h[(b * 8 + w) * 2] >> 4) & 3]++;
        two_per_simd += (cnt[0] == 2 && cnt[1] == 2 && cnt[2] == 2 && cnt[3] == 2);
        const unsigned hw = h[b * 16], xcc = h[b * 16 + 1];
        const unsigned cu = ((hw >> 8) & 15) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5) | (xcc << 8);
        cu_blocks[cu].push_back(b);
    }
    for (auto& kv : cu_blocks) {
        if (kv.second.size() != 2) continue;
        ++cu_pairs;
        const unsigned t0 = (h[kv.second[0] * 16] >> 16) & 15, t1 = (h[kv.second[1] * 16] >> 16) & 15;
        tg_par_differ += ((t0 ^ t1) & 1) != 0;
    }
    printf("{\"blocks\": %d, \"cus\": %zu, \"two_waves_per_simd\": %d, \"cus_with_two_blocks\": %d, "
           "\"tg_parity_differs\": %d, \"block0_simds\": [", nb, cu_blocks.size(), two_per_simd, cu_pairs, tg_par_differ);
    for (int w = 0; w < 8; ++w) printf("%u%s", (h[w * 2] >> 4) & 3, w < 7 ? ", " : "");
    printf("], \"block0_tg\": %u}\n", (h[0] >> 16) & 15);
    return 0;
}
