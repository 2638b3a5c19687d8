// Wave placement probe (diagnostic, not product): for a workgroup of NW waves with enough LDS that
// only K workgroups fit on a CU, which SIMD does each wave land on, and how do the K co-resident
// workgroups of a CU relate?  Every wave records XCC_ID << 32 | HW_ID (wave [3:0], simd [5:4],
// cu [11:8], sh [12], se [15:13], tg [19:16]) and spins until the whole grid is resident.
//   hipcc --offload-arch=gfx950 -O2 -o tools/ubench_place tools/ubench_place.hip && ./tools/ubench_place
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <string>
#include <vector>

__global__ void probe(unsigned long long* out, unsigned int* arrived, int total_waves) {
    extern __shared__ int lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
    lds[threadIdx.x] = (int)hw;
    if (lane == 0) {
        out[(size_t)blockIdx.x * (blockDim.x >> 6) + wave] = ((unsigned long long)xcc << 32) | hw;
        __hip_atomic_fetch_add(arrived, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // spin (bounded) until every wave of the grid has arrived: all co-resident
    for (int it = 0; it < 200000; ++it) {
        unsigned v = __hip_atomic_load(arrived, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_readfirstlane(v) >= (unsigned)total_waves) break;
        __builtin_amdgcn_s_sleep(8);
    }
    __syncthreads();
    if (lds[(threadIdx.x + 64) % blockDim.x] == -1) out[0] = 0;  // keep the LDS allocation
}

static void run(int nw, int per_cu, int n_cu) {
    const int grid = per_cu * n_cu;
    const size_t lds = (160 * 1024) / per_cu - 1024;
    unsigned long long* d = nullptr;
    unsigned int* arr = nullptr;
    (void)hipMalloc(&d, sizeof(unsigned long long) * grid * nw);
    (void)hipMalloc(&arr, sizeof(unsigned));
    (void)hipMemset(arr, 0, sizeof(unsigned));
    hipLaunchKernelGGL(probe, dim3(grid), dim3(64 * nw), lds, 0, d, arr, grid * nw);
    hipError_t e = hipDeviceSynchronize();
    std::vector<unsigned long long> h((size_t)grid * nw);
    (void)hipMemcpy(h.data(), d, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost);
    unsigned got = 0;
    (void)hipMemcpy(&got, arr, sizeof(unsigned), hipMemcpyDeviceToHost);
    printf("=== NW=%d per_cu=%d grid=%d lds=%zu: %s, arrived %u/%d\n", nw, per_cu, grid, lds, hipGetErrorString(e), got,
           grid * nw);
    // per CU: the workgroups on it, each as its SIMD sequence; histogram of CU patterns
    std::map<unsigned long long, std::vector<std::pair<int, std::string>>> cus;
    std::map<std::string, int> wg_pat;
    for (int b = 0; b < grid; ++b) {
        std::string s;
        unsigned long long key = 0;
        int tg = 0;
        for (int w = 0; w < nw; ++w) {
            const unsigned long long v = h[(size_t)b * nw + w];
            const unsigned hw = (unsigned)v, xcc = (unsigned)(v >> 32) & 0xF;
            s += (char)('0' + ((hw >> 4) & 3));
            key = ((unsigned long long)xcc << 16) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF);
            tg = (hw >> 16) & 0xF;
        }
        cus[key].push_back({b, s});
        wg_pat[s]++;
        (void)tg;
    }
    printf("distinct CUs %zu\n", cus.size());
    std::map<std::string, int> cu_pat;
    for (auto& kv : cus) {
        std::string p;
        for (auto& x : kv.second) p += x.second + " ";
        cu_pat[p]++;
    }
    int shown = 0;
    for (auto& kv : wg_pat) {
        if (shown++ < 12) printf("  wg simd seq %s : %d\n", kv.first.c_str(), kv.second);
    }
    shown = 0;
    for (auto& kv : cu_pat) {
        if (shown++ < 16) printf("  cu pattern [%s] : %d\n", kv.first.c_str(), kv.second);
    }
    printf("  (%zu cu patterns)\n", cu_pat.size());
    (void)hipFree(d);
    (void)hipFree(arr);
}

int main() {
    int n_cu = 0;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d\n", n_cu);
    run(4, 4, n_cu);
    run(8, 2, n_cu);
    run(6, 2, n_cu);
    run(12, 1, n_cu);
    run(16, 1, n_cu);
    run(8, 1, n_cu);
    return 0;
}
