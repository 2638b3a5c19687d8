// Micro-benchmark (diagnostic, never shipped): issue-to-issue cycles of the instruction kinds the Brent
// continuation's dependency chain is made of, for ONE wave alone on its SIMD (the continuation's
// situation at small batch, and nearly so at full load where the path wave has the highest priority).
// Each test runs a chain of 64 copies of a short sequence inside inline asm between two s_memtime
// reads; "dep" chains feed each result into the next instruction, "ind" runs four independent chains
// interleaved.  Prints cycles per sequence.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_lat tools/ubench_lat.hip && ./tools/ubench_lat
#include <hip/hip_runtime.h>

#include <cstdio>

#define N_REP "64"

__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    return t;
}

__global__ __launch_bounds__(64) void lat(unsigned long long* out, double seed, int iseed) {
    __shared__ double lds[512];
    __shared__ unsigned idx[64];
    const int lane = threadIdx.x;
    for (int k = lane; k < 512; k += 64) lds[k] = seed + k;
    using L32 = __attribute__((address_space(3))) unsigned;
    using L64 = __attribute__((address_space(3))) double;
    const unsigned self = (unsigned)(size_t)(L32*)&idx[lane];
    idx[lane] = self;  // pointer chase: each lane's word holds its own LDS address
    __syncthreads();
    double x = seed + lane, y = seed * 0.5 + 1.0, z = seed + 2.0, w = seed + 3.0, v = 1.000001;
    unsigned long long t0, t1;
    int slot = 0;
#define RUN(body, ...)                                          \
    t0 = now();                                                 \
    asm volatile(".rept " N_REP "\n" body "\n.endr" __VA_ARGS__); \
    t1 = now();                                                 \
    if (lane == 0) out[slot] = t1 - t0;                         \
    ++slot;
    // 0: v_add_f64 dependent
    RUN("v_add_f64 %0, %0, %1", : "+v"(x) : "v"(v))
    // 1: v_add_f64, four independent chains
    RUN("v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4",
        : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(v))
    // 2: v_mul_f64 dependent
    RUN("v_mul_f64 %0, %0, %1", : "+v"(x) : "v"(v))
    // 3: v_fma_f64 dependent
    RUN("v_fma_f64 %0, %0, %1, %2", : "+v"(x) : "v"(v), "v"(y))
    // 4: v_cmp_lt_f64 -> v_cndmask_b32 x2 (a 64-bit select on a fresh compare), dependent through x
    t0 = now();
    asm volatile("v_mov_b64 v[10:11], %0\n v_mov_b64 v[12:13], %1\n s_nop 4\n"
                 ".rept " N_REP "\n v_cmp_lt_f64 vcc, v[10:11], v[12:13]\n v_cndmask_b32 v10, v12, v10, vcc\n"
                 " v_cndmask_b32 v11, v13, v11, vcc\n.endr" :: "v"(x), "v"(y) : "v10", "v11", "v12", "v13", "vcc");
    t1 = now();
    if (lane == 0) out[slot] = t1 - t0;
    ++slot;
    // 5: v_rcp_f64 dependent
    RUN("v_rcp_f64 %0, %0", : "+v"(x))
    // 6: v_cmp_lt_f64 into an SGPR pair, then s_and_b64 reading it (VALU -> SALU), dependent via x
    {
        t0 = now();
        asm volatile("v_mov_b64 v[10:11], %0\n v_mov_b64 v[12:13], %1\n s_nop 4\n"
                     ".rept " N_REP "\n v_cmp_lt_f64 s[40:41], v[10:11], v[12:13]\n s_and_b64 s[40:41], s[40:41], exec\n"
                     " v_cndmask_b32 v10, v12, v10, s[40:41]\n v_cndmask_b32 v11, v13, v11, s[40:41]\n.endr"
                     :: "v"(x), "v"(y) : "v10", "v11", "v12", "v13", "s40", "s41", "scc");
        t1 = now();
        if (lane == 0) out[slot] = t1 - t0;
        ++slot;
    }
    // 7: LDS pointer chase (ds_read_b32 of the address just read)
    {
        unsigned a = self;
        RUN("ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)", : "+v"(a))
        if (a == 12345u) out[63] = 1;
    }
    // 8: ds_read_b64 issued, waited, then one dependent v_add_f64 (load-use)
    {
        unsigned a = (unsigned)(size_t)(L64*)&lds[lane];
        double r;
        RUN("ds_read_b64 %1, %2\n s_waitcnt lgkmcnt(0)\n v_add_f64 %0, %0, %1", : "+v"(x), "=&v"(r) : "v"(a))
    }
    // 9: v_mov_b64 dependent
    RUN("v_mov_b64 %0, %0", : "+v"(x))
    // 10: v_add_u32 dependent
    {
        int q = iseed + lane;
        RUN("v_add_u32 %0, %0, %1", : "+v"(q) : "v"(iseed))
        if (q == 12345) out[62] = 1;
    }
    // 11: v_max_f64 dependent
    RUN("v_max_f64 %0, %0, %1", : "+v"(x) : "v"(y))
    // 12: v_cmp -> s_cbranch on vccz (VALU writes VCC, a branch reads it)
    RUN("v_cmp_lt_f64 vcc, %0, %1\n s_cbranch_vccz 1f\n 1:\n v_add_f64 %0, %0, %2", : "+v"(x) : "v"(y), "v"(v) : "vcc")
    // 13: v_div_scale / v_div_fmas / v_div_fixup full double division chain (the library sequence)
    {
        double q = x;
        for (int k = 0; k < 64; ++k) q = q / (y + (double)k * 1e-300);
        t0 = now();
        double r = x;
#pragma unroll 1
        for (int k = 0; k < 64; ++k) r = r / y;
        t1 = now();
        if (lane == 0) out[slot] = t1 - t0;
        ++slot;
        x += r + q;
    }
    // 14: v_sqrt_f64 dependent
    RUN("v_sqrt_f64 %0, %0", : "+v"(x))
    // 15: v_fma_f64 with 2 independent chains (what a pair of envs per lane would give)
    RUN("v_fma_f64 %0, %0, %2, %3\n v_fma_f64 %1, %1, %2, %3", : "+v"(x), "+v"(z) : "v"(v), "v"(y))
    // 16: v_cmp (vcc) issued, 8 independent adds, then s_cbranch_vccz (condition long ready, not taken)
    RUN("v_cmp_gt_f64 vcc, %1, %2\n v_add_f64 %0, %0, %2\n v_add_f64 %0, %0, %2\n v_add_f64 %0, %0, %2\n"
        " v_add_f64 %0, %0, %2\n v_add_f64 %0, %0, %2\n v_add_f64 %0, %0, %2\n v_add_f64 %0, %0, %2\n"
        " v_add_f64 %0, %0, %2\n s_cbranch_vccz 1f\n 1:", : "+v"(x) : "v"(y), "v"(v) : "vcc")
    // 17: the same 8 adds without the compare and branch (baseline of 16)
    RUN("v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n"
        " v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1", : "+v"(x) : "v"(v))
    // 18: v_cmp into an SGPR pair -> v_cndmask reading it directly (no SALU), dependent via x
    t0 = now();
    asm volatile("v_mov_b64 v[10:11], %0\n v_mov_b64 v[12:13], %1\n s_nop 4\n"
                 ".rept " N_REP "\n v_cmp_lt_f64 s[40:41], v[10:11], v[12:13]\n"
                 " v_cndmask_b32 v10, v12, v10, s[40:41]\n v_cndmask_b32 v11, v13, v11, s[40:41]\n.endr"
                 :: "v"(x), "v"(y) : "v10", "v11", "v12", "v13", "s40", "s41");
    t1 = now();
    if (lane == 0) out[slot] = t1 - t0;
    ++slot;
    // 19: ballot idiom: v_cmp -> s_cmp_lg_u64 -> s_cbranch_scc0 -> dependent add
    RUN("v_cmp_lt_f64 s[40:41], %0, %1\n s_cmp_lg_u64 s[40:41], 0\n s_cbranch_scc0 1f\n 1:\n v_add_f64 %0, %0, %2",
        : "+v"(x) : "v"(y), "v"(v) : "s40", "s41", "scc")
    // 20: exec-mask loop step: v_cmp -> s_and_saveexec_b64 -> s_cbranch_execz -> add -> s_or exec
    RUN("v_cmp_lt_f64 s[40:41], %0, %1\n s_and_saveexec_b64 s[42:43], s[40:41]\n s_cbranch_execz 1f\n"
        " v_add_f64 %0, %0, %2\n 1:\n s_or_b64 exec, exec, s[42:43]", : "+v"(x) : "v"(y), "v"(v)
        : "s40", "s41", "s42", "s43", "scc")
    // 21: v_div_scale/fmas/fixup-free correctly rounded division of the product (div_normal's 8 ops)
    RUN("v_rcp_f64 v[14:15], %1\n v_fma_f64 v[16:17], -%1, v[14:15], 1.0\n v_fma_f64 v[14:15], v[14:15], v[16:17], v[14:15]\n"
        " v_fma_f64 v[16:17], -%1, v[14:15], 1.0\n v_fma_f64 v[14:15], v[14:15], v[16:17], v[14:15]\n"
        " v_mul_f64 v[16:17], %0, v[14:15]\n v_fma_f64 v[18:19], -%1, v[16:17], %0\n v_fma_f64 %0, v[18:19], v[14:15], v[16:17]",
        : "+v"(x) : "v"(y) : "v14", "v15", "v16", "v17", "v18", "v19")
    if (x == 12345.0 || y == 1.0 || z == 2.0 || w == 3.0) out[61] = 1;
}

int main() {
    unsigned long long* d;
    (void)hipMalloc(&d, 64 * sizeof(unsigned long long));
    (void)hipMemset(d, 0, 64 * sizeof(unsigned long long));
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, d, 1.5, 3);
    (void)hipDeviceSynchronize();
    unsigned long long h[64];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[] = {"add_f64_dep", "add_f64_ind4", "mul_f64_dep", "fma_f64_dep", "cmp_sel64_dep",
                           "rcp_f64_dep", "cmp_salu_sel_dep", "ds_read_chase", "ds_read_use", "mov_b64_dep",
                           "add_u32_dep", "max_f64_dep", "cmp_vccz_branch_add", "div_f64_lib_dep", "sqrt_f64_dep",
                           "fma_f64_2chains", "cmp_8add_vccz_ready", "8add_base", "cmp_sgpr_sel_dep",
                           "ballot_branch_add", "saveexec_branch_add", "div_normal_dep"};
    printf("{");
    for (int k = 0; k < 22; ++k) printf("%s\"%s\": %.1f", k ? ", " : "", names[k], h[k] / 64.0);
    printf("}\n");
    return 0;
}
