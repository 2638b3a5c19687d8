// Micro-benchmark (diagnostic, never shipped): what the fp32 trade of DESIGN.md ("The 40 % HBM-roofline
// target") would buy on the physics role.  One lane per env runs the joint sweep of one cpSpaceStep
// (preStep, cached impulses, 10 Gauss-Seidel sweeps over the 6 pivots) from a random pivot-triple
// state, at K1's occupancy (256-thread workgroups, 4 per CU, every wave sweeping):
//   mode 0  fp64, the product's phys_velocities<false> (d2d_device.h), registers only
//   mode 1  the same operation sequence in fp32 (scalar)
//   mode 2  fp32 with the (x, y) pairs as 2-vectors (packed v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32)
// Prints ns per env-sweep for each mode and the largest relative velocity / impulse difference of
// the fp32 modes against fp64 after one step.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../drone-2d-custom-gym-env-for-reinforcement-learning_amd/csrc/d2d_device.h"

using namespace d2d;
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int NV = 9, NJ = 12, NIN = 6 + 3 + 3 + NV + NJ + 2;  // pos, fx fy tq, cs sn... see fill()

// state of env i: pos[6], (fx, fy, tq), vel[9], j[12], angles of the 3 bodies
struct In {
    double pos[6], f[3], vel[NV], j[NJ], ang[3];
};

template <typename T>
struct ArmsT {
    T m7c[2], m7s[2], f47c, f47s, f40c, f40s, f33c, f33s;
};
template <typename T>
__device__ __forceinline__ void armT(const ArmsT<T>& A, int k, T& r1x, T& r1y, T& r2x, T& r2y) {
    const int m = k < 3 ? 0 : 1, q = k % 3;
    r1x = (q == 0) ? -A.m7c[m] : ((q == 1) ? T(0) : A.m7c[m]);
    r1y = (q == 0) ? -A.m7s[m] : ((q == 1) ? T(0) : A.m7s[m]);
    const T c = (k == 0 || k == 5) ? A.f47c : ((k == 1 || k == 4) ? A.f40c : A.f33c);
    const T s = (k == 0 || k == 5) ? A.f47s : ((k == 1 || k == 4) ? A.f40s : A.f33s);
    r2x = (k < 3) ? -c : c;
    r2y = (k < 3) ? -s : s;
}

// phys_velocities<false> restated over float (same operations, same order)
__device__ __forceinline__ void sweep_f32(const ArmsT<float>& A, const float pos[6], float damping_dt, float fx,
                                          float fy, float tq, float vel[9], float j[12]) {
    const float MIM = (float)MI_M, MIF = (float)MI_F, IIM = (float)II_M, IIF = (float)II_F, dt = (float)DT;
    const float bias_coef = -1.0f / dt;
    float kk[6][5];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int m = k < 3 ? 1 : 2;
        float r1x, r1y, r2x, r2y;
        armT(A, k, r1x, r1y, r2x, r2y);
        const float ms = MIM + MIF;
        float k11 = ms, k12 = 0.0f, k22 = ms;
        k11 += r1y * r1y * IIM; k12 += -r1x * r1y * IIM; k22 += r1x * r1x * IIM;
        k11 += r2y * r2y * IIF; k12 += -r2x * r2y * IIF; k22 += r2x * r2x * IIF;
        const float di = 1.0f / (k11 * k22 - k12 * k12);
        kk[k][0] = k22 * di; kk[k][1] = -k12 * di; kk[k][2] = k11 * di;
        kk[k][3] = ((pos[0] + r2x) - (pos[2 * m] + r1x)) * bias_coef;
        kk[k][4] = ((pos[1] + r2y) - (pos[2 * m + 1] + r1y)) * bias_coef;
    }
    vel[0] = vel[0] * damping_dt + (fx * MIF) * dt;
    vel[1] = vel[1] * damping_dt + ((float)GRAV_Y + fy * MIF) * dt;
    vel[2] = vel[2] * damping_dt + tq * IIF * dt;
#pragma unroll
    for (int b = 1; b < 3; ++b) {
        vel[3 * b] = vel[3 * b] * damping_dt;
        vel[3 * b + 1] = vel[3 * b + 1] * damping_dt + (float)GRAV_Y * dt;
        vel[3 * b + 2] = vel[3 * b + 2] * damping_dt;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int m = k < 3 ? 1 : 2;
        float r1x, r1y, r2x, r2y;
        armT(A, k, r1x, r1y, r2x, r2y);
        const float jx = j[2 * k], jy = j[2 * k + 1];
        vel[3 * m] -= jx * MIM; vel[3 * m + 1] -= jy * MIM;
        vel[3 * m + 2] += IIM * (r1x * (-jy) - r1y * (-jx));
        vel[0] += jx * MIF; vel[1] += jy * MIF;
        vel[2] += IIF * (r2x * jy - r2y * jx);
    }
    for (int it = 0; it < 10; ++it) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int m = k < 3 ? 1 : 2;
            float r1x, r1y, r2x, r2y;
            armT(A, k, r1x, r1y, r2x, r2y);
            const bool za = k % 3 == 1;
            const float v1x = za ? vel[3 * m] : vel[3 * m] + (-r1y) * vel[3 * m + 2];
            const float v1y = za ? vel[3 * m + 1] : vel[3 * m + 1] + r1x * vel[3 * m + 2];
            const float v2x = vel[0] + (-r2y) * vel[2], v2y = vel[1] + r2x * vel[2];
            const float ux = kk[k][3] - (v2x - v1x), uy = kk[k][4] - (v2y - v1y);
            float jx = ux * kk[k][0] + uy * kk[k][1], jy = ux * kk[k][1] + uy * kk[k][2];
            const float ox = j[2 * k], oy = j[2 * k + 1], nx = ox + jx, ny = oy + jy;
            j[2 * k] = nx; j[2 * k + 1] = ny;
            jx = nx - ox; jy = ny - oy;
            vel[3 * m] += (-jx) * MIM; vel[3 * m + 1] += (-jy) * MIM;
            if (!za) vel[3 * m + 2] += IIM * (r1x * (-jy) - r1y * (-jx));
            vel[0] += jx * MIF; vel[1] += jy * MIF;
            vel[2] += IIF * (r2x * jy - r2y * jx);
        }
    }
}

// the same with (x, y) as 2-vectors: the linear velocity updates and the impulse arithmetic pack
__device__ __forceinline__ void sweep_pk(const ArmsT<float>& A, const float pos[6], float damping_dt, float fx,
                                         float fy, float tq, float vel[9], float j[12]) {
    const float MIM = (float)MI_M, MIF = (float)MI_F, IIM = (float)II_M, IIF = (float)II_F, dt = (float)DT;
    const float bias_coef = -1.0f / dt;
    f2 ka[6], kb[6], bb[6], J[6];
    f2 lv[3] = {f2{vel[0], vel[1]}, f2{vel[3], vel[4]}, f2{vel[6], vel[7]}};
    float w[3] = {vel[2], vel[5], vel[8]};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int m = k < 3 ? 1 : 2;
        float r1x, r1y, r2x, r2y;
        armT(A, k, r1x, r1y, r2x, r2y);
        const float ms = MIM + MIF;
        float k11 = ms, k12 = 0.0f, k22 = ms;
        k11 += r1y * r1y * IIM; k12 += -r1x * r1y * IIM; k22 += r1x * r1x * IIM;
        k11 += r2y * r2y * IIF; k12 += -r2x * r2y * IIF; k22 += r2x * r2x * IIF;
        const float di = 1.0f / (k11 * k22 - k12 * k12);
        ka[k] = f2{k22 * di, -k12 * di};   // column 0 of K^-1
        kb[k] = f2{-k12 * di, k11 * di};   // column 1
        bb[k] = f2{(pos[0] + r2x) - (pos[2 * m] + r1x), (pos[1] + r2y) - (pos[2 * m + 1] + r1y)} * bias_coef;
        J[k] = f2{j[2 * k], j[2 * k + 1]};
    }
    const f2 g{0.0f, (float)GRAV_Y * dt};
    lv[0] = lv[0] * damping_dt + f2{fx * MIF, fy * MIF} * dt + g;
    w[0] = w[0] * damping_dt + tq * IIF * dt;
    lv[1] = lv[1] * damping_dt + g;
    lv[2] = lv[2] * damping_dt + g;
    w[1] *= damping_dt;
    w[2] *= damping_dt;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int m = k < 3 ? 1 : 2;
        float r1x, r1y, r2x, r2y;
        armT(A, k, r1x, r1y, r2x, r2y);
        lv[m] -= J[k] * MIM;
        w[m] += IIM * (r1x * (-J[k].y) - r1y * (-J[k].x));
        lv[0] += J[k] * MIF;
        w[0] += IIF * (r2x * J[k].y - r2y * J[k].x);
    }
    for (int it = 0; it < 10; ++it) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int m = k < 3 ? 1 : 2;
            float r1x, r1y, r2x, r2y;
            armT(A, k, r1x, r1y, r2x, r2y);
            const bool za = k % 3 == 1;
            const f2 v1 = za ? lv[m] : lv[m] + f2{-r1y, r1x} * w[m];
            const f2 v2 = lv[0] + f2{-r2y, r2x} * w[0];
            const f2 u = bb[k] - (v2 - v1);
            f2 jj = ka[k] * u.x + kb[k] * u.y;
            const f2 o = J[k], nn = o + jj;
            J[k] = nn;
            jj = nn - o;
            lv[m] -= jj * MIM;
            if (!za) w[m] += IIM * (r1x * (-jj.y) - r1y * (-jj.x));
            lv[0] += jj * MIF;
            w[0] += IIF * (r2x * jj.y - r2y * jj.x);
        }
    }
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        vel[3 * b] = lv[b].x;
        vel[3 * b + 1] = lv[b].y;
        vel[3 * b + 2] = w[b];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        j[2 * k] = J[k].x;
        j[2 * k + 1] = J[k].y;
    }
}

__global__ __launch_bounds__(256, 4) void k_sweep(const In* in, double* out, int n, int reps, int mode, double ddt) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const In& s = in[i];
    double acc[NV + NJ] = {};
    for (int r = 0; r < reps; ++r) {
        double cs[3], sn[3];
        for (int b = 0; b < 3; ++b) sincos(s.ang[b] + 1e-12 * r, &sn[b], &cs[b]);
        if (mode == 0) {
            const Arms A = make_arms(cs, sn);
            double vel[NV], j[NJ];
            for (int k = 0; k < NV; ++k) vel[k] = s.vel[k];
            for (int k = 0; k < NJ; ++k) j[k] = s.j[k];
            phys_velocities<false>(A, s.pos, ddt, s.f[0], s.f[1], s.f[2], vel, j, nullptr, 0);
            for (int k = 0; k < NV; ++k) acc[k] += vel[k];
            for (int k = 0; k < NJ; ++k) acc[NV + k] += j[k];
        } else {
            ArmsT<float> A;
            A.m7c[0] = (float)(cs[1] * 7.0); A.m7s[0] = (float)(sn[1] * 7.0);
            A.m7c[1] = (float)(cs[2] * 7.0); A.m7s[1] = (float)(sn[2] * 7.0);
            A.f47c = (float)(cs[0] * 47.0); A.f47s = (float)(sn[0] * 47.0);
            A.f40c = (float)(cs[0] * 40.0); A.f40s = (float)(sn[0] * 40.0);
            A.f33c = (float)(cs[0] * 33.0); A.f33s = (float)(sn[0] * 33.0);
            float pos[6], vel[NV], j[NJ];
            for (int k = 0; k < 6; ++k) pos[k] = (float)s.pos[k];
            for (int k = 0; k < NV; ++k) vel[k] = (float)s.vel[k];
            for (int k = 0; k < NJ; ++k) j[k] = (float)s.j[k];
            if (mode == 1) sweep_f32(A, pos, (float)ddt, (float)s.f[0], (float)s.f[1], (float)s.f[2], vel, j);
            else sweep_pk(A, pos, (float)ddt, (float)s.f[0], (float)s.f[1], (float)s.f[2], vel, j);
            for (int k = 0; k < NV; ++k) acc[k] += vel[k];
            for (int k = 0; k < NJ; ++k) acc[NV + k] += j[k];
        }
    }
    for (int k = 0; k < NV + NJ; ++k) out[(size_t)k * n + i] = acc[k] / reps;
}

int main() {
    const int n = 65536 * 4, reps = 8;
    std::vector<In> h(n);
    unsigned long long x = 88172645463325252ull;
    auto rnd = [&]() {  // xorshift, U(-1, 1)
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        return (double)(x >> 11) * (2.0 / 9007199254740992.0) - 1.0;
    };
    for (auto& s : h) {
        const double a = 0.3 * rnd(), px = 400 + 200 * rnd(), py = 300 + 200 * rnd();
        const double c = std::cos(a), sn = std::sin(a);
        s.ang[0] = a; s.ang[1] = a + 1e-3 * rnd(); s.ang[2] = a + 1e-3 * rnd();
        s.pos[0] = px; s.pos[1] = py;
        s.pos[2] = px - 40 * c + 0.05 * rnd(); s.pos[3] = py - 40 * sn + 0.05 * rnd();
        s.pos[4] = px + 40 * c + 0.05 * rnd(); s.pos[5] = py + 40 * sn + 0.05 * rnd();
        s.f[0] = -sn * 30 * (1 + rnd()); s.f[1] = c * 30 * (1 + rnd()); s.f[2] = 200 * rnd();
        for (double& v : s.vel) v = 50 * rnd();
        for (double& v : s.j) v = 2 * rnd();
    }
    In* din;
    double* dout[3];
    (void)hipMalloc(&din, sizeof(In) * n);
    (void)hipMemcpy(din, h.data(), sizeof(In) * n, hipMemcpyHostToDevice);
    for (auto& p : dout) (void)hipMalloc(&p, sizeof(double) * (NV + NJ) * n);
    const double ddt = std::pow(0.9, 1.0 / 60.0);  // a damping of 0.9 per second
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best[3] = {1e30f, 1e30f, 1e30f};
    for (int round = 0; round < 5; ++round)
        for (int mode = 0; mode < 3; ++mode) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k_sweep, dim3(n / 256), dim3(256), 0, 0, din, dout[mode], n, reps, mode, ddt);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best[mode]) best[mode] = ms;
        }
    std::vector<double> r[3];
    for (int mode = 0; mode < 3; ++mode) {
        r[mode].resize((size_t)(NV + NJ) * n);
        (void)hipMemcpy(r[mode].data(), dout[mode], sizeof(double) * r[mode].size(), hipMemcpyDeviceToHost);
    }
    const char* name[3] = {"fp64 (product sweep)", "fp32 scalar", "fp32 packed 2-vectors"};
    for (int mode = 0; mode < 3; ++mode) {
        double ev = 0.0, ej = 0.0;
        for (int k = 0; k < NV + NJ; ++k)
            for (int i = 0; i < n; ++i) {
                const double a = r[0][(size_t)k * n + i], b = r[mode][(size_t)k * n + i];
                const double e = std::fabs(a - b) / std::max(1.0, std::fabs(a));
                if (k < NV) ev = std::max(ev, e);
                else ej = std::max(ej, e);
            }
        printf("%-24s %8.3f ms for %d env-sweeps x %d reps: %7.3f ns per env-sweep; max rel diff vs fp64: vel %.2e, impulse %.2e\n",
               name[mode], best[mode], n, reps, 1e6 * best[mode] / ((double)n * reps), ev, ej);
    }
    return 0;
}
