/* d2d_pmath.h -- deterministic sin / cos / log for the curriculum generator (plain C and HIP).
 *
 * The fresh-curriculum generator (d2d_curriculum.h on the device, oracle/d2d_oracle.c on the host)
 * draws its own random scenarios (the reference's draws come from NumPy's global RandomState, which
 * no parallel generator reproduces), so the generator's output is pinned against itself: the device
 * and the CPU oracle must draw bit-identical paths.  The only operations whose last bit differs
 * between the device library (ocml) and glibc are the transcendental functions; the generator uses
 * these instead -- fdlibm's kernels (__kernel_sin / __kernel_cos / __ieee754_log polynomials) with a
 * simple Cody-Waite reduction, every operation an IEEE add / mul / div (compile with
 * -ffp-contract=off on both sides), so both builds round identically.  Accuracy: within a few ulp of
 * libm for the arguments the generator uses (|x| <= 8, 0 < s <= 1); tests/test_curriculum.py checks
 * it against NumPy.
 */
#ifndef D2D_PMATH_H
#define D2D_PMATH_H
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define D2D_PM_FN __host__ __device__ static inline
#else
#define D2D_PM_FN static inline
#endif

D2D_PM_FN double d2d_pm_bits2d(uint64_t b) {
    double d;
    memcpy(&d, &b, sizeof d);
    return d;
}
D2D_PM_FN uint64_t d2d_pm_d2bits(double d) {
    uint64_t b;
    memcpy(&b, &d, sizeof b);
    return b;
}

/* fdlibm k_sin.c / k_cos.c on |r| <= pi/4 (y = 0 tail dropped: the reduction below is exact to
 * well below an ulp for |x| <= 8) */
D2D_PM_FN double d2d_pm_ksin(double x) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double z = x * x, v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    return x + v * (S1 + z * r);
}
D2D_PM_FN double d2d_pm_kcos(double x) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}
/* sin and cos of x (|x| <= 8): k = nearest integer to x * 2/pi, r = x - k * pi/2 in three parts */
D2D_PM_FN void d2d_pm_sincos(double x, double* s, double* c) {
    const double INV_PIO2 = 6.36619772367581382433e-01;
    /* fdlibm pio2_1, pio2_2, pio2_3: 33 significant bits each, so k * P1 and k * P2 are exact */
    const double P1 = 1.57079632673412561417e+00, P2 = 6.07710050630396597660e-11,
                 P3 = 2.02226624871116645580e-21;
    double kf = x * INV_PIO2;
    kf = (kf >= 0.0) ? (double)(int64_t)(kf + 0.5) : -(double)(int64_t)(0.5 - kf);
    const double r = ((x - kf * P1) - kf * P2) - kf * P3;
    const double sr = d2d_pm_ksin(r), cr = d2d_pm_kcos(r);
    const int q = (int)((int64_t)kf & 3);
    *s = (q == 0) ? sr : ((q == 1) ? cr : ((q == 2) ? -sr : -cr));
    *c = (q == 0) ? cr : ((q == 1) ? -sr : ((q == 2) ? -cr : sr));
}
/* natural log of a positive normal x (fdlibm e_log.c) */
D2D_PM_FN double d2d_pm_log(double x) {
    const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    uint64_t b = d2d_pm_d2bits(x);
    int k = (int)((b >> 52) & 0x7ff) - 1023;
    uint64_t m = b & 0x000fffffffffffffull;
    /* scale the mantissa into [sqrt(2)/2, sqrt(2)) */
    if (m > 0x6a09e667f3bcdull) {  /* m >= sqrt(2) - 1 (mantissa bits of sqrt(2)) */
        m |= 0x3fe0000000000000ull;  /* m / 2 */
        k += 1;
    } else {
        m |= 0x3ff0000000000000ull;
    }
    const double f = d2d_pm_bits2d(m) - 1.0;
    const double s = f / (2.0 + f), dk = (double)k;
    const double z = s * s, w = z * z;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const double R = t2 + t1, hfsq = 0.5 * f * f;
    return dk * LN2_HI - ((hfsq - (s * (hfsq + R) + dk * LN2_LO)) - f);
}
#endif /* D2D_PMATH_H */
