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
/* fdlibm s_atan.c: atan(x), |error| < 1 ulp; the same operations on host and device */
D2D_PM_FN double d2d_pm_atan(double x) {
    static const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                     9.82793723247329054082e-01, 1.57079632679489655800e+00};
    static const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                     1.39033110312309984516e-17, 6.12323399573676603587e-17};
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    const uint64_t b = d2d_pm_d2bits(x);
    const int32_t hx = (int32_t)(b >> 32);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x44100000) { /* |x| >= 2^66 */
        if (ix > 0x7ff00000 || (ix == 0x7ff00000 && (uint32_t)b != 0u)) return x + x; /* NaN */
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3fdc0000) { /* |x| < 0.4375 */
        if (ix < 0x3e400000) return x; /* |x| < 2^-27 (fdlibm: huge + x > one, inexact) */
        id = -1;
    } else {
        x = x < 0.0 ? -x : x;
        if (ix < 0x3ff30000) {     /* |x| < 1.1875 */
            if (ix < 0x3fe60000) { /* 7/16 <= |x| < 11/16 */
                id = 0;
                x = (2.0 * x - 1.0) / (2.0 + x);
            } else { /* 11/16 <= |x| < 19/16 */
                id = 1;
                x = (x - 1.0) / (x + 1.0);
            }
        } else {
            if (ix < 0x40038000) { /* |x| < 2.4375 */
                id = 2;
                x = (x - 1.5) / (1.0 + 1.5 * x);
            } else { /* 2.4375 <= |x| < 2^66 */
                id = 3;
                x = -1.0 / x;
            }
        }
    }
    const double z = x * x, w = z * z;
    const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    const double r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}
/* fdlibm e_atan2.c: atan2(y, x) with its signed-zero / infinity cases */
D2D_PM_FN double d2d_pm_atan2(double y, double x) {
    const double pi_o_4 = 7.8539816339744827900E-01, pi_o_2 = 1.5707963267948965580E+00,
                 pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
    const uint64_t bx = d2d_pm_d2bits(x), by = d2d_pm_d2bits(y);
    const int32_t hx = (int32_t)(bx >> 32), hy = (int32_t)(by >> 32);
    const uint32_t lx = (uint32_t)bx, ly = (uint32_t)by;
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (((uint32_t)ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u ||
        ((uint32_t)iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
        return x + y; /* NaN */
    if (hx == 0x3ff00000 && lx == 0u) return d2d_pm_atan(y); /* x = 1.0 */
    const int m = (int)(((uint32_t)hy >> 31) & 1u) | (int)(((uint32_t)hx >> 30) & 2u); /* 2 sign(x) + sign(y) */
    if ((iy | (int32_t)ly) == 0) { /* y = +-0 */
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi;
            default: return -pi;
        }
    }
    if ((ix | (int32_t)lx) == 0) return hy < 0 ? -pi_o_2 : pi_o_2; /* x = +-0 */
    if (ix == 0x7ff00000) {
        if (iy == 0x7ff00000) {
            switch (m) {
                case 0: return pi_o_4;
                case 1: return -pi_o_4;
                case 2: return 3.0 * pi_o_4;
                default: return -3.0 * pi_o_4;
            }
        }
        switch (m) {
            case 0: return 0.0;
            case 1: return -0.0;
            case 2: return pi;
            default: return -pi;
        }
    }
    if (iy == 0x7ff00000) return hy < 0 ? -pi_o_2 : pi_o_2;
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = pi_o_2 + 0.5 * pi_lo; /* |y / x| > 2^60 */
    else if (hx < 0 && k < -60) z = 0.0;  /* |y| / x < -2^60 */
    else {
        const double q = y / x;
        z = d2d_pm_atan(q < 0.0 ? -q : q);
    }
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}
#endif /* D2D_PMATH_H */
