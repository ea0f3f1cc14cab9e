// rtw_math.h — small fp64 kernels shared by the device code and the host
// tests (tests/cpp/sincos_check.cpp).
#pragma once

#include <stdint.h>
#if defined(__HIPCC__)
#define RTW_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define RTW_HD inline
#endif

namespace rtwd {

// sin and cos of x in [0, 2*pi] (the azimuth 2*pi*r1 of the direction
// samplers), fdlibm-style: Cody-Waite reduction by pi/2 in two steps
// (pio2_1 / pio2_2 carry 33 significant bits, so n*pio2_1 and n*pio2_2 are
// exact for the n <= 4 that occur; the remainder is kept as r + rt) and the
// __kernel_sin / __kernel_cos polynomials with tail on [-pi/4, pi/4].  Within
// an ulp of glibc's sin/cos (which the reference calls) and about half the
// instructions of the general ocml sincos (no large-argument path).
RTW_HD void sincos_azimuth(double x, double& sn, double& cs) {
    constexpr double inv_pio2 = 6.36619772367581382433e-01;
    constexpr double pio2_1 = 1.57079632673412561417e+00;   // 0x3FF921FB54400000
    constexpr double pio2_1t = 6.07710050650619224932e-11;  // pi/2 - pio2_1
    constexpr double pio2_2 = 6.07710050630396597660e-11;   // 0x3DD0B4611A600000
    constexpr double pio2_2t = 2.02226624879595063154e-21;  // pi/2 - pio2_1 - pio2_2
    const double n = __builtin_rint(x * inv_pio2);
    const double t = x - n * pio2_1;  // exact
    double w = n * pio2_2;            // exact
    const double r0 = t - w;
    w = n * pio2_2t - ((t - r0) - w);
    const double r = r0 - w;          // remainder r + rt, |r| <= pi/4
    const double rt = (r0 - r) - w;
    const double z = r * r;
    // __kernel_sin(r, rt)
    const double v = z * r;
    const double sp = 8.33333333332248946124e-03 +
                      z * (-1.98412698298579493134e-04 +
                           z * (2.75573137070700676789e-06 +
                                z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
    const double sr = r - ((z * (0.5 * rt - v * sp) - rt) - v * -1.66666666666666324348e-01);
    // __kernel_cos(r, rt)
    const double cp = z * (4.16666666666666019037e-02 +
                           z * (-1.38888888888741095749e-03 +
                                z * (2.48015872894767294178e-05 +
                                     z * (-2.75573143513906633035e-07 +
                                          z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
    const double hz = 0.5 * z;
    const double wc = 1.0 - hz;
    const double cr = wc + (((1.0 - wc) - hz) + (z * cp - r * rt));
    const int q = (int)n & 3;
    const double s0 = (q & 1) ? cr : sr;
    const double c0 = (q & 1) ? sr : cr;
    sn = (q & 2) ? -s0 : s0;
    cs = ((q + 1) & 2) ? -c0 : c0;
}

// sin(x) for |x| <= 2^19 (sin_wide_ok) with sincos_azimuth's reduction and
// kernel: n = rint(x * 2/pi) stays below 2^19, so n * pio2_1 and n * pio2_2
// (33 significant bits each) are still exact and the remainder carries 119
// bits of pi/2.  Within an ulp of glibc's sin over that range
// (tests/cpp/sincos_check.cpp); callers take their own path outside it.
// x^5 in double-double (exact products through fma), rounded once: within
// a hair of the correctly rounded x^5, i.e. at least as accurate as glibc's
// pow(x, 5) the reference calls (material.h:44-49, < 0.52 ulp) and far
// cheaper than ocml pow.
RTW_HD double pow5(double x) {
    const double x2 = x * x, e2 = __builtin_fma(x, x, -x2);
    const double x4 = x2 * x2, e4 = __builtin_fma(x2, x2, -x4) + 2.0 * x2 * e2;
    const double x5 = x4 * x, e5 = __builtin_fma(x4, x, -x5) + e4 * x;
    return x5 + e5;
}

RTW_HD bool sin_wide_ok(double x) { return __builtin_fabs(x) <= 0x1p19; }
RTW_HD double sin_wide(double x) {
    double s, c;
    sincos_azimuth(x, s, c);
    return s;
}

// log(x) for x positive, normal and finite (log_pos_ok): fdlibm's
// __ieee754_log (e_log.c, < 1 ulp).  x = 2^k (1 + f) with 1 + f in
// [sqrt(2)/2, sqrt(2)), s = f / (2 + f), log(1 + f) = f - (hfsq - s (hfsq + R))
// with R(s^2) a degree-14 polynomial; fdlibm's k == 0 forms are the same
// arithmetic with the exact zero terms left out, so one form serves all k.
// The constants come from coef(i) (i = 0 ln2_hi, 1 ln2_lo, 2..8 Lg1..Lg7):
// the device reads them from a table where the log is evaluated, so they are
// not held in registers across a kernel's loop.  Within an ulp of glibc's
// log (tests/cpp/sincos_check.cpp).
constexpr double kLogCoef[9] = {
    6.93147180369123816490e-01, 1.90821492927058770002e-10, 6.666666666666735130e-01, 3.999999999940941908e-01,
    2.857142874366239149e-01,   2.222219843214978396e-01,   1.818357216161805012e-01, 1.531383769920937332e-01,
    1.479819860511658591e-01};
RTW_HD bool log_pos_ok(double x) { return x >= 0x1p-1022 && x <= 1.7976931348623157e308; }
template <class C>
RTW_HD double log_pos(double x, C coef) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    int32_t hx = (int32_t)(b >> 32);
    int k = (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i = (hx + 0x95f64) & 0x100000;
    const uint64_t nb = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (b & 0xffffffffull);
    k += i >> 20;
    const double f = __builtin_bit_cast(double, nb) - 1.0;  // x or x/2 normalised, minus 1
    const double dk = (double)k;
    if ((0x000fffff & (2 + hx)) < 3) {  // -2^-20 <= f < 2^-20
        if (f == 0.0) return k == 0 ? 0.0 : dk * coef(0) + dk * coef(1);
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        return dk * coef(0) - ((R - dk * coef(1)) - f);
    }
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double w = z * z;
    const int32_t ii = (hx - 0x6147a) | (0x6b851 - hx);
    const double t1 = w * (coef(3) + w * (coef(5) + w * coef(7)));
    const double t2 = z * (coef(2) + w * (coef(4) + w * (coef(6) + w * coef(8))));
    const double R = t2 + t1;
    if (ii > 0) {
        const double hfsq = 0.5 * f * f;
        return dk * coef(0) - ((hfsq - (s * (hfsq + R) + dk * coef(1))) - f);
    }
    return dk * coef(0) - ((s * (f - R) - dk * coef(1)) - f);
}

}  // namespace rtwd
