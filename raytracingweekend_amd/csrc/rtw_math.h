// rtw_math.h — small fp64 kernels shared by the device code and the host
// tests (tests/cpp/sincos_check.cpp).
#pragma once

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

}  // namespace rtwd
