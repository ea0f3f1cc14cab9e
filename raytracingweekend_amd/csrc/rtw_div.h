// rtw_div.h — correctly rounded fp64 division without the hardware divide
// sequence, for divisors whose reciprocal is known or shared.
//
// gfx950 has no fp64 divide instruction: a / b compiles to div_scale x2,
// a quarter-rate v_rcp_f64, five fma, div_fmas and div_fixup.  Where the
// divisor is a constant with a known reciprocal -- generate_canonical's
// R*R, divided once per random draw -- Markstein's theorem gives the same
// correctly rounded quotient from fma alone, with y = RN(1/b):
//
//   q0 = RN(a*y)                      within 1.5 ulp of a/b
//   q1 = RN(q0 + RN(a - b*q0) * y)    within 1 ulp
//   q  = RN(q1 + RN(a - b*q1) * y)    = RN(a/b)   (Markstein: y within 1/2 ulp
//                                                  of 1/b, q1 within 1 ulp,
//                                                  no over/underflow)
//
// The no-over/underflow condition is the guard below (callers outside it
// divide directly).  tests/test_division.py checks the identity against IEEE
// division bit for bit on random, midpoint-adversarial and edge operands.
// (Measured: using it for shared-divisor quotients such as vec3 / length
// costs more in registers and branches than it saves; only the canonical
// draw uses it.)
#pragma once

#if defined(__HIPCC__)
#define RTW_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define RTW_HD inline
#endif

namespace rtwd {

// a / b from y = RN(1/b); valid when div_rcp_ok(a, b).
RTW_HD double div_rcp(double a, double b, double y) {
    const double q0 = a * y;
    const double r0 = __builtin_fma(-b, q0, a);
    const double q1 = __builtin_fma(r0, y, q0);
    const double r1 = __builtin_fma(-b, q1, a);
    return a == 0.0 ? q0 : __builtin_fma(r1, y, q1);  // q0 carries 0's sign rule
}

// Quotient, reciprocal and remainders stay normal: |b| in [2^-500, 2^500],
// a = 0 or |a| in [2^-500, 2^500].  (NaN / inf operands fail the test.)
RTW_HD bool div_rcp_ok_b(double b) {
    const double m = __builtin_fabs(b);
    return m >= 0x1p-500 && m <= 0x1p500;
}
RTW_HD bool div_rcp_ok_a(double a) {
    const double m = __builtin_fabs(a);
    return a == 0.0 || (m >= 0x1p-500 && m <= 0x1p500);
}

}  // namespace rtwd
