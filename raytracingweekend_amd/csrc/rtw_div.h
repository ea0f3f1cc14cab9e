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

#include <cassert>
#if defined(__HIPCC__)
#define RTW_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#include <cstdint>
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

// generate_canonical's sum / (R * R), R * R rounded to b = 2^62 - 2^33 (the
// divisor libstdc++ forms, kCanonDiv), for 0 <= sum <= 2^62: ONE correction
// step.  y = RN(1/b) = 2^-62 (1 + 2^-29) lies within 2^-57.9 (relative) of
// 1/b = 2^-62 (1 + 2^-29 + 2^-58 + ...), so q0 = RN(sum * y) is within
// 0.534 ulp of sum / b -- faithful -- and Markstein's theorem (y = RN(1/b),
// q0 within 1 ulp, r = fma(-b, q0, sum) exact) makes fma(r, y, q0) the
// correctly rounded quotient; sum = +0 gives +0.  div_rcp's second step and
// its zero select are not needed (tests/cpp/div_check.cpp: every canonical
// sum form, bit for bit against IEEE division).
RTW_HD double div_canon(double sum) {
    constexpr double b = 4611686009837453312.0;  // 2^62 - 2^33
    constexpr double y = 0x1.00000008p-62;       // RN(1 / b) = 2^-62 (1 + 2^-29)
    const double q0 = sum * y;
    return __builtin_fma(__builtin_fma(-b, q0, sum), y, q0);
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

// Unsigned 32-bit division by a divisor fixed for a launch (the sample id
// -> pixel, row decomposition): Granlund-Montgomery's round-up method.  With
// l = ceil(log2 d) and m = floor(2^32 (2^l - d) / d) + 1 (< 2^32),
//   t = mulhi(m, n),  n / d = (t + ((n - t) >> s1)) >> s2,  s1 = min(l, 1), s2 = max(l - 1, 0)
// for every n, d in [1, 2^32) -- one multiply-high, a subtract, an add and two
// shifts where the compiler's n / d with a run-time d expands to ~18
// instructions (float reciprocal and two corrections).
// tests/cpp/udiv_check.cpp: exhaustive over n near every multiple of the
// image sizes' divisors and random 32-bit operands.
struct udiv32 {
    uint32_t m, s1, s2;
};
inline udiv32 udiv_magic(uint32_t d) {  // host, d >= 1
    assert(d >= 1 && "udiv_magic: divisor 0");  // callers pass validated sizes (npix, nx, S_pass)
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) ++l;
    const uint64_t m = (((1ull << 32) * ((1ull << l) - d)) / d) + 1;
    return udiv32{(uint32_t)m, l ? 1u : 0u, l ? l - 1u : 0u};
}
RTW_HD uint32_t udiv_fast(uint32_t n, const udiv32& D) {
    const uint32_t t = (uint32_t)(((uint64_t)D.m * n) >> 32);
    return (t + ((n - t) >> D.s1)) >> D.s2;
}

// x mod (2^31 - 2) for a 64-bit x (the per-sample seed, rtw_path_seed): as
// 2^31 = 2 (mod 2^31 - 2), x = a 2^31 + b folds to 2a + b < 2^35, which folds
// once more below 2^31 + 18, and one conditional subtract ends it -- 32-bit
// shifts, masks and adds where a 64-bit remainder by a constant costs a
// 64 x 64 multiply-high (tests/cpp/udiv_check.cpp: equal to x % m).
RTW_HD uint32_t mod_2p31m2(uint64_t x) {
    constexpr uint32_t m = 2147483646u;
    const uint64_t y = ((x >> 31) << 1) + (x & 0x7fffffffu);
    const uint32_t z = (uint32_t)((y >> 31) << 1) + (uint32_t)(y & 0x7fffffffu);
    return z >= m ? z - m : z;
}

#if defined(__HIPCC__)
// Shared-divisor quotients, bit for bit the compiler's own a / b.
//
// hipcc expands an fp64 a / b on gfx950 into
//   ns = div_scale(b), y0 = rcp(ns), two Newton steps y = fma(y, fma(-ns, y, 1), y),
//   ns' = div_scale(a), q = ns' * y, r = fma(-ns, q, ns'), div_fmas(r, y, q),
//   div_fixup(., b, a)
// where div_scale / div_fmas only rescale operands with extreme exponents and
// div_fixup only repairs zeros, infinities, NaNs and over/underflow.  When
// |b| is in [2^-200, 2^200] and |a| in [2^-800, 2^100] none of them acts, and
// the sequence is exactly rcp_hw(b) followed by div_hw(a, b, y): the
// reciprocal part depends on b alone, so several quotients by one divisor
// (a ray direction component, a vector length, a pdf) pay the quarter-rate
// v_rcp_f64 and its refinement once.  tests/cpp/div_hw_check.hip checks the
// identity on the card; callers keep exact a / b for lanes outside the range.
__device__ __forceinline__ double rcp_hw(double b) {
    const double y0 = __builtin_amdgcn_rcp(b);
    const double y1 = __builtin_fma(y0, __builtin_fma(-b, y0, 1.0), y0);
    return __builtin_fma(y1, __builtin_fma(-b, y1, 1.0), y1);
}
__device__ __forceinline__ double div_hw(double a, double b, double y) {
    const double q = a * y;
    return __builtin_fma(__builtin_fma(-b, q, a), y, q);
}
__device__ __forceinline__ bool div_hw_ok_b(double b) {
    const double m = __builtin_fabs(b);
    return m >= 0x1p-200 && m <= 0x1p200;
}
__device__ __forceinline__ bool div_hw_ok_a(double a) {
    const double m = __builtin_fabs(a);
    return m >= 0x1p-800 && m <= 0x1p100;
}
// The same ranges (slightly narrower at the top: |b| < 2^200, |a| < 2^100)
// from the biased exponent in the high word: 32-bit integer work, no 64-bit
// constants to hold in registers.  div_hw_ok_a0 also admits a zero numerator.
__device__ __forceinline__ uint32_t exp_bits(double v) {
    return ((uint32_t)(__builtin_bit_cast(unsigned long long, v) >> 52)) & 0x7ffu;
}
__device__ __forceinline__ bool div_hw_ok_b_exp(double b) { return exp_bits(b) - 823u < 400u; }
__device__ __forceinline__ bool div_hw_ok_a0_exp(double a) { return a == 0.0 || exp_bits(a) - 223u < 900u; }

// fp64 square root without the compiler's range handling.  hipcc expands
// sqrt(x) on gfx950 as: s = x < 2^-767 ? 256 : 0; x' = ldexp(x, s); y =
// rsq(x'); the Goldschmidt / Newton refinement below; ldexp(g, -s/2); and a
// class fixup returning x' for +-0 and +inf.  For positive finite x >= 2^-766
// the scale and fixup are identities, leaving exactly this sequence, so the
// result is bit for bit the compiler's sqrt (tests/cpp/sqrt_check.hip on the
// card) for 7 fewer instructions (two of them fp64 ldexp).
__device__ __forceinline__ double sqrt_core(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
// x positive, finite, >= 2^-766 (the sign and biased exponent in the high word)
__device__ __forceinline__ bool sqrt_core_ok(double x) {
    const uint32_t hi = (uint32_t)(__builtin_bit_cast(unsigned long long, x) >> 32);
    return (hi >> 20) - 257u < 1790u;
}
// sqrt for a wave: the core sequence when every active lane is in its range
// (wave-uniform branch), else the compiler's sqrt -- the same value either way
__device__ __forceinline__ double sqrt_w(double x) {
    if (__builtin_amdgcn_ballot_w64(!sqrt_core_ok(x)) == 0) return sqrt_core(x);
    return __builtin_sqrt(x);
}
#endif

}  // namespace rtwd
