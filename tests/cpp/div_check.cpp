// Checks rtw_div.h's Markstein division against IEEE a / b, bit for bit:
// random operands over wide exponent ranges, quotients placed next to rounding
// midpoints (the hard cases for a correction scheme), the constant divisors
// the kernels use, and the guard's edges.  Usage: div_check N  (prints the
// number of cases and mismatches; exit 1 on any mismatch).
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>

#include "rtw_div.h"

static uint64_t st = 0x243F6A8885A308D3ull;
static uint64_t next() {
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double mant() { return 1.0 + (double)(next() >> 12) * 0x1p-52; }
static double wide(int emax) {
    const int e = (int)(next() % (uint64_t)(2 * emax + 1)) - emax;
    const double s = (next() & 1) ? -1.0 : 1.0;
    return s * std::ldexp(mant(), e);
}
static uint64_t bits(double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}

static long long cases = 0, bad = 0;
static void check(double a, double b) {
    using namespace rtwd;
    if (!div_rcp_ok_b(b) || !div_rcp_ok_a(a)) return;
    const double y = 1.0 / b;
    const double q = div_rcp(a, b, y);
    const double want = a / b;
    ++cases;
    if (bits(q) != bits(want)) {
        if (++bad <= 10) std::printf("mismatch a=%a b=%a got=%a want=%a\n", a, b, q, want);
    }
}

// div_canon: generate_canonical's sum = (e1 + e2 * R) for raw draws e1, e2 in
// [0, 2^31 - 3] (R = 2^31 - 2, libstdc++'s two-draw form, rtw_device.h
// canon_raw) divided by kCanonDiv
static long long ccases = 0, cbad = 0;
static void check_canon(uint64_t e1, uint64_t e2) {
    const double R = 2147483646.0, b = 4611686009837453312.0;
    double sum = 0.0 + (double)e1 * 1.0;
    sum = sum + (double)e2 * R;
    const double q = rtwd::div_canon(sum), want = sum / b;
    ++ccases;
    if (bits(q) != bits(want) && ++cbad <= 10) std::printf("canon mismatch sum=%a got=%a want=%a\n", sum, q, want);
}

int main(int argc, char** argv) {
    const long long n = argc > 1 ? std::atoll(argv[1]) : 1000000;
    {
        if (rtwd::div_canon(0.0) != 0.0 || std::signbit(rtwd::div_canon(0.0))) ++cbad;
        const uint64_t top = 2147483645ull;  // 2^31 - 3
        for (uint64_t e2 : {(uint64_t)0, (uint64_t)1, (uint64_t)2, top - 1, top})
            for (uint64_t e1 = 0; e1 < 200000; ++e1) check_canon(e1, e2), check_canon(top - e1, e2);
        for (long long k = 0; k < 20 * n; ++k) check_canon(next() % (top + 1), next() % (top + 1));
        // sums next to every power of two (binade edges, where q0's error bound is widest)
        for (int e = 31; e <= 62; ++e)
            for (int d = -3000; d <= 3000; ++d) {
                const double s = std::ldexp(1.0, e) + d * std::ldexp(1.0, e - 52 > 0 ? e - 52 : 0);
                const double want = s / 4611686009837453312.0;
                ++ccases;
                if (bits(rtwd::div_canon(s)) != bits(want) && ++cbad <= 10)
                    std::printf("canon mismatch edge sum=%a\n", s);
            }
        std::printf("canon cases %lld mismatches %lld\n", ccases, cbad);
    }
    const double consts[] = {3.14159265358979323846, 4611686009837453312.0, 2147483646.0, 6.283185307179586,
                             0.1, 3.0, 555.0};
    for (long long k = 0; k < n; ++k) {
        // 1. wide random
        check(wide(60), wide(60));
        // 2. quotient next to a rounding midpoint: a = RN(m * b), m halfway
        //    between two doubles (long double carries the extra bits)
        {
            const double b = wide(40), q = wide(40);
            const long double m = (long double)q + (long double)(std::nextafter(q, INFINITY) - q) / 2;
            const double a = (double)(m * (long double)b);
            check(a, b);
            check(std::nextafter(a, INFINITY), b);
            check(std::nextafter(a, -INFINITY), b);
        }
        // 3. the kernels' constant divisors, canonical sums, unit-range values
        {
            const double b = consts[next() % 7];
            const double e1 = (double)(next() % 2147483646ull), e2 = (double)(next() % 2147483646ull);
            check(e1 + e2 * 2147483646.0, b);
            check((double)(next() >> 11) * 0x1p-53, b);
            check(wide(8), b);
        }
        // 4. vector / length shapes
        {
            const double x = wide(12), yv = wide(12), z = wide(12);
            const double len = std::sqrt(x * x + yv * yv + z * z);
            check(x, len);
            check(yv, len);
            check(z, len);
        }
    }
    // guard edges and signed zeros
    const double edge[] = {0.0, -0.0, 0x1p-500, -0x1p-500, 0x1p500, 0x1.fffffffffffffp499, 1.0, -1.0};
    for (double a : edge)
        for (double b : edge) check(a, b);
    std::printf("cases %lld mismatches %lld\n", cases, bad);
    return (bad || cbad) ? 1 : 0;
}
