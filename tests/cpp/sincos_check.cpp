// sincos_azimuth (rtw_math.h) against glibc sin/cos over [0, 2*pi]: maximum
// error in ulps of the glibc value (glibc's double sin/cos are < 1 ulp).
// Usage: sincos_check N   -> prints "max_ulp_sin X max_ulp_cos Y"
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <initializer_list>
#include "rtw_math.h"

static double ulp_diff(double a, double b) {
    if (a == b) return 0.0;
    const double u = std::fabs(std::nextafter(b, INFINITY) - b);
    return std::fabs(a - b) / (u > 0 ? u : 1e-300);
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 1000000;
    const double two_pi = 2 * 3.14159265358979323846;
    double ms = 0, mc = 0, ams = 0, amc = 0;
    uint64_t st = 12345;
    for (long k = 0; k <= n; ++k) {
        // the samplers' argument: 2*pi times a canonical draw in [0, 1)
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        const double r1 = (k < n / 2) ? (double)k / (double)(n / 2) : (double)(st >> 11) * 0x1p-53;
        const double x = two_pi * r1;
        double s, c;
        rtwd::sincos_azimuth(x, s, c);
        const double rs = std::sin(x), rc = std::cos(x);
        ms = std::fmax(ms, ulp_diff(s, rs));
        mc = std::fmax(mc, ulp_diff(c, rc));
        ams = std::fmax(ams, std::fabs(s - rs));
        amc = std::fmax(amc, std::fabs(c - rc));
    }
    // points next to the quadrant boundaries
    for (int q = 0; q <= 4; ++q)
        for (int d = -2000; d <= 2000; ++d) {
            const double x = std::nextafter(q * (two_pi / 4), 0.0) + d * 1e-12;
            if (x < 0 || x > two_pi) continue;
            double s, c;
            rtwd::sincos_azimuth(x, s, c);
            ams = std::fmax(ams, std::fabs(s - std::sin(x)));
            amc = std::fmax(amc, std::fabs(c - std::cos(x)));
        }
    // sin_wide over [-2^19, 2^19] (the marble texture's argument): random
    // arguments at every scale and the doubles next to multiples of pi / 2
    double mw = 0;
    for (long k = 0; k <= n; ++k) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        const int e = (int)((st >> 40) % 40) - 20;  // |x| in [2^-20, 2^19]
        double x = std::ldexp(1.0 + (double)(st >> 12 & 0xFFFFFFFFFFFull) * 0x1p-44, e);
        if (x > 0x1p19) x = 0x1p19;
        if (st & 1) x = -x;
        mw = std::fmax(mw, ulp_diff(rtwd::sin_wide(x), std::sin(x)));
    }
    for (long m = 1; m <= 333772; m += (m < 4096 ? 1 : 97)) {  // m * pi/2 <= 2^19
        const double c = m * (two_pi / 4);
        for (double x : {c, std::nextafter(c, 0.0), std::nextafter(c, INFINITY)}) {
            if (!rtwd::sin_wide_ok(x)) continue;
            mw = std::fmax(mw, ulp_diff(rtwd::sin_wide(x), std::sin(x)));
            mw = std::fmax(mw, ulp_diff(rtwd::sin_wide(-x), std::sin(-x)));
        }
    }
    // log_pos over the media's arguments (canonical draws in [2^-62, 1)) and
    // over every binade of the normal range
    double ml = 0;
    auto lc = [](int i) { return rtwd::kLogCoef[i]; };
    for (long k = 0; k <= n; ++k) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        const double u = (double)(st >> 11) * 0x1p-53;
        const double x1 = u > 0x1p-62 ? u : 0x1p-62;
        ml = std::fmax(ml, ulp_diff(rtwd::log_pos(x1, lc), std::log(x1)));
        const int e = (int)((st >> 20) % 2046) - 1022;
        const double x2 = std::ldexp(1.0 + (double)(st & 0xFFFFFFFFFFFFFull) * 0x1p-52, e);
        if (rtwd::log_pos_ok(x2)) ml = std::fmax(ml, ulp_diff(rtwd::log_pos(x2, lc), std::log(x2)));
        const double x3 = 1.0 + ((double)(st >> 11) * 0x1p-53 - 0.5) * 0x1p-18;  // near 1 (the small-f form)
        ml = std::fmax(ml, ulp_diff(rtwd::log_pos(x3, lc), std::log(x3)));
    }
    for (double x : {1.0, 2.0, 0.5, 0x1p-1022, 1.7976931348623157e308, std::nextafter(1.0, 0.0), 0x1p-62})
        ml = std::fmax(ml, ulp_diff(rtwd::log_pos(x, lc), std::log(x)));
    std::printf("max_ulp_sin %.3f max_ulp_cos %.3f max_abs_sin %.3g max_abs_cos %.3g max_ulp_sin_wide %.3f "
                "max_ulp_log %.3f\n", ms, mc, ams, amc, mw, ml);
    return 0;
}
