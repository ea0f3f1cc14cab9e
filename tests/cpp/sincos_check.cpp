// sincos_azimuth (rtw_math.h) against glibc sin/cos over [0, 2*pi]: maximum
// error in ulps of the glibc value (glibc's double sin/cos are < 1 ulp).
// Usage: sincos_check N   -> prints "max_ulp_sin X max_ulp_cos Y"
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
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
    std::printf("max_ulp_sin %.3f max_ulp_cos %.3f max_abs_sin %.3g max_abs_cos %.3g\n", ms, mc, ams, amc);
    return 0;
}
