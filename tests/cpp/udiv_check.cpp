// Checks rtw_div.h's udiv_fast (Granlund-Montgomery magic-number division)
// against n / d for the divisors the kernels use -- image widths and pixel
// counts -- and random ones, over n next to every multiple of d (the hard
// cases), the ends of the range and random values.  Usage: udiv_check N
// (random operands per divisor); prints the case count and mismatches, exit
// 1 on any mismatch.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rtw_div.h"

static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint64_t next() {
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const long per = argc > 1 ? std::atol(argv[1]) : 100000;
    std::vector<uint32_t> ds;
    for (uint32_t d = 1; d <= 4096; ++d) ds.push_back(d);
    for (uint32_t nx : {100u, 200u, 400u, 600u, 800u, 1200u, 1600u, 1920u, 3840u, 8192u})
        for (uint32_t ny : {1u, 2u, 3u, 50u, 100u, 200u, 400u, 600u, 800u, 1080u, 1600u, 2160u, 8192u})
            ds.push_back(nx * ny);
    for (int k = 0; k < 32; ++k) ds.push_back(1u << k), ds.push_back((1u << k) + 1), ds.push_back(~0u >> k);
    for (int k = 0; k < 2000; ++k) ds.push_back((uint32_t)(next() >> (32 + next() % 32)) | 1u);
    uint64_t cases = 0, bad = 0;
    auto check = [&](uint32_t n, uint32_t d, const rtwd::udiv32& D) {
        ++cases;
        if (rtwd::udiv_fast(n, D) != n / d) {
            if (bad++ < 10) std::printf("mismatch n=%u d=%u got %u want %u\n", n, d, rtwd::udiv_fast(n, D), n / d);
        }
    };
    for (uint32_t d : ds) {
        if (!d) continue;
        const rtwd::udiv32 D = rtwd::udiv_magic(d);
        for (uint32_t n : {0u, 1u, d - 1, d, d + 1, ~0u, ~0u - 1, ~0u - d}) check(n, d, D);
        // next to multiples of d over the whole range
        const uint64_t step = std::max<uint64_t>(d, ((1ull << 32) / 4096) / d * d);
        for (uint64_t k = d; k < (1ull << 32); k += step)
            for (int64_t o = -2; o <= 2; ++o) {
                const int64_t n = (int64_t)k + o;
                if (n >= 0 && n < (int64_t)(1ull << 32)) check((uint32_t)n, d, D);
            }
        for (long k = 0; k < per; ++k) check((uint32_t)next(), d, D);
    }
    // the seed fold: x mod (2^31 - 2) for 64-bit x
    const unsigned long long M = 2147483646ull;
    uint64_t mcases = 0, mbad = 0;
    auto mcheck = [&](uint64_t x) {
        ++mcases;
        if (rtwd::mod_2p31m2(x) != x % M && mbad++ < 10)
            std::printf("mod mismatch x=%llu\n", (unsigned long long)x);
    };
    for (uint64_t x : {0ull, 1ull, M - 1, M, M + 1, 2 * M, ~0ull, ~0ull - 1, (1ull << 31) - 1, 1ull << 31,
                       (1ull << 32) - 1, 1ull << 32, (1ull << 35) - 1})
        mcheck(x);
    for (uint64_t k = 1; k < (1ull << 33); k += 1 + (next() & 0xfffff))  // next to multiples of M
        for (int64_t o = -3; o <= 3; ++o) mcheck(k * M + (uint64_t)o);
    for (long k = 0; k < 100 * per; ++k) mcheck(next());
    for (long k = 0; k < 100 * per; ++k) mcheck(next() >> (next() % 64));
    bad += mbad;
    std::printf("mod cases %llu mismatches %llu\n", (unsigned long long)mcases, (unsigned long long)mbad);
    std::printf("udiv cases %llu mismatches %llu\n", (unsigned long long)cases, (unsigned long long)bad);
    return bad ? 1 : 0;
}
