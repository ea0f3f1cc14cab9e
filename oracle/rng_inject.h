// rng_inject.h — TEST INFRASTRUCTURE ONLY (oracle).  Pre-included by
// oracle/ref_harness.cpp before the reference headers.
//
// Every std::minstd_rand the reference declares (utility.h:17, material.h:210,
// hittable.h:64,433, camera.h:72-73, noise.h:169,192,203, Scene/scene.h:104,
// and the render loop's own engine RayTracingWeekend.cpp:208) is redirected to
// rtw_path_rng.  While a path key is active on the calling thread, every
// instance draws from ONE thread-local minstd_rand stream owned by the current
// (pixel, sample): the per-path stream of include/rtw_gpu.h.  With no key
// active each instance behaves exactly like a default-seeded std::minstd_rand
// (own state, seed 1), so scene construction (Scene/scene.h:103-158) and the
// Perlin tables (noise.h:166-213) come out as in the unmodified reference.
//
// min() = 1, max() = 2147483646 as std::minstd_rand, so libstdc++'s
// generate_canonical<double,53> still consumes two raw draws per double.
#pragma once
#include <random>
#include <cstdint>

inline thread_local bool rtw_inject_active = false;
inline thread_local uint64_t rtw_inject_state = 1;
inline thread_local uint64_t rtw_inject_draws = 0;

struct rtw_path_rng {
    typedef std::uint_fast32_t result_type;
    static constexpr result_type multiplier = 48271;
    static constexpr result_type increment = 0;
    static constexpr result_type modulus = 2147483647;
    static constexpr result_type default_seed = 1;
    static constexpr result_type min() { return 1; }
    static constexpr result_type max() { return 2147483646; }

    rtw_path_rng() : x(1) {}
    explicit rtw_path_rng(result_type s) { seed(s); }
    void seed(result_type s = default_seed) {
        x = s % modulus;
        if (x == 0) x = 1;
    }
    result_type operator()() {
        if (rtw_inject_active) {
            rtw_inject_state = (rtw_inject_state * 48271u) % 2147483647u;
            ++rtw_inject_draws;
            return (result_type)rtw_inject_state;
        }
        x = (x * 48271u) % 2147483647u;
        return x;
    }
    void discard(unsigned long long z) { for (; z; --z) (*this)(); }

    uint64_t x;
};

namespace std { using ::rtw_path_rng; }
#define minstd_rand rtw_path_rng

// splitmix64 finaliser (Steele, Lea, Flood 2014)
static inline uint64_t rtw_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// rtw_path_seed of include/rtw_gpu.h
static inline uint32_t rtw_inject_seed(uint64_t seed, uint32_t pixel, uint32_t s) {
    uint64_t k = ((uint64_t)s << 32) ^ (uint64_t)pixel;
    uint64_t h = rtw_splitmix64(rtw_splitmix64(seed) ^ k);
    return (uint32_t)(1u + h % 2147483646ull);
}

static inline void rtw_inject_begin(uint64_t seed, uint32_t pixel, uint32_t s) {
    rtw_inject_state = rtw_inject_seed(seed, pixel, s);
    rtw_inject_active = true;
}
static inline void rtw_inject_end() { rtw_inject_active = false; }
