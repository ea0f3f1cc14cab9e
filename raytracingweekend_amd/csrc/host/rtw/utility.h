// utility.h surface of the host scene API (reference utility.h:6-81): the
// global random_double engine and the direction samplers, for scene code
// written against the reference (random_balls-style layouts, custom pdfs),
// and the engines the host classes' hit / scatter / get_ray draw from.
//
// Every engine of the host API (random_double's, the dielectric's and the
// medium's function-static ones, the camera's two members, a render loop's
// own) is an rtw::engine: std::minstd_rand's recurrence and range, default
// seed 1, consumed by libstdc++'s generate_canonical<double, 53> as two raw
// draws per double.  While an rtw::path_stream is alive on a thread, every
// rtw::engine on that thread draws from that stream instead: the per-sample
// stream of include/rtw_gpu.h (rtw_path_seed(seed, pixel, sample)), which is
// what the device kernels draw from, so a host render that opens one stream
// per camera sample reproduces the GPU's and the oracle's paths.
// Where the reference builds vec3(random_double(), ...) from several draws,
// g++ evaluates the arguments right to left; the draws are made explicitly in
// that order here (z, y, x), so the values do not depend on the compiler.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <random>
#include "vec3.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

namespace rtw {

// The stream a thread's engines draw from while a path_stream is open (0: none).
struct stream_state {
    uint64_t x = 0;       // minstd_rand state of the open stream, 0 = no stream open
    uint64_t draws = 0;   // raw draws taken from it
};
inline stream_state& current_stream() {
    static thread_local stream_state s;
    return s;
}

// rtw_path_seed (include/rtw_gpu.h): splitmix64 finaliser (Steele, Lea,
// Flood 2014) of the seed, mixed with (sample << 32) ^ pixel, into [1, 2^31-2]
inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
inline uint32_t path_seed(uint64_t seed, uint32_t pixel, uint32_t sample) {
    const uint64_t key = ((uint64_t)sample << 32) ^ (uint64_t)pixel;
    return (uint32_t)(1u + splitmix64(splitmix64(seed) ^ key) % 2147483646ull);
}

// std::minstd_rand's generator (48271 x mod 2^31 - 1), redirected to the
// thread's open path stream when there is one.
class engine {
public:
    typedef std::uint_fast32_t result_type;
    static constexpr result_type min() { return 1; }
    static constexpr result_type max() { return 2147483646; }
    engine() {}
    explicit engine(result_type s) { seed(s); }
    void seed(result_type s = 1) {
        state_ = s % 2147483647u;
        if (state_ == 0) state_ = 1;
    }
    result_type operator()() {
        stream_state& st = current_stream();
        uint64_t& x = st.x ? st.x : state_;
        if (st.x) ++st.draws;
        x = x * 48271u % 2147483647u;
        return (result_type)x;
    }

private:
    uint64_t state_ = 1;
};

// Opens the per-sample stream rtw_path_seed(seed, pixel, sample) on this
// thread for its lifetime (camera sample = one path_stream).
class path_stream {
public:
    path_stream(uint64_t seed, uint32_t pixel, uint32_t sample) : saved_(current_stream()) {
        current_stream() = stream_state{path_seed(seed, pixel, sample), 0};
    }
    ~path_stream() { current_stream() = saved_; }
    uint64_t draws() const { return current_stream().draws; }
    path_stream(const path_stream&) = delete;
    path_stream& operator=(const path_stream&) = delete;

private:
    stream_state saved_;
};

}  // namespace rtw

// utility.h:6-12 (the free function; sphere_base keeps its own copy)
inline void get_sphere_uv(const vec3& p, double& u, double& v) {
    const double phi = std::atan2(p.z, p.x);
    const double theta = std::asin(p.y);
    u = 1 - (phi + M_PI) / (2.0 * M_PI);
    v = (theta + M_PI / 2) / M_PI;
}

// utility.h:14-20: one engine for the whole program (an inline function's
// statics are shared by every translation unit)
inline double random_double(double a = 0.0, double b = 1.0) {
    static std::uniform_real_distribution<double> uniform;
    static rtw::engine engine;
    return a + (b - a) * uniform(engine);
}

// utility.h:22-25
inline int random_int(int a, int b) { return a + std::min(b - a, (int)((b - a + 1) * random_double())); }

// utility.h:27-35 (z drawn first, as g++ evaluates vec3(U, U, U))
inline vec3 random_in_unit_sphere() {
    vec3 p(0, 0, 0);
    do {
        const double z = random_double();
        const double y = random_double();
        const double x = random_double();
        p = 2.0 * vec3(x, y, z) - vec3(1, 1, 1);
    } while (dot(p, p) >= 1.0);
    return p;
}

namespace rtw {
// sin and cos of one angle.  g++ -O2 (the reference's build) turns the
// reference's cos(phi) ... sin(phi) pairs into ONE glibc sincos() call, and
// glibc's sincos and its separate sin / cos can differ in the last ulp; the
// host API makes that call explicitly, so its values do not depend on the
// compiler that builds it (clang keeps two calls).
inline void sin_cos(double phi, double& s, double& c) { ::sincos(phi, &s, &c); }
}  // namespace rtw

// utility.h:37-43 (a before z: two statements in the reference)
inline vec3 random_unit_vector() {
    const double a = random_double() * 2.0 * M_PI;
    const double z = random_double() * 2.0 - 1.0;
    const double r = std::sqrt(1 - z * z);
    double s, c;
    rtw::sin_cos(a, s, c);
    return vec3(r * c, r * s, z);
}

// utility.h:45-52
inline vec3 random_in_hemisphere(const vec3& normal) {
    const vec3 in_unit_sphere = random_in_unit_sphere();
    return dot(in_unit_sphere, normal) > 0.0 ? in_unit_sphere : -in_unit_sphere;
}

// utility.h:54-67: cosine-weighted direction about +z
inline vec3 random_cosine_direction() {
    const double r1 = random_double();
    const double r2 = random_double();
    const double z = std::sqrt(1 - r2);
    const double phi = 2 * M_PI * r1;
    double s, c;
    rtw::sin_cos(phi, s, c);
    const double x = c * std::sqrt(r2);
    const double y = s * std::sqrt(r2);
    return vec3(x, y, z);
}

// utility.h:69-81: uniform direction in the cone of a sphere of `radius`
// seen from distance sqrt(distance_squared), about +z
inline vec3 random_to_sphere(double radius, double distance_squared) {
    const double r1 = random_double();
    const double r2 = random_double();
    const double z = 1 + r2 * (std::sqrt(1 - radius * radius / distance_squared) - 1);
    const double phi = 2 * M_PI * r1;
    double s, c;
    rtw::sin_cos(phi, s, c);
    const double x = c * std::sqrt(1 - z * z);
    const double y = s * std::sqrt(1 - z * z);
    return vec3(x, y, z);
}
