// utility.h surface of the host scene API (reference utility.h:6-81): the
// global random_double engine and the direction samplers, for scene code
// written against the reference (random_balls-style layouts, custom pdfs).
//
// Host only.  Renders draw on the device from per-sample streams
// (rtw_path_seed) with these same formulas (rtw_device.h); this engine is
// the reference's single function-static std::minstd_rand, default seeded,
// with libstdc++'s generate_canonical<double, 53> (two raw draws per double).
// Where the reference builds vec3(random_double(), ...) from several draws,
// g++ evaluates the arguments right to left; the draws are made explicitly in
// that order here (z, y, x), so the values do not depend on the compiler.
#pragma once
#include <algorithm>
#include <cmath>
#include <random>
#include "vec3.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

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
    static std::minstd_rand engine;
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

// utility.h:37-43 (a before z: two statements in the reference)
inline vec3 random_unit_vector() {
    const double a = random_double() * 2.0 * M_PI;
    const double z = random_double() * 2.0 - 1.0;
    const double r = std::sqrt(1 - z * z);
    return vec3(r * std::cos(a), r * std::sin(a), z);
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
    const double x = std::cos(phi) * std::sqrt(r2);
    const double y = std::sin(phi) * std::sqrt(r2);
    return vec3(x, y, z);
}

// utility.h:69-81: uniform direction in the cone of a sphere of `radius`
// seen from distance sqrt(distance_squared), about +z
inline vec3 random_to_sphere(double radius, double distance_squared) {
    const double r1 = random_double();
    const double r2 = random_double();
    const double z = 1 + r2 * (std::sqrt(1 - radius * radius / distance_squared) - 1);
    const double phi = 2 * M_PI * r1;
    const double x = std::cos(phi) * std::sqrt(1 - z * z);
    const double y = std::sin(phi) * std::sqrt(1 - z * z);
    return vec3(x, y, z);
}
