// texture.h / noise.h surface of the host scene API.
// Reference: texture.h:10-71 (constant, checker, noise) and noise.h:71-225
// (perlin lookup tables).  The per-point evaluation (value(), noise(), turb())
// runs on the device; the host only owns the tables, which it generates with
// the reference's algorithm so that the device sees identical lattices.
#pragma once
#include <memory>
#include "vec3.h"

class texture {
public:
    virtual ~texture() {}
};

class constant_texture : public texture {
public:
    constant_texture() {}
    constant_texture(vec3 c) : color(c) {}
    vec3 color;
};

class checker_texture : public texture {
public:
    checker_texture() {}
    checker_texture(std::shared_ptr<texture>& t0, std::shared_ptr<texture>& t1) : odd(t1), even(t0) {}
    std::shared_ptr<texture> odd;
    std::shared_ptr<texture> even;
};

// Perlin tables (noise.h:154-223).  Every table is generated from its own
// freshly default-seeded std::minstd_rand, exactly as the reference does, so
// perm_x, perm_y and perm_z come out identical.
class perlin {
public:
    static constexpr int SIZE = 256;
    static const double* ranfloat();  // SIZE
    static const vec3* ranvec();      // SIZE, normalised
    static const int* perm_x();
    static const int* perm_y();
    static const int* perm_z();
};

class noise_texture : public texture {
public:
    noise_texture() : scale(5.f) {}
    noise_texture(double sc) : scale(sc) {}
    perlin noise;
    double scale;
};
