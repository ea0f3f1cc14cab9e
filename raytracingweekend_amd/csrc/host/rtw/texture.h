// texture.h / noise.h surface of the host scene API.
// Reference: texture.h:10-71 (constant, checker, noise) and noise.h:9-225
// (Perlin lattice noise and its tables).  value(), noise() and turb() are
// evaluated on the host with the reference's arithmetic (IEEE fp64, glibc
// sin); the device kernels have their own restatement for renders and read
// the same tables, which the host generates with the reference's algorithm
// (scene_api.cpp) so both see identical lattices.
#pragma once
#include <cmath>
#include <memory>
#include "vec3.h"

class texture {
public:
    virtual ~texture() {}
    virtual vec3 value(double u, double v, const vec3& p) const = 0;
};

class constant_texture : public texture {
public:
    constant_texture() {}
    constant_texture(vec3 c) : color(c) {}
    vec3 value(double, double, const vec3&) const override { return color; }
    vec3 color;
};

// texture.h:29-49: alternates by the sign of sin(10x) sin(10y) sin(10z)
class checker_texture : public texture {
public:
    checker_texture() {}
    checker_texture(std::shared_ptr<texture>& t0, std::shared_ptr<texture>& t1) : odd(t1), even(t0) {}
    vec3 value(double u, double v, const vec3& p) const override {
        const double sines = std::sin(10.0 * p.x) * std::sin(10.0 * p.y) * std::sin(10.0 * p.z);
        return (sines < 0 ? odd : even)->value(u, v, p);
    }
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

    // noise.h:100-146 (the PERLIN interpolation the reference selects): the
    // eight lattice gradients around p, each dotted with p's offset from its
    // corner, blended with Hermite-smoothed weights (noise.h:9-12, 40-58);
    // in [-1, 1]
    double noise(const vec3& p) const {
        const double fx = std::floor(p.x), fy = std::floor(p.y), fz = std::floor(p.z);
        const double u = p.x - fx, v = p.y - fy, w = p.z - fz;
        const int i = (int)fx, j = (int)fy, k = (int)fz;
        const double su = u * u * (3 - 2 * u), sv = v * v * (3 - 2 * v), sw = w * w * (3 - 2 * w);
        const vec3* g = ranvec();
        const int *px = perm_x(), *py = perm_y(), *pz = perm_z();
        double sum = 0;
        for (int di = 0; di < 2; ++di)
            for (int dj = 0; dj < 2; ++dj)
                for (int dk = 0; dk < 2; ++dk) {
                    const vec3& grad = g[px[(i + di) & 255] ^ py[(j + dj) & 255] ^ pz[(k + dk) & 255]];
                    // a corner's weight is the smoothed fraction (far corner) or its
                    // complement (near corner): i*uu + (1-i)*(1-uu) in the reference
                    const double wi = di ? su : 1 - su, wj = dj ? sv : 1 - sv, wk = dk ? sw : 1 - sw;
                    sum += wi * wj * wk * dot(grad, vec3(u - di, v - dj, w - dk));
                }
        return sum;
    }
    // noise.h:74-86: |sum of depth octaves|, each at twice the frequency and
    // half (0.5f) the weight of the last
    double turb(const vec3& p, int depth = 7) const {
        double sum = 0, weight = 1.0;
        vec3 q = p;
        for (int octave = 0; octave < depth; ++octave) {
            sum += weight * noise(q);
            weight *= 0.5f;
            q *= 2;
        }
        return std::fabs(sum);
    }
};

// texture.h:52-71: marble stripes along z, 0.5 (1 + sin(scale z + 10
// turb(p))) -- turbulence of p itself, not of scale * p
class noise_texture : public texture {
public:
    noise_texture() : scale(5.f) {}
    noise_texture(double sc) : scale(sc) {}
    vec3 value(double, double, const vec3& p) const override {
        const double phase = 1 + std::sin(scale * p.z + 10 * noise.turb(p));
        return vec3(1, 1, 1) * 0.5f * phase;
    }
    perlin noise;
    double scale;
};
