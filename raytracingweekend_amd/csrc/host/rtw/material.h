// material.h surface of the host scene API (reference material.h:59-265).
// Materials are descriptions here; scatter/emitted/scattering_pdf are
// evaluated by the device shade kernel (raytracingweekend_amd/csrc/rtw_device.h).
#pragma once
#include <memory>
#include <random>  // as the reference's material.h:3: scene code draws with std::minstd_rand
#include "texture.h"

class material {
public:
    virtual ~material() {}
};

class lambertian : public material {
public:
    explicit lambertian(std::shared_ptr<texture> a) : albedo(a) {}
    std::shared_ptr<texture> albedo;
};

class metal : public material {
public:
    explicit metal(const vec3& a, double f) : albedo(a), fuzz(f) {}  // no fuzz clamp (material.h:127)
    vec3 albedo;
    double fuzz;
};

class dielectric : public material {
public:
    explicit dielectric(double ri) : ref_idx(ri) {}
    double ref_idx;
};

class diffuse_light : public material {
public:
    diffuse_light(std::shared_ptr<texture> a) : emit(a) {}
    std::shared_ptr<texture> emit;
};

class isotropic : public material {
public:
    isotropic(std::shared_ptr<texture> t) : albedo(t) {}
    std::shared_ptr<texture> albedo;
};
