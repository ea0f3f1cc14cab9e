// material.h surface of the host scene API (reference material.h:1-264).
// The five materials with the reference's constructors and fields, and the
// evaluating interface color() calls (RayTracingWeekend.cpp:45-160):
// scatter (into a scatter_record: a specular continuation ray, or a pdf to
// importance-sample), emitted and scattering_pdf, with the reference's fp64
// arithmetic.  Draws come from utility.h's engines (the thread's path stream
// while one is open).  Renders never call these: the device's shade_core
// (raytracingweekend_amd/csrc/rtw_device.h) restates them.
#pragma once
#include <cmath>
#include <memory>
#include <random>  // as the reference's material.h:3: scene code draws with std::minstd_rand
#include "hittable.h"
#include "pdf.h"
#include "texture.h"

// material.h:10-13: mirror v about n
inline vec3 reflect(const vec3& v, const vec3& n) { return v - 2.0 * dot(v, n) * n; }

// material.h:17-39: Snell's law for the normalised v (ni_over_nt = n_i / n_t);
// false on total internal reflection
inline bool refract(const vec3& v, const vec3& n, double ni_over_nt, vec3& refracted) {
    const vec3 uv = normalize(v);
    const double cos_i = dot(uv, n);
    const double cos_t2 = 1.0 - ni_over_nt * ni_over_nt * (1 - cos_i * cos_i);
    if (!(cos_t2 > 0)) return false;
    refracted = ni_over_nt * (uv - n * cos_i) - n * std::sqrt(cos_t2);
    return true;
}

// material.h:44-49: Schlick's Fresnel reflectance
inline double schlick(double cosine, double ref_idx) {
    const double r = (1 - ref_idx) / (1 + ref_idx);
    const double r0 = r * r;
    return r0 + (1 - r0) * std::pow((1 - cosine), 5);
}

// material.h:51-57: either a continuation ray whose direction is fixed
// (pdf_ptr null: metal, dielectric, isotropic) or a pdf to sample
struct scatter_record {
    ray scattered_ray_without_pdf;
    std::shared_ptr<pdf> pdf_ptr;
    vec3 attenuation;
};

class material {
public:
    virtual ~material() {}
    virtual bool scatter(const ray& r_in, const hit_record& rec, scatter_record& srec) const = 0;
    virtual double scattering_pdf(const ray& r_in, const hit_record& rec, const ray& scattered) const { return 0.0; }
    virtual vec3 emitted(const ray& r_in, const hit_record& rec, double u, double v, const vec3& p) const {
        return vec3(0, 0, 0);
    }
};

// material.h:81-122: cosine-weighted diffuse reflection
class lambertian : public material {
public:
    explicit lambertian(std::shared_ptr<texture> a) : albedo(a) {}
    bool scatter(const ray&, const hit_record& rec, scatter_record& srec) const override {
        srec.attenuation = albedo->value(rec.u, rec.v, rec.p);
        srec.pdf_ptr = std::make_shared<cosine_pdf>(rec.normal);
        return true;
    }
    double scattering_pdf(const ray&, const hit_record& rec, const ray& scattered) const override {
        const double cosine = dot(rec.normal, normalize(scattered.direction()));
        return cosine < 0 ? 0 : cosine / M_PI;
    }
    std::shared_ptr<texture> albedo;
};

// material.h:124-140: mirror reflection of the normalised direction,
// perturbed by fuzz * a point of the unit ball; never absorbs
class metal : public material {
public:
    explicit metal(const vec3& a, double f) : albedo(a), fuzz(f) {}  // no fuzz clamp (material.h:127)
    bool scatter(const ray& r_in, const hit_record& rec, scatter_record& srec) const override {
        const vec3 mirrored = reflect(normalize(r_in.direction()), rec.normal);
        srec.scattered_ray_without_pdf = ray(rec.p, mirrored + fuzz * random_in_unit_sphere(), r_in.time());
        srec.attenuation = albedo;
        srec.pdf_ptr = nullptr;
        return true;
    }
    vec3 albedo;
    double fuzz;
};

// material.h:142-225: glass.  Leaving the surface (d . n > 0) the Schlick
// cosine is the refracted angle's, sqrt(1 - n^2 (1 - c^2)) (the corrected
// form, material.h:165-173).  One uniform draw always decides between the
// reflected and the refracted ray, total internal reflection included
// (reflect_prob 1), from the material's own engine.
class dielectric : public material {
public:
    explicit dielectric(double ri) : ref_idx(ri) {}
    bool scatter(const ray& r_in, const hit_record& rec, scatter_record& srec) const override {
        static std::uniform_real_distribution<double> uniform;
        static rtw::engine engine;
        srec.attenuation = vec3(1.0, 1.0, 1.0);
        const vec3 d = r_in.direction();
        const bool leaving = dot(d, rec.normal) > 0;
        const vec3 outward_normal = leaving ? -rec.normal : rec.normal;
        const double ni_over_nt = leaving ? ref_idx : 1.0 / ref_idx;
        double cosine;
        if (leaving) {
            const double c = dot(d, rec.normal) / d.length();
            cosine = std::sqrt(1 - ref_idx * ref_idx * (1 - c * c));
        } else {
            cosine = -dot(d, rec.normal) / d.length();
        }
        const vec3 reflected = reflect(d, rec.normal);
        vec3 refracted;
        const double reflect_prob = refract(d, outward_normal, ni_over_nt, refracted) ? schlick(cosine, ref_idx) : 1.0;
        const bool mirror = uniform(engine) < reflect_prob;
        srec.scattered_ray_without_pdf = ray(rec.p, mirror ? reflected : refracted, r_in.time());
        return true;
    }
    double ref_idx;
};

// material.h:227-245: emits its texture on the side its normal faces
// (dot(normal, d) > 0); never scatters
class diffuse_light : public material {
public:
    diffuse_light(std::shared_ptr<texture> a) : emit(a) {}
    bool scatter(const ray&, const hit_record&, scatter_record&) const override { return false; }
    vec3 emitted(const ray& r_in, const hit_record& rec, double u, double v, const vec3& p) const override {
        if (dot(rec.normal, r_in.direction()) > 0) return emit->value(u, v, p);
        return vec3(0, 0, 0);
    }
    std::shared_ptr<texture> emit;
};

// material.h:247-262: phase function of a medium: a direction from the unit
// ball (not normalised), attenuated by the texture
class isotropic : public material {
public:
    isotropic(std::shared_ptr<texture> t) : albedo(t) {}
    bool scatter(const ray& r_in, const hit_record& rec, scatter_record& srec) const override {
        srec.scattered_ray_without_pdf = ray(rec.p, random_in_unit_sphere(), r_in.time());
        srec.attenuation = albedo->value(rec.u, rec.v, rec.p);
        return true;
    }
    std::shared_ptr<texture> albedo;
};
