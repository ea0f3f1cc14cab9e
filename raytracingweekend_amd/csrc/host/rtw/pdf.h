// pdf.h surface of the host scene API (reference pdf.h:6-79): the
// importance-sampling densities color() mixes at every lambertian bounce
// (RayTracingWeekend.cpp:117-124).
//
// The render evaluates them on the device (rtw_device.h mixture_generate,
// lights_pdf_value); these host classes give scene and tool code the same
// objects, drawing from utility.h's engine: cosine_pdf, hittable_pdf over any
// hittable (its pdf_value / random overrides: xz_rect, sphere, moving_sphere,
// hittable_list -- hittable.h, sphere.h, hittable_list.h) and the 50/50
// mixture_pdf.
#pragma once
#include <memory>
#include "hittable.h"
#include "onb.h"
#include "utility.h"

class pdf {
public:
    virtual ~pdf() {}
    virtual double value(const vec3& direction) const = 0;
    virtual vec3 generate() const = 0;
};

// pdf.h:15-33
class cosine_pdf : public pdf {
public:
    cosine_pdf(const vec3& w) { uvw.build_from_w(w); }
    double value(const vec3& direction) const override {
        const double cosine = dot(normalize(direction), uvw.w());
        return (cosine <= 0) ? 0 : cosine / M_PI;
    }
    vec3 generate() const override { return uvw.local(random_cosine_direction()); }

private:
    onb uvw;
};

// pdf.h:35-53
class hittable_pdf : public pdf {
public:
    hittable_pdf(std::shared_ptr<hittable> p, const vec3& origin) : o(origin), ptr(p) {}
    double value(const vec3& direction) const override { return ptr->pdf_value(o, direction); }
    vec3 generate() const override { return ptr->random(o); }

    vec3 o;
    std::shared_ptr<hittable> ptr;
};

// pdf.h:55-79
class mixture_pdf : public pdf {
public:
    mixture_pdf(std::shared_ptr<pdf> p0, std::shared_ptr<pdf> p1) {
        p[0] = p0;
        p[1] = p1;
    }
    double value(const vec3& direction) const override {
        return 0.5 * p[0]->value(direction) + 0.5 * p[1]->value(direction);
    }
    vec3 generate() const override { return random_double() < 0.5 ? p[0]->generate() : p[1]->generate(); }

private:
    std::shared_ptr<pdf> p[2];
};
