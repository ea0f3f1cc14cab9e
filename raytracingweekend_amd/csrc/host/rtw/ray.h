// ray.h surface of the host scene API (reference ray.h:5-21).
#pragma once
#include "vec3.h"

class ray {
public:
    ray() {}
    ray(const vec3& origin, const vec3& direction, double time) : o_(origin), d_(direction), t_(time) {}
    vec3 origin() const { return o_; }
    vec3 direction() const { return d_; }  // not normalised
    double time() const { return t_; }
    vec3 point_at_parameter(double t) const { return o_ + d_ * t; }

private:
    vec3 o_, d_;
    double t_ = 0.0;
};
#include "aabb.h"  // scene code reaches aabb through the ray / hittable headers
