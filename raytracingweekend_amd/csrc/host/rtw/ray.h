// ray.h / aabb.h surface of the host scene API (reference: ray.h:5-21,
// aabb.h:10-65).  aabb::hit is kept for API compatibility and host-side tests
// of the reference's slab semantics (std::max/std::min, reject tmax <= tmin).
#pragma once
#include <utility>
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

class aabb {
public:
    aabb() {}
    aabb(const vec3& lo, const vec3& hi) : _min(lo), _max(hi) {}
    vec3 min() const { return _min; }
    vec3 max() const { return _max; }

    bool hit(const ray& r, double tmin, double tmax) const {
        for (int a = 0; a < 3; ++a) {
            const double inv = 1.0 / r.direction()[a];
            double ta = (_min[a] - r.origin()[a]) * inv;
            double tb = (_max[a] - r.origin()[a]) * inv;
            if (inv < 0.0) std::swap(ta, tb);
            tmin = std::max(ta, tmin);
            tmax = std::min(tb, tmax);
            if (tmax <= tmin) return false;
        }
        return true;
    }

    static aabb surrounding(const aabb& p, const aabb& q) {
        return aabb(vec3(std::fmin(p._min.x, q._min.x), std::fmin(p._min.y, q._min.y), std::fmin(p._min.z, q._min.z)),
                    vec3(std::fmax(p._max.x, q._max.x), std::fmax(p._max.y, q._max.y), std::fmax(p._max.z, q._max.z)));
    }

    vec3 _min, _max;
};
