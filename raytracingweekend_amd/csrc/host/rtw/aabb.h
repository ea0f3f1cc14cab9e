// aabb.h surface of the host scene API (reference aabb.h:10-65).  aabb::hit
// keeps the reference's slab semantics (std::max / std::min, so a NaN slab
// keeps the running bound; reject tmax <= tmin) for API compatibility and the
// reference's own unit tests (CppTest/unittest1.cpp:72-109); the device walks
// its own fp32 boxes (rtw_device.h slab32).
#pragma once
#include <utility>
#include "vec3.h"

class ray;

class aabb {
public:
    aabb() {}
    aabb(const vec3& lo, const vec3& hi) : _min(lo), _max(hi) {}
    vec3 min() const { return _min; }
    vec3 max() const { return _max; }

    inline bool hit(const ray& r, double tmin, double tmax) const;

    static aabb surrounding(const aabb& p, const aabb& q) {
        return aabb(vec3(std::fmin(p._min.x, q._min.x), std::fmin(p._min.y, q._min.y), std::fmin(p._min.z, q._min.z)),
                    vec3(std::fmax(p._max.x, q._max.x), std::fmax(p._max.y, q._max.y), std::fmax(p._max.z, q._max.z)));
    }

    vec3 _min, _max;
};

#include "ray.h"

inline bool aabb::hit(const ray& r, double tmin, double tmax) const {
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
