// sphere.h surface of the host scene API (reference sphere.h:6-131).
#pragma once
#include "hittable.h"

struct movement_none {
    vec3 center(const vec3& center0, double) const { return center0; }
    bool bounding_box(const vec3& c, double r, double, double, aabb& box) const {
        box = aabb(c - vec3(r, r, r), c + vec3(r, r, r));
        return true;
    }
};

struct movement_linear {
    vec3 center(const vec3& center0, double time) const {
        return center0 + ((time - time0) / (time1 - time0)) * (center1 - center0);
    }
    bool bounding_box(const vec3& c, double r, double, double, aabb& box) const {
        aabb a(c - vec3(r, r, r), c + vec3(r, r, r));
        aabb b(center1 - vec3(r, r, r), center1 + vec3(r, r, r));
        box = aabb::surrounding(a, b);
        return true;
    }
    vec3 center1;
    double time0 = 0.0;
    double time1 = 1.0;
};

template <typename movement_type>
class sphere_base : public hittable {
public:
    sphere_base() : center(0, 0, 0), radius(0), mat(nullptr) {}
    sphere_base(vec3 cen, double r, std::shared_ptr<material> m) : center(cen), radius(r), mat(m) {}
    bool bounding_box(double t0, double t1, aabb& box) const override {
        return movement.bounding_box(center, radius, t0, t1, box);
    }
    void set_movement(const movement_type& m) { movement = m; }

    vec3 center;
    double radius;
    std::shared_ptr<material> mat;
    movement_type movement;
};

typedef sphere_base<movement_none> sphere;
typedef sphere_base<movement_linear> moving_sphere;
