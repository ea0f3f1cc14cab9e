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

    // sphere.h:88-99: uniform density over the cone the sphere subtends,
    // where a ray of time FLT_MAX along v hits it in (0.001, +inf)
    // (sphere.h:46-81's roots about the centre at that time)
    double pdf_value(const vec3& o, const vec3& v) const override {
        const ray r(o, v, FLT_MAX);
        const vec3 oc = r.origin() - movement.center(center, r.time());
        const double a = dot(r.direction(), r.direction());
        const double b = dot(oc, r.direction());
        const double c = dot(oc, oc) - radius * radius;
        const double disc = b * b - a * c;
        const double t_max = std::numeric_limits<double>::infinity();
        if (!(disc > 0)) return 0.0;
        double temp = (-b - std::sqrt(disc)) / a;
        if (!(temp < t_max && temp > 0.001)) {
            temp = (-b + std::sqrt(disc)) / a;
            if (!(temp < t_max && temp > 0.001)) return 0.0;
        }
        const double cos_theta_max = std::sqrt(1 - radius * radius / (center - o).length_squared());
        const double solid_angle = 2.0 * M_PI * (1.0 - cos_theta_max);
        return 1.0 / solid_angle;
    }
    // sphere.h:101-108
    vec3 random(const vec3& o) const override {
        const vec3 direction = center - o;
        const double distance_squared = direction.length_squared();
        onb uvw;
        uvw.build_from_w(direction);
        return uvw.local(random_to_sphere(radius, distance_squared));
    }

    vec3 center;
    double radius;
    std::shared_ptr<material> mat;
    movement_type movement;
};

typedef sphere_base<movement_none> sphere;
typedef sphere_base<movement_linear> moving_sphere;
