// sphere.h surface of the host scene API (reference sphere.h:6-131).
#pragma once
#include "hittable.h"
#include "material.h"

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
    // sphere.h:46-81: the half-b quadratic about the centre at the ray's
    // time; the near root, else the far one, strictly inside (t_min, t_max);
    // normal (p - c) / radius (inward for a negative radius: hollow glass)
    bool hit(const ray& r, double t_min, double t_max, hit_record& rec) const override {
        const vec3 c_now = movement.center(center, r.time());
        const vec3 oc = r.origin() - c_now;
        const double a = dot(r.direction(), r.direction());
        const double b = dot(oc, r.direction());
        const double c = dot(oc, oc) - radius * radius;
        const double disc = b * b - a * c;
        if (!(disc > 0)) return false;
        for (int side = -1; side <= 1; side += 2) {
            const double root = (-b + side * std::sqrt(disc)) / a;
            if (root < t_max && root > t_min) {
                rec.t = root;
                rec.p = r.point_at_parameter(root);
                rec.normal = (rec.p - c_now) / radius;
                get_sphere_uv(rec.normal, rec.u, rec.v);
                rec.mat_ptr = mat.get();
                return true;
            }
        }
        return false;
    }
    bool bounding_box(double t0, double t1, aabb& box) const override {
        return movement.bounding_box(center, radius, t0, t1, box);
    }
    void set_movement(const movement_type& m) { movement = m; }

    // sphere.h:88-99: uniform density over the cone the sphere subtends,
    // where a ray of time FLT_MAX along v hits it in (0.001, +inf)
    double pdf_value(const vec3& o, const vec3& v) const override {
        hit_record rec;
        if (!hit(ray(o, v, FLT_MAX), 0.001, std::numeric_limits<double>::infinity(), rec)) return 0.0;
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

    // sphere.h:115-122: longitude / latitude of a unit normal
    static void get_sphere_uv(const vec3& p, double& u, double& v) { ::get_sphere_uv(p, u, v); }

    vec3 center;
    double radius;
    std::shared_ptr<material> mat;
    movement_type movement;
};

typedef sphere_base<movement_none> sphere;
typedef sphere_base<movement_linear> moving_sphere;
