// hittable_list.h surface of the host scene API (reference hittable_list.h:5-114).
#pragma once
#include "material.h"
#include "sphere.h"

class hittable_list : public hittable {
public:
    hittable_list() {}
    hittable_list(const std::vector<std::shared_ptr<hittable>>& l) : objects(l) {}
    // hittable_list.h:11-37: closest hit over the objects, walked TWICE with
    // the closest distance carried over.  For deterministic shapes the second
    // walk re-accepts only hits at exactly that distance (rects: t == t_max
    // is accepted), so ties go to the last such object; a medium draws a
    // fresh free-flight distance in each walk.
    bool hit(const ray& r, double t_min, double t_max, hit_record& rec) const override {
        hit_record cand;
        bool any = false;
        double closest = t_max;
        for (int walk = 0; walk < 2; ++walk) {
            for (const auto& object : objects) {
                if (!object->hit(r, t_min, closest, cand)) continue;
                any = true;
                closest = cand.t;
                rec = cand;
            }
        }
        return any;
    }
    // As the reference (hittable_list.h:39-42): reports true without setting `box`.
    bool bounding_box(double, double, aabb&) const override { return true; }
    // hittable_list.h:44-53: the members' densities, equally weighted
    double pdf_value(const vec3& o, const vec3& v) const override {
        const double weight = 1.0 / objects.size();
        double sum = 0.0;
        for (const auto& object : objects) sum += weight * object->pdf_value(o, v);
        return sum;
    }
    // hittable_list.h:55-59: a uniformly chosen member's direction
    vec3 random(const vec3& o) const override {
        const int int_size = static_cast<int>(objects.size());
        return objects[random_int(0, int_size - 1)]->random(o);
    }
    std::vector<std::shared_ptr<hittable>> objects;
};

// Axis-aligned box as six rects (hittable_list.h:65-114): +z, -z(flipped),
// +y, -y(flipped), +x, -x(flipped) — the order matters for tie-breaking.
class box : public hittable {
public:
    box() {}
    box(const vec3& p0, const vec3& p1, std::shared_ptr<material> mat);
    // hittable_list.h:106-110: the six rects' list (its own double walk)
    bool hit(const ray& r, double t0, double t1, hit_record& rec) const override { return list_ptr.hit(r, t0, t1, rec); }
    bool bounding_box(double, double, aabb& b) const override {
        b = aabb(pmin, pmax);
        return true;
    }
    vec3 pmin, pmax;
    hittable_list list_ptr;
};
