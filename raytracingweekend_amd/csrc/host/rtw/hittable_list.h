// hittable_list.h surface of the host scene API (reference hittable_list.h:5-114).
#pragma once
#include "sphere.h"

class hittable_list : public hittable {
public:
    hittable_list() {}
    hittable_list(const std::vector<std::shared_ptr<hittable>>& l) : objects(l) {}
    // As the reference (hittable_list.h:39-42): reports true without setting `box`.
    bool bounding_box(double, double, aabb&) const override { return true; }
    std::vector<std::shared_ptr<hittable>> objects;
};

// Axis-aligned box as six rects (hittable_list.h:65-114): +z, -z(flipped),
// +y, -y(flipped), +x, -x(flipped) — the order matters for tie-breaking.
class box : public hittable {
public:
    box() {}
    box(const vec3& p0, const vec3& p1, std::shared_ptr<material> mat);
    bool bounding_box(double, double, aabb& b) const override {
        b = aabb(pmin, pmax);
        return true;
    }
    vec3 pmin, pmax;
    hittable_list list_ptr;
};
