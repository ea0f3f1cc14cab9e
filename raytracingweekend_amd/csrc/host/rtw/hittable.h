// hittable.h surface of the host scene API (reference hittable.h:31-489).
//
// The classes keep the reference's names, constructor signatures and public
// fields, so scene code written against the reference compiles unchanged.
// They describe geometry; closest-hit queries (hit) are answered by the
// device kernels after rtw_flatten_scene() has turned the graph into an
// rtw_scene_desc.  bounding_box() keeps the reference's results (including
// the +-0.0001f rect slabs and rotate_y's rotated corner box), and the light
// sampling surface pdf_value() / random() (hittable.h:36-37, the xz_rect,
// sphere and hittable_list overrides) is evaluated on the host with the
// reference's arithmetic for pdf.h's hittable_pdf.
#pragma once
#include <cfloat>
#include <cmath>
#include <limits>
#include <memory>
#include <vector>
#include "aabb.h"
#include "material.h"
#include "onb.h"
#include "utility.h"

class hittable {
public:
    virtual ~hittable() {}
    virtual bool bounding_box(double t0, double t1, aabb& box) const = 0;
    // hittable.h:36-37: the defaults for objects that are not light shapes
    virtual double pdf_value(const vec3& o, const vec3& v) const { return 0.0; }
    virtual vec3 random(const vec3& o) const { return vec3(1, 0, 0); }
};

class xy_rect : public hittable {
public:
    xy_rect() {}
    xy_rect(double _x0, double _x1, double _y0, double _y1, double _k, std::shared_ptr<material> mat)
        : x0(_x0), x1(_x1), y0(_y0), y1(_y1), k(_k), mp(mat) {}
    bool bounding_box(double, double, aabb& box) const override {
        box = aabb(vec3(x0, y0, k - 0.0001f), vec3(x1, y1, k + 0.0001f));
        return true;
    }
    double x0, x1, y0, y1, k;
    std::shared_ptr<material> mp;
};

class xz_rect : public hittable {
public:
    xz_rect() {}
    xz_rect(double _x0, double _x1, double _z0, double _z1, double _k, std::shared_ptr<material> mat)
        : x0(_x0), x1(_x1), z0(_z0), z1(_z1), k(_k), mp(mat) {}
    bool bounding_box(double, double, aabb& box) const override {
        box = aabb(vec3(x0, k - 0.0001f, z0), vec3(x1, k + 0.0001f, z1));
        return true;
    }
    // hittable.h:208-222: the solid-angle density of a hit of the rect along
    // v, through xz_rect::hit (:184-200) on a ray of time FLT_MAX, t in
    // (0.001, +inf]
    double pdf_value(const vec3& origin, const vec3& v) const override {
        const ray r(origin, v, FLT_MAX);
        const double t = (k - r.origin().y) / r.direction().y;
        if (t < 0.001 || t > std::numeric_limits<double>::infinity()) return 0;
        const double x = r.origin().x + t * r.direction().x;
        const double z = r.origin().z + t * r.direction().z;
        if (x < x0 || x > x1 || z < z0 || z > z1) return 0;
        const double area = (x1 - x0) * (z1 - z0);
        const double distance_squared = t * t * v.length_squared();
        const double cosine = std::fabs(dot(v, vec3(0, 1, 0)) / v.length());
        return distance_squared / (cosine * area);
    }
    // hittable.h:224-228 (z drawn first, as g++ evaluates the vec3 arguments)
    vec3 random(const vec3& origin) const override {
        const double rz = random_double(z0, z1);
        const double rx = random_double(x0, x1);
        return vec3(rx, k, rz) - origin;
    }
    double x0, x1, z0, z1, k;
    std::shared_ptr<material> mp;
};

class yz_rect : public hittable {
public:
    yz_rect() {}
    yz_rect(double _y0, double _y1, double _z0, double _z1, double _k, std::shared_ptr<material> mat)
        : y0(_y0), y1(_y1), z0(_z0), z1(_z1), k(_k), mp(mat) {}
    bool bounding_box(double, double, aabb& box) const override {
        box = aabb(vec3(k - 0.0001f, y0, z0), vec3(k + 0.0001f, y1, z1));
        return true;
    }
    double y0, y1, z0, z1, k;
    std::shared_ptr<material> mp;
};

class flip_normals : public hittable {
public:
    flip_normals(std::shared_ptr<hittable> p) : ptr(p) {}
    bool bounding_box(double t0, double t1, aabb& box) const override { return ptr->bounding_box(t0, t1, box); }
    std::shared_ptr<hittable> ptr;
};

class translate : public hittable {
public:
    translate(std::shared_ptr<hittable> p, const vec3& displacement) : ptr(p), offset(displacement) {}
    bool bounding_box(double t0, double t1, aabb& box) const override {
        if (!ptr->bounding_box(t0, t1, box)) return false;
        box = aabb(box.min() + offset, box.max() + offset);
        return true;
    }
    std::shared_ptr<hittable> ptr;
    vec3 offset;
};

class rotate_y : public hittable {
public:
    rotate_y(std::shared_ptr<hittable> p, double angle);
    bool bounding_box(double, double, aabb& box) const override {
        box = bbox;
        return hasbox;
    }
    std::shared_ptr<hittable> ptr;
    double sin_theta;
    double cos_theta;
    bool hasbox;
    aabb bbox;
};

class constant_medium : public hittable {
public:
    constant_medium(std::shared_ptr<hittable> b, double d, std::shared_ptr<material> mat)
        : boundary(b), density(d), mp(mat) {}
    bool bounding_box(double t0, double t1, aabb& box) const override { return boundary->bounding_box(t0, t1, box); }
    std::shared_ptr<hittable> boundary;
    double density;
    std::shared_ptr<material> mp;
};

// bvh_node: the reference's version (hittable.h:41-140) never assigns `right`,
// tests `left` twice and sorts n-1 elements, and no scene uses
// it.  Here it is a correct container: its objects are flattened as a group
// and the library builds a device BVH over them, whose closest hit equals the
// flat hittable_list's (same comparison operators and tie order).
class bvh_node : public hittable {
public:
    bvh_node() {}
    bvh_node(hittable** l, int n, double time0, double time1);
    bvh_node(const std::vector<std::shared_ptr<hittable>>& l, double time0, double time1);
    bool bounding_box(double, double, aabb& b) const override {
        b = box;
        return true;
    }
    std::vector<std::shared_ptr<hittable>> objects;
    aabb box;
};
