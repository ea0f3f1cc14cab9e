// scene_api.cpp — out-of-line parts of the host scene API: Perlin tables,
// rotate_y's box, box's six rects, camera basis, bvh_node container.
#include <cmath>
#include <mutex>
#include <random>
#include "rtw/scene.h"
#include "rtw/texture.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

// ---------------------------------------------------------------- perlin
// noise.h:154-213.  Each generator owns a fresh default-seeded minstd_rand,
// so the three permutations are the same permutation.
namespace {
struct perlin_tables {
    double ranfloat[perlin::SIZE];
    vec3 ranvec[perlin::SIZE];
    int perm[3][perlin::SIZE];

    static void permutation(int* p) {
        for (int i = 0; i < perlin::SIZE; ++i) p[i] = i;
        std::uniform_real_distribution<double> U;
        std::minstd_rand eng;
        for (int i = perlin::SIZE - 1; i > 0; --i) {  // noise.h:171-177
            const int target = int(U(eng) * (i + 1));
            std::swap(p[i], p[target]);
        }
    }

    perlin_tables() {
        {
            std::uniform_real_distribution<double> U;
            std::minstd_rand eng;
            for (int i = 0; i < perlin::SIZE; ++i) ranfloat[i] = U(eng);  // noise.h:189-198
        }
        {
            // noise.h:200-213.  The reference builds vec3(f(), f(), f()); g++
            // evaluates those constructor arguments right to left, so the
            // first draw is z.  Spelled out explicitly here.
            std::uniform_real_distribution<double> U;
            std::minstd_rand eng;
            for (int i = 0; i < perlin::SIZE; ++i) {
                const double z = -1.0 + 2.0 * U(eng);
                const double y = -1.0 + 2.0 * U(eng);
                const double x = -1.0 + 2.0 * U(eng);
                ranvec[i] = normalize(vec3(x, y, z));
            }
        }
        for (int a = 0; a < 3; ++a) permutation(perm[a]);
    }
};

const perlin_tables& tables() {
    static const perlin_tables t;  // thread-safe lazy init (C++11 magic statics)
    return t;
}
}  // namespace

const double* perlin::ranfloat() { return tables().ranfloat; }
const vec3* perlin::ranvec() { return tables().ranvec; }
const int* perlin::perm_x() { return tables().perm[0]; }
const int* perlin::perm_y() { return tables().perm[1]; }
const int* perlin::perm_z() { return tables().perm[2]; }

// ---------------------------------------------------------------- rotate_y
// hittable.h:334-372: rotate the child's box corners about +y.  The
// reference indexes all three coordinates with the outer loop variable, so
// only the min and max corners are visited; kept for field parity (the public
// `bbox` is not used for rendering — the flattener computes its own bounds).
rotate_y::rotate_y(std::shared_ptr<hittable> p, double angle) : ptr(p) {
    const double radians = ((double)M_PI / 180.0) * angle;
    sin_theta = std::sin(radians);
    cos_theta = std::cos(radians);
    hasbox = ptr->bounding_box(0, 1, bbox);
    const double big = std::numeric_limits<double>::max();
    vec3 lo(big, big, big), hi(-big, -big, -big);
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
                const double x = i * bbox.max().x + (1 - i) * bbox.min().x;
                const double y = i * bbox.max().y + (1 - i) * bbox.min().y;
                const double z = i * bbox.max().z + (1 - i) * bbox.min().z;
                const vec3 c(cos_theta * x + sin_theta * z, y, -sin_theta * x + cos_theta * z);
                for (int a = 0; a < 3; ++a) {
                    if (c[a] > hi[a]) hi[a] = c[a];
                    if (c[a] < lo[a]) lo[a] = c[a];
                }
            }
    bbox = aabb(lo, hi);
}

// ---------------------------------------------------------------- box
box::box(const vec3& p0, const vec3& p1, std::shared_ptr<material> mat) : pmin(p0), pmax(p1) {
    auto& o = list_ptr.objects;
    o.push_back(std::make_shared<xy_rect>(p0.x, p1.x, p0.y, p1.y, p1.z, mat));
    o.push_back(std::make_shared<flip_normals>(std::make_shared<xy_rect>(p0.x, p1.x, p0.y, p1.y, p0.z, mat)));
    o.push_back(std::make_shared<xz_rect>(p0.x, p1.x, p0.z, p1.z, p1.y, mat));
    o.push_back(std::make_shared<flip_normals>(std::make_shared<xz_rect>(p0.x, p1.x, p0.z, p1.z, p0.y, mat)));
    o.push_back(std::make_shared<yz_rect>(p0.y, p1.y, p0.z, p1.z, p1.x, mat));
    o.push_back(std::make_shared<flip_normals>(std::make_shared<yz_rect>(p0.y, p1.y, p0.z, p1.z, p0.x, mat)));
}

// ---------------------------------------------------------------- bvh_node
static aabb union_of(const std::vector<std::shared_ptr<hittable>>& objs, double t0, double t1) {
    aabb acc;
    bool first = true;
    for (const auto& o : objs) {
        aabb b;
        if (!o->bounding_box(t0, t1, b)) continue;
        acc = first ? b : aabb::surrounding(acc, b);
        first = false;
    }
    return acc;
}

bvh_node::bvh_node(hittable** l, int n, double time0, double time1) {
    // The raw pointers are borrowed (the reference leaks them too); wrap
    // them without taking ownership.
    for (int i = 0; i < n; ++i) objects.push_back(std::shared_ptr<hittable>(l[i], [](hittable*) {}));
    box = union_of(objects, time0, time1);
}

bvh_node::bvh_node(const std::vector<std::shared_ptr<hittable>>& l, double time0, double time1) : objects(l) {
    box = union_of(objects, time0, time1);
}

// ---------------------------------------------------------------- camera
// camera.h:13-34, same fp64 operation order.
camera::camera(const vec3& lookfrom, const vec3& lookat, const vec3& vup, double vfov, double aspect,
               double aperture, double focus_dist, double t0, double t1) {
    time0 = t0;
    time1 = t1;
    lens_radius = aperture / 2;
    const double theta = vfov * static_cast<double>(M_PI) / 180.0;
    const double half_height = std::tan(theta / 2);
    const double half_width = aspect * half_height;
    origin = lookfrom;
    w = normalize(lookfrom - lookat);
    u = normalize(cross(vup, w));
    v = cross(w, u);
    lower_left_corner = origin - half_width * focus_dist * u - half_height * focus_dist * v - focus_dist * w;
    horizontal = 2.0 * half_width * focus_dist * u;
    vertical = 2.0 * half_height * focus_dist * v;
}

rtw_camera_desc camera::desc() const {
    rtw_camera_desc d;
    for (int a = 0; a < 3; ++a) {
        d.origin[a] = origin[a];
        d.lower_left[a] = lower_left_corner[a];
        d.horizontal[a] = horizontal[a];
        d.vertical[a] = vertical[a];
        d.u[a] = u[a];
        d.v[a] = v[a];
        d.w[a] = w[a];
    }
    d.time0 = time0;
    d.time1 = time1;
    d.lens_radius = lens_radius;
    return d;
}
