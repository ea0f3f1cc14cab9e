// scene_api.cpp — out-of-line parts of the host scene API: Perlin tables,
// rotate_y's box, box's six rects, camera basis, bvh_node container.
#include <algorithm>
#include <cmath>
#include <limits>
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
namespace {
// A box grown by a relative margin, so that rounding in aabb::hit never
// culls a hit the object's own test accepts (the walk only narrows the
// candidates; the objects decide).
aabb widened(const aabb& b) {
    vec3 lo = b.min(), hi = b.max();
    for (int a = 0; a < 3; ++a) {
        const double m = 1e-9 * (std::fabs(lo[a]) + std::fabs(hi[a]) + 1.0);
        lo[a] -= m;
        hi[a] += m;
    }
    return aabb(lo, hi);
}
// A box that really bounds h over [t0, t1].  The reference's own boxes are
// not always that: hittable_list::bounding_box reports true without setting
// the box (hittable_list.h:39-42), so a translate / rotate_y over a list
// inherits garbage, and rotate_y rotates only two corners of its child's box
// (hittable.h:334-372).  Lists are unioned, transforms re-derived from their
// child's true box (all eight corners), inverted boxes (negative radii)
// reordered, anything unknown without a box is unbounded.
bool true_box(const hittable* h, double t0, double t1, aabb& out) {
    const double inf = std::numeric_limits<double>::infinity();
    if (auto l = dynamic_cast<const hittable_list*>(h)) {
        bool any = false;
        for (const auto& o : l->objects) {
            aabb b;
            if (!true_box(o.get(), t0, t1, b)) {
                out = aabb(vec3(-inf), vec3(inf));
                return true;
            }
            out = any ? aabb::surrounding(out, b) : b;
            any = true;
        }
        if (!any) out = aabb(vec3(inf), vec3(-inf));  // empty: overlaps nothing
        return true;
    }
    if (auto f = dynamic_cast<const flip_normals*>(h)) return true_box(f->ptr.get(), t0, t1, out);
    if (auto m = dynamic_cast<const constant_medium*>(h)) return true_box(m->boundary.get(), t0, t1, out);
    if (auto tr = dynamic_cast<const translate*>(h)) {
        if (!true_box(tr->ptr.get(), t0, t1, out)) return false;
        out = aabb(out.min() + tr->offset, out.max() + tr->offset);
        return true;
    }
    if (auto ro = dynamic_cast<const rotate_y*>(h)) {
        aabb c;
        if (!true_box(ro->ptr.get(), t0, t1, c)) return false;
        vec3 lo(inf), hi(-inf);
        for (int corner = 0; corner < 8; ++corner) {
            const double x = (corner & 1) ? c.max().x : c.min().x;
            const double y = (corner & 2) ? c.max().y : c.min().y;
            const double z = (corner & 4) ? c.max().z : c.min().z;
            const vec3 q(ro->cos_theta * x + ro->sin_theta * z, y, -ro->sin_theta * x + ro->cos_theta * z);
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::fmin(lo[a], q[a]);
                hi[a] = std::fmax(hi[a], q[a]);
            }
        }
        out = aabb(lo, hi);
        return true;
    }
    if (!h->bounding_box(t0, t1, out)) return false;
    // a negative radius (hollow glass) gives sphere boxes with min > max
    vec3 lo = out.min(), hi = out.max();
    for (int a = 0; a < 3; ++a)
        if (lo[a] > hi[a]) std::swap(lo[a], hi[a]);
    out = aabb(lo, hi);
    return true;
}

// a ray's overlap with the slabs of b on [tmin, tmax], inclusive at the ends
bool slab_overlap(const aabb& b, const ray& r, double tmin, double tmax, double& entry) {
    for (int a = 0; a < 3; ++a) {
        const double inv = 1.0 / r.direction()[a];
        double t0 = (b.min()[a] - r.origin()[a]) * inv;
        double t1 = (b.max()[a] - r.origin()[a]) * inv;
        if (inv < 0.0) std::swap(t0, t1);
        if (t0 > tmin) tmin = t0;  // a NaN slab (0 * inf) leaves the range alone
        if (t1 < tmax) tmax = t1;
        if (tmax < tmin) return false;
    }
    entry = tmin;
    return true;
}
}  // namespace

// does `h` hold a constant_medium (itself, or below lists, boxes, bvh_nodes
// and transforms)?
bool holds_medium(const hittable* h) {
    if (!h) return false;
    if (dynamic_cast<const constant_medium*>(h)) return true;
    if (auto l = dynamic_cast<const hittable_list*>(h)) {
        for (const auto& o : l->objects)
            if (holds_medium(o.get())) return true;
        return false;
    }
    if (auto b = dynamic_cast<const bvh_node*>(h)) return b->media;
    if (auto f = dynamic_cast<const flip_normals*>(h)) return holds_medium(f->ptr.get());
    if (auto t = dynamic_cast<const translate*>(h)) return holds_medium(t->ptr.get());
    if (auto y = dynamic_cast<const rotate_y*>(h)) return holds_medium(y->ptr.get());
    return false;
}

void bvh_node::build(double time0, double time1) {
    media = false;
    for (const auto& o : objects) media = media || holds_medium(o.get());
    // per object: its box over the shutter (an object without one is kept
    // in every leaf's candidate walk: the box of everything)
    const int n = (int)objects.size();
    std::vector<aabb> boxes(n);
    std::vector<bool> boxed(n);
    bool first = true;
    for (int k = 0; k < n; ++k) {
        aabb b;
        boxed[k] = true_box(objects[k].get(), time0, time1, b);
        boxes[k] = widened(b);
        if (!boxed[k]) continue;
        box = first ? b : aabb::surrounding(box, b);
        first = false;
    }
    const aabb all(vec3(-std::numeric_limits<double>::infinity()), vec3(std::numeric_limits<double>::infinity()));
    for (int k = 0; k < n; ++k)
        if (!boxed[k]) boxes[k] = all;
    order.resize(n);
    for (int k = 0; k < n; ++k) order[k] = k;
    nodes.clear();
    // median split on the widest axis of the centres, leaves of <= 2
    struct item { int first, count, node; };
    std::vector<item> todo;
    nodes.push_back(node{});
    todo.push_back({0, n, 0});
    while (!todo.empty()) {
        const item it = todo.back();
        todo.pop_back();
        aabb b = boxes[order[it.first]];
        vec3 clo(std::numeric_limits<double>::infinity()), chi(-std::numeric_limits<double>::infinity());
        for (int k = it.first; k < it.first + it.count; ++k) {
            const aabb& o = boxes[order[k]];
            b = aabb::surrounding(b, o);
            for (int a = 0; a < 3; ++a) {
                const double c = 0.5 * (o.min()[a] + o.max()[a]);
                clo[a] = std::fmin(clo[a], c);
                chi[a] = std::fmax(chi[a], c);
            }
        }
        nodes[it.node].bounds = b;
        if (it.count <= 2) {
            nodes[it.node].first = it.first;
            nodes[it.node].count = it.count;
            continue;
        }
        int axis = 0;
        for (int a = 1; a < 3; ++a)
            if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
        const int half = it.count / 2;
        std::nth_element(order.begin() + it.first, order.begin() + it.first + half, order.begin() + it.first + it.count,
                         [&](int x, int y) {
                             const double cx = boxes[x].min()[axis] + boxes[x].max()[axis];
                             const double cy = boxes[y].min()[axis] + boxes[y].max()[axis];
                             return cx < cy || (cx == cy && x < y);
                         });
        const int l = (int)nodes.size();
        nodes.push_back(node{});
        nodes.push_back(node{});
        nodes[it.node].left = l;
        nodes[it.node].right = l + 1;
        todo.push_back({it.first, half, l});
        todo.push_back({it.first + half, it.count - half, l + 1});
    }
}

bvh_node::bvh_node(hittable** l, int n, double time0, double time1) {
    // The raw pointers are borrowed (the reference leaks them too); wrap
    // them without taking ownership.
    for (int i = 0; i < n; ++i) objects.push_back(std::shared_ptr<hittable>(l[i], [](hittable*) {}));
    build(time0, time1);
}

bvh_node::bvh_node(const std::vector<std::shared_ptr<hittable>>& l, double time0, double time1) : objects(l) {
    build(time0, time1);
}

bool bvh_node::hit(const ray& r, double t_min, double t_max, hit_record& rec) const {
    if (objects.empty()) return false;
    if (media) {
        // hittable_list::hit (hittable_list.h:11-36): every object twice, in
        // list order, each below the closest so far -- the media draw exactly
        // as in the list (the distance search below would call a
        // medium's hit with other bounds, or more often)
        hit_record tmp;
        bool found = false;
        double bound = t_max;
        for (int walk = 0; walk < 2; ++walk)
            for (const auto& o : objects)
                if (o->hit(r, t_min, bound, tmp)) {
                    found = true;
                    bound = tmp.t;
                    rec = tmp;
                }
        return found;
    }
    // 1. the closest distance: nearest-first walk, each object tested below
    //    the closest found so far (the set of hits below a bound does not
    //    depend on the order, so neither does its minimum)
    double closest = t_max;
    bool any = false;
    hit_record tmp;
    std::vector<int> stack{0};
    double entry;
    while (!stack.empty()) {
        const node& nd = nodes[stack.back()];
        stack.pop_back();
        if (!slab_overlap(nd.bounds, r, t_min, closest, entry)) continue;
        if (nd.count || nd.left < 0) {
            for (int k = nd.first; k < nd.first + nd.count; ++k)
                if (objects[order[k]]->hit(r, t_min, closest, tmp)) {
                    any = true;
                    closest = tmp.t;
                }
            continue;
        }
        double el, er;
        const bool hl = slab_overlap(nodes[nd.left].bounds, r, t_min, closest, el);
        const bool hr = slab_overlap(nodes[nd.right].bounds, r, t_min, closest, er);
        if (hl && hr) {
            stack.push_back(el <= er ? nd.right : nd.left);
            stack.push_back(el <= er ? nd.left : nd.right);
        } else if (hl) {
            stack.push_back(nd.left);
        } else if (hr) {
            stack.push_back(nd.right);
        }
    }
    if (!any) return false;
    // 2. every object whose box reaches that distance, in list order, through
    //    hittable_list::hit's double walk from the caller's t_max: only the
    //    objects with a hit at exactly `closest` can decide its record
    std::vector<int> cand;
    stack.assign(1, 0);
    while (!stack.empty()) {
        const node& nd = nodes[stack.back()];
        stack.pop_back();
        if (!slab_overlap(nd.bounds, r, t_min, closest, entry)) continue;
        if (nd.count || nd.left < 0) {
            for (int k = nd.first; k < nd.first + nd.count; ++k) cand.push_back(order[k]);
            continue;
        }
        stack.push_back(nd.left);
        stack.push_back(nd.right);
    }
    std::sort(cand.begin(), cand.end());
    bool found = false;
    double bound = t_max;
    for (int walk = 0; walk < 2; ++walk)
        for (const int k : cand)
            if (objects[k]->hit(r, t_min, bound, tmp)) {
                found = true;
                bound = tmp.t;
                rec = tmp;
            }
    return found;
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
