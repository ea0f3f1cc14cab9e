// flatten.cpp — hittable graph -> rtw_scene_desc, plus the BVH builder.
//
// The world hittable_list (hittable_list.h:5-62) becomes a list of entries in
// the same order.  Each entry is a chain of transform ops (translate /
// rotate_y / flip_normals, outermost first) over a group of leaf primitives
// (rects, spheres) whose closest hit is taken as one unit; constant_medium
// entries keep their boundary the same way.  Flattening a nested list into a
// group is exact: a nested hittable_list started with t_max = the outer
// closest-so-far (hittable_list.h:15) picks the same winner, with the same
// tie order, as the same primitives inlined at that position.
//
// Nesting of any depth: a list (or box, bvh_node, flip_normals, translate,
// rotate_y) whose subtree holds transforms or media is taken apart -- its
// children become entries of their own, in list order, each carrying the
// op chain of every transform above it (the enclosing ops first).  A
// deterministic subtree is inlined with one walk: hittable_list::hit walks
// its objects twice (hittable_list.h:16-34), and for objects without random
// draws the second walk re-accepts only what the first kept.  A list that
// holds media is not: each medium draws again in the second walk.  Such
// scenes get a visit program (rtw_scene_desc::visits): the entries in the
// order the reference's nested walks call them, both walks of every list
// that holds media, second-walk visits flagged RTW_VISIT_REPLAY (a
// deterministic replay can only re-accept an exact tie; the GPU skips those,
// the oracle runs them all).
//
// Light list members become rtw_light records with their own primitive copy
// (entry = -1): hittable_pdf only ever queries them through their own
// pdf_value/random overrides (pdf.h:35-53).
#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>
#include "rtw/flatten.h"
#include "rtw/scene.h"
#include "rtw_host_util.h"

namespace {

struct bvh_item {
    double lo[3], hi[3];
    int32_t id;
};

// Binned-SAH BVH over `items`; appends nodes/items, returns the root.
// Leaves hold at most `leaf_max` items.  Bounds are padded outward by a
// relative 1e-9 so the (independently rounded) device slab test never culls
// a primitive that the exact closest-hit test would accept.
struct bvh_builder {
    std::vector<rtw_bvh_node>& nodes;
    std::vector<int32_t>& out_items;
    int leaf_max;

    static void grow(double* lo, double* hi, const bvh_item& it) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], it.lo[a]);
            hi[a] = std::max(hi[a], it.hi[a]);
        }
    }
    static double area(const double* lo, const double* hi) {
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }

    int build(std::vector<bvh_item>& items, int begin, int end) {
        const int me = (int)nodes.size();
        nodes.push_back(rtw_bvh_node{});
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        double clo[3] = {1e300, 1e300, 1e300}, chi[3] = {-1e300, -1e300, -1e300};
        for (int i = begin; i < end; ++i) {
            grow(lo, hi, items[i]);
            for (int a = 0; a < 3; ++a) {
                const double c = 0.5 * (items[i].lo[a] + items[i].hi[a]);
                clo[a] = std::min(clo[a], c);
                chi[a] = std::max(chi[a], c);
            }
        }
        const int n = end - begin;
        auto make_leaf = [&]() {
            rtw_bvh_node& nd = nodes[me];
            pad_into(nd, lo, hi);
            nd.left = (int32_t)out_items.size();
            nd.count = n;
            nd.right = -1;
            for (int i = begin; i < end; ++i) out_items.push_back(items[i].id);
            return me;
        };
        if (n <= leaf_max) return make_leaf();

        // binned SAH
        const int B = 16;
        int best_axis = -1, best_split = -1;
        double best_cost = 1e300;
        for (int a = 0; a < 3; ++a) {
            const double ext = chi[a] - clo[a];
            if (!(ext > 0)) continue;
            int cnt[B] = {0};
            double blo[B][3], bhi[B][3];
            for (int b = 0; b < B; ++b)
                for (int k = 0; k < 3; ++k) blo[b][k] = 1e300, bhi[b][k] = -1e300;
            for (int i = begin; i < end; ++i) {
                const double c = 0.5 * (items[i].lo[a] + items[i].hi[a]);
                int b = (int)((c - clo[a]) / ext * B);
                b = std::min(std::max(b, 0), B - 1);
                cnt[b]++;
                grow(blo[b], bhi[b], items[i]);
            }
            for (int s = 1; s < B; ++s) {
                double llo[3] = {1e300, 1e300, 1e300}, lhi[3] = {-1e300, -1e300, -1e300};
                double rlo[3] = {1e300, 1e300, 1e300}, rhi[3] = {-1e300, -1e300, -1e300};
                int nl = 0, nr = 0;
                for (int b = 0; b < s; ++b)
                    if (cnt[b]) {
                        nl += cnt[b];
                        for (int k = 0; k < 3; ++k) llo[k] = std::min(llo[k], blo[b][k]), lhi[k] = std::max(lhi[k], bhi[b][k]);
                    }
                for (int b = s; b < B; ++b)
                    if (cnt[b]) {
                        nr += cnt[b];
                        for (int k = 0; k < 3; ++k) rlo[k] = std::min(rlo[k], blo[b][k]), rhi[k] = std::max(rhi[k], bhi[b][k]);
                    }
                if (!nl || !nr) continue;
                const double cost = nl * area(llo, lhi) + nr * area(rlo, rhi);
                if (cost < best_cost) best_cost = cost, best_axis = a, best_split = s;
            }
        }
        int mid;
        if (best_axis < 0) {
            mid = begin + n / 2;  // all centroids coincide: split by count
        } else {
            const double ext = chi[best_axis] - clo[best_axis];
            auto it = std::partition(items.begin() + begin, items.begin() + end, [&](const bvh_item& x) {
                const double c = 0.5 * (x.lo[best_axis] + x.hi[best_axis]);
                int b = (int)((c - clo[best_axis]) / ext * B);
                b = std::min(std::max(b, 0), B - 1);
                return b < best_split;
            });
            mid = (int)(it - items.begin());
            if (mid == begin || mid == end) mid = begin + n / 2;
        }
        const int l = build(items, begin, mid);
        const int r = build(items, mid, end);
        rtw_bvh_node& nd = nodes[me];
        pad_into(nd, lo, hi);
        nd.left = l;
        nd.right = r;
        nd.count = 0;
        return me;
    }

    static void pad_into(rtw_bvh_node& nd, const double* lo, const double* hi) {
        for (int a = 0; a < 3; ++a) {
            const double m = 1e-9 * (std::fabs(lo[a]) + std::fabs(hi[a]) + (hi[a] - lo[a])) + 1e-12;
            nd.bmin[a] = lo[a] - m;
            nd.bmax[a] = hi[a] + m;
        }
    }
};

struct flattener {
    std::vector<rtw_prim> prims;
    std::vector<rtw_entry> entries;
    std::vector<rtw_material> mats;
    std::vector<rtw_texture> texs;
    std::vector<rtw_light> lights;
    std::vector<rtw_prim> light_prims;
    std::vector<rtw_bvh_node> nodes;
    std::vector<int32_t> items;
    std::map<const material*, int> mat_ids;
    std::map<const texture*, int> tex_ids;
    std::set<int> box_starts;  // first prims of boxes' six-rect runs
    bool perlin = false;
    std::string err;
    bool nesting = false;  // collect() met a transform or medium
    bool any_media = false;
    // the camera's shutter interval: rays carry times in [shutter0, shutter1]
    // (camera.h:41), so a moving sphere's BVH box must cover its centres over
    // that interval -- movement_linear extrapolates outside [time0, time1]
    double shutter0 = 0.0, shutter1 = 0.0;

    int texture_id(const texture* t) {
        auto f = tex_ids.find(t);
        if (f != tex_ids.end()) return f->second;
        rtw_texture x;
        std::memset(&x, 0, sizeof x);
        if (auto c = dynamic_cast<const constant_texture*>(t)) {
            x.type = RTW_TEX_CONSTANT;
            x.color[0] = c->color.x, x.color[1] = c->color.y, x.color[2] = c->color.z;
        } else if (auto n = dynamic_cast<const noise_texture*>(t)) {
            x.type = RTW_TEX_NOISE;
            x.scale = n->scale;
            perlin = true;
        } else if (auto ch = dynamic_cast<const checker_texture*>(t)) {
            // register the children after this entry's slot is reserved
            const int id = (int)texs.size();
            tex_ids[t] = id;
            texs.push_back(x);
            const int odd = texture_id(ch->odd.get());
            const int even = texture_id(ch->even.get());
            texs[id].type = RTW_TEX_CHECKER;
            texs[id].odd = odd;
            texs[id].even = even;
            return id;
        } else {
            err = "unsupported texture type (image_texture has no loader in this build)";
            return -1;
        }
        const int id = (int)texs.size();
        tex_ids[t] = id;
        texs.push_back(x);
        return id;
    }

    int material_id(const material* m) {
        if (!m) {
            err = "primitive without material";
            return -1;
        }
        auto f = mat_ids.find(m);
        if (f != mat_ids.end()) return f->second;
        rtw_material x;
        std::memset(&x, 0, sizeof x);
        x.texture = -1;
        if (auto l = dynamic_cast<const lambertian*>(m)) {
            x.type = RTW_MAT_LAMBERTIAN;
            x.texture = texture_id(l->albedo.get());
        } else if (auto me = dynamic_cast<const metal*>(m)) {
            x.type = RTW_MAT_METAL;
            x.albedo[0] = me->albedo.x, x.albedo[1] = me->albedo.y, x.albedo[2] = me->albedo.z;
            x.fuzz = me->fuzz;
        } else if (auto d = dynamic_cast<const dielectric*>(m)) {
            x.type = RTW_MAT_DIELECTRIC;
            x.ref_idx = d->ref_idx;
        } else if (auto dl = dynamic_cast<const diffuse_light*>(m)) {
            x.type = RTW_MAT_DIFFUSE_LIGHT;
            x.texture = texture_id(dl->emit.get());
        } else if (auto is = dynamic_cast<const isotropic*>(m)) {
            x.type = RTW_MAT_ISOTROPIC;
            x.texture = texture_id(is->albedo.get());
        } else {
            err = "unsupported material type";
            return -1;
        }
        if (!err.empty()) return -1;
        const int id = (int)mats.size();
        mat_ids[m] = id;
        mats.push_back(x);
        return id;
    }

    // A leaf primitive as an rtw_prim (no entry / flip yet); false if `h` is
    // not a leaf.
    bool leaf(const hittable* h, rtw_prim& p) {
        std::memset(&p, 0, sizeof p);
        if (auto r = dynamic_cast<const xy_rect*>(h)) {
            p.type = RTW_PRIM_RECT_XY;
            p.p[0] = r->x0, p.p[1] = r->x1, p.p[2] = r->y0, p.p[3] = r->y1, p.p[4] = r->k;
            p.material = material_id(r->mp.get());
        } else if (auto r = dynamic_cast<const xz_rect*>(h)) {
            p.type = RTW_PRIM_RECT_XZ;
            p.p[0] = r->x0, p.p[1] = r->x1, p.p[2] = r->z0, p.p[3] = r->z1, p.p[4] = r->k;
            p.material = material_id(r->mp.get());
        } else if (auto r = dynamic_cast<const yz_rect*>(h)) {
            p.type = RTW_PRIM_RECT_YZ;
            p.p[0] = r->y0, p.p[1] = r->y1, p.p[2] = r->z0, p.p[3] = r->z1, p.p[4] = r->k;
            p.material = material_id(r->mp.get());
        } else if (auto s = dynamic_cast<const sphere*>(h)) {
            p.type = RTW_PRIM_SPHERE;
            p.p[0] = s->center.x, p.p[1] = s->center.y, p.p[2] = s->center.z, p.p[3] = s->radius;
            p.material = material_id(s->mat.get());
        } else if (auto s = dynamic_cast<const moving_sphere*>(h)) {
            p.type = RTW_PRIM_MOVING_SPHERE;
            p.p[0] = s->center.x, p.p[1] = s->center.y, p.p[2] = s->center.z, p.p[3] = s->radius;
            p.p[4] = s->movement.center1.x, p.p[5] = s->movement.center1.y, p.p[6] = s->movement.center1.z;
            p.p[7] = s->movement.time0, p.p[8] = s->movement.time1;
            p.material = material_id(s->mat.get());
        } else {
            return false;
        }
        p.entry = -1;
        return true;
    }

    // Append the leaves under `h` (a group: leaf / flip_normals / box /
    // hittable_list / bvh_node) to prims, in list order.
    bool collect(const hittable* h, int flip, int entry) {
        rtw_prim p;
        if (leaf(h, p)) {
            if (!err.empty()) return false;
            p.flip = flip;
            p.entry = entry;
            prims.push_back(p);
            return true;
        }
        if (auto f = dynamic_cast<const flip_normals*>(h)) return collect(f->ptr.get(), flip + 1, entry);
        if (auto b = dynamic_cast<const box*>(h)) {
            const size_t first = prims.size();
            if (!collect(&b->list_ptr, flip, entry)) return false;
            // a box's six rects in its list order (hittable_list.h:65-114):
            // one item of a group BVH (RTW_ITEM_BOX)
            static const int kBoxTypes[6] = {RTW_PRIM_RECT_XY, RTW_PRIM_RECT_XY, RTW_PRIM_RECT_XZ,
                                             RTW_PRIM_RECT_XZ, RTW_PRIM_RECT_YZ, RTW_PRIM_RECT_YZ};
            bool is_box = prims.size() == first + 6;
            for (int j = 0; j < 6 && is_box; ++j) is_box = prims[first + j].type == kBoxTypes[j];
            if (is_box) box_starts.insert((int)first);
            return true;
        }
        if (auto l = dynamic_cast<const hittable_list*>(h)) {
            for (const auto& o : l->objects)
                if (!collect(o.get(), flip, entry)) return false;
            return true;
        }
        if (auto bn = dynamic_cast<const bvh_node*>(h)) {
            for (const auto& o : bn->objects)
                if (!collect(o.get(), flip, entry)) return false;
            return true;
        }
        nesting = true;  // a transform or medium below: the caller takes the subtree apart
        return false;
    }

    // Peel translate / rotate_y / flip_normals-around-non-leaf into ops.
    const hittable* peel_ops(const hittable* h, rtw_entry& e) {
        for (;;) {
            int op = 0;
            const hittable* inner = nullptr;
            double prm[3] = {0, 0, 0};
            if (auto t = dynamic_cast<const translate*>(h)) {
                op = RTW_OP_TRANSLATE, inner = t->ptr.get();
                prm[0] = t->offset.x, prm[1] = t->offset.y, prm[2] = t->offset.z;
            } else if (auto r = dynamic_cast<const rotate_y*>(h)) {
                op = RTW_OP_ROTATE_Y, inner = r->ptr.get();
                prm[0] = r->sin_theta, prm[1] = r->cos_theta;
            } else if (auto f = dynamic_cast<const flip_normals*>(h)) {
                // A flip with no transform below it negates the normal right
                // after the leaf produced it (through any nesting of lists and
                // boxes), which is exactly a per-prim flip: fold it (collect()).
                // Only a flip over a transform stays an op in the chain.
                const hittable* in = f->ptr.get();
                if (!dynamic_cast<const translate*>(in) && !dynamic_cast<const rotate_y*>(in)) return h;
                op = RTW_OP_FLIP, inner = in;
            } else {
                return h;
            }
            if (e.n_ops >= RTW_MAX_OPS) {
                err = "more than RTW_MAX_OPS nested transforms";
                return nullptr;
            }
            e.op[e.n_ops] = op;
            for (int a = 0; a < 3; ++a) e.op_param[e.n_ops][a] = prm[a];
            e.n_ops++;
            h = inner;
        }
    }

    // One entry over `body` (a group of leaves, or a medium's boundary) with
    // the ops `chain` (outermost first).
    bool make_entry(rtw_entry e, const hittable* body) {
        const int id = (int)entries.size();
        e.first_prim = (int)prims.size();
        nesting = false;
        if (!collect(body, 0, id)) {
            if (nesting && err.empty()) err = "a constant_medium boundary must not hold transforms or media";
            return false;
        }
        e.n_prims = (int)prims.size() - e.first_prim;
        if (e.n_prims == 0) {
            err = "empty group";
            return false;
        }
        entry_bounds(e);
        entries.push_back(e);
        return true;
    }

    // Append `ops` to the chain of entry `e`.
    bool push_ops(rtw_entry& e, const std::vector<std::pair<int, std::array<double, 3>>>& ops) {
        for (const auto& o : ops) {
            if (e.n_ops >= RTW_MAX_OPS) {
                err = "more than RTW_MAX_OPS nested transforms";
                return false;
            }
            e.op[e.n_ops] = o.first;
            for (int a = 0; a < 3; ++a) e.op_param[e.n_ops][a] = o.second[a];
            e.n_ops++;
        }
        return true;
    }

    using op_chain = std::vector<std::pair<int, std::array<double, 3>>>;

    // Flatten one object of a list: entries for it (appended in list order)
    // and the visits one call of its hit() makes (`out`).  `prefix`: the ops
    // of the transforms enclosing it, outermost first.
    bool flatten_node(const hittable* h, const op_chain& prefix, std::vector<int32_t>& out, bool& media) {
        rtw_entry e;
        std::memset(&e, 0, sizeof e);
        e.phase_material = -1;
        e.bvh_root = -1;
        e.kind = RTW_ENTRY_GROUP;
        if (!push_ops(e, prefix)) return false;
        if (auto cm = dynamic_cast<const constant_medium*>(h)) {
            e.kind = RTW_ENTRY_MEDIUM;
            e.density = cm->density;
            e.phase_material = material_id(cm->mp.get());
            if (e.phase_material < 0) return false;
            e.n_outer_ops = e.n_ops;  // the enclosing transforms; the boundary's own follow
            const hittable* body = peel_ops(cm->boundary.get(), e);
            if (!body) return false;
            const int id = (int)entries.size();
            if (!make_entry(e, body)) return false;
            out.push_back(id);
            media = true;
            any_media = true;
            return true;
        }
        const hittable* body = peel_ops(h, e);
        if (!body) return false;
        // a deterministic group of leaves: one entry
        {
            const size_t np = prims.size();
            const int id = (int)entries.size();
            nesting = false;
            e.first_prim = (int)np;
            if (collect(body, 0, id)) {
                e.n_prims = (int)prims.size() - e.first_prim;
                if (e.n_prims == 0) {
                    err = "empty group";
                    return false;
                }
                entry_bounds(e);
                entries.push_back(e);
                out.push_back(id);
                return true;
            }
            if (!nesting || !err.empty()) return false;
            prims.resize(np);  // take it apart instead
        }
        // the chain peeled so far becomes the children's prefix
        op_chain inner;
        for (int k = 0; k < e.n_ops; ++k)
            inner.push_back({e.op[k], {e.op_param[k][0], e.op_param[k][1], e.op_param[k][2]}});
        std::vector<const hittable*> kids;
        if (auto f = dynamic_cast<const flip_normals*>(body)) {  // flip over a subtree with transforms
            inner.push_back({RTW_OP_FLIP, {0, 0, 0}});
            kids.push_back(f->ptr.get());
        } else if (auto b = dynamic_cast<const box*>(body)) {
            kids.push_back(&b->list_ptr);
        } else if (auto l = dynamic_cast<const hittable_list*>(body)) {
            for (const auto& o : l->objects) kids.push_back(o.get());
        } else if (auto bn = dynamic_cast<const bvh_node*>(body)) {
            for (const auto& o : bn->objects) kids.push_back(o.get());
        } else {
            err = "unsupported hittable in the scene graph";
            return false;
        }
        const bool is_list = !dynamic_cast<const flip_normals*>(body);
        std::vector<int32_t> seq;
        bool m = false;
        for (const hittable* k : kids) {
            if (!k) {
                err = "null object";
                return false;
            }
            if (!flatten_node(k, inner, seq, m)) return false;
        }
        if (m && dynamic_cast<const bvh_node*>(body)) {
            // the reference's bvh_node::hit walks `left` twice and never
            // `right` (hittable.h:82-110): there is no walk order whose media
            // draws could be reproduced, so refuse rather than guess
            err = "a bvh_node holding a constant_medium is unsupported (the reference's bvh_node::hit is broken, "
                  "hittable.h:82-110)";
            return false;
        }
        out.insert(out.end(), seq.begin(), seq.end());
        if (m && is_list) {  // the list's second walk (hittable_list.h:26-34)
            for (int32_t v : seq) out.push_back(v | RTW_VISIT_REPLAY);
        }
        media = media || m;
        return true;
    }

    // --------------------------------------------------------- bounds
    void prim_bounds(const rtw_prim& p, double* lo, double* hi) const {
        const double* q = p.p;
        switch (p.type) {
        case RTW_PRIM_SPHERE:
        case RTW_PRIM_MOVING_SPHERE: {
            const double r = std::fabs(q[3]);
            for (int a = 0; a < 3; ++a) lo[a] = q[a] - r, hi[a] = q[a] + r;
            if (p.type == RTW_PRIM_MOVING_SPHERE) {
                // the centre moves along a line: its extremes over the shutter
                // are the centres at the shutter's ends (sphere.h:22-25), plus
                // center0 / center1 for good measure
                for (int a = 0; a < 3; ++a) lo[a] = std::min(lo[a], q[4 + a] - r), hi[a] = std::max(hi[a], q[4 + a] + r);
                for (double t : {shutter0, shutter1}) {
                    const double f = (t - q[7]) / (q[8] - q[7]);
                    for (int a = 0; a < 3; ++a) {
                        const double c = q[a] + f * (q[4 + a] - q[a]);
                        lo[a] = std::min(lo[a], c - r), hi[a] = std::max(hi[a], c + r);
                    }
                }
            }
            return;
        }
        case RTW_PRIM_RECT_XY: lo[0] = q[0], hi[0] = q[1], lo[1] = q[2], hi[1] = q[3], lo[2] = hi[2] = q[4]; break;
        case RTW_PRIM_RECT_XZ: lo[0] = q[0], hi[0] = q[1], lo[2] = q[2], hi[2] = q[3], lo[1] = hi[1] = q[4]; break;
        case RTW_PRIM_RECT_YZ: lo[1] = q[0], hi[1] = q[1], lo[2] = q[2], hi[2] = q[3], lo[0] = hi[0] = q[4]; break;
        }
        for (int a = 0; a < 3; ++a) lo[a] = std::min(lo[a], hi[a]), hi[a] = std::max(hi[a], lo[a]);
    }

    void entry_bounds(rtw_entry& e) {
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (int i = e.first_prim; i < e.first_prim + e.n_prims; ++i) {
            double a[3], b[3];
            prim_bounds(prims[i], a, b);
            for (int k = 0; k < 3; ++k) lo[k] = std::min(lo[k], a[k]), hi[k] = std::max(hi[k], b[k]);
        }
        // apply ops innermost -> outermost (object space -> world space)
        for (int o = e.n_ops - 1; o >= 0; --o) {
            if (e.op[o] == RTW_OP_TRANSLATE) {
                for (int k = 0; k < 3; ++k) lo[k] += e.op_param[o][k], hi[k] += e.op_param[o][k];
            } else if (e.op[o] == RTW_OP_ROTATE_Y) {
                const double s = e.op_param[o][0], c = e.op_param[o][1];
                double nlo[3] = {1e300, lo[1], 1e300}, nhi[3] = {-1e300, hi[1], -1e300};
                for (int i = 0; i < 4; ++i) {
                    const double x = (i & 1) ? hi[0] : lo[0], z = (i & 2) ? hi[2] : lo[2];
                    const double nx = c * x + s * z, nz = -s * x + c * z;
                    nlo[0] = std::min(nlo[0], nx), nhi[0] = std::max(nhi[0], nx);
                    nlo[2] = std::min(nlo[2], nz), nhi[2] = std::max(nhi[2], nz);
                }
                for (int k = 0; k < 3; ++k) lo[k] = nlo[k], hi[k] = nhi[k];
            }
        }
        for (int k = 0; k < 3; ++k) e.bounds[k] = lo[k], e.bounds[3 + k] = hi[k];
    }

    bool add_light(const hittable* h) {
        rtw_light l;
        l.kind = RTW_LIGHT_DEFAULT;
        l.prim = -1;
        rtw_prim p;
        if (dynamic_cast<const xz_rect*>(h) && leaf(h, p)) {
            l.kind = RTW_LIGHT_XZ_RECT;
        } else if ((dynamic_cast<const sphere*>(h) || dynamic_cast<const moving_sphere*>(h)) && leaf(h, p)) {
            l.kind = RTW_LIGHT_SPHERE;
        }
        if (!err.empty()) return false;
        if (l.kind != RTW_LIGHT_DEFAULT) {
            l.prim = (int)light_prims.size();  // rebased after the world prims below
            light_prims.push_back(p);
        }
        lights.push_back(l);
        return true;
    }
};

}  // namespace

int rtw_flatten_scene(const scene& sc, int use_bvh, rtw_scene_desc** out) {
    return rtw_flatten_world(sc.GetWorld(), sc.GetLights().get(), sc.GetCamera(), static_cast<int>(sc.GetRenderType()),
                             static_cast<int>(sc.GetBackgroundType()), use_bvh, out);
}

int rtw_flatten_world(const hittable_list& world, const hittable_list* lights, const camera& cam, int render_type,
                      int background, int use_bvh, rtw_scene_desc** out) {
    if (!out) return rtw_fail(RTW_ERR_INVALID, "rtw_flatten_scene: null output");
    *out = nullptr;
    if (render_type != RTW_RENDER_SHADED && render_type != RTW_RENDER_NORMAL)
        return rtw_fail(RTW_ERR_INVALID, "rtw_flatten_scene: unknown render type");
    if (background != RTW_BG_BLACK && background != RTW_BG_GRADIENT)
        return rtw_fail(RTW_ERR_INVALID, "rtw_flatten_scene: unknown background type");
    flattener f;
    {
        const rtw_camera_desc cd = cam.desc();
        f.shutter0 = std::min(cd.time0, cd.time1);
        f.shutter1 = std::max(cd.time0, cd.time1);
    }
    // the world list, one call of its hit(): both walks when it holds media
    std::vector<int32_t> visits;
    for (const auto& o : world.objects) {
        bool m = false;
        if (!o || !f.flatten_node(o.get(), {}, visits, m))
            return rtw_fail(RTW_ERR_UNSUPPORTED, "rtw_flatten_scene: " + (f.err.empty() ? std::string("null object") : f.err));
    }
    if (f.any_media) {
        const size_t n = visits.size();
        for (size_t k = 0; k < n; ++k) visits.push_back(visits[k] | RTW_VISIT_REPLAY);
    } else {
        visits.clear();  // one walk over the entries is the reference's two
    }
    if (lights) {
        for (const auto& o : lights->objects)
            if (!o || !f.add_light(o.get())) return rtw_fail(RTW_ERR_UNSUPPORTED, "rtw_flatten_scene: light: " + f.err);
    }
    const int n_world = (int)f.prims.size();
    for (auto& l : f.lights)
        if (l.prim >= 0) l.prim += n_world;
    for (auto& p : f.light_prims) f.prims.push_back(p);

    bool has_media = false;
    for (const auto& e : f.entries) has_media |= (e.kind == RTW_ENTRY_MEDIUM);

    int world_root = -1;
    if (use_bvh) {
        // leaf sizes, measured on 1 MI355X (random_balls world BVH: 1 item
        // +8 % over 2; Book-2 group BVHs: 2 items, 1 -8 %, 4 -9 %);
        // RTW_BVH_LEAF_MAX / RTW_BVH_WORLD_LEAF_MAX override them for tuning
        auto env_leaf = [](const char* name, int dflt) {
            const char* v = std::getenv(name);
            return v && *v ? std::max(1, std::min(16, std::atoi(v))) : dflt;
        };
        const int leaf_max = env_leaf("RTW_BVH_LEAF_MAX", 2);
        const int world_leaf_max = env_leaf("RTW_BVH_WORLD_LEAF_MAX", 1);
        // a box is one BVH item (its six rects tested together in list
        // order) rather than six: a third of the nodes for a group of boxes
        // (RTW_BVH_BOX_ITEMS=0: six items, for A/B)
        const char* bx = std::getenv("RTW_BVH_BOX_ITEMS");
        const bool box_items = !(bx && *bx && std::atoi(bx) == 0);
        // group BVHs over large groups
        for (auto& e : f.entries) {
            if (e.n_prims <= 8) continue;
            std::vector<bvh_item> its;
            for (int i = e.first_prim; i < e.first_prim + e.n_prims; ++i) {
                bvh_item it;
                f.prim_bounds(f.prims[i], it.lo, it.hi);
                it.id = i;
                if (box_items && f.box_starts.count(i) && i + 6 <= e.first_prim + e.n_prims) {
                    for (int j = 1; j < 6; ++j) {
                        double lo[3], hi[3];
                        f.prim_bounds(f.prims[i + j], lo, hi);
                        for (int k = 0; k < 3; ++k) it.lo[k] = std::min(it.lo[k], lo[k]), it.hi[k] = std::max(it.hi[k], hi[k]);
                    }
                    it.id = i | RTW_ITEM_BOX;
                    i += 5;
                }
                its.push_back(it);
            }
            bvh_builder b{f.nodes, f.items, leaf_max};
            e.bvh_root = b.build(its, 0, (int)its.size());
        }
        // world BVH over entries (media keep list order: see DESIGN.md)
        if (!has_media && f.entries.size() > 8) {
            std::vector<bvh_item> its;
            for (int i = 0; i < (int)f.entries.size(); ++i) {
                bvh_item it;
                for (int k = 0; k < 3; ++k) it.lo[k] = f.entries[i].bounds[k], it.hi[k] = f.entries[i].bounds[3 + k];
                it.id = i;
                its.push_back(it);
            }
            bvh_builder b{f.nodes, f.items, world_leaf_max};
            world_root = b.build(its, 0, (int)its.size());
        }
    }

    // one allocation owns the desc and every array
    rtw_scene_desc* d = new rtw_scene_desc;
    std::memset(d, 0, sizeof *d);
    d->abi_version = RTW_ABI_VERSION;
    d->render_type = render_type;
    d->background = background;
    d->n_prims = (int)f.prims.size();
    d->n_entries = (int)f.entries.size();
    d->n_materials = (int)f.mats.size();
    d->n_textures = (int)f.texs.size();
    d->n_lights = (int)f.lights.size();
    d->n_bvh_nodes = (int)f.nodes.size();
    d->n_bvh_items = (int)f.items.size();
    d->world_bvh_root = world_root;
    d->has_perlin = f.perlin ? 1 : 0;
    d->prims = rtw_dup(f.prims);
    d->entries = rtw_dup(f.entries);
    d->materials = rtw_dup(f.mats);
    d->textures = rtw_dup(f.texs);
    d->lights = rtw_dup(f.lights);
    d->bvh_nodes = rtw_dup(f.nodes);
    d->bvh_items = rtw_dup(f.items);
    d->n_visits = (int)visits.size();
    d->visits = visits.empty() ? nullptr : rtw_dup(visits);
    if (f.perlin) {
        std::vector<double> rv(perlin::SIZE * 3);
        std::vector<int32_t> pm(perlin::SIZE * 3);
        for (int i = 0; i < perlin::SIZE; ++i) {
            for (int a = 0; a < 3; ++a) rv[i * 3 + a] = perlin::ranvec()[i][a];
            pm[i] = perlin::perm_x()[i];
            pm[perlin::SIZE + i] = perlin::perm_y()[i];
            pm[2 * perlin::SIZE + i] = perlin::perm_z()[i];
        }
        d->perlin_ranvec = rtw_dup(rv);
        d->perlin_perm = rtw_dup(pm);
    }
    d->camera = cam.desc();
    *out = d;
    return RTW_OK;
}

extern "C" void rtw_scene_desc_free(rtw_scene_desc* d) {
    if (!d) return;
    free((void*)d->prims);
    free((void*)d->entries);
    free((void*)d->materials);
    free((void*)d->textures);
    free((void*)d->lights);
    free((void*)d->bvh_nodes);
    free((void*)d->bvh_items);
    free((void*)d->perlin_ranvec);
    free((void*)d->perlin_perm);
    free((void*)d->visits);
    delete d;
}

extern "C" int rtw_scene_builtin(const char* name, double aspect, int use_bvh, rtw_scene_desc** out) {
    if (!name || !out) return rtw_fail(RTW_ERR_INVALID, "rtw_scene_builtin: null argument");
    auto sc = make_builtin_scene(name, aspect);
    if (!sc) return rtw_fail(RTW_ERR_INVALID, std::string("rtw_scene_builtin: unknown scene '") + name + "'");
    return rtw_flatten_scene(*sc, use_bvh, out);
}
