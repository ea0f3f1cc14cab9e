// rtw_fast.h — device code of the fp32 fast mode (RTW_PRECISION_FP32).
//
// The same path tracer as rtw_device.h -- RayTracingWeekend.cpp:45-160's
// color() over the flattened scene: world walks in list order (or a BVH),
// the media walk with its replays, transforms, the five materials, the
// cosine / light mixture pdf, textures and Perlin marble -- in single
// precision, for users who accept statistical parity with the reference
// instead of its double arithmetic (vec3.h:35-44).  Nothing here has to
// round like the reference, so it is written for the fp32 VALU: hardware
// reciprocals / square roots, v_sin / v_cos in revolutions, one raw
// minstd_rand draw per uniform (libstdc++'s generate_canonical<float, 24>),
// the numerically stable sphere discriminant.  Each sample still owns its
// (seed, pixel, sample) stream (rtw_path_seed), so results do not depend on
// how samples are split over lanes or GPUs.
//
// Scene data: fp32 mirrors of the prims, entries, ops, materials, textures,
// Perlin vectors and rect frames (rtw_scene_upload builds them); BVH nodes
// (already fp32, rounded outward), items, world runs and the media walk are
// the fp64 path's own arrays.
#pragma once
#include "rtw_device.h"

namespace rtwf {

using rtwd::bvh_node32;
using rtwd::ld;
using rtwd::world_run;

constexpr float kPiF = 3.14159265358979f;
constexpr float kTMinF = 0.001f;                // RayTracingWeekend.cpp:52
constexpr float kStepF = 0.0001f;               // hittable.h:447
constexpr float kFltMaxF = 3.40282347e38f;

// ------------------------------------------------------------------ math
struct f3 {
    float x, y, z;
};
RTW_D f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RTW_D f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RTW_D f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
RTW_D f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
RTW_D f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
RTW_D float dot(f3 a, f3 b) { return __builtin_fmaf(a.x, b.x, __builtin_fmaf(a.y, b.y, a.z * b.z)); }
RTW_D float len2(f3 a) { return dot(a, a); }
RTW_D float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
RTW_D float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
RTW_D float len(f3 a) { return fsqrt(len2(a)); }
RTW_D f3 normalize(f3 v) { return v * __builtin_amdgcn_rsqf(len2(v)); }
RTW_D f3 cross(f3 a, f3 b) { return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
RTW_D f3 ldf3(const float* p) { return f3{p[0], p[1], p[2]}; }
RTW_D float comp(const f3& v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }
// sin / cos of 2 pi x (v_sin_f32 / v_cos_f32 take revolutions)
RTW_D float sin_rev(float x) { return __builtin_amdgcn_sinf(x); }
RTW_D float cos_rev(float x) { return __builtin_amdgcn_cosf(x); }

struct fray {
    f3 o, d;
    float t;
};
RTW_D f3 at(const fray& r, float t) { return r.o + r.d * t; }

// one raw minstd_rand draw per uniform in [0, 1)
RTW_D float u01(uint32_t& s) {
    const float r = (float)(rtwd::mr_next(s) - 1u) * 4.65661287525e-10f;  // / (2^31 - 2)
    return r < 1.0f ? r : 0x1.fffffep-1f;
}

// ------------------------------------------------------------------ scene
// p: sphere  c0 xyz, r, c1 - c0 xyz, time0, 1 / (time1 - time0), r^2
//    rect    lo_a, hi_a, lo_b, hi_b, k
struct prim32 {
    int32_t type, material, flip, entry;
    float p[10];
    int32_t pad[2];
};  // 64 B
struct ent32 {
    int32_t kind, first_prim, n_prims, n_ops, first_op, phase_material, bvh_root, n_outer_ops;
    float neg_inv_density;  // -1 / density (hittable.h:450)
    int32_t pad[3];
};  // 48 B
struct op32 {
    int32_t type;
    float p[3];
};  // 16 B
struct mat32 {
    int32_t type, texture;
    float albedo[3], fuzz, ref_idx, inv_ref_idx, r0;
    int32_t pad;
};  // 40 B
struct tex32 {
    int32_t type, odd, even;
    float scale;
    float color[3];
    int32_t pad;
};  // 32 B

struct fscene {
    const prim32* prims;
    const ent32* entries;
    const op32* ops;
    const mat32* materials;
    const tex32* textures;
    const rtw_light* lights;
    const float* ranvec;    // 256 x 3
    const int32_t* perm;    // 3 x 256
    const float* frames;    // per rect prim: world-normal onb (u, v, w)
    const rtwd::node_store* nodes;
    const int32_t* items;
    const world_run* runs;
    const int32_t* media;
    const float* ysph;  // the y-sphere runs' pair-interleaved fp32 records (rtw_scene_upload)
    const float* boxes;  // box items' planes, as rtwd::scene::boxes
    float light_weight;
    float mv_t0, mv_inv_den;  // the common motion interval of the y-sphere runs' movers
    int32_t n_lights, world_bvh_root, render_type, background, n_media, n_runs, n_nodes;
    // the BVH node packet in LDS (k_fast with LDS stacks: the top n_lnodes
    // nodes of the BFS numbering, set by the kernel; 0 elsewhere)
    const rtwd::node_store* lnodes;
    int32_t n_lnodes;
};

// uniform (scalar) loads of a prim's fields
RTW_D prim32 uprim(const prim32* P, int i) {
    prim32 q;
    q.type = ld(&P[i].type);
    q.material = ld(&P[i].material);
    q.flip = ld(&P[i].flip);
    q.entry = ld(&P[i].entry);
#pragma unroll
    for (int k = 0; k < 10; ++k) q.p[k] = ld(&P[i].p[k]);
    return q;
}
template <bool U, typename T>
RTW_D T rd(const T* p) {
    if constexpr (U) return ld(p);
    else return *p;
}

// ------------------------------------------------------------------ hits
struct fhit {
    float t;
    int32_t prim;  // -1 none, <= -2 medium entry -(2 + e)
    bool rect;
};
// list-order tie rule of hittable_list::hit for any visiting order (rtwd::better)
RTW_D bool better(float t, int idx, bool rectlike, const fhit& h) {
    if (t < h.t) return true;
    if (t != h.t) return false;
    const bool has = h.prim != -1;
    if (rectlike) return !has || !h.rect || idx > h.prim;
    return has && !h.rect && idx < h.prim;
}

RTW_D f3 sphere_center(const prim32& q, float time) {
    const f3 c0{q.p[0], q.p[1], q.p[2]};
    if (q.type != RTW_PRIM_MOVING_SPHERE) return c0;
    return c0 + f3{q.p[4], q.p[5], q.p[6]} * ((time - q.p[7]) * q.p[8]);  // sphere.h:22-25
}
// sphere.h:46-81's roots, near then far, from the stable form of the
// discriminant: b^2 - a c = a (r^2 - |oc - (b/a) d|^2)
RTW_D bool sphere_t(const prim32& q, const fray& r, float tmin, float tmax, float& t) {
    const f3 oc = r.o - sphere_center(q, r.t);
    const float ia = rcp(dot(r.d, r.d));
    const float tb = dot(oc, r.d) * ia;
    const f3 l = oc - r.d * tb;
    const float h = q.p[9] - dot(l, l);
    if (!(h > 0)) return false;
    const float sq = fsqrt(h * ia);
    t = -tb - sq;
    if (t < tmax && t > tmin) return true;
    t = -tb + sq;
    return t < tmax && t > tmin;
}
// hittable.h:149-165 / 184-200 / 241-257 (K plane axis, A / B in-plane axes)
template <int K, int A, int B, class Q = prim32>
RTW_D bool rect_axis_t(const Q& q, const fray& r, float t0, float t1, float& t) {
    t = (q.p[4] - comp(r.o, K)) * rcp(comp(r.d, K));
    if (t < t0 || t > t1) return false;
    const float a = __builtin_fmaf(t, comp(r.d, A), comp(r.o, A));
    const float b = __builtin_fmaf(t, comp(r.d, B), comp(r.o, B));
    return !(a < q.p[0] || a > q.p[1] || b < q.p[2] || b > q.p[3]);
}
RTW_D bool rect_t(const prim32& q, const fray& r, float t0, float t1, float& t) {
    if (q.type == RTW_PRIM_RECT_XY) return rect_axis_t<2, 0, 1>(q, r, t0, t1, t);
    if (q.type == RTW_PRIM_RECT_XZ) return rect_axis_t<1, 0, 2>(q, r, t0, t1, t);
    return rect_axis_t<0, 1, 2>(q, r, t0, t1, t);
}
RTW_D f3 rect_normal(int type) {
    return type == RTW_PRIM_RECT_XY ? f3{0, 0, 1} : (type == RTW_PRIM_RECT_XZ ? f3{0, 1, 0} : f3{1, 0, 0});
}

// transforms (hittable.h:299-311, 373-404)
template <bool U>
RTW_D void op_ray_in(const op32* O, int k, fray& r) {
    const int op = rd<U>(&O[k].type);
    if (op == RTW_OP_TRANSLATE) {
        r.o = r.o - f3{rd<U>(&O[k].p[0]), rd<U>(&O[k].p[1]), rd<U>(&O[k].p[2])};
    } else if (op == RTW_OP_ROTATE_Y) {
        const float s = rd<U>(&O[k].p[0]), c = rd<U>(&O[k].p[1]);
        const f3 o = r.o, d = r.d;
        r.o.x = c * o.x - s * o.z;
        r.o.z = s * o.x + c * o.z;
        r.d.x = c * d.x - s * d.z;
        r.d.z = s * d.x + c * d.z;
    }
}
template <bool U>
RTW_D void op_rec_out(const op32* O, int k, f3& p, f3& n) {
    const int op = rd<U>(&O[k].type);
    if (op == RTW_OP_TRANSLATE) {
        p = p + f3{rd<U>(&O[k].p[0]), rd<U>(&O[k].p[1]), rd<U>(&O[k].p[2])};
    } else if (op == RTW_OP_ROTATE_Y) {
        const float s = rd<U>(&O[k].p[0]), c = rd<U>(&O[k].p[1]);
        const f3 p0 = p, n0 = n;
        p.x = c * p0.x + s * p0.z;
        p.z = -s * p0.x + c * p0.z;
        n.x = c * n0.x + s * n0.z;
        n.z = -s * n0.x + c * n0.z;
    } else if (op == RTW_OP_FLIP) {
        n = -n;
    }
}
struct ent_v {
    const ent32* p;
    const op32* ops;
    int kind, first_prim, n_prims, n_ops, bvh_root;
};
template <bool U>
RTW_D ent_v view_entry(const fscene& S, int i) {
    const ent32* E = S.entries;
    ent_v e;
    e.p = E + i;
    e.ops = S.ops + rd<U>(&E[i].first_op);
    e.kind = rd<U>(&E[i].kind);
    e.first_prim = rd<U>(&E[i].first_prim);
    e.n_prims = rd<U>(&E[i].n_prims);
    e.n_ops = rd<U>(&E[i].n_ops);
    e.bvh_root = rd<U>(&E[i].bvh_root);
    return e;
}
template <bool U>
RTW_D fray ops_in(const ent_v& e, fray r, int k0, int k1) {
    for (int k = k0; k < k1; ++k) op_ray_in<U>(e.ops, k, r);
    return r;
}
template <bool U>
RTW_D void ops_out(const ent_v& e, int k1, f3& p, f3& n) {
    for (int k = k1 - 1; k >= 0; --k) op_rec_out<U>(e.ops, k, p, n);
}

// closest hit over prims [first, first + n) in list order (uniform loads)
RTW_D void group_scan(const fscene& S, int first, int n, const fray& r, float tmin, fhit& h) {
    for (int i = first; i < first + n; ++i) {
        const prim32 q = uprim(S.prims, i);
        float t;
        if (rtwd::is_sphere(q.type)) {
            if (sphere_t(q, r, tmin, h.t, t)) h.t = t, h.prim = i, h.rect = false;
        } else {
            if (rect_t(q, r, tmin, h.t, t)) h.t = t, h.prim = i, h.rect = true;
        }
    }
}

// A y-sphere run (WORLD_RUN_YSPHERES: spheres moving along y at most, the
// Book-1 random_balls list): the discriminants of two spheres per packed
// fp32 instruction (v_pk_fma_f32) from the upload's pair-interleaved records
// {cx, cy, cz, dy, r^2}, and the full test -- list order, strict t < t_max
// only for spheres some lane of the wave may hit.  fc = the walk's motion
// fraction.  Spheres the records do not bound (r^2 = +inf: the ground) always
// pass to the full test.
RTW_D void ysphere_scan(const fscene& S, int first, int n, const fray& r, float tmin, fhit& h, float fc) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const float a = dot(r.d, r.d);
    auto full = [&](int i) {
        const prim32 q = uprim(S.prims, first + i);
        float t;
        if (sphere_t(q, r, tmin, h.t, t)) h.t = t, h.prim = first + i, h.rect = false;
    };
    // the ray's components splatted into pairs from register copies (built
    // from the struct itself, the compiler kept the caller's ray in scratch)
    float ox = r.o.x, oy = r.o.y, oz = r.o.z, dx = r.d.x, dy = r.d.y, dz = r.d.z;
    asm volatile("" : "+v"(ox), "+v"(oy), "+v"(oz), "+v"(dx), "+v"(dy), "+v"(dz));
    const f2 ox2 = ox, oy2 = oy, oz2 = oz, dx2 = dx, dy2 = dy, dz2 = dz, fc2 = fc, a2 = a;
    auto disc = [&](f2 cx, f2 cy, f2 cz, f2 dy, f2 rr, f2& slack) {
        const f2 ocx = ox2 - cx, ocz = oz2 - cz;
        const f2 ocy = __builtin_elementwise_fma(-dy, fc2, oy2 - cy);
        const f2 b = __builtin_elementwise_fma(ocx, dx2, __builtin_elementwise_fma(ocy, dy2, ocz * dz2));
        const f2 q = __builtin_elementwise_fma(ocx, ocx, __builtin_elementwise_fma(ocy, ocy, ocz * ocz));
        slack = 0x1p-18f * a2 * (q + rr);  // the filter's own rounding, generously
        return __builtin_elementwise_fma(b, b, -(a2 * (q - rr)));
    };
    const f2* g0 = reinterpret_cast<const f2*>(S.ysph + 8 * (size_t)first);
    const int np = n >> 1;
    for (int p = 0; p < np; ++p) {
        const f2* g = g0 + 8 * p;
        f2 e;
        const f2 d = disc(ld(g), ld(g + 1), ld(g + 2), ld(g + 3), ld(g + 4), e);
        if (__builtin_amdgcn_ballot_w64(!(d.x <= -e.x))) full(2 * p);
        if (__builtin_amdgcn_ballot_w64(!(d.y <= -e.y))) full(2 * p + 1);
    }
    if (n & 1) {  // the last sphere of an odd run keeps a plain record
        const float* g = S.ysph + 8 * (size_t)(first + n - 1);
        f2 e;
        const f2 d = disc(f2(ld(g)), f2(ld(g + 1)), f2(ld(g + 2)), f2(ld(g + 3)), f2(ld(g + 4)), e);
        if (__builtin_amdgcn_ballot_w64(!(d.x <= -e.x))) full(n - 1);
    }
}

// any-order test of prim i against the running best (BVH leaves)
RTW_D void arbitrate(const fscene& S, int i, const fray& r, float tmin, fhit& h) {
    const prim32& q = S.prims[i];
    const bool rl = !rtwd::is_sphere(q.type);
    float t;
    if (rl) {
        if (!rect_t(q, r, tmin, h.t, t)) return;
    } else {
        if (!sphere_t(q, r, tmin, __builtin_inff(), t) || t > h.t) return;
    }
    if (better(t, i, rl, h)) h.t = t, h.prim = i, h.rect = rl;
}
template <int K, int A, int B>
RTW_D void rect_arbitrate(const fscene& S, int i, const fray& r, float tmin, fhit& h) {
    float t;
    if (rect_axis_t<K, A, B>(S.prims[i], r, tmin, h.t, t) && better(t, i, true, h)) h.t = t, h.prim = i, h.rect = true;
}
struct rect_vf {
    float p[5];
};
template <int K, int A, int B>
RTW_D void rect_arbitrate_v(const rect_vf& q, int i, const fray& r, float tmin, fhit& h) {
    float t;
    if (rect_axis_t<K, A, B>(q, r, tmin, h.t, t) && better(t, i, true, h)) h.t = t, h.prim = i, h.rect = true;
}
RTW_D void arbitrate_item(const fscene& S, int it, const fray& r, float tmin, fhit& h) {
    if (it & RTW_ITEM_BOX) {  // a box's six rects in list order (hittable_list.h:65-114)
        const int b = it & RTW_ITEM_INDEX;
        // the six rects from the box's 32-B record where the scene has one (a
        // wave-uniform test; rtwd::box_arbitrate's reason): C5 fp32 32-spp
        // slice 979 vs 862 Msamples/s (+14 %, profiles/r06/ab_r6u_C5f.log;
        // bit-identical, parity_r6v_boxtab.log)
        if (S.boxes) {  // (b is the record; the record names the first rect)
            const float* q = S.boxes + 8 * (size_t)b;
            const float x0 = q[0], x1 = q[1], y0 = q[2], y1 = q[3], z0 = q[4], z1 = q[5];
            const int f = *reinterpret_cast<const int32_t*>(q + 6);
            rect_arbitrate_v<2, 0, 1>(rect_vf{{x0, x1, y0, y1, z1}}, f, r, tmin, h);
            rect_arbitrate_v<2, 0, 1>(rect_vf{{x0, x1, y0, y1, z0}}, f + 1, r, tmin, h);
            rect_arbitrate_v<1, 0, 2>(rect_vf{{x0, x1, z0, z1, y1}}, f + 2, r, tmin, h);
            rect_arbitrate_v<1, 0, 2>(rect_vf{{x0, x1, z0, z1, y0}}, f + 3, r, tmin, h);
            rect_arbitrate_v<0, 1, 2>(rect_vf{{y0, y1, z0, z1, x1}}, f + 4, r, tmin, h);
            rect_arbitrate_v<0, 1, 2>(rect_vf{{y0, y1, z0, z1, x0}}, f + 5, r, tmin, h);
            return;
        }
        rect_arbitrate<2, 0, 1>(S, b, r, tmin, h);
        rect_arbitrate<2, 0, 1>(S, b + 1, r, tmin, h);
        rect_arbitrate<1, 0, 2>(S, b + 2, r, tmin, h);
        rect_arbitrate<1, 0, 2>(S, b + 3, r, tmin, h);
        rect_arbitrate<0, 1, 2>(S, b + 4, r, tmin, h);
        rect_arbitrate<0, 1, 2>(S, b + 5, r, tmin, h);
    } else {
        arbitrate(S, it, r, tmin, h);
    }
}

// BVH walks: nodes padded outward by the builder and rounded outward to fp32
struct slab_rayf {
    f3 inv, oi;  // t = x * inv + oi per axis
};
RTW_D slab_rayf make_slab(const fscene& S, const fray& r) {
    slab_rayf s;
    s.inv = f3{rcp(r.d.x), rcp(r.d.y), rcp(r.d.z)};
    s.oi = f3{-r.o.x * s.inv.x, -r.o.y * s.inv.y, -r.o.z * s.inv.z};
    (void)S;
    return s;
}
RTW_D bool slab(const bvh_node32& nd, const slab_rayf& s, float t0, float t1) {
    const float x0 = __builtin_fmaf(nd.lo[0], s.inv.x, s.oi.x), x1 = __builtin_fmaf(nd.hi[0], s.inv.x, s.oi.x);
    const float y0 = __builtin_fmaf(nd.lo[1], s.inv.y, s.oi.y), y1 = __builtin_fmaf(nd.hi[1], s.inv.y, s.oi.y);
    const float z0 = __builtin_fmaf(nd.lo[2], s.inv.z, s.oi.z), z1 = __builtin_fmaf(nd.hi[2], s.inv.z, s.oi.z);
    const float tn = __builtin_fmaxf(__builtin_fmaxf(t0, __builtin_fminf(x0, x1)),
                                     __builtin_fmaxf(__builtin_fminf(y0, y1), __builtin_fminf(z0, z1)));
    const float tf = __builtin_fminf(__builtin_fminf(t1, __builtin_fmaxf(x0, x1)),
                                     __builtin_fminf(__builtin_fmaxf(y0, y1), __builtin_fmaxf(z0, z1)));
    return tn <= tf * 1.00000024f;  // a 2-ulp allowance for the fp32 slab arithmetic
}
// (explicit address spaces, as rtwd::node_at: an LDS read for packet nodes,
// a global read for the rest)
// PALL: the all-in-packet shortcut is compiled in (every fp32 BVH kernel
// since round 6; with 16-entry stacks the media kernel's packet never held
// every node and the branch cost it a spilled register: C5 fp32 -1.4 %,
// profiles/r05/ab_r5f_fpall.log)
template <bool PALL = true>
RTW_D bvh_node32 node_at(const fscene& S, int i) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    using lds_v4 = const __attribute__((address_space(3))) v4u;
    using glb_v4 = const __attribute__((address_space(1))) v4u;
    v4u a, b;
    if (PALL && S.n_lnodes >= S.n_nodes) {  // every node in the packet: wave-uniform
        lds_v4* p = (lds_v4*)(S.lnodes + i);
        a = p[0], b = p[1];
    } else if (i < S.n_lnodes) {
        lds_v4* p = (lds_v4*)(S.lnodes + i);
        a = p[0], b = p[1];
    } else {
        glb_v4* p = (glb_v4*)(S.nodes + i);
        a = p[0], b = p[1];
        asm volatile("" ::"v"(a.x));  // keeps the two loads apart (else they become one flat load)
    }
    bvh_node32 nd;
    __builtin_memcpy(&nd, &a, 16);
    __builtin_memcpy(reinterpret_cast<char*>(&nd) + 16, &b, 16);
    return nd;
}

// (The speculative while-while of the fp64 world walk, without its child
// test, measured C3 fp32 -12 % here: the 8-wave kernel spills more around
// the two-level loop.)
// Workgroup size of k_fast: the LDS node packet is one per workgroup, so
// larger workgroups at the same waves per CU share a larger packet (as
// rtwd::kPBlock for k_persist); 1 024 threads = two workgroups of 16 waves
// per CU at 8 waves per SIMD (rtw_kernels.hip RTW_FAST_BVH_WAVES: measured).
constexpr int kFastBlock = 1024;
// ... and of the media kernel (F_MEDIA: Book 2).  Measured (1 MI355X, A/B,
// profiles/r05/ab_r5e_fmedia.log, C5 fp32 slice): 1 024 threads at 8 waves
// (64 VGPRs, 17 spilled) 843; 896 at 7 (72 VGPRs, 9 spilled, a 1 632-node
// packet) 472; 768 at 6 (spill-free, every node in the packet, its fetch
// shortcut) 751.  1 024 stays.
constexpr int fast_block(int F) { return kFastBlock; }
// LDS stack entries per lane.  The media kernel's walks are group walks
// from an empty stack (a scene with media has no world BVH), which hold at
// most D entries for a tree of depth D (launch_fast: group_depth), so 12
// entries serve Book 2's trees (depths 10 and 12) where the general bound
// (world + group depth + 2) asks for 16.  The 8 KB this frees per
// workgroup grows the node packet from 1 534 to all 1 668 of Book 2's nodes
// at two 1 024-thread workgroups per CU, and every node is then an LDS
// read (node_at<PALL>): C5 fp32 32-spp slice 856 vs 828 Msamples/s
// (+3.4 %, profiles/r06/ab_r6o_C5f.log; bit-identical, parity_r6o_mstack.log).
constexpr int kMediaStack = 12;
constexpr int fast_stack(int F) { return (F & rtwd::F_MEDIA) ? kMediaStack : rtwd::kLdsStack; }
// the all-in-packet node fetch (node_at<PALL>, a wave-uniform test)
constexpr bool fast_pall(int F) { return true; }

// traversal stacks: a column of 16-bit node ids per lane in LDS (column
// stride: the workgroup size), or a private array
template <int BLK, int CAP = rtwd::kLdsStack>
struct lds_stackf_t {
    static constexpr int cap = CAP;
    uint16_t* p;
    RTW_D uint16_t& at(int i) { return p[i * BLK]; }
};
using lds_stackf = lds_stackf_t<kFastBlock>;
struct priv_stackf {
    static constexpr int cap = rtwd::kStack;
    int s[rtwd::kStack];
    RTW_D int& at(int i) { return s[i]; }
};

template <bool PALL = true, class STK>
RTW_D void group_bvh(const fscene& S, int root, const fray& r, float tmin, fhit& h, STK& stk, int base) {
    const slab_rayf sr = make_slab(S, r);
    const float t0 = tmin > 0 ? tmin * 0.5f : tmin * 2.0f - 1e-6f;
    int sp = base;
    stk.at(sp++) = root;
    while (sp > base) {
        const bvh_node32 nd = node_at<PALL>(S, stk.at(--sp));
        if (!slab(nd, sr, t0, h.t)) continue;
        if (nd.b < 0) {
            // (the fp32 node copy: b == -1 one item, in a; b < -16 two items,
            // a and b's low bits; else an index and a count)
            const bool inl = nd.b == -1 || nd.b < -16;
            const int n = nd.b == -1 ? 1 : (nd.b < -16 ? 2 : -nd.b);
            for (int k = 0; k < n; ++k) {
                int it;
                if (inl)
                    it = k == 0 ? nd.a : (nd.b & 0x7fffffff);
                else
                    it = S.items[nd.a + k];
                arbitrate_item(S, it, r, tmin, h);
            }
        } else if (sp + 2 <= STK::cap) {
            stk.at(sp++) = nd.b & 0x0fffffff;
            stk.at(sp++) = nd.a;
        }
    }
}

template <int F, class STK>
RTW_D void group_closest(const fscene& S, const ent_v& e, const fray& r, float tmin, fhit& h, STK& stk, int base) {
    if ((F & rtwd::F_GBVH) && e.bvh_root >= 0)
        group_bvh<fast_pall(F)>(S, e.bvh_root, r, tmin, h, stk, base);
    else
        group_scan(S, e.first_prim, e.n_prims, r, tmin, h);
}

// constant_medium::hit hittable.h:430-479 in the medium's frame
template <int F, class STK>
RTW_D bool medium_t(const fscene& S, const ent_v& e, const fray& rw, float tmin, float tmax, uint32_t& rng,
                    float& t_out, STK& stk) {
    const int outer = ld(&e.p->n_outer_ops);
    const fray r = ops_in<true>(e, rw, 0, outer);
    const fray lr = ops_in<true>(e, r, outer, e.n_ops);
    fhit b1{kFltMaxF, -1, false};
    group_closest<F>(S, e, lr, -kFltMaxF, b1, stk, 0);
    if (b1.prim == -1) return false;
    fhit b2{kFltMaxF, -1, false};
    group_closest<F>(S, e, lr, b1.t + kStepF, b2, stk, 0);
    if (b2.prim == -1) return false;
    float t1 = b1.t, t2 = b2.t;
    if (t1 < tmin) t1 = tmin;
    if (t2 > tmax) t2 = tmax;
    if (t1 >= t2) return false;
    if (t1 < 0) t1 = 0;
    const float dl = len(r.d);
    const float inside = (t2 - t1) * dl;
    const float hit_distance = ld(&e.p->neg_inv_density) * __logf(u01(rng));
    if (hit_distance < inside) {
        t_out = t1 + hit_distance * rcp(dl);
        return true;
    }
    return false;
}

// hittable_list::hit over the world (hittable_list.h:11-37)
template <int F, class STK>
RTW_D fhit world_closest(const fscene& S, const fray& r, uint32_t& rng, STK& stk) {
    fhit h{kFltMaxF, -1, false};
    if constexpr ((F & rtwd::F_WBVH) != 0 && (F & rtwd::F_MEDIA) == 0) {
        const slab_rayf sr = make_slab(S, r);
        const float t0 = kTMinF * 0.5f;
        int sp = 0;
        stk.at(sp++) = S.world_bvh_root;
        while (sp > 0) {
            const bvh_node32 nd = node_at<fast_pall(F)>(S, stk.at(--sp));
            if (!slab(nd, sr, t0, h.t)) continue;
            if (nd.b >= 0) {
                if (sp + 2 <= STK::cap) stk.at(sp++) = nd.b & 0x0fffffff, stk.at(sp++) = nd.a;
                continue;
            }
            for (int k = 0; k < -nd.b; ++k) {
                // (a one-item world leaf holds its item: launch-time fp32 nodes)
                const int it = nd.b == -1 ? nd.a : S.items[nd.a + k];
                if (it < 0) {  // a plain one-prim entry: ~prim
                    arbitrate(S, ~it, r, kTMinF, h);
                    continue;
                }
                const ent_v e = view_entry<false>(S, it);
                const fray lr = ops_in<false>(e, r, 0, e.n_ops);
                if ((F & rtwd::F_GBVH) && e.bvh_root >= 0)
                    group_bvh<fast_pall(F)>(S, e.bvh_root, lr, kTMinF, h, stk, sp);
                else
                    for (int i = 0; i < e.n_prims; ++i) arbitrate(S, e.first_prim + i, lr, kTMinF, h);
            }
        }
    } else if constexpr ((F & rtwd::F_MEDIA) != 0) {
        // the media walk: entries in the reference's visit order, media
        // drawn again in the second walk
        for (int k = 0; k < S.n_media; ++k) {
            const int ei = ld(&S.media[k]) & rtwd::kVisitEntry;  // (the fp64 walk's cache slots unused here)
            const ent_v e = view_entry<true>(S, ei);
            if (e.kind == RTW_ENTRY_MEDIUM) {
                float t;
                if (medium_t<F>(S, e, r, kTMinF, h.t, rng, t, stk)) h.t = t, h.prim = -(2 + ei), h.rect = false;
            } else {
                const fray lr = ops_in<true>(e, r, 0, e.n_ops);
                group_closest<F>(S, e, lr, kTMinF, h, stk, 0);
            }
        }
    } else {
        for (int ri = 0; ri < S.n_runs; ++ri) {
            const int ei = ld(&S.runs[ri].entry);
            if (ei == rtwd::WORLD_RUN_YSPHERES) {
                const float fc = ld(&S.runs[ri].movers) ? (r.t - S.mv_t0) * S.mv_inv_den : 0.0f;
                ysphere_scan(S, ld(&S.runs[ri].first_prim), ld(&S.runs[ri].n_prims), r, kTMinF, h, fc);
                continue;
            }
            // (two scan sites rather than one over a conditionally
            // transformed copy of the ray: that copy was kept in scratch)
            if (ei >= 0) {
                const ent_v e = view_entry<true>(S, ei);
                const fray lr = ops_in<true>(e, r, 0, e.n_ops);
                if ((F & rtwd::F_GBVH) && e.bvh_root >= 0) {
                    group_bvh<fast_pall(F)>(S, e.bvh_root, lr, kTMinF, h, stk, 0);
                    continue;
                }
                group_scan(S, ld(&S.runs[ri].first_prim), ld(&S.runs[ri].n_prims), lr, kTMinF, h);
            } else {
                group_scan(S, ld(&S.runs[ri].first_prim), ld(&S.runs[ri].n_prims), r, kTMinF, h);
            }
        }
    }
    return h;
}

// the hit record of the winner (leaf hit, then ops outward)
RTW_D void hit_record(const fscene& S, const fray& r, const fhit& h, f3& p, f3& n, int& mat, int& frame_prim) {
    frame_prim = -1;
    if (h.prim <= -2) {
        const ent_v e = view_entry<false>(S, -h.prim - 2);
        const int outer = e.p->n_outer_ops;
        const fray mr = ops_in<false>(e, r, 0, outer);
        p = at(mr, h.t);
        n = f3{1, 0, 0};
        ops_out<false>(e, outer, p, n);
        mat = e.p->phase_material;
        return;
    }
    const prim32& q = S.prims[h.prim];
    const ent_v e = view_entry<false>(S, q.entry);
    const fray lr = ops_in<false>(e, r, 0, e.n_ops);
    p = at(lr, h.t);
    const int type = q.type;
    if (rtwd::is_sphere(type)) {
        n = (p - sphere_center(q, lr.t)) * rcp(q.p[3]);
    } else {
        n = rect_normal(type);
        frame_prim = h.prim;
    }
    if (q.flip & 1) n = -n;
    ops_out<false>(e, e.n_ops, p, n);
    mat = q.material;
}

// ------------------------------------------------------------------ textures
RTW_D float perlin_noise(const float* ranvec, const int32_t* perm, f3 p) {  // noise.h:89-151
    const float fx = __builtin_floorf(p.x), fy = __builtin_floorf(p.y), fz = __builtin_floorf(p.z);
    const float u = p.x - fx, v = p.y - fy, w = p.z - fz;
    const int i = (int)fx, j = (int)fy, k = (int)fz;
    const float uu = u * u * (3 - 2 * u), vv = v * v * (3 - 2 * v), ww = w * w * (3 - 2 * w);
    float accum = 0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int idx = perm[(i + a) & 255] ^ perm[256 + ((j + b) & 255)] ^ perm[512 + ((k + c) & 255)];
                const f3 g = ldf3(ranvec + 3 * idx);
                accum += (a ? uu : 1 - uu) * (b ? vv : 1 - vv) * (c ? ww : 1 - ww) * dot(g, f3{u - a, v - b, w - c});
            }
    return accum;
}
RTW_D float turb(const float* ranvec, const int32_t* perm, f3 p) {  // noise.h:74-86
    float accum = 0, weight = 1.0f;
    for (int i = 0; i < 7; ++i) {
        accum += weight * perlin_noise(ranvec, perm, p);
        weight *= 0.5f;
        p = p * 2.0f;
    }
    return __builtin_fabsf(accum);
}
// NOISE = false: the scene has no noise texture (kernels for such scenes
// compile the marble branch out: its seven octaves of eight gradients are
// the widest register peak of the fp32 kernels, and inlined they set the
// register budget of every path -- the list kernel spilled in shading for it
// though Cornell has no noise texture)
template <bool NOISE = true>
RTW_D f3 texture_value(const fscene& S, int id, f3 p) {
    for (int guard = 0; guard < 8; ++guard) {
        const tex32& t = S.textures[id];
        if (t.type == RTW_TEX_CONSTANT) return ldf3(t.color);
        if (t.type == RTW_TEX_CHECKER) {  // texture.h:38-49
            const float sines = __sinf(10 * p.x) * __sinf(10 * p.y) * __sinf(10 * p.z);
            id = sines < 0 ? t.odd : t.even;
            continue;
        }
        if constexpr (!NOISE) return f3{0, 0, 0};  // unreachable: no noise texture in the scene
        const float v = 0.5f * (1 + sinf(t.scale * p.z + 10 * turb(S.ranvec, S.perm, p)));  // texture.h:57-68
        return f3{v, v, v};
    }
    return f3{0, 0, 0};
}

// ------------------------------------------------------------------ sampling
struct onbf {
    f3 u, v, w;
};
RTW_D onbf onb_from_w(f3 n) {  // onb.h:32-38
    onbf b;
    b.w = normalize(n);
    const f3 a = (__builtin_fabsf(b.w.x) > 0.9f) ? f3{0, 1, 0} : f3{1, 0, 0};
    b.v = normalize(cross(b.w, a));
    b.u = cross(b.w, b.v);
    return b;
}
RTW_D f3 local(const onbf& b, f3 a) { return b.u * a.x + b.v * a.y + b.w * a.z; }
RTW_D onbf frame(const fscene& S, f3 n, int frame_prim) {
    if (frame_prim >= 0) {
        const float* f = S.frames + 9 * (size_t)frame_prim;
        return onbf{ldf3(f), ldf3(f + 3), ldf3(f + 6)};
    }
    return onb_from_w(n);
}
RTW_D f3 random_in_unit_sphere(uint32_t& s) {  // utility.h:27-35
    f3 p;
    do {
        p = f3{u01(s), u01(s), u01(s)} * 2.0f - f3{1, 1, 1};
    } while (dot(p, p) >= 1.0f);
    return p;
}
RTW_D f3 cone_dir(float r1, float z) {  // shared tail of the cosine / sphere-cone samplers
    const float sq = fsqrt(__builtin_fmaxf(0.0f, 1 - z * z));
    return f3{cos_rev(r1) * sq, sin_rev(r1) * sq, z};
}
RTW_D float light_pdf_value(const fscene& S, const rtw_light& L, f3 o, f3 v) {
    const fray r{o, v, kFltMaxF};
    float t;
    if (L.kind == RTW_LIGHT_XZ_RECT) {  // hittable.h:208-222
        const prim32& q = S.prims[L.prim];
        if (!rect_axis_t<1, 0, 2>(q, r, 0.001f, __builtin_inff(), t)) return 0;
        const float area = (q.p[1] - q.p[0]) * (q.p[3] - q.p[2]);
        const float vv = len2(v);
        return (t * t * vv) / (__builtin_fabsf(v.y) * __builtin_amdgcn_rsqf(vv) * area);
    }
    if (L.kind == RTW_LIGHT_SPHERE) {  // sphere.h:88-99
        const prim32& q = S.prims[L.prim];
        if (!sphere_t(q, r, 0.001f, __builtin_inff(), t)) return 0;
        const float cos_theta_max = fsqrt(__builtin_fmaxf(0.0f, 1 - q.p[9] * rcp(len2(f3{q.p[0], q.p[1], q.p[2]} - o))));
        return rcp(2 * kPiF * (1.0f - cos_theta_max));
    }
    return 0;
}
// mixture_pdf(cosine_pdf, hittable_pdf(lights))::generate (pdf.h:55-79)
RTW_D f3 mixture_generate(const fscene& S, const onbf& fr, f3 o, uint32_t& rng) {
    if (u01(rng) < 0.5f) {
        const float r1 = u01(rng), r2 = u01(rng);
        return local(fr, cone_dir(r1, fsqrt(1 - r2)));
    }
    const int span = (int)(S.n_lights * u01(rng));
    const rtw_light L = S.lights[span < S.n_lights - 1 ? span : S.n_lights - 1];
    if (L.kind == RTW_LIGHT_XZ_RECT) {  // hittable.h:224-228
        const prim32& q = S.prims[L.prim];
        const float rz = q.p[2] + (q.p[3] - q.p[2]) * u01(rng);
        const float rx = q.p[0] + (q.p[1] - q.p[0]) * u01(rng);
        return f3{rx, q.p[4], rz} - o;
    }
    if (L.kind == RTW_LIGHT_SPHERE) {  // sphere.h:101-108, utility.h:69-81
        const prim32& q = S.prims[L.prim];
        const f3 dir = f3{q.p[0], q.p[1], q.p[2]} - o;
        const float r1 = u01(rng), r2 = u01(rng);
        const float z = 1 + r2 * (fsqrt(__builtin_fmaxf(0.0f, 1 - q.p[9] * rcp(len2(dir)))) - 1);
        return local(onb_from_w(dir), cone_dir(r1, z));
    }
    return f3{1, 0, 0};  // hittable.h:37
}
RTW_D float lights_pdf_value(const fscene& S, f3 o, f3 v) {  // hittable_list.h:44-53
    float sum = 0;
    for (int i = 0; i < S.n_lights; ++i) sum += light_pdf_value(S, S.lights[i], o, v);
    return sum * S.light_weight;
}

RTW_D f3 reflect(f3 v, f3 n) { return v - n * (2.0f * dot(v, n)); }  // material.h:10-13

// ------------------------------------------------------------------ shading
// One segment of color() (RayTracingWeekend.cpp:52-159) for a path whose
// world hit is h: the path ends with radiance thr * w (emission or
// background; w = 0 for an absorbed path), or continues with thr *= w along
// `next` (depth - 1).  rng advances by the draws the branch takes.
struct seg_f {
    bool cont;
    f3 w;
    fray next;
};
template <bool NOISE = true>
RTW_D seg_f shade(const fscene& S, const fray& r, const fhit& h, uint32_t& rng, uint32_t depth) {
    seg_f o{false, f3{0, 0, 0}, r};
    if (h.prim == -1) {  // background :141-159
        if (S.background == RTW_BG_GRADIENT) {
            const float t = 0.5f * (normalize(r.d).y + 1.0f);
            o.w = f3{1, 1, 1} * (1.0f - t) + f3{0.5f, 0.7f, 1.0f} * t;
        }
        return o;
    }
    f3 p, n;
    int mat, fp;
    hit_record(S, r, h, p, n, mat, fp);
    if (S.render_type == RTW_RENDER_NORMAL) {  // :135-136
        o.w = (n + f3{1, 1, 1}) * 0.5f;
        return o;
    }
    // The material's type and texture are read here; its other fields where
    // a branch uses them, through an opaque copy of the index (a material
    // pointer formed once was held in a VGPR pair across every branch, and
    // spilled to scratch: most of the fp32 kernels' write traffic).
    const int type = S.materials[mat].type;
    const int tex = S.materials[mat].texture;
    auto mat_now = [&]() -> const mat32& {
        int m = mat;
        asm volatile("" : "+v"(m));
        return S.materials[m];
    };
    if (type == RTW_MAT_DIFFUSE_LIGHT) {  // material.h:232-244, one-sided
        if (dot(n, r.d) > 0) o.w = texture_value<NOISE>(S, tex, p);
        return o;
    }
    f3 f{1, 1, 1}, dir;
    if (type == RTW_MAT_METAL) {  // material.h:128-136
        const mat32& M = mat_now();
        dir = reflect(normalize(r.d), n) + random_in_unit_sphere(rng) * M.fuzz;
        f = ldf3(M.albedo);
    } else if (type == RTW_MAT_DIELECTRIC) {  // material.h:146-222
        const mat32& M = mat_now();
        const float dn = dot(r.d, n), il = __builtin_amdgcn_rsqf(len2(r.d));
        const float ri = M.ref_idx;
        f3 outward;
        float ni, cosine;
        if (dn > 0) {
            outward = -n;
            ni = ri;
            cosine = dn * il;
            cosine = fsqrt(__builtin_fmaxf(0.0f, 1 - ri * ri * (1 - cosine * cosine)));
        } else {
            outward = n;
            ni = M.inv_ref_idx;
            cosine = -dn * il;
        }
        const f3 uv = r.d * il;
        const float dt = dot(uv, outward);
        const float disc = 1.0f - ni * ni * (1 - dt * dt);
        f3 refracted{0, 0, 0};
        float reflect_prob = 1.0f;
        if (disc > 0) {
            refracted = (uv - outward * dt) * ni - outward * fsqrt(disc);
            const float x = 1 - cosine, x2 = x * x;
            reflect_prob = M.r0 + (1 - M.r0) * (x2 * x2 * x);
        }
        dir = u01(rng) < reflect_prob ? reflect(r.d, n) : refracted;
    } else if (type == RTW_MAT_ISOTROPIC) {  // material.h:257-262
        dir = random_in_unit_sphere(rng);
        f = texture_value<NOISE>(S, tex, p);
    } else {  // lambertian material.h:81-119 + RayTracingWeekend.cpp:112-132
        const onbf fr = frame(S, n, fp);
        float pdf_val;
        if (S.n_lights > 0) {
            dir = mixture_generate(S, fr, p, rng);
            const float cw = dot(normalize(dir), fr.w);
            pdf_val = 0.5f * (cw <= 0 ? 0.0f : cw * (1.0f / kPiF)) + 0.5f * lights_pdf_value(S, p, dir);
        } else {
            const float r1 = u01(rng), r2 = u01(rng);
            dir = local(fr, cone_dir(r1, fsqrt(1 - r2)));
            const float cw = dot(normalize(dir), fr.w);
            pdf_val = cw <= 0 ? 0.0f : cw * (1.0f / kPiF);
        }
        if (!(pdf_val > 0)) return o;  // :126-127 returns emitted (0)
        const float cosine = dot(n, normalize(dir));
        const float spdf = cosine < 0 ? 0.0f : cosine * (1.0f / kPiF);
        f = texture_value<NOISE>(S, tex, p) * (spdf * rcp(pdf_val));
    }
    if (depth <= 1) return o;  // the next color() call has depth 0: returns 0
    o.cont = true;
    o.w = f;
    o.next = fray{p, dir, r.t};
    return o;
}

// the material class of a hit, the key the regrouping kernel sorts by
// (the sorted block's order, as k_persist_sort's: material order,
// path-ending keys last)
enum { FK_LAMB = 0, FK_DIEL, FK_METAL, FK_ISO, FK_EMIT, FK_MISS, FK_IDLE, FK_N };
RTW_D int hit_key(const fscene& S, const fhit& h) {
    if (h.prim == -1) return FK_MISS;
    const int mat = h.prim <= -2 ? S.entries[-h.prim - 2].phase_material : S.prims[h.prim].material;
    const int ty = S.materials[mat].type;
    return ty == RTW_MAT_LAMBERTIAN ? FK_LAMB
           : ty == RTW_MAT_DIELECTRIC ? FK_DIEL
           : ty == RTW_MAT_METAL ? FK_METAL
           : ty == RTW_MAT_ISOTROPIC ? FK_ISO
                                     : FK_EMIT;
}

// ------------------------------------------------------------------ camera
struct cam32 {
    float origin[3], lower_left[3], horizontal[3], vertical[3], u[3], v[3];
    float time0, dtime, lens_radius;
};
// camera::get_ray camera.h:36-50 (thin lens, shutter time)
RTW_D fray camera_ray(const cam32& c, float s, float t, uint32_t& rng) {
    f3 rd{0, 0, 0};
    if (c.lens_radius > 0) {  // random_in_unit_disk camera.h:61-69
        f3 p;
        do {
            p = f3{u01(rng), u01(rng), 0} * 2.0f - f3{1, 1, 0};
        } while (dot(p, p) >= 1.0f);
        rd = p * c.lens_radius;
    }
    const f3 offset = ldf3(c.u) * rd.x + ldf3(c.v) * rd.y;
    const float time = c.time0 + u01(rng) * c.dtime;
    const f3 dir = ldf3(c.lower_left) + ldf3(c.horizontal) * s + ldf3(c.vertical) * t - ldf3(c.origin) - offset;
    return fray{ldf3(c.origin) + offset, normalize(dir), time};
}

}  // namespace rtwf
