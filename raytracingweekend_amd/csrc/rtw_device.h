// rtw_device.h — gfx950 device code of the path tracer: fp64 vector math,
// per-path minstd_rand, primitive / group / world closest-hit, materials,
// pdfs, textures and camera ray generation.
//
// Every function restates one reference function (file:line cited) with the
// same fp64 operation order; the translation unit is compiled with
// -ffp-contract=off so no multiply-add is fused (x86-64 g++ fuses none), and
// fp64 division / sqrt are the IEEE correctly rounded sequences.  What can
// differ from the host reference is the last ulp of ocml's sin/cos/pow/log
// against glibc's ("Parity").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "rtw_gpu.h"
#include "rtw_div.h"
#include "rtw_math.h"

#define RTW_D __device__ __forceinline__
// vector helpers also used by the host to precompute per-primitive frames
// with the very same arithmetic (see upload_scene)
#define RTW_HD __host__ __device__ __forceinline__

namespace rtwd {

constexpr double kPi = 3.14159265358979323846;
constexpr double kTwoPi = 2 * kPi;                 // `2 * M_PI` (exact doubling)
constexpr double kInvPi = 1.0 / kPi;

// RTW_RADIANCE_FAST: a path's radiance is the product of per-bounce factors
// (attenuation * scattering_pdf / pdf) and the emission it ends on; those
// values never steer a path -- no branch, ray or random draw of the
// reference reads them, only the SIGN of pdf_val (RayTracingWeekend.cpp:
// 126-127) -- so they may be formed with fewer divisions: the lambertian
// factor as texture * (cosine / (pi pdf_val)) (one division instead of
// four), cosine / pi as cosine * (1 / pi) (the same sign: both round the same
// positive real), the rect light's distance^2 / (cosine area) with one
// division.  Paths, traversal counts and every decision stay the
// reference's; the radiance moves by a few ulps (the parity bound is 1e-4).
// RTW_STRICT_RADIANCE (a build of its own, librtw_strict.so: tests and
// maintainers' checks): the reference's radiance arithmetic exactly -- these
// reorderings off, and each path's factors folded inside-out at its end as
// the recursion of color() folds them (rtw_kernels.hip, k_persist).
#ifndef RTW_STRICT_RADIANCE
#define RTW_STRICT_RADIANCE 0
#endif
#ifndef RTW_RADIANCE_FAST
#define RTW_RADIANCE_FAST (!RTW_STRICT_RADIANCE)
#endif
#if RTW_STRICT_RADIANCE && RTW_RADIANCE_FAST
#error "RTW_STRICT_RADIANCE needs RTW_RADIANCE_FAST 0"
#endif
// ... and (RTW_RADIANCE_RCP) the remaining radiance-only quotients -- the
// lambertian factor, the rect light's pdf, the sphere light's 1 / solid angle -- as
// products with rcp_hw's reciprocal (within an ulp of 1 / x; a wave with a
// lane outside [2^-200, 2^200] divides exactly, so zeros and infinities keep
// division's results).
// Measured (1 MI355X, A/B, profiles/r04/ab_radrcp_r4n.log; GPU suite green
// with it): T 4 460 vs 4 446, C5 slice 663 vs 661.
#ifndef RTW_RADIANCE_RCP
#define RTW_RADIANCE_RCP RTW_RADIANCE_FAST
#endif
constexpr double kDblMax = 1.7976931348623157e308; // std::numeric_limits<double>::max()
constexpr double kFltMax = 3.4028234663852886e38;  // FLT_MAX widened
constexpr double kTMin = (double)0.001f;           // RayTracingWeekend.cpp:52 (float literal)
constexpr double kStep = (double)0.0001f;          // hittable.h:447
constexpr double kOneMinusUlp = 0.99999999999999989; // nextafter(1.0, 0.0)
// generate_canonical's divisor: (double)((long double)R * R), R = 2^31 - 2
constexpr double kCanonDiv = 4611686009837453312.0;
constexpr double kCanonR = 2147483646.0;
constexpr double kCanonRcp = 1.0 / kCanonDiv;  // RN(1/x): constant folding is IEEE

// A value materialised where it is used (an opaque VGPR copy the compiler can
// neither hoist out of a loop nor merge with another use): 64-bit constants
// the persistent kernels need inside their loop (the initial closest t, a
// zero radiance) are otherwise held in VGPR pairs across the whole loop and
// spilled to scratch.
// (The two v_mov are emitted by the asm itself: an opaque copy of a
// constant would still be fed from the loop-carried register.)
template <uint64_t B>
__device__ __forceinline__ double in_place() {
    uint32_t lo, hi;
    asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %3" : "=v"(lo), "=v"(hi) : "i"((uint32_t)B), "i"((uint32_t)(B >> 32)));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
constexpr uint64_t kDblMaxBits = 0x7FEFFFFFFFFFFFFFull;  // == kDblMax

// ------------------------------------------------------------------ libm
// sin of the textures (texture.h:45, :66) and log of the media (hittable.h:
// 450): rtw_math.h's sin_wide / log_pos (within an ulp of glibc's, which the
// reference calls) in their ranges, ocml's functions in separate functions
// beyond.  ocml's inlined sin and log hold fifteen 64-bit polynomial
// constants the media kernels kept in VGPR pairs across their loop and
// spilled; log_pos reads its constants from a table where it runs.
__device__ __attribute__((noinline)) double sin_far(double x) { return sin(x); }
__device__ __attribute__((noinline)) double log_far(double x) { return log(x); }
RTW_D double sin_tex(double x) {
    double s = sin_wide(x);
    if (__builtin_expect(!sin_wide_ok(x), 0)) {
        asm volatile("");
        s = sin_far(x);
    }
    return s;
}
__constant__ double c_log_coef[9] = {kLogCoef[0], kLogCoef[1], kLogCoef[2], kLogCoef[3], kLogCoef[4],
                                     kLogCoef[5], kLogCoef[6], kLogCoef[7], kLogCoef[8]};
RTW_D double log_dev(double x) {
    const __attribute__((address_space(4))) double* t = (const __attribute__((address_space(4))) double*)c_log_coef;
    asm volatile("" : "+s"(t));  // the table's loads are issued here, not hoisted
    double l = log_pos(x, [&](int i) { return t[i]; });
    if (__builtin_expect(!log_pos_ok(x), 0)) {
        asm volatile("");
        l = log_far(x);
    }
    return l;
}

// ------------------------------------------------------------------ vec3
struct d3 {
    double x, y, z;
};
RTW_HD d3 mk(double x, double y, double z) { return d3{x, y, z}; }
RTW_HD d3 operator+(d3 a, d3 b) { return d3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RTW_HD d3 operator-(d3 a, d3 b) { return d3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RTW_HD d3 operator*(d3 a, d3 b) { return d3{a.x * b.x, a.y * b.y, a.z * b.z}; }
RTW_HD d3 operator*(d3 a, double s) { return d3{a.x * s, a.y * s, a.z * s}; }
// d3 / double (vec3.h operator/): three IEEE divisions.  (Sharing one
// reciprocal behind a range vote measured T -3.3 %: EXPERIMENTS.md.)
RTW_HD d3 operator/(d3 a, double s) { return d3{a.x / s, a.y / s, a.z / s}; }
RTW_HD d3 operator-(d3 a) { return d3{-a.x, -a.y, -a.z}; }
// a / b for a quantity that only scales radiance (RTW_RADIANCE_RCP)
__device__ __forceinline__ double rad_div(double a, double b) {
#if RTW_RADIANCE_RCP
    if (__builtin_amdgcn_ballot_w64(!div_hw_ok_b_exp(b)) == 0) return a * rcp_hw(b);
#endif
    return a / b;
}
RTW_HD double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RTW_HD double len2(d3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
// fp64 square roots as rtw_div.h's sqrt_w (the compiler's own sequence
// without its range scaling and class fixup, taken when the whole wave is in
// range; bit for bit the same value) or sqrt_core where the range is known
// (1 - a canonical draw).  Measured T +0.5 %, C5 +1.7 % (EXPERIMENTS.md).
#if defined(__HIP_DEVICE_COMPILE__)
#define RTW_SQRT(x) sqrt_w(x)
#define RTW_SQRT_POS(x) sqrt_core(x)  // x in [2^-766, 2^1024): callers argue it
#else
#define RTW_SQRT(x) __builtin_sqrt(x)
#define RTW_SQRT_POS(x) __builtin_sqrt(x)
#endif
RTW_HD double len(d3 a) { return __builtin_sqrt(len2(a)); }
RTW_HD d3 cross(d3 a, d3 b) {  // vec3.h:54-59
    return d3{a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x};
}
// (normalize keeps the compiler's sqrt: sqrt_w's wave-uniform branch in
// every normalization cost SGPRs, T -1.3 %)
RTW_HD d3 normalize(d3 v) { return v / len(v); }  // vec3.h:61-67
// (the compiler's sqrt: in onb_from_w a wave-uniform branch inside the
// frame's normalizations turned the onb into a scratch object)
RTW_HD d3 normalize_b(d3 v) { return v / len(v); }
RTW_HD d3 ld3(const double* p) { return d3{p[0], p[1], p[2]}; }

struct ray {
    d3 o, d;
    double t;
};
RTW_D d3 at(const ray& r, double t) { return r.o + r.d * t; }  // ray.h:103

// ------------------------------------------------------------------ RNG
// std::minstd_rand: x <- 48271 x mod (2^31 - 1), via the Mersenne fold.
RTW_D uint32_t mr_next(uint32_t& s) {
    const uint64_t p = (uint64_t)s * 48271u;
    uint32_t r = (uint32_t)(p & 0x7fffffffu) + (uint32_t)(p >> 31);
    if (r >= 0x7fffffffu) r -= 0x7fffffffu;
    s = r;
    return r;
}

// The engine k steps ahead: x <- (48271^k mod m) x mod m, one multiply and
// the same fold as mr_next (a product of two values below 2^31 folds to below
// 2m, so one conditional subtract finishes it).  The fp32-decided rejection
// loops below test only the even draws of a try (the canonical draws'
// leading terms), so a try jumps two draws at a time and the odd draws are
// formed only where a try needs its exact fp64 point (T +0.7 %, C3 +1.3 %).
constexpr uint32_t kMrA = 48271u;
constexpr uint32_t kMrA2 = 182605794u;  // 48271^2 mod (2^31 - 1)
RTW_D uint32_t mr_jump(uint32_t s, uint32_t c) {
    const uint64_t p = (uint64_t)s * c;
    uint32_t r = (uint32_t)(p & 0x7fffffffu) + (uint32_t)(p >> 31);
    if (r >= 0x7fffffffu) r -= 0x7fffffffu;
    return r;
}

// libstdc++ generate_canonical<double,53>(minstd_rand): two raw draws.
RTW_D double canon_raw(uint32_t r1, uint32_t r2) {
    const double e1 = (double)(r1 - 1u);
    const double e2 = (double)(r2 - 1u);
    double sum = 0.0 + e1 * 1.0;
    sum = sum + e2 * kCanonR;
    // sum in [0, 2^62]: one Markstein step (rtw_div.h div_canon)
    const double r = div_canon(sum);
    // libstdc++'s clamp (as one v_min_f64: T -0.2 %, its constant holds an
    // SGPR pair through the loop)
    return r >= 1.0 ? kOneMinusUlp : r;
}
RTW_D double canon(uint32_t& s) {
    const uint32_t r1 = mr_next(s);
    const uint32_t r2 = mr_next(s);
    return canon_raw(r1, r2);
}
RTW_D double rnd01(uint32_t& s) { return canon(s) * (1.0 - 0.0) + 0.0; }
RTW_D double rnd(uint32_t& s, double a, double b) { return a + (b - a) * rnd01(s); }  // utility.h:14-20

RTW_D uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// rtw_path_seed (include/rtw_gpu.h); seed_mix = splitmix64(seed)
RTW_D uint32_t path_seed(uint64_t seed_mix, uint32_t pixel, uint32_t s) {
    const uint64_t k = ((uint64_t)s << 32) ^ (uint64_t)pixel;
    return (uint32_t)(1u + splitmix64(seed_mix ^ k) % 2147483646ull);
}

RTW_D int random_int(uint32_t& s, int a, int b) {  // utility.h:22-25
    const int span = (int)((b - a + 1) * rnd01(s));
    return a + ((b - a) < span ? (b - a) : span);
}

// utility.h:27-35 — vec3(U, U, U) is built right to left by g++: z, y, x.
// The rejection loop decided in fp32: a wave runs its
// longest lane's number of tries (~4 for the metal lanes of a random_balls
// wave, ~6 for the isotropic lanes of a Book-2 wave), so each try draws its
// six raw values and tests 2 (e2 / R) - 1 -- the canonical draw's leading
// term, within 2^-22.4 of it -- in fp32: |d32 - d| < 2^-18 for d = |p|^2, so
// d32 < 1 - 2^-14 accepts and d32 >= 1 + 2^-14 rejects exactly as the fp64
// test would, and a try in between takes the fp64 test.  The accepted try's
// p is then formed from its raw draws in fp64, once: the same draws, the
// same value, the same engine state as the reference's loop.
RTW_D d3 random_in_unit_sphere(uint32_t& s) {
    constexpr float k2Rf = (float)(2.0 / kCanonR);  // 2 / R rounded
    auto lead = [&](uint32_t raw) { return __builtin_fmaf((float)(raw - 1u), k2Rf, -1.0f); };
    auto exact = [&](uint32_t z1, uint32_t z2, uint32_t y1, uint32_t y2, uint32_t x1, uint32_t x2) {
        const double z = canon_raw(z1, z2) * (1.0 - 0.0) + 0.0;
        const double y = canon_raw(y1, y2) * (1.0 - 0.0) + 0.0;
        const double x = canon_raw(x1, x2) * (1.0 - 0.0) + 0.0;
        return d3{x, y, z} * 2.0 - d3{1.0, 1.0, 1.0};
    };
    uint32_t z1, z2, y1, y2, x1, x2;
    // a try is draws 1..6 from s0: the even ones by two-step jumps, the odd
    // ones (z1 = a s0, y1 = a z2, x1 = a y2) only where the point is formed
    uint32_t s0;
    for (;;) {
        s0 = s;
        z2 = mr_jump(s0, kMrA2), y2 = mr_jump(z2, kMrA2), x2 = mr_jump(y2, kMrA2);
        s = x2;
        const float px = lead(x2), py = lead(y2), pz = lead(z2);
        const float d32 = __builtin_fmaf(px, px, __builtin_fmaf(py, py, pz * pz));
        if (d32 < 1.0f - 0x1p-14f) break;
        if (!(d32 < 1.0f + 0x1p-14f)) continue;
        z1 = mr_jump(s0, kMrA), y1 = mr_jump(z2, kMrA), x1 = mr_jump(y2, kMrA);
        const d3 q = exact(z1, z2, y1, y2, x1, x2);
        if (dot(q, q) < 1.0) break;
    }
    z1 = mr_jump(s0, kMrA), y1 = mr_jump(z2, kMrA), x1 = mr_jump(y2, kMrA);
    return exact(z1, z2, y1, y2, x1, x2);
}

RTW_D d3 random_cosine_direction(uint32_t& s) {  // utility.h:54-67
    const double r1 = rnd01(s);
    const double r2 = rnd01(s);
    const double z = RTW_SQRT_POS(1 - r2);  // r2 <= 1 - 2^-53: 1 - r2 >= 2^-53
    const double phi = kTwoPi * r1;
    const double sq = RTW_SQRT(r2);
    double sp, cp;
    sincos_azimuth(phi, sp, cp);
    return d3{cp * sq, sp * sq, z};
}

// ------------------------------------------------------------------ onb
struct onb {
    d3 u, v, w;
};
// Vectors whose length is known to be about 1 are normalised
// with rtw_div.h's bare sqrt sequence (sqrt_core: the compiler's sqrt for x
// >= 2^-766, without its range and class handling -- no branch, no vote):
// the second axis of every frame (cross(w, a) with w unit and |w.x| <= 0.9
// when a = x, so |.|^2 >= 0.19 -- or >= 0.81), and frame_w of a lambertian
// surface's normal (hit_record: (p - c) / r of a sphere, an axis normal,
// rotated orthogonally; surf_frame::unit, a constant where shade_core builds
// the frame -- a per-lane choice of the two forms made the frame a scratch
// object).  A non-finite vector gives NaN either way.  T +0.25 %, C3 +0.25 %
// (profiles/r05/ab_r5r_sqrt_unit.log).
RTW_HD d3 normalize_unit(d3 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return v / sqrt_core(len2(v));
#else
    return normalize_b(v);
#endif
}
RTW_HD onb onb_from_w(d3 n) {  // onb.h:32-38
    onb b;
    b.w = normalize_b(n);
    const d3 a = (fabs(b.w.x) > 0.9) ? d3{0, 1, 0} : d3{1, 0, 0};
    b.v = normalize_unit(cross(b.w, a));
    b.u = cross(b.w, b.v);
    return b;
}
RTW_HD d3 local(const onb& b, d3 a) { return b.u * a.x + b.v * a.y + b.w * a.z; }  // onb.h:21-24

// ------------------------------------------------------------------ scene
// entry >= 0: one world-list entry; WORLD_RUN_PLAIN: consecutive plain
// entries (one untransformed group each) scanned as their contiguous prims;
// WORLD_RUN_YSPHERES: the same, all spheres for ysphere_scan.
enum : int { WORLD_RUN_PLAIN = -1, WORLD_RUN_YSPHERES = -2 };
struct bvh_node32;
// Device BVH node format (rtw_scene_upload writes it, node_at reads it):
// 32-B nodes with fp32 bounds.  (16-B fp16 nodes, twice the nodes per LDS
// packet, measured C5 -6 %, C3 -9 %: the packet already holds every node of
// C3 and C5 and the fp16 decode costs more; EXPERIMENTS.md.)
using node_store = bvh_node32;
struct world_run {
    int32_t entry, first_prim, n_prims, movers;  // movers: the prims hold DP_MOVING_COMMON*
};
// Device form of a world-list entry (rtw_entry, built by the upload): the
// header alone, its transform ops in one pool (scene::ops) -- 48 B instead of
// the ABI's 312, so a scene's entries stay small in the LDS shading prefix
// whatever RTW_MAX_OPS is, and op chains have no length limit here.
struct dev_entry {
    int32_t kind, first_prim, n_prims, n_ops;
    int32_t first_op;     // ops [first_op, first_op + n_ops) of scene::ops, outermost first
    int32_t phase_material, bvh_root;
    int32_t n_outer_ops;  // MEDIUM: ops enclosing the medium (rtw_entry::n_outer_ops)
    int32_t movers;       // the group holds DP_MOVING_COMMON* spheres
    int32_t pad;
    double neg_inv_density;  // MEDIUM: -(1 / density) (hittable.h:451), IEEE on the host at upload
};
struct dev_op {
    int32_t type, pad;
    double p[3];
};
// The media walk (scene::media) lists entry indices in visit order.
// (A boundary cache for a medium's second visit measured C5 -8 %, and fused
// walks of two group trees -11 %: EXPERIMENTS.md.)
constexpr int32_t kVisitEntry = (1 << 20) - 1;
struct scene {
    const rtw_prim* prims;
    const dev_entry* entries;
    const dev_op* ops;
    const rtw_material* materials;
    const rtw_texture* textures;
    const rtw_light* lights;
    const node_store* nodes;  // device BVH nodes (rtw_scene_upload)
    const int32_t* items;
    const double* ranvec;
    const int32_t* perm;
    const double* prim_onb;  // per rect prim: onb of its world normal (u, v, w), host-built
    const double* mat_aux;   // per material: 1/ref_idx, schlick's r0^2 (host-built, same expressions)
    double light_weight;     // 1.0 / n_lights (hittable_list.h:45), host-computed
    int32_t n_entries, n_lights, world_bvh_root, render_type, background;
    int32_t has_media;
    int32_t n_media;
    const int32_t* media;  // the media walk: entry indices in visit order (upload_scene)
    // World list as runs (world_closest)
    const world_run* runs;
    int32_t n_runs;
    int32_t mv_common;     // some prims are DP_MOVING_COMMON*
    double mv_t0, mv_den;  // their time0 and time1 - time0
    int32_t fast_div;      // shared-divisor sphere roots allowed in world walks (ysphere_scan)
    double bvh_bound;      // largest |coordinate| of any device BVH node (make_slab_ray)
    // ysphere_scan's fp32 prefilter: per prim {cx, cy, cz, dy, r^2, 0, 0, 0}
    // (r^2 = +inf: never filtered), and the largest |cx|, |cy|, |dy|, |cz|
    // and r^2 of the filtered spheres
    const float* ysph;
    float ysb_cx, ysb_cy, ysb_dy, ysb_cz, ysb_r2;
    // box items' planes: per box item a 64-B record {x0, x1, y0, y1, z0, z1,
    // first rect (int)}, the items then RTW_ITEM_BOX | record
    // (rtw_scene_upload, when every box's six rects match them; nullptr: the
    // items are RTW_ITEM_BOX | first rect and the walks read the rects)
    const double* boxes;
    // BVH node packets staged in LDS: the upload numbers the nodes of every
    // BVH breadth-first from all roots together, so nodes [0, n_lnodes) are
    // the top levels of every tree; the persistent BVH kernels copy them to
    // LDS (lnodes) once per workgroup (n_lnodes = 0: all from memory)
    const node_store* lnodes;
    int32_t n_lnodes;
    int32_t n_nodes;  // device BVH nodes in all
};

// Scene features a traversal kernel is specialised for.
// F_YSPH: the world list holds y-sphere runs (ysphere_scan); without it such
// runs take group_scan (same results), which keeps the prefilter's code and
// registers out of the kernels of other scenes (Cornell).
// F_STATIC: no moving spheres, so a ray's time is never read (sphere.h:22-25
// is its only reader); the persistent kernels then keep no time per path
// (the camera still draws it: the RNG sequence is the reference's).
// F_LIGHTS: the scene has lights, so every lambertian bounce samples the
// mixture pdf (RayTracingWeekend.cpp:112-132) and the lights-free branch is
// compiled out.
// F_BLACK: black background and colour rendering (RayTracingWeekend.cpp:
// 135-159): a miss emits 0 and the normal-visualisation branch is compiled out.
// F_NOLIGHTS: the scene has no lights, so the mixture-pdf branch of the
// lambertian bounce is compiled out instead.
enum : int { F_MEDIA = 1, F_WBVH = 2, F_GBVH = 4, F_YSPH = 8, F_STATIC = 16, F_LIGHTS = 32, F_BLACK = 64,
             F_NOLIGHTS = 128,
             // every camera ray of the render starts at the camera's origin (a
             // pinhole camera, lens_radius 0, whose origin has no zero
             // coordinate: origin + offset is then exactly origin, camera.h:48)
             F_PIN = 256 };

// Uniform scene reads.  The scene is read-only for a whole launch; reading
// it through the constant address space lets the compiler use scalar loads
// (s_load, one per wave, through the scalar cache) wherever the index is
// wave-uniform — the linear scans of the world list and of groups.
template <typename T>
using cptr = const __attribute__((address_space(4))) T*;
template <typename T>
RTW_D T ld(const T* p) { return *(cptr<T>)p; }

RTW_D rtw_prim uprim(const rtw_prim* P, int i) {
    rtw_prim q;
    q.type = ld(&P[i].type);
    q.material = ld(&P[i].material);
    q.flip = ld(&P[i].flip);
    q.entry = ld(&P[i].entry);
#pragma unroll
    for (int k = 0; k < 10; ++k) q.p[k] = ld(&P[i].p[k]);
    return q;
}

// Loads that are scalar (s_load through the constant address space) when
// U, i.e. when the index is wave-uniform, else ordinary per-lane loads.
template <bool U, typename T>
RTW_D T rd(const T* p) {
    if constexpr (U) return ld(p);
    else return *p;
}

// A world-list entry as the kernels use it: the header in registers; op
// types and parameters (up to 4 ops x 3 doubles) read where an op is applied,
// not all up front.
struct entry_v {
    const dev_entry* p;
    const dev_op* ops;  // its op chain
    int kind, first_prim, n_prims, n_ops, bvh_root;
    bool movers;  // the group holds DP_MOVING_COMMON* spheres (dev_entry::movers)
};
template <bool U>
RTW_D entry_v view_entry(const scene& S, int i) {
    const dev_entry* E = S.entries;
    entry_v e;
    e.p = E + i;
    e.ops = S.ops + rd<U>(&E[i].first_op);
    e.kind = rd<U>(&E[i].kind);
    e.first_prim = rd<U>(&E[i].first_prim);
    e.n_prims = rd<U>(&E[i].n_prims);
    e.n_ops = rd<U>(&E[i].n_ops);
    e.bvh_root = rd<U>(&E[i].bvh_root);
    e.movers = rd<U>(&E[i].movers) != 0;
    return e;
}

// Device primitive types.  rtw_scene_upload rewrites the sphere records it
// copies to the GPU (the caller's rtw_scene_desc is untouched), each value
// with the reference's own expression, evaluated once instead of per test:
//   spheres:         p[9] = radius * radius                  (sphere.h:52)
//   moving spheres:  p[4..6] = center1 - center0, p[8] = time1 - time0
//                                                             (sphere.h:24)
// and moving spheres whose (time0, time1) equal the scene's common interval
// (scene::mv_t0 / mv_den) get DP_MOVING_COMMON: their fraction
// (time - time0) / (time1 - time0) is computed once per walk (motion_frac)
// instead of once per sphere.  DP_MOVING_COMMON_Y: in addition
// center1 - center0 = (0, dy, 0) and center0.x, center0.z are nonzero, so
// center0.x + 0 * f == center0.x exactly (f is finite: upload checks the
// interval) and only y moves.
enum : int { DP_MOVING_COMMON = 5, DP_MOVING_COMMON_Y = 6 };
RTW_HD bool is_sphere(int type) { return type < RTW_PRIM_RECT_XY || type > RTW_PRIM_RECT_YZ; }

// The moving-sphere fraction (time - time0) / (time1 - time0) of the
// scene's common interval, computed once per walk over prims that hold
// DP_MOVING_COMMON* spheres (world_run::movers, dev_entry::movers; the
// walk's transforms keep the ray's time), else not at all.
RTW_D double motion_frac(const scene& S, double time, bool movers) {
    return movers ? (time - S.mv_t0) / S.mv_den : 0.0;
}

// sphere.h:22-25: center0 + ((time - time0) / (time1 - time0)) * (center1 - center0),
// fc = motion_frac(...)
RTW_D d3 sphere_center(const rtw_prim& s, double time, double fc) {
    const d3 c0 = ld3(s.p);
    if (s.type == RTW_PRIM_SPHERE) return c0;
    if (s.type == DP_MOVING_COMMON_Y) return d3{c0.x, c0.y + s.p[5] * fc, c0.z};
    const double f = s.type == DP_MOVING_COMMON ? fc : (time - s.p[7]) / s.p[8];
    return c0 + ld3(s.p + 4) * f;
}

// sphere.h:46-81: near root if in (t_min, t_max), else far root.
RTW_D bool sphere_t(const rtw_prim& s, const ray& r, double t_min, double t_max, double& t_out, double fc) {
    const d3 cc = sphere_center(s, r.t, fc);
    const d3 oc = r.o - cc;
    const double a = dot(r.d, r.d);
    const double b = dot(oc, r.d);
    const double c = dot(oc, oc) - s.p[9];  // radius * radius
    const double disc = b * b - a * c;
    if (disc > 0) {
        const double sq = RTW_SQRT(disc);
        double temp = (-b - sq) / a;
        if (temp < t_max && temp > t_min) {
            t_out = temp;
            return true;
        }
        temp = (-b + sq) / a;
        if (temp < t_max && temp > t_min) {
            t_out = temp;
            return true;
        }
    }
    return false;
}

// hittable.h:149-165 / 184-200 / 241-257: plane axis K, in-plane axes A, B
// (XY: K=z A=x B=y; XZ: K=y A=x B=z; YZ: K=x A=y B=z).
template <int K, int A, int B>
RTW_D bool rect_axis_t(const rtw_prim& q, const ray& r, double t0, double t1, double& t_out) {
    const double ok = K == 0 ? r.o.x : (K == 1 ? r.o.y : r.o.z);
    const double od = K == 0 ? r.d.x : (K == 1 ? r.d.y : r.d.z);
    const double t = (q.p[4] - ok) / od;
    if (t < t0 || t > t1) return false;
    const double a = (A == 0 ? r.o.x : r.o.y) + t * (A == 0 ? r.d.x : r.d.y);
    const double b = (B == 1 ? r.o.y : r.o.z) + t * (B == 1 ? r.d.y : r.d.z);
    if (a < q.p[0] || a > q.p[1] || b < q.p[2] || b > q.p[3]) return false;
    t_out = t;
    return true;
}

RTW_D bool rect_t(const rtw_prim& q, const ray& r, double t0, double t1, double& t_out) {
    if (q.type == RTW_PRIM_RECT_XY) return rect_axis_t<2, 0, 1>(q, r, t0, t1, t_out);
    if (q.type == RTW_PRIM_RECT_XZ) return rect_axis_t<1, 0, 2>(q, r, t0, t1, t_out);
    return rect_axis_t<0, 1, 2>(q, r, t0, t1, t_out);
}

RTW_D bool prim_t(const rtw_prim& q, const ray& r, double t0, double t1, double& t_out, double fc) {
    return is_sphere(q.type) ? sphere_t(q, r, t0, t1, t_out, fc) : rect_t(q, r, t0, t1, t_out);
}

RTW_HD d3 rect_normal(int type) {
    return type == RTW_PRIM_RECT_XY ? d3{0, 0, 1} : (type == RTW_PRIM_RECT_XZ ? d3{0, 1, 0} : d3{1, 0, 0});
}

// translate::hit hittable.h:299-311, rotate_y::hit :373-404 (ray inward)
template <bool U>
RTW_D void op_ray_in(const dev_op* O, int k, ray& r) {
    const int op = rd<U>(&O[k].type);
    if (op == RTW_OP_TRANSLATE) {
        r.o = r.o - d3{rd<U>(&O[k].p[0]), rd<U>(&O[k].p[1]), rd<U>(&O[k].p[2])};
    } else if (op == RTW_OP_ROTATE_Y) {
        const double s = rd<U>(&O[k].p[0]), c = rd<U>(&O[k].p[1]);
        const d3 o = r.o, d = r.d;
        r.o.x = c * o.x - s * o.z;
        r.o.z = s * o.x + c * o.z;
        r.d.x = c * d.x - s * d.z;
        r.d.z = s * d.x + c * d.z;
    }
}
// ... and the record outward (p, normal), innermost op first
template <bool U>
RTW_D void op_rec_out(const dev_op* O, int k, d3& p, d3& n) {
    const int op = rd<U>(&O[k].type);
    if (op == RTW_OP_TRANSLATE) {
        p = p + d3{rd<U>(&O[k].p[0]), rd<U>(&O[k].p[1]), rd<U>(&O[k].p[2])};
    } else if (op == RTW_OP_ROTATE_Y) {
        const double s = rd<U>(&O[k].p[0]), c = rd<U>(&O[k].p[1]);
        const d3 p0 = p, n0 = n;
        p.x = c * p0.x + s * p0.z;
        p.z = -s * p0.x + c * p0.z;
        n.x = c * n0.x + s * n0.z;
        n.z = -s * n0.x + c * n0.z;
    } else if (op == RTW_OP_FLIP) {
        n = -n;
    }
}

// Ops [k0, k1) of an entry's chain on the way in, and [0, k1) on the way
// out.  The first kOpsUnrolled are statically indexed (unrolled, each behind
// its count test); longer chains (nested transforms) continue in a loop.
#ifndef RTW_OPS_UNROLLED
#define RTW_OPS_UNROLLED 4
#endif
constexpr int kOpsUnrolled = RTW_OPS_UNROLLED;
template <bool U>
RTW_D ray ops_in(const entry_v& e, ray r, int k0, int k1) {
#pragma unroll
    for (int k = 0; k < kOpsUnrolled; ++k)
        if (k >= k0 && k < k1) op_ray_in<U>(e.ops, k, r);
    for (int k = kOpsUnrolled; k < k1; ++k)
        if (k >= k0) op_ray_in<U>(e.ops, k, r);
    return r;
}
template <bool U>
RTW_D void ops_out(const entry_v& e, int k1, d3& p, d3& n) {
    for (int k = k1 - 1; k >= kOpsUnrolled; --k) op_rec_out<U>(e.ops, k, p, n);
#pragma unroll
    for (int k = kOpsUnrolled - 1; k >= 0; --k)
        if (k < k1) op_rec_out<U>(e.ops, k, p, n);
}
template <bool U>
RTW_D ray entry_local_ray(const entry_v& e, ray r) {
    return ops_in<U>(e, r, 0, e.n_ops);
}
template <bool U>
RTW_D void entry_rec_out(const entry_v& e, d3& p, d3& n) {
    ops_out<U>(e, e.n_ops, p, n);
}

// ------------------------------------------------------------------ traversal
// Candidate comparison that reproduces the list-order winner of
// hittable_list::hit for a BVH (any visiting order): a candidate at the same
// t as the best wins iff list order would have let it overwrite: a rect
// (accepts t == t_max) beats every sphere and lower-indexed rects; among
// spheres (strict t < t_max) the lowest index is kept.
RTW_D bool better(double t, int idx, bool rectlike, double bt, int bidx, bool brect, bool has) {
    if (t < bt) return true;
    if (t != bt) return false;
    if (rectlike) return !has || !brect || idx > bidx;
    return has && !brect && idx < bidx;
}

struct hit_state {
    double t;     // closest so far (the t_max of the next test)
    int32_t prim; // winner, -1 none, <= -2 medium entry -(2+e)
    bool rect;    // winner accepts equal t (for BVH tie order)
};

// Shared-divisor rect tests (rtw_div.h rcp_hw / div_hw): every rect test of
// a walk divides by one of the ray's three direction components
// (t = (k - o.K) / d.K, hittable.h:149-165), so a scan computes the three
// reciprocals once and each test pays a multiply and two fma instead of a
// full division -- bit-identical to the division when |d.K| is in
// [2^-200, 2^200] and the numerator in [2^-800, 2^100]:
//  * divisor: checked per walk and axis (false for 0, NaN, inf);
//  * numerator above: scene::fast_div bounds every rect coordinate by 2^40
//    and the walk checks |o| <= 2^40, so |k - o.K| <= 2^41;
//  * numerator below 2^-800: both quotients are below 2^-599 and rejected
//    alike by t < t_min -- so only walks with t_min >= 0.001 (the world
//    walks; not the media boundary probes) use it.
// Lanes outside the ranges divide exactly.
struct rect_rcp {
    double y[3];
    bool ok[3];
};
RTW_D rect_rcp make_rect_rcp(const scene& S, const ray& r) {
    constexpr double kB = 0x1p40;
    const bool base = S.fast_div != 0 && __builtin_fabs(r.o.x) <= kB && __builtin_fabs(r.o.y) <= kB &&
                      __builtin_fabs(r.o.z) <= kB;
    rect_rcp q;
    const double d[3] = {r.d.x, r.d.y, r.d.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        q.y[k] = rcp_hw(d[k]);
        q.ok[k] = base && div_hw_ok_b(d[k]);
    }
    return q;
}
// rect_axis_t with the walk's shared reciprocal of d.K.  BL (the world list
// walk's rects): the same comparisons without the early
// return -- a and b formed for every lane, one branch level less of
// exec-mask bookkeeping on the scalar unit per rect.  Measured (1 MI355X,
// A/B, profiles/r05/ab_r5u_rect_branchless.log; bit-identical images): T
// 4 811 vs 4 747 (+1.3 %); in the BVH leaves' box faces (mostly missed, the
// early return skips their a, b) C5 -1.2 %, so those keep it.
template <int K, int A, int B, bool BL = false, class Q = rtw_prim>
RTW_D bool rect_axis_rcp(const Q& q, const ray& r, const rect_rcp& rr, double t0, double t1,
                         double& t_out) {
    const double ok = K == 0 ? r.o.x : (K == 1 ? r.o.y : r.o.z);
    const double od = K == 0 ? r.d.x : (K == 1 ? r.d.y : r.d.z);
    const double num = q.p[4] - ok;
    double t = div_hw(num, od, rr.y[K]);
    if (__builtin_expect(!rr.ok[K], 0)) {
        asm volatile("");  // keeps the exact division behind the branch
        t = num / od;
    }
    if constexpr (BL) {
        const double a = (A == 0 ? r.o.x : r.o.y) + t * (A == 0 ? r.d.x : r.d.y);
        const double b = (B == 1 ? r.o.y : r.o.z) + t * (B == 1 ? r.d.y : r.d.z);
        const bool hit = !(t < t0 || t > t1) && !(a < q.p[0] || a > q.p[1] || b < q.p[2] || b > q.p[3]);
        t_out = t;
        return hit;
    }
    if (t < t0 || t > t1) return false;
    const double a = (A == 0 ? r.o.x : r.o.y) + t * (A == 0 ? r.d.x : r.d.y);
    const double b = (B == 1 ? r.o.y : r.o.z) + t * (B == 1 ? r.d.y : r.d.z);
    if (a < q.p[0] || a > q.p[1] || b < q.p[2] || b > q.p[3]) return false;
    t_out = t;
    return true;
}
RTW_D bool rect_t_rcp(const rtw_prim& q, const ray& r, const rect_rcp& rr, double t0, double t1, double& t_out) {
    constexpr bool BL = true;  // (the world list walk's rects)
    if (q.type == RTW_PRIM_RECT_XY) return rect_axis_rcp<2, 0, 1, BL>(q, r, rr, t0, t1, t_out);
    if (q.type == RTW_PRIM_RECT_XZ) return rect_axis_rcp<1, 0, 2, BL>(q, r, rr, t0, t1, t_out);
    return rect_axis_rcp<0, 1, 2, BL>(q, r, rr, t0, t1, t_out);
}


// Shared-divisor quotients (rtw_div.h rcp_hw / div_hw) for the sphere roots
// of a world walk: every root is (-b -+ sqrt(disc)) / dot(d, d), so a scan
// over many spheres computes 1 / dot(d, d) once and each root pays one
// multiply and two fma instead of a full division.  Bit-identical to a / b
// when the divisor lies in [2^-200, 2^200] and the numerator in
// [2^-800, 2^100]:
//  * divisor: checked per walk (false for NaN too);
//  * numerators: bounded above because the scene is (upload sets
//    scene::fast_div only when every prim coordinate and radius is within
//    2^40 and every mover shares the common interval) and the walk's ray is
//    (|o|, |d| <= 2^40, |fc| <= 2^8, checked here), so |-b -+ sqrt(disc)| < 2^95;
//  * a numerator below 2^-800 (a grazing root) gives quotients below 2^-599
//    by either route, rejected alike by t > t_min = 0.001.
// Lanes that fail the check divide exactly (the branch is skipped when no
// lane of the wave takes it).  Measured: +3 % random_balls flat (485
// spheres per walk).  The same sharing for rect tests (1 / d.x, 1 / d.y,
// 1 / d.z), for scans holding one sphere and for BVH walks cost more in
// registers than the divisions it saved (Cornell -0.6 ... -2.5 %, random_balls
// BVH -6 %), so those divide directly.
RTW_D bool walk_ray_ok(const scene& S, const ray& r, double fc) {
    constexpr double kB = 0x1p40;
    return S.fast_div != 0 && __builtin_fabs(r.o.x) <= kB && __builtin_fabs(r.o.y) <= kB &&
           __builtin_fabs(r.o.z) <= kB && __builtin_fabs(r.d.x) <= kB && __builtin_fabs(r.d.y) <= kB &&
           __builtin_fabs(r.d.z) <= kB && __builtin_fabs(fc) <= 0x1p8;
}
// num / den via the shared reciprocal y, exact a / b on lanes without `ok`
RTW_D double walk_quot(double num, double den, double y, bool ok) {
    double q = div_hw(num, den, y);
    if (__builtin_expect(!ok, 0)) {
        asm volatile("");  // keeps the exact division behind the branch
        q = num / den;
    }
    return q;
}

// Linear closest hit over prims [first, first+n) of one group, in list order
// (t range (t_min, closest]) with the reference's own comparisons; the
// primitive data are wave-uniform scalar loads.
// (STATIC: the scene has no moving spheres, centres are center0.  WORLD: a
// world walk, t_min = 0.001: rect tests share the direction's reciprocals.)
template <bool STATIC = false, bool WORLD = false>
RTW_D void group_scan(const scene& S, int first, int n, const ray& r, double t_min, hit_state& h, bool movers) {
    const double fc = STATIC ? 0.0 : motion_frac(S, r.t, movers);
    const double a = dot(r.d, r.d);  // sphere.h:50, the same for every sphere
    constexpr bool kRcp = WORLD;
    rect_rcp rr;
    if (kRcp) rr = make_rect_rcp(S, r);
    for (int i = 0; i < n; ++i) {
        const rtw_prim q = uprim(S.prims, first + i);
        if (is_sphere(q.type)) {
            // sphere_t inlined so the winner is written where it is found
            // (no per-prim merge of the running best on the common miss path)
            const d3 oc = r.o - (STATIC ? ld3(q.p) : sphere_center(q, r.t, fc));
            const double b = dot(oc, r.d);
            const double c = dot(oc, oc) - q.p[9];
            const double disc = b * b - a * c;
            if (disc > 0) {
                const double sq = RTW_SQRT(disc);
                double temp = (-b - sq) / a;
                bool ok = temp < h.t && temp > t_min;
                if (!ok) {
                    temp = (-b + sq) / a;
                    ok = temp < h.t && temp > t_min;
                }
                if (ok) {
                    h.t = temp;
                    h.prim = first + i;
                    h.rect = false;
                }
            }
        } else {
            double t;
            if (kRcp ? rect_t_rcp(q, r, rr, t_min, h.t, t) : rect_t(q, r, t_min, h.t, t)) {
                h.t = t;
                h.prim = first + i;
                h.rect = true;
            }
        }
    }
}


// group_scan for a run of spheres that all move along y only (or not at
// all): centre (c0.x, c0.y + p[5] * fc, c0.z).  The upload forms such runs
// (WORLD_RUN_YSPHERES) from DP_MOVING_COMMON_Y spheres and static spheres
// with c0.y != 0, whose p[5] it sets to 0 (c0.y + 0 * fc == c0.y exactly,
// fc finite), so one branch-free body serves the whole run: the Book-1
// random_balls list.  Same arithmetic as sphere.h:46-81 per sphere.
#ifndef RTW_YS_AHEAD
#define RTW_YS_AHEAD 4
#endif
#ifndef RTW_YS_GROUP
#define RTW_YS_GROUP 4  // packed pairs filtered together per iteration (2: -1.7 %, 3: -2.5 %)
#endif
constexpr int kYsGroup = RTW_YS_GROUP;
constexpr int kYsAhead = RTW_YS_AHEAD;  // fp32 records in flight ahead of the filtered one
RTW_D void ysphere_scan(const scene& S, int first, int n, const ray& r, double t_min, hit_state& h, double fc) {
    const double a = dot(r.d, r.d);
    const bool oka = walk_ray_ok(S, r, fc) && div_hw_ok_b(a);  // world walk: t_min = 0.001
    const double ya = rcp_hw(a);
    // fp32 prefilter (twice the fp64 rate): disc32 below -E proves the fp64
    // disc <= 0 for that lane (no root, nothing to test), so a sphere no lane
    // of the wave can reach skips the fp64 test altogether.  Each fp32 op is
    // off by at most u = 2^-24 relative; carried through oc, b, q, c = q - r^2
    // and disc = b^2 - a c (with b^2 <= a Q, Cauchy-Schwarz) that gives
    // |disc32 - disc64| <= u a (37 Q + 9 r^2), Q = sum_i (|o_i| + |c_i|)^2;
    // E = 2^-16 a (Q + r^2) bounds it with |c_i| and r^2 at their scene
    // maxima over the filtered spheres (host, rounded up) -- about 14 times
    // over.  NaN anywhere makes the filter pass the sphere on (!(x <= -E)).
    const float oxf = (float)r.o.x, oyf = (float)r.o.y, ozf = (float)r.o.z;
    const float dxf = (float)r.d.x, dyf = (float)r.d.y, dzf = (float)r.d.z, fcf = (float)fc;
    const float af = __builtin_fmaf(dxf, dxf, __builtin_fmaf(dyf, dyf, dzf * dzf));
    const float R0 = __builtin_fabsf(oxf) + S.ysb_cx;
    const float R1 = __builtin_fabsf(oyf) + __builtin_fmaf(S.ysb_dy, __builtin_fabsf(fcf), S.ysb_cy);
    const float R2 = __builtin_fabsf(ozf) + S.ysb_cz;
    const float E = 0x1p-16f * af * (R0 * R0 + R1 * R1 + R2 * R2 + S.ysb_r2) + 0x1p-60f;  // + denormal slack
    // software-pipelined scalar loads of the fp32 records: the records of
    // the next kYsAhead spheres are in flight while sphere i is filtered (a
    // ring of registers, the loop unrolled by its length)
    // the reference's test, sphere.h:46-81 (exact fp64), for a sphere the
    // prefilter could not exclude
    auto exact = [&](int i) {
        const double* p = S.prims[first + i].p;
        const d3 oc{r.o.x - ld(p), r.o.y - (ld(p + 1) + ld(p + 5) * fc), r.o.z - ld(p + 2)};
        const double b = dot(oc, r.d);
        const double c = dot(oc, oc) - ld(p + 9);
        const double disc = b * b - a * c;
        if (disc > 0) {
            const double sq = RTW_SQRT(disc);
            double temp = walk_quot(-b - sq, a, ya, oka);
            bool ok = temp < h.t && temp > t_min;
            if (!ok) {
                temp = walk_quot(-b + sq, a, ya, oka);
                ok = temp < h.t && temp > t_min;
            }
            if (ok) {
                h.t = temp;
                h.prim = first + i;
                h.rect = false;
            }
        }
    };
    // Two spheres per instruction: gfx950's packed fp32 VALU ops (v_pk_fma /
    // v_pk_mul / v_pk_add_f32) run the filter of spheres 2p and 2p + 1
    // side by side -- the same IEEE fp32 operations per sphere as the scalar
    // form, so the bound above holds unchanged.  The upload interleaves the
    // records of a run pairwise ({cx, cx', cy, cy', cz, cz', dy, dy', rr,
    // rr'}), so one scalar load brings each pair's operands in adjacent
    // registers.  The exact tests still run in list order (2p, then 2p + 1).
    // A run of odd length ends with one sphere in the plain record, filtered
    // alone.  (Runs hold at least two spheres: np >= 1.)
    typedef float f2 __attribute__((ext_vector_type(2)));
    struct ysrec2 {
        f2 cx, cy, cz, dy, rr;
    };
    const int np = n >> 1;
    // (each load is the run's base plus a constant offset: no index clamp,
    // every pair read lies inside the run)
    const f2* const g0 = reinterpret_cast<const f2*>(S.ysph + 8 * (size_t)first);
    auto load2 = [&](int p) {
        const f2* g = g0 + 8 * p;
        return ysrec2{ld(g), ld(g + 1), ld(g + 2), ld(g + 3), ld(g + 4)};
    };
    const f2 ox2 = oxf, oy2 = oyf, oz2 = ozf, dx2 = dxf, dy2 = dyf, dz2 = dzf, fc2 = fcf, af2 = af;
    // ocy as (oy - cy) - dy fc: each instruction then reads one scalar pair
    // (one SGPR operand per VALU instruction), where oy - (dy fc + cy)
    // needed cy copied to vector registers first; two roundings either way,
    // within the same 2u (|oy| + |cy| + |dy fc|) the bound above allows for
    auto filt = [&](const ysrec2& c) {
        const f2 ocx = ox2 - c.cx, ocz = oz2 - c.cz;
        const f2 ocy = __builtin_elementwise_fma(-c.dy, fc2, oy2 - c.cy);
        const f2 b32 = __builtin_elementwise_fma(ocx, dx2, __builtin_elementwise_fma(ocy, dy2, ocz * dz2));
        const f2 q32 = __builtin_elementwise_fma(ocx, ocx, __builtin_elementwise_fma(ocy, ocy, ocz * ocz));
        return __builtin_elementwise_fma(b32, b32, -(af2 * (q32 - c.rr)));
    };
    // kYsGroup pairs per iteration: all their filters first (independent
    // chains the scheduler interleaves, so no hazard stalls between
    // dependent packed instructions), then the ballots, then the exact tests
    // in list order
    int p = 0;
    for (; p + kYsGroup <= np; p += kYsGroup) {
        f2 d[kYsGroup];
#pragma unroll
        for (int j = 0; j < kYsGroup; ++j) d[j] = filt(load2(p + j));
        unsigned long long m[2 * kYsGroup];
#pragma unroll
        for (int j = 0; j < kYsGroup; ++j) {
            m[2 * j] = __builtin_amdgcn_ballot_w64(!(d[j].x <= -E));
            m[2 * j + 1] = __builtin_amdgcn_ballot_w64(!(d[j].y <= -E));
        }
#pragma unroll
        for (int k = 0; k < 2 * kYsGroup; ++k)
            if (m[k]) exact(2 * p + k);
    }
    for (; p < np; ++p) {
        const f2 d0 = filt(load2(p));
        if (__builtin_amdgcn_ballot_w64(!(d0.x <= -E))) exact(2 * p);
        if (__builtin_amdgcn_ballot_w64(!(d0.y <= -E))) exact(2 * p + 1);
    }
    if (n & 1) {
        const float* g = S.ysph + 8 * (size_t)(first + n - 1);
        const float ocx = oxf - ld(g), ocy = oyf - __builtin_fmaf(ld(g + 3), fcf, ld(g + 1)), ocz = ozf - ld(g + 2);
        const float b32 = __builtin_fmaf(ocx, dxf, __builtin_fmaf(ocy, dyf, ocz * dzf));
        const float q32 = __builtin_fmaf(ocx, ocx, __builtin_fmaf(ocy, ocy, ocz * ocz));
        const float d32 = __builtin_fmaf(b32, b32, -(af * (q32 - ld(g + 4))));
        if (__builtin_amdgcn_ballot_w64(!(d32 <= -E))) exact(n - 1);
    }
}

// Tie-exact test of prim `pi` against the running best, valid for ANY
// visiting order (BVH): same acceptance ranges as the reference tests, ties
// arbitrated by better().  A sphere is probed with an open upper bound so an
// exact tie reaches the arbiter; its root choice is unchanged (if the near root
// lies beyond h.t so does the far one).
// (Shared-reciprocal rect tests, as in group_scan's world walks, measured
// −0.8 % C3 / −0.6 % C5 here: not used.)
RTW_D void arbitrate(const scene& S, int pi, const ray& r, double t_min, hit_state& h, double fc) {
    const rtw_prim& q = S.prims[pi];  // fields read where the test uses them
    const bool rl = !is_sphere(q.type);
    double t;
    if (rl) {
        if (!rect_t(q, r, t_min, h.t, t)) return;
    } else {
        if (!sphere_t(q, r, t_min, kDblMax, t, fc) || t > h.t) return;
    }
    if (better(t, pi, rl, h.t, h.prim, h.rect, h.prim != -1)) {
        h.t = t;
        h.prim = pi;
        h.rect = rl;
    }
}

// A box item of a group BVH (RTW_ITEM_BOX): its six rects in the box's list
// order (hittable_list.h:65-114: +z, -z, +y, -y, +x, -x), each with the
// reference's own test and better()'s tie rule -- exactly six arbitrate
// calls, with each rect's plane axis known instead of read from its type.
// A box's six rect tests divide by only three values, d.x, d.y and d.z
// (each face pair shares its plane axis), so a box computes the three
// reciprocals once (rtw_div.h rcp_hw) and each face's t = (k - o.K) / d.K
// costs a multiply and two fma (div_hw) instead of a full division --
// bit-identical under make_rect_rcp's conditions (scene::fast_div, |o| <=
// 2^40, |d.K| in [2^-200, 2^200]) when t_min >= 0.001 (a numerator below
// 2^-800 then gives quotients that t_min rejects alike); other lanes, and
// boxes probed as a medium's boundary (t_min = -DBL_MAX), divide exactly.
template <int K, int A, int B>
RTW_D void rect_arbitrate_rcp(const scene& S, int pi, const ray& r, const rect_rcp& rr, double t_min, hit_state& h) {
    double t;
    const rtw_prim& q = S.prims[pi];  // fields read where the test uses them
    if (!rect_axis_rcp<K, A, B>(q, r, rr, t_min, h.t, t)) return;
    if (better(t, pi, true, h.t, h.prim, h.rect, h.prim != -1)) {
        h.t = t;
        h.prim = pi;
        h.rect = true;
    }
}
// make_rect_rcp with the quotient rule's t_min condition folded in
RTW_D rect_rcp make_rect_rcp_t(const scene& S, const ray& r, double t_min) {
    rect_rcp rr = make_rect_rcp(S, r);
    const bool tmin_ok = t_min >= kTMin;
#pragma unroll
    for (int k = 0; k < 3; ++k) rr.ok[k] = rr.ok[k] && tmin_ok;
    return rr;
}
struct rect_v {  // a rect's planes as rtw_prim::p holds them (a0, a1, b0, b1, k)
    double p[5];
};
template <int K, int A, int B>
RTW_D void rect_arbitrate_v(const rect_v& q, int pi, const ray& r, const rect_rcp& rr, double t_min, hit_state& h) {
    double t;
    if (!rect_axis_rcp<K, A, B>(q, r, rr, t_min, h.t, t)) return;
    if (better(t, pi, true, h.t, h.prim, h.rect, h.prim != -1)) {
        h.t = t;
        h.prim = pi;
        h.rect = true;
    }
}
RTW_D void box_arbitrate(const scene& S, int idx, const ray& r, double t_min, hit_state& h) {
    const rect_rcp rr = make_rect_rcp_t(S, r, t_min);
    // The six rects from the box's 64-B record (scene::boxes) where the scene
    // has one (a wave-uniform test): one cache line per box where the six
    // 96-B rect records take five.  Measured (1 MI355X, A/B; bit-identical):
    // C5 16-spp slice 702.5 vs 679.1 Msamples/s (+3.4 %), the fp32 kernel's
    // form (rtw_fast.h arbitrate_item) +14 % (profiles/r06/ab_r6v_C5.log,
    // ab_r6u_C5f.log, parity_r6v_boxtab.log, records at the first rect's
    // index); the records packed densely, the 400 ground boxes in 25 KB
    // (12.5 KB in fp32) instead of spread over 150 KB: +0.8 % / +0.4 %
    // (ab_r6dn_*.log, parity_r6dn.log).
    if (S.boxes) {
        const double* b = S.boxes + 8 * (size_t)idx;  // record idx
        const double x0 = b[0], x1 = b[1], y0 = b[2], y1 = b[3], z0 = b[4], z1 = b[5];
        const int first = *reinterpret_cast<const int32_t*>(b + 6);
        rect_arbitrate_v<2, 0, 1>(rect_v{{x0, x1, y0, y1, z1}}, first, r, rr, t_min, h);
        rect_arbitrate_v<2, 0, 1>(rect_v{{x0, x1, y0, y1, z0}}, first + 1, r, rr, t_min, h);
        rect_arbitrate_v<1, 0, 2>(rect_v{{x0, x1, z0, z1, y1}}, first + 2, r, rr, t_min, h);
        rect_arbitrate_v<1, 0, 2>(rect_v{{x0, x1, z0, z1, y0}}, first + 3, r, rr, t_min, h);
        rect_arbitrate_v<0, 1, 2>(rect_v{{y0, y1, z0, z1, x1}}, first + 4, r, rr, t_min, h);
        rect_arbitrate_v<0, 1, 2>(rect_v{{y0, y1, z0, z1, x0}}, first + 5, r, rr, t_min, h);
        return;
    }
    const int first = idx;  // (no table: the item names the first rect)
    rect_arbitrate_rcp<2, 0, 1>(S, first, r, rr, t_min, h);
    rect_arbitrate_rcp<2, 0, 1>(S, first + 1, r, rr, t_min, h);
    rect_arbitrate_rcp<1, 0, 2>(S, first + 2, r, rr, t_min, h);
    rect_arbitrate_rcp<1, 0, 2>(S, first + 3, r, rr, t_min, h);
    rect_arbitrate_rcp<0, 1, 2>(S, first + 4, r, rr, t_min, h);
    rect_arbitrate_rcp<0, 1, 2>(S, first + 5, r, rr, t_min, h);
}
// a group-BVH leaf item: a prim, or a box's six rects
RTW_D void arbitrate_item(const scene& S, int it, const ray& r, double t_min, hit_state& h, double fc) {
    if (it & RTW_ITEM_BOX)
        box_arbitrate(S, it & RTW_ITEM_INDEX, r, t_min, h);
    else
        arbitrate(S, it, r, t_min, h, fc);
}
// arbitrate for a world walk's one-prim leaves with the walk's shared
// 1 / dot(d, d) (walk_quot's rules; t_min = 0.001)
RTW_D void arbitrate_a(const scene& S, int pi, const ray& r, double t_min, hit_state& h, double fc, double ya,
                       bool oka) {
    const rtw_prim& q = S.prims[pi];
    const bool rl = !is_sphere(q.type);
    double t;
    if (rl) {
        if (!rect_t(q, r, t_min, h.t, t)) return;
    } else {
        const d3 oc = r.o - sphere_center(q, r.t, fc);
        const double a = dot(r.d, r.d);
        const double b = dot(oc, r.d);
        const double c = dot(oc, oc) - q.p[9];
        const double disc = b * b - a * c;
        if (!(disc > 0)) return;
        const double sq = RTW_SQRT(disc);
        t = walk_quot(-b - sq, a, ya, oka);
        if (!(t < kDblMax && t > t_min)) {
            t = walk_quot(-b + sq, a, ya, oka);
            if (!(t < kDblMax && t > t_min)) return;
        }
        if (t > h.t) return;
    }
    if (better(t, pi, rl, h.t, h.prim, h.rect, h.prim != -1)) {
        h.t = t;
        h.prim = pi;
        h.rect = rl;
    }
}

// The items of a group-BVH leaf.  (Reciprocals shared across the leaf's
// boxes and spheres measured C5 -7 %: 10 more spilled VGPRs, EXPERIMENTS.md.)
RTW_D void leaf_items(const scene& S, int la, int lc, const ray& r, double t_min, hit_state& h, double fc) {
    for (int k = 0; k < lc; ++k) arbitrate_item(S, S.items[la + k], r, t_min, h, fc);
}

// Device BVH node (rtw_scene_upload): the builder's padded fp64 bounds
// rounded OUTWARD to fp32, children / leaf range in two ints.  32 B instead
// of rtw_bvh_node's 64, and the slab test below runs in fp32 (twice the fp64
// rate on gfx950).
struct bvh_node32 {
    float lo[3], hi[3];
    int32_t a;  // inner: left child; leaf: first item
    int32_t b;  // inner: right child | pad << 28 (push_children); leaf: -count
};
RTW_HD int node_count(const bvh_node32& n) { return n.b < 0 ? -n.b : 0; }
// Per-walk fp32 form of the ray for the slab tests: t = x * inv + oi per
// axis, with oi = -o * inv moved down (oin, near planes) and up (oif, far
// planes) by eps = (2^-21 + 2^-22) (B + |o|) |inv| + 2^-120, B the largest
// node coordinate (scene::bvh_bound).  The 2^-21 part covers the fp32
// rounding of inv (x * inv is off by at most 2^-23.9 B |inv|) and of oi
// itself, so x * inv + oin <= (x - o) / d <= x * inv + oif in real
// arithmetic; the 2^-22 part covers the rounding of the slab test's own fma
// (its result is at most (B + |o|) |inv| (1 + 2^-20) in magnitude, so it is
// off by less than 2^-23.9 of that), and 2^-120 a flushed denormal result.
// An axis whose |inv| or eps exceeds 2^90 (d.K ~ 0, NaN) never culls:
// inv = 0, oin = -inf, oif = +inf.
// inv is the hardware fp32 reciprocal of fl32(d) instead of
// fl32(1.0 / d) -- within 2^-22.4 |1 / d| (2^-24 for the conversion, 1 ulp
// for v_rcp_f32), and oi = -o * inv in fp64 within 2^-22.4 |o / d|; with the
// final rounding of oi +- eps that is under 2^-21.9 (B + |o|) |1 / d|, inside
// the 2^-21 part (eps itself computed from |inv| loses a 2^-22 relative) --
// three fp64 divisions fewer per walk.
struct slab_ray {
    float inv[3], oin[3], oif[3];
};
RTW_D slab_ray make_slab_ray(const scene& S, const ray& r) {
    slab_ray s;
    const double dd[3] = {r.d.x, r.d.y, r.d.z}, oo[3] = {r.o.x, r.o.y, r.o.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double inv = (double)__builtin_amdgcn_rcpf((float)dd[k]);
        const double oi = -oo[k] * inv;
        const double eps = 0x1.8p-21 * (S.bvh_bound + __builtin_fabs(oo[k])) * __builtin_fabs(inv) + 0x1p-120;
        const bool ok = __builtin_fabs(inv) <= 0x1p90 && eps <= 0x1p90;
        s.inv[k] = ok ? (float)inv : 0.0f;
        s.oin[k] = ok ? (float)(oi - eps) : -__builtin_inff();
        s.oif[k] = ok ? (float)(oi + eps) : __builtin_inff();
    }
    return s;
}

// Slab test of a node over [t0, t1]: true whenever the real-arithmetic slab
// test against the builder's padded fp64 bounds is (the fp64 test this
// replaces was itself conservative that way), so it may keep a node that test
// would drop, never the reverse.  Per axis the near / far planes' t are
// bracketed by the fma results (make_slab_ray's eps covers their rounding),
// min / max are exact, and t0 <= t_min, t1 >= t_max are the caller's (t_lo32,
// t_hi32): no adjustment is left for the comparison.  Node coordinates are
// finite and within 2^90 (upload), so no NaN arises.
RTW_D bool slab32(const bvh_node32& nd, const slab_ray& s, float t0, float t1) {
    float tn = t0, tf = t1;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float an = __builtin_fmaf(nd.lo[k], s.inv[k], s.oin[k]);
        const float bn = __builtin_fmaf(nd.hi[k], s.inv[k], s.oin[k]);
        const float af = __builtin_fmaf(nd.lo[k], s.inv[k], s.oif[k]);
        const float bf = __builtin_fmaf(nd.hi[k], s.inv[k], s.oif[k]);
        tn = __builtin_fmaxf(tn, __builtin_fminf(an, bn));
        tf = __builtin_fminf(tf, __builtin_fmaxf(af, bf));
    }
    return tn <= tf;
}

// BVH traversal stacks.  A private array (scratch memory) by default; the
// persistent kernels give each lane a column of an LDS array instead (one
// bank per lane, no scratch round trips).  Nested walks (a group BVH inside
// a world-BVH leaf) share one stack above the outer walk's entries; the host
// checks at upload that the deepest nesting fits (rtw_scene_upload).
constexpr int kStack = 48;
constexpr int kLdsStack = 16;  // LDS stack entries per lane
struct local_stack {
    static constexpr int cap = kStack;
    int s[kStack];
    RTW_D int& at(int i) { return s[i]; }
};
// Workgroup size of the persistent BVH kernel (k_persist): its LDS node
// packet is one per workgroup, so larger workgroups at the same waves per CU
// share one larger packet.  1 024 threads = the CU's 16 waves in one
// workgroup: one ~36 KB packet (1 152 nodes: all 969 of random_balls' tree)
// instead of four ~8 KB copies (256 nodes each).  k_persist has no block
// barrier in its loop, so the larger workgroup costs nothing else.
// Measured (1 MI355X, A/B against 256, profiles/r03/ab_persist_block.log):
// C3 slice 2 783 vs 2 607 Msamples/s (+6.7 %), C5 slice 623 vs 600 (+3.8 %).
#ifndef RTW_PERSIST_BLOCK
#define RTW_PERSIST_BLOCK 1024
#endif
constexpr int kPBlock = RTW_PERSIST_BLOCK;
struct lds_stack {  // 16-bit node indices (LDS stacks need < 65536 nodes: upload)
    static constexpr int cap = kLdsStack;
    uint16_t* p;  // &column[0][lane]; entry i at p[i * kPBlock]
    RTW_D uint16_t& at(int i) { return p[i * kPBlock]; }
};

// A BVH node: from the LDS packet when it is one of the top n_lnodes, else
// from memory.
RTW_D bvh_node32 node_at(const scene& S, int i) {
    // explicit address spaces: an LDS read for packet lanes, a global read
    // for the rest (one flat load through a selected pointer is what the
    // compiler makes of the plain form, with a flat load's latency)
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    using lds_v4 = const __attribute__((address_space(3))) v4u;
    using glb_v4 = const __attribute__((address_space(1))) v4u;
    v4u a, b;
    if (S.n_lnodes >= S.n_nodes) {
        // every node is in the packet (wave-uniform: a scalar branch, no
        // per-lane address-space test; Book 2's 1 668 nodes with F_PIN)
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

// Inner nodes carry their children's split axis (pad & 3) and whether the
// left child lies on the upper side of it (pad & 4), set at upload: the
// child nearer along the ray is pushed last, so it is visited first and the
// closest hit tightens early.  (Visiting order never changes the result:
// arbitrate reproduces the list order's tie rule.)
// dneg: bit k set iff !(d.k >= 0), once per walk (dir_mask), so choosing the
// order is integer bit work, not a branchy per-lane pick of a component.
RTW_D int dir_mask(const d3& d) { return (d.x >= 0 ? 0 : 1) | (d.y >= 0 ? 0 : 2) | (d.z >= 0 ? 0 : 4); }
template <class STK>
RTW_D void push_children(const bvh_node32& nd, int dneg, STK& stk, int& sp) {
    const int pad = nd.b >> 28, right = nd.b & 0x0fffffff;
    const bool left_first = (((dneg >> (pad & 3)) ^ (pad >> 2)) & 1) == 0;
    stk.at(sp++) = left_first ? right : nd.a;
    stk.at(sp++) = left_first ? nd.a : right;
}

// Speculative while-while for the world child-test walk (Aila & Laine 2009):
// lanes that already hold their leaf keep walking until every lane of the
// wave has one, so the inner loop runs with more lanes busy.  Nodes are then
// sometimes tested against a closest t the pending leaf would have
// tightened: more work per lane, never a different winner (better() makes
// it order-independent).

RTW_D double widen_lo(double t) { return t > 0 ? t * 0.5 : t * 2.0 - 1e-9; }
RTW_D double widen_hi(double t) { return t * (1 + 1e-12) + 1e-9; }
// fp32 bounds of a walk's t range for slab32: t_lo32(t) <= t (widen_lo leaves
// a factor of two, the conversion is off by 2^-24 relative); t_hi32(t) >= t
// (the conversion of widen_hi(t) may round down by 2^-24 relative, so the
// result is moved up by 2^-23 relative + 2^-126 -- once per closest-hit
// update, not per node)
RTW_D float t_lo32(double t) { return (float)widen_lo(t); }
RTW_D float t_hi32(double t) {
    const float f = (float)widen_hi(t);
    return __builtin_fmaf(__builtin_fabsf(f), 0x1p-23f, f) + 0x1p-126f;
}

// One step of the child-test walks: the inner node (ca, cb)
// (its a / b fields) loads both children and slab-tests them together; the
// nearer passing child becomes (ca, cb), the other passing one is stacked.
// Returns false when neither passes.
template <class STK>
RTW_D bool expand_children(const scene& S, const slab_ray& sr, float t0, float t1, int dneg, STK& stk, int& sp,
                           int& ca, int& cb) {
    const int pad = cb >> 28, right = cb & 0x0fffffff;
    const bvh_node32 L = node_at(S, ca), R = node_at(S, right);
    const bool hl = slab32(L, sr, t0, t1), hr = slab32(R, sr, t0, t1);
    const bool left_first = (((dneg >> (pad & 3)) ^ (pad >> 2)) & 1) == 0;
    const bool hn = left_first ? hl : hr, hf = left_first ? hr : hl;
    const int far_i = left_first ? right : ca;
    const int na = left_first ? L.a : R.a, nb = left_first ? L.b : R.b;
    const int fa = left_first ? R.a : L.a, fb = left_first ? R.b : L.b;
    if (hn && hf && sp + 1 <= STK::cap) stk.at(sp++) = far_i;  // always fits: depth checked at upload
    ca = hn ? na : fa;
    cb = hn ? nb : fb;
    return hn || hf;
}

// BVH over the prims of one group (items = prim indices).  (Packet walks of
// a wave-uniform root, 4-wide nodes and fused walks of two group trees all
// measured slower: EXPERIMENTS.md.)
template <class STK>
RTW_D void group_bvh(const scene& S, int root, const ray& r, double t_min, hit_state& h, STK& stk, int base,
                     bool movers) {
    const double fc = motion_frac(S, r.t, movers);
    const slab_ray sr = make_slab_ray(S, r);
    const int dneg = dir_mask(r.d);
    const float t0 = t_lo32(t_min);
    int sp = base;
    stk.at(sp++) = root;
    // while-while, as in world_closest (+6.6 % Book 2 BVH, whose 1 000-sphere
    // cluster is a group BVH).  (The world walk's child-test form measured
    // -0.4 % here, C5.)
    for (;;) {
        int la = 0, lc = 0;
        while (lc == 0 && sp > base) {
            const bvh_node32 nd = node_at(S, stk.at(--sp));
            if (!slab32(nd, sr, t0, t_hi32(h.t))) continue;
            lc = node_count(nd);
            la = nd.a;
            if (lc == 0 && sp + 2 <= STK::cap) push_children(nd, dneg, stk, sp);
        }
        if (lc == 0) break;
        leaf_items(S, la, lc, r, t_min, h, fc);
    }
}

// (called with wave-uniform entries only: the media walk)
template <int F, class STK>
RTW_D void group_closest(const scene& S, const entry_v& e, const ray& r, double t_min, hit_state& h, STK& stk) {
    if ((F & F_GBVH) && e.bvh_root >= 0)
        group_bvh(S, e.bvh_root, r, t_min, h, stk, 0, e.movers);
    else
        group_scan(S, e.first_prim, e.n_prims, r, t_min, h, e.movers);
}

// Closest t of a medium's boundary in (t0, t1) (hittable.h:438-449); the
// boundary is the entry's ops after the enclosing ones + group, `r` the ray
// in the medium's frame.
template <int F, class STK>
RTW_D bool boundary_t(const scene& S, const entry_v& e, const ray& r, double t0, double t1, double& t, STK& stk) {
    const ray lr = ops_in<true>(e, r, rd<true>(&e.p->n_outer_ops), e.n_ops);
    hit_state h{t1, -1, false};
    group_closest<F>(S, e, lr, t0, h, stk);
    if (h.prim == -1) return false;
    t = h.t;
    return true;
}

// Both boundary probes of a one-sphere boundary from one quadratic.
// Measured (1 MI355X, A/B, profiles/r04/ab_pin_quad_boxrcp.log): C5 slice
// 656.1 vs 639.3 Msamples/s.
// The boundary distances of constant_medium::hit (hittable.h:438-449): the
// closest boundary hit t1 in (-DBL_MAX, DBL_MAX), then the closest beyond
// t1 + 0.0001f; false when either probe misses.  `r` is the ray in the
// frame of the transforms enclosing the medium.
template <int F, class STK>
RTW_D bool medium_bounds(const scene& S, const entry_v& e, const ray& r, int n_outer, double& t1, double& t2,
                         STK& stk) {
    if (e.n_prims == 1 && e.bvh_root < 0 && is_sphere(ld(&S.prims[e.first_prim].type))) {
        // A boundary that is one sphere (wave-uniform: the media walk's
        // entries are): both probes (hittable.h:438-449) are that sphere's
        // test on the same ray, so its quadratic is solved once and each
        // probe applies its own range to the two roots, as group_scan would
        // (near root if in (t_lo, DBL_MAX), else the far one).
        const ray lr = ops_in<true>(e, r, n_outer, e.n_ops);
        const rtw_prim q = uprim(S.prims, e.first_prim);
        const d3 oc = lr.o - sphere_center(q, lr.t, motion_frac(S, lr.t, e.movers));
        const double a = dot(lr.d, lr.d);
        const double b = dot(oc, lr.d);
        const double c = dot(oc, oc) - q.p[9];
        const double disc = b * b - a * c;
        if (!(disc > 0)) return false;
        const double sq = RTW_SQRT(disc);
        const double r0 = (-b - sq) / a, r1 = (-b + sq) / a;
        if (r0 < kDblMax && r0 > -kDblMax)
            t1 = r0;
        else if (r1 < kDblMax && r1 > -kDblMax)
            t1 = r1;
        else
            return false;
        const double lo = t1 + kStep;
        if (r0 < kDblMax && r0 > lo)
            t2 = r0;
        else if (r1 < kDblMax && r1 > lo)
            t2 = r1;
        else
            return false;
    } else {
        if (!boundary_t<F>(S, e, r, -kDblMax, kDblMax, t1, stk)) return false;
        if (!boundary_t<F>(S, e, r, t1 + kStep, kDblMax, t2, stk)) return false;
    }
    return true;
}

// constant_medium::hit hittable.h:430-479 (at most one draw per call), in
// the frame of the transforms enclosing the medium (translate / rotate_y
// hand it their moved ray, hittable.h:299-311, 373-404)
template <int F, class STK>
RTW_D bool medium_t(const scene& S, const entry_v& e, const ray& rw, double t_min, double t_max, uint32_t& rng,
                    double& t_out, STK& stk) {
    const int n_outer = rd<true>(&e.p->n_outer_ops);
    const ray r = ops_in<true>(e, rw, 0, n_outer);
    double t1, t2;
    if (!medium_bounds<F>(S, e, r, n_outer, t1, t2, stk)) return false;
    if (t1 < t_min) t1 = t_min;
    if (t2 > t_max) t2 = t_max;
    if (t1 >= t2) return false;
    if (t1 < 0) t1 = 0;
    const double dl = len(r.d);
    const double inside = (t2 - t1) * dl;
    const double hit_distance = rd<true>(&e.p->neg_inv_density) * log_dev(rnd01(rng));
    if (hit_distance < inside) {
        t_out = t1 + hit_distance / dl;
        return true;
    }
    return false;
}


#ifdef RTW_PROF_WALK
__device__ unsigned long long g_walk[32][64];  // clock per media-walk position (sampled walks), per lane slot
#endif

// World closest hit (hittable_list::hit hittable_list.h:11-37).  Without
// media, one walk in list order equals the reference's two walks (every
// primitive is deterministic; the second walk re-accepts only what the first
// kept).  With media, the second walk can only change the result through the
// media's fresh draws, so it re-evaluates just the media, in list order.
template <int F, class STK>
RTW_D hit_state world_closest(const scene& S, const ray& r, uint32_t& rng, STK& stk) {
    hit_state h{in_place<kDblMaxBits>(), -1, false};
    if constexpr ((F & F_WBVH) != 0 && (F & F_MEDIA) == 0) {
        const double fc = motion_frac(S, r.t, S.mv_common != 0);  // transforms keep the ray's time
        const slab_ray sr = make_slab_ray(S, r);
        const int dneg = dir_mask(r.d);
        const float t0 = t_lo32(kTMin);
        int sp = 0;
        stk.at(sp++) = S.world_bvh_root;
        // Leaf items: prims (~prim) or entries (their groups, flat or BVH)
        const double a = dot(r.d, r.d);
        const bool oka = walk_ray_ok(S, r, fc) && div_hw_ok_b(a);
        const double ya = rcp_hw(a);
        auto leaf = [&](int la, int lc) {
            for (int k = 0; k < lc; ++k) {
                const int it = S.items[la + k];
                if (it < 0) {  // plain one-prim entry, its prim stored as ~prim by the upload
                    arbitrate_a(S, ~it, r, kTMin, h, fc, ya, oka);
                    continue;
                }
                const entry_v e = view_entry<false>(S, it);
                const ray lr = entry_local_ray<false>(e, r);
                if ((F & F_GBVH) && e.bvh_root >= 0) {
                    group_bvh(S, e.bvh_root, lr, kTMin, h, stk, sp, S.mv_common != 0);
                } else {
                    for (int i = 0; i < e.n_prims; ++i) arbitrate(S, e.first_prim + i, lr, kTMin, h, fc);
                }
            }
        };
        if constexpr ((F & F_GBVH) == 0) {
            // Children tested by their parent's iteration: expanding an inner
            // node loads both children and slab-tests them together; a lane
            // continues with the nearer child that passes and stacks the
            // other, so a child whose box fails costs no iteration of its
            // own.  A stacked node's box is tested again when it is popped
            // (the closest hit may have tightened since).  While-while as
            // below: lanes run inner iterations until each holds a leaf.
            int ca = 0, cb = 0;  // the node this lane expands next: its a / b fields
            bool have = false;
            {
                const bvh_node32 rt = node_at(S, S.world_bvh_root);
                if (slab32(rt, sr, t0, t_hi32(h.t))) ca = rt.a, cb = rt.b, have = true;
            }
            sp = 0;
            for (;;) {
                int la = 0, lc = 0;  // this lane's pending leaf: first item, count
                // speculative while-while: a lane that holds its leaf keeps
                // walking (with the closest t it has) while other lanes of the
                // wave still look for theirs, and stops at its next leaf,
                // which it keeps as its current node for the next round
                for (;;) {
                    const bool done = !have && sp == 0;
                    if (__builtin_amdgcn_ballot_w64(lc == 0 && !done) == 0) break;
                    if (done || (have && cb < 0 && lc != 0)) continue;
                    if (!have) {
                        const bvh_node32 nd = node_at(S, stk.at(--sp));
                        if (!slab32(nd, sr, t0, t_hi32(h.t))) continue;
                        ca = nd.a, cb = nd.b, have = true;
                    }
                    if (cb < 0) {  // a leaf
                        if (lc == 0) la = ca, lc = -cb, have = false;
                        continue;
                    }
                    have = expand_children(S, sr, t0, t_hi32(h.t), dneg, stk, sp, ca, cb);
                }
                if (__builtin_amdgcn_ballot_w64(lc != 0) == 0) break;
                if (lc != 0) leaf(la, lc);
            }
        } else {
            while (sp > 0) {
                const bvh_node32 nd = node_at(S, stk.at(--sp));
                if (!slab32(nd, sr, t0, t_hi32(h.t))) continue;
                const int cnt = node_count(nd);
                if (cnt > 0) {
                    leaf(nd.a, cnt);
                } else if (sp + 2 <= STK::cap) {  // always true: depth checked at upload
                    push_children(nd, dneg, stk, sp);
                }
            }
        }
        return h;
    } else {
        if constexpr ((F & F_MEDIA) != 0) {
            // the media walk: entries in the order the reference's nested
            // list walks call them (scene::media; with media the run form
            // spills more registers than it saves, measured on Book-2 BVH)
#ifdef RTW_PROF_WALK  // profiling builds: clock per visit of the media walk, by entry (g_walk)
            const bool pw = (rng & 63) == 0;  // a sample of the walks
            uint64_t pw_t = pw ? clock64() : 0;
#endif
            for (int k = 0; k < S.n_media; ++k) {
                const int visit = ld(&S.media[k]);
                const int ei = visit & kVisitEntry;
                const entry_v e = view_entry<true>(S, ei);
                if (e.kind == RTW_ENTRY_MEDIUM) {
                    double t;
                    if (medium_t<F>(S, e, r, kTMin, h.t, rng, t, stk)) {
                        h.t = t;
                        h.prim = -(2 + ei);
                        h.rect = false;
                    }
                } else {
                    const ray lr = entry_local_ray<true>(e, r);
                    group_closest<F>(S, e, lr, kTMin, h, stk);
                }
#ifdef RTW_PROF_WALK
                if (pw) {
                    const uint64_t now = clock64();
                    atomicAdd(&g_walk[k < 31 ? k : 31][threadIdx.x & 63], (unsigned long long)(now - pw_t));
                    pw_t = now;
                }
#endif
            }
        } else {
            for (int ri = 0; ri < S.n_runs; ++ri) {
                // one scan site for plain runs and transformed groups alike
                const int ei = ld(&S.runs[ri].entry);
                if ((F & F_YSPH) && ei == WORLD_RUN_YSPHERES) {
                    ysphere_scan(S, ld(&S.runs[ri].first_prim), ld(&S.runs[ri].n_prims), r, kTMin, h,
                                 motion_frac(S, r.t, ld(&S.runs[ri].movers)));
                    continue;
                }
                ray lr = r;
                if (ei >= 0) {
                    const entry_v e = view_entry<true>(S, ei);
                    lr = entry_local_ray<true>(e, r);
                    if ((F & F_GBVH) && e.bvh_root >= 0) {
                        group_bvh(S, e.bvh_root, lr, kTMin, h, stk, 0, e.movers);
                        continue;
                    }
                }
                group_scan<(F & F_STATIC) != 0, true>(S, ld(&S.runs[ri].first_prim), ld(&S.runs[ri].n_prims), lr,
                                                      kTMin, h, ld(&S.runs[ri].movers));
            }
        }
        return h;
    }
}
template <int F>
RTW_D hit_state world_closest(const scene& S, const ray& r, uint32_t& rng) {
    local_stack stk;
    return world_closest<F>(S, r, rng, stk);
}

// Reconstruct the hit record (p, normal, material) of a winner exactly as
// the reference produced it (leaf hit, then ops outward).
// (MEDIA false: the scene has no isotropic material, hence no medium whose
// hit this could be.)
template <bool MEDIA = true, bool STATIC = false>
RTW_D void hit_record(const scene& S, const ray& r, const hit_state& h, d3& p, d3& n, int& mat, bool& rect) {
    rect = false;
    if (MEDIA && h.prim <= -2) {  // constant_medium, hittable.h:469-472, then its enclosing ops outward
        const entry_v e = view_entry<false>(S, -h.prim - 2);
        const int n_outer = e.p->n_outer_ops;
        const ray mr = ops_in<false>(e, r, 0, n_outer);
        p = at(mr, h.t);
        n = d3{1, 0, 0};
        ops_out<false>(e, n_outer, p, n);
        mat = S.entries[-h.prim - 2].phase_material;
        return;
    }
    const rtw_prim q = S.prims[h.prim];
    const entry_v e = view_entry<false>(S, q.entry);
    const ray lr = entry_local_ray<false>(e, r);
    p = at(lr, h.t);
    if (is_sphere(q.type)) {
        const d3 cc = STATIC ? ld3(q.p) : sphere_center(q, lr.t, motion_frac(S, lr.t, q.type >= DP_MOVING_COMMON));
        n = (p - cc) / q.p[3];
    } else {
        n = rect_normal(q.type);
        rect = true;
    }
    if (q.flip & 1) n = -n;
    entry_rec_out<false>(e, p, n);
    mat = q.material;
}

// ------------------------------------------------------------------ textures

RTW_D double smooth(double x) { return x * x * (3 - 2 * x); }  // noise.h:9-12

RTW_D double perlin_noise(const scene& S, d3 p) {  // noise.h:89-151 (PERLIN branch)
    const double fx = floor(p.x), fy = floor(p.y), fz = floor(p.z);
    const double u = p.x - fx, v = p.y - fy, w = p.z - fz;
    const int i = (int)fx, j = (int)fy, k = (int)fz;
    const double uu = smooth(u), vv = smooth(v), ww = smooth(w);
    double accum = 0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int idx = S.perm[(i + a) & 255] ^ S.perm[256 + ((j + b) & 255)] ^ S.perm[512 + ((k + c) & 255)];
                const d3 g = ld3(S.ranvec + 3 * idx);
                const d3 wv = d3{u - a, v - b, w - c};
                accum += (a * uu + (1 - a) * (1 - uu)) * (b * vv + (1 - b) * (1 - vv)) *
                         (c * ww + (1 - c) * (1 - ww)) * dot(g, wv);
            }
    return accum;
}

RTW_D double turb(const scene& S, d3 p) {  // noise.h:74-86
    double accum = 0;
    double weight = 1.0;
    for (int i = 0; i < 7; ++i) {
        accum += weight * perlin_noise(S, p);
        weight *= 0.5f;
        p = p * 2.0;
    }
    return fabs(accum);
}

// Shade-kernel specialisation by the scene's material / texture set.
enum : int { SF_NOISE = 1, SF_CHECKER = 2, SF_METAL = 4, SF_DIEL = 8, SF_ISO = 16, SF_ALL = 31 };

template <int M>
RTW_D d3 texture_value(const scene& S, int id, d3 p) {
    for (int guard = 0; guard < 8; ++guard) {
        const rtw_texture& t = S.textures[id];
        if (!(M & (SF_NOISE | SF_CHECKER)) || t.type == RTW_TEX_CONSTANT) return ld3(t.color);
        if ((M & SF_CHECKER) && t.type == RTW_TEX_CHECKER) {  // texture.h:38-49
            const double sines = sin_tex(10.0 * p.x) * sin_tex(10.0 * p.y) * sin_tex(10.0 * p.z);
            id = sines < 0 ? t.odd : t.even;
            continue;
        }
        if (M & SF_NOISE) {
            // texture.h:57-68: vec3(1,1,1) * 0.5f * (1 + sin(scale*p.z + 10*turb(p)))
            const double v = (1.0 * (double)0.5f) * (1 + sin_tex(t.scale * p.z + 10 * turb(S, p)));
            return d3{v, v, v};
        }
        return ld3(t.color);
    }
    return d3{0, 0, 0};
}

// ------------------------------------------------------------------ lights
template <bool STATIC>
RTW_D double light_pdf_value(const scene& S, const rtw_light& L, d3 o, d3 v) {
    if (L.kind == RTW_LIGHT_XZ_RECT) {  // hittable.h:208-222
        // xz_rect::hit (hittable.h:184-200, validate: an XZ light is an xz
        // rect) without its early returns: t, a, b and the pdf are formed for
        // every lane and a miss selects 0 -- one branch level less of
        // exec-mask bookkeeping per light per bounce (the world walk's rects
        // likewise, rect_axis_rcp<BL>); a missing lane's values are never
        // used.  Measured T +0.27 % (profiles/r05/ab_r5w_light_rect_branchless.log).
        const rtw_prim& q = S.prims[L.prim];
        const double t = (q.p[4] - o.y) / v.y;
        const double a = o.x + t * v.x;
        const double b = o.z + t * v.z;
        const bool hit = !(t < 0.001 || t > __builtin_inf()) && !(a < q.p[0] || a > q.p[1] || b < q.p[2] || b > q.p[3]);
        const double area = (q.p[1] - q.p[0]) * (q.p[3] - q.p[2]);
        const double distance_squared = t * t * len2(v);
#if RTW_RADIANCE_FAST
        // |dot(v, n)| / |v| folded into one quotient (v.y != 0 where the rect
        // was hit; a missing lane divides by 1, so rad_div's wave vote is
        // the hitting lanes' as before)
        const double pdf = rad_div(distance_squared * len(v), hit ? fabs(v.y) * area : 1.0);
#else
        const double cosine = fabs(dot(v, d3{0, 1, 0}) / len(v));
        const double pdf = distance_squared / (cosine * area);
#endif
        return hit ? pdf : 0.0;
    }
    if (L.kind == RTW_LIGHT_SPHERE) {  // sphere.h:88-99
        const rtw_prim& q = S.prims[L.prim];
        const ray r{o, v, kFltMax};
        double t;
        // (STATIC: no moving spheres, the fraction is never read)
        if (!sphere_t(q, r, 0.001, __builtin_inf(), t, STATIC ? 0.0 : motion_frac(S, r.t, q.type >= DP_MOVING_COMMON)))
            return 0.0;
#if RTW_RADIANCE_FAST
        // (magnitude only: the pdf's sign is that of the hit above; r^2 / d^2
        // stays a division, so 1 - r^2 / d^2 rounds as the reference's does
        // next to the sphere, where it cancels)
        const double cos_theta_max = RTW_SQRT(1 - q.p[9] / len2(ld3(q.p) - o));
        return rad_div(1.0, kTwoPi * (1.0 - cos_theta_max));
#else
        const double cos_theta_max = RTW_SQRT(1 - q.p[9] / len2(ld3(q.p) - o));  // p[9] = radius * radius
        const double solid_angle = kTwoPi * (1.0 - cos_theta_max);
        return 1.0 / solid_angle;
#endif
    }
    return 0.0;  // hittable.h:36
}

// The frame (onb::build_from_w(normal), onb.h:32-38) of a lambertian hit,
// kept as what it is built from and built only where it is used: a rect's
// world normal is fixed, so its frame comes from the host-built table
// (scene::prim_onb, same arithmetic); anything else's from its normal.  The
// 18 registers of a built frame are then never live across the light
// sampling and the pdfs.
struct surf_frame {
    d3 n;
    int32_t prim;
    bool rect;
    bool unit;  // n is a surface normal (length about 1: normalize_unit)
};
RTW_D onb frame_onb(const scene& S, const surf_frame& s) {
    if (s.rect) {
        const double* f = S.prim_onb + 9 * (size_t)s.prim;
        return onb{ld3(f), ld3(f + 3), ld3(f + 6)};
    }
    return onb_from_w(s.n);
}
RTW_D d3 frame_w(const scene& S, const surf_frame& s) {  // == frame_onb(S, s).w
    return s.rect ? ld3(S.prim_onb + 9 * (size_t)s.prim + 6) : (s.unit ? normalize_unit(s.n) : normalize(s.n));
}

// mixture_pdf(cosine_pdf(n), hittable_pdf(lights, o))::generate (pdf.h:55-79)
// as one code path: the cosine lobe (utility.h:54-67) and a sphere light
// (sphere.h:101-108, utility.h:69-81) share their sqrt / sincos / onb tail,
// so a wave whose lanes took different branches pays for one sincos, not
// two.  Every lane draws and rounds exactly as its own branch would.
RTW_D d3 mixture_generate(const scene& S, const surf_frame& sf, d3 o, uint32_t& rng, uint32_t pre = 0) {
    // (pre: the choice already drawn -- 1 cosine, 2 lights; 0 draws it here)
    const bool cosine = pre ? pre == 1 : rnd01(rng) < 0.5;
    rtw_light L{RTW_LIGHT_DEFAULT, 0};
    int kind = -1;  // the cosine lobe
    if (!cosine) {
        L = S.lights[random_int(rng, 0, S.n_lights - 1)];
        kind = L.kind;
    }
    if (kind == RTW_LIGHT_DEFAULT) return d3{1, 0, 0};  // hittable.h:37
    const double r1 = rnd01(rng);
    const double r2 = rnd01(rng);
    if (kind == RTW_LIGHT_XZ_RECT) {  // hittable.h:224-228, z drawn first
        const rtw_prim& q = S.prims[L.prim];
        const double rz = q.p[2] + (q.p[3] - q.p[2]) * r1;
        const double rx = q.p[0] + (q.p[1] - q.p[0]) * r2;
        return d3{rx, q.p[4], rz} - o;
    }
    const bool sph = kind == RTW_LIGHT_SPHERE;
    surf_frame bf = sf;  // the lobe's frame: the surface's, or the light direction's
    double a1 = 1 - r2;
    if (sph) {
        const rtw_prim& q = S.prims[L.prim];
        const d3 direction = ld3(q.p) - o;
        const double distance_squared = len2(direction);
        bf.n = direction;
        bf.rect = false;
        bf.unit = false;
        a1 = 1 - q.p[9] / distance_squared;  // radius * radius / distance_squared
    }
    const double s1 = RTW_SQRT(a1);
    const double z = sph ? 1 + r2 * (s1 - 1) : s1;
    const double sq = RTW_SQRT(sph ? 1 - z * z : r2);
    const double phi = kTwoPi * r1;
    double sp, cp;
    sincos_azimuth(phi, sp, cp);
    return local(frame_onb(S, bf), d3{cp * sq, sp * sq, z});
}

template <bool STATIC = false>
RTW_D double lights_pdf_value(const scene& S, d3 o, d3 v) {  // hittable_list.h:44-53
    const double weight = S.light_weight;  // 1.0 / (double)n_lights, computed once on the host
    double sum = 0.0;
    for (int i = 0; i < S.n_lights; ++i) sum += weight * light_pdf_value<STATIC>(S, S.lights[i], o, v);
    return sum;
}

// ------------------------------------------------------------------ materials
RTW_D d3 reflect(d3 v, d3 n) { return v - n * (2.0 * dot(v, n)); }  // material.h:10-13

RTW_D bool refract(d3 v, d3 n, double ni_over_nt, d3& refracted) {  // material.h:17-39
    const d3 uv = normalize(v);
    const double dt = dot(uv, n);
    const double disc = 1.0 - ni_over_nt * ni_over_nt * (1 - dt * dt);
    if (disc > 0) {
        refracted = (uv - n * dt) * ni_over_nt - n * RTW_SQRT(disc);
        return true;
    }
    return false;
}

// pow(x, 5) of schlick: rtw_math.h pow5 (double-double, shared with the
// strict-radiance oracle build)

// material.h:44-49 with r0 = ((1 - ref_idx) / (1 + ref_idx))^2 precomputed
// per material on the host (same expression, same rounding)
RTW_D double schlick_r0(double cosine, double r0) { return r0 + (1 - r0) * pow5(1 - cosine); }

// ------------------------------------------------------------------ camera
// camera::get_ray camera.h:36-50, random_in_unit_disk :61-69 (y drawn first)
// (the rejection loop decided in fp32 as random_in_unit_sphere's)
// A pinhole camera (`pin`, the host's camera_is_pinhole: lens_radius 0, no
// zero origin coordinate, finite u and v) draws the disk point only to
// advance the engine: rd = 0 * p is a signed zero, so is the offset
// u * rd.x + v * rd.y, so origin + offset == origin, and (x - origin) - offset ==
// x - origin (that difference is never -0: x - origin is exactly zero only
// for x == origin != 0, which rounds to +0) -- the point is not formed and
// the offset not computed.  The draws, the time and the ray are the
// reference's (camera.h:36-50).
RTW_D ray camera_ray(const rtw_camera_desc& c, double s, double t, uint32_t& rng, bool pin) {
    d3 p;  // (pin is wave-uniform: the job's or the camera's)
    {
        constexpr float k2Rf = (float)(2.0 / kCanonR);
        auto lead = [&](uint32_t raw) { return __builtin_fmaf((float)(raw - 1u), k2Rf, -1.0f); };
        auto exact = [&](uint32_t y1, uint32_t y2, uint32_t x1, uint32_t x2) {
            const double y = canon_raw(y1, y2) * (1.0 - 0.0) + 0.0;
            const double x = canon_raw(x1, x2) * (1.0 - 0.0) + 0.0;
            return d3{x, y, 0} * 2.0 - d3{1, 1, 0};
        };
        uint32_t y1, y2, x1, x2;
        // draws 1..4 of a try from s0: y2, x2 by two-step jumps, y1 = a s0 and
        // x1 = a y2 only where the point is formed (never for a pinhole)
        uint32_t s0;
        for (;;) {
            s0 = rng;
            y2 = mr_jump(s0, kMrA2), x2 = mr_jump(y2, kMrA2);
            rng = x2;
            const float px = lead(x2), py = lead(y2);
            const float d32 = __builtin_fmaf(px, px, py * py);
            if (d32 < 1.0f - 0x1p-14f) break;
            if (!(d32 < 1.0f + 0x1p-14f)) continue;
            y1 = mr_jump(s0, kMrA), x1 = mr_jump(y2, kMrA);
            const d3 q = exact(y1, y2, x1, x2);
            if (dot(q, q) < 1.0) break;
        }
        if (!pin) {
            y1 = mr_jump(s0, kMrA), x1 = mr_jump(y2, kMrA);
            p = exact(y1, y2, x1, x2);
        }
    }
    if (pin) {
        const double time = c.time0 + rnd01(rng) * (c.time1 - c.time0);
        const d3 dir = ld3(c.lower_left) + ld3(c.horizontal) * s + ld3(c.vertical) * t - ld3(c.origin);
        return ray{ld3(c.origin), normalize(dir), time};
    }
    const d3 rd = p * c.lens_radius;
    const d3 offset = ld3(c.u) * rd.x + ld3(c.v) * rd.y;
    const double time = c.time0 + rnd01(rng) * (c.time1 - c.time0);
    const d3 dir = ld3(c.lower_left) + ld3(c.horizontal) * s + ld3(c.vertical) * t - ld3(c.origin) - offset;
    return ray{ld3(c.origin) + offset, normalize(dir), time};
}

}  // namespace rtwd
