// rtw_kernels.hip — the wavefront path tracer for gfx950 and the C ABI
// around it (include/rtw_gpu.h).
//
// Replaces the triple `_for` of RayTracingWeekend.cpp:211-250.  The recursion
// of color() (RayTracingWeekend.cpp:45-160) is unrolled into an iterative
// wavefront over a pool of in-flight paths kept as SoA arrays in HBM:
//
//   k_fill + k_regen   empty pool, then camera ray-gen for the first samples
//   repeat:
//     k_intersect  one world closest-hit query per live path   (traversal)
//     k_shade      emission / scatter / mixture-pdf sampling per path; a
//                  path that ends writes its 24-byte radiance record to its
//                  sample's slot of the pass's radiance buffer and empties
//                  its pool slot
//     k_regen      (until the sample queue is drained) refills empty slots:
//                  per-block compaction of the empty slots, one atomic on a
//                  sharded sample queue per 1024 slots, camera rays written
//                  densely to a staging buffer, a 4-byte marker per slot
//     k_compact    (tail only, once the sample queue is drained) stream
//                  compaction of live paths, __ballot/prefix-sum per tile
//   k_reduce     per-pixel sum of the samples in increasing sample order
//
// Paths are independent (the RNG is keyed by (seed, pixel, sample)), so the
// pool order never changes a result, only its speed.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>
#include "rtw_device.h"
#include "rtw_fast.h"
#include "host/rtw_host_util.h"

using namespace rtwd;

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kPWaves = kPBlock / 64;  // k_persist's workgroup (rtw_device.h kPBlock)

// Path pool (SoA, one element per slot).  depth word of a slot:
//   0                    empty
//   1..max_depth         live path: the depth argument of its next color() call
//   kFresh | k           a new camera sample whose ray / time / rng / sample id
//                        sit in staging entry k (written densely by k_regen);
//                        its throughput is 1 and its depth max_depth
constexpr uint32_t kFresh = 0x80000000u;

struct paths_t {
    double *ox, *oy, *oz, *dx, *dy, *dz, *tm, *tr, *tg, *tb;
    uint32_t *rng, *depth, *qid;
};

struct fresh_t {  // staging of new camera rays, indexed like the pool
    double *ox, *oy, *oz, *dx, *dy, *dz, *tm;
    uint32_t *rng, *qid;
};

// The sample queue is sharded over kQShards counters to spread the atomics:
// shard s owns the chunks c = s, s + kQShards, ... of kQChunk consecutive
// samples, and its j-th sample is  q = ((j / kQChunk) * kQShards + s) * kQChunk
// + j % kQChunk.
constexpr int kQShards = 8;
constexpr uint32_t kQChunk = 1024;

// Counters hit by many workgroups live on 256-byte lines of their own: all
// words of one line are served by one L2 channel, which serialises them
// (one word saturates at ~88 atomics/us).  Shard k is used by the blocks with
// blockIdx % 8 == k, i.e. by one XCD.
struct alignas(256) ctr_line {
    unsigned long long v;
    unsigned long long pad[31];
};

struct ctrs_t {
    ctr_line qshard[kQShards];  // per-shard count of samples handed out
    ctr_line segments[8];       // world hit queries (live paths intersected)
    unsigned int n;                      // slots in the current pool
    unsigned int n_out;                  // compaction output count
    unsigned int pad[4];
};

__host__ __device__ inline uint64_t shard_sample(int s, uint64_t j) {
    return ((j / kQChunk) * kQShards + (uint64_t)s) * kQChunk + j % kQChunk;
}
// number of the pass's `total` samples that shard s owns (its ids 0..limit-1)
__host__ __device__ inline uint64_t shard_limit(int s, uint64_t total) {
    const uint64_t full = total / kQChunk, rem = total % kQChunk;
    const uint64_t nfull = full > (uint64_t)s ? (full - (uint64_t)s + kQShards - 1) / kQShards : 0;
    return nfull * kQChunk + ((full % kQShards) == (uint64_t)s ? rem : 0);
}

struct job_t {
    const rtw_camera_desc* cam;  // device copy (read where rays are made, see camera_sample)
    uint64_t seed_mix;   // splitmix64(seed)
    uint32_t total;      // samples in this pass
    uint32_t npix;       // pixels of this call (n_rows * nx)
    int32_t nx, ny, row_begin, row_step, s_begin, max_depth;
    uint32_t spp_pass;   // samples per pixel in this pass
    uint32_t cam_pin;    // camera_is_pinhole(camera): camera_ray's pinhole shortcut applies
    rtwd::udiv32 div_npix, div_nx, div_spp;  // magic numbers of npix, nx, spp_pass (sample_coords)
    double* L;           // per-sample radiance, L[3q + c] (pass-local sample id q)
#if RTW_STRICT_RADIANCE
    // per-thread factor logs of the strict build: bounce k of the path on
    // global thread g at flog[4 (k * flog_threads + g)] = (m.x, m.y, m.z, pdf)
    double* flog;
    uint32_t flog_threads;
#endif
};

// Pass-local sample ids are sample-major: q = sample * npix + pixel, so a
// wave's 64 consecutive ids are 64 neighbouring pixels and k_reduce reads
// each sample plane coalesced.  (Pixel-major ids fill whole lines with a
// wave's records but make k_reduce stage each pixel's run through LDS: the
// step -0.5 %, profiles/r03/ab_pixel_major.log.)  Results do not depend on
// the order: the RNG is keyed by (pixel, sample) and each pixel's records are
// summed in sample order.

// A sample's radiance record.  (Non-temporal stores measured +-0 on T and
// C5, profiles/r05/ab_r5b_*.log.)
template <typename T>
__device__ __forceinline__ void store_record(T* o, T x, T y, T z) {
    o[0] = x, o[1] = y, o[2] = z;
}

// pass-local sample id -> pixel (i, j) and global sample index s
__device__ __forceinline__ void sample_coords(const job_t& J, uint32_t q, int& i, int& j, int& s) {
// (the quotients by exact magic-number division, rtw_div.h udiv_fast)
    const uint32_t sl = udiv_fast(q, J.div_npix);
    const uint32_t rem = q - sl * J.npix;
    const uint32_t k = udiv_fast(rem, J.div_nx);
    i = (int)(rem - k * (uint32_t)J.nx);
    j = J.row_begin + (int)k * J.row_step;
    s = J.s_begin + (int)sl;
}

// Render-loop body RayTracingWeekend.cpp:227-231 for sample q: jitter,
// camera::get_ray -> staging entry k.
// JPIN: the pinhole shortcut applies per the job's host-computed flag
// (J.cam_pin), else per the device camera's own lens_radius == 0 and nonzero
// origin -- the host gives a lens-less camera with a non-finite u or v a NaN
// lens_radius in the device copy, so both say the same.  (The two forms
// measure differently through code layout alone: J.cam_pin T +0.6 %, the
// camera test C3 +1.5 %, profiles/r06/ab_r6h_*.log; each kernel takes its
// better one.)
template <bool JPIN = true>
__device__ __forceinline__ ray camera_sample(const job_t& J, uint32_t q, uint32_t& rng) {
    int i, j, s;
    sample_coords(J, q, i, j, s);
    rng = path_seed(J.seed_mix, (uint32_t)(j * J.nx + i), (uint32_t)s);
    // The camera (23 doubles) is loaded here, with scalar loads, each time
    // rays are made: an opaque pointer stops the compiler from hoisting it
    // into loop-carried SGPRs of the persistent loop, where it spills.
    const rtw_camera_desc* cp = J.cam;
    asm volatile("" : "+s"(cp));
    // u = (i + U) / nx, v = (j + U) / ny with the device's own reciprocals of
    // nx, ny (k_recips, stored after the camera): rtw_div.h's div_hw is the
    // compiler's division sequence bit for bit when the divisor is in
    // [2^-200, 2^200] and the numerator 0 or in [2^-800, 2^100] -- here the
    // divisor is an image size and the numerator 0 or at least 2^-62 (a
    // canonical draw's grain) and below 2^32; +0 / n gives +0 either way.
    // With the magic-number sample decomposition, measured (1 MI355X, A/B,
    // profiles/r05/ab_r5m_udiv_recips.log; bit-identical images,
    // parity_r5m.log): T 4 741 vs 4 705 (+0.8 %), C3 +1.2 %, C5 -0.5 %,
    // T fp32 -0.3 %.
    const double* yr = reinterpret_cast<const double*>(cp + 1);
    const double u = div_hw((double)(i + rnd01(rng)), (double)J.nx, ld(yr));
    const double v = div_hw((double)(j + rnd01(rng)), (double)J.ny, ld(yr + 1));
    rtw_camera_desc c;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        c.origin[k] = ld(&cp->origin[k]);
        c.lower_left[k] = ld(&cp->lower_left[k]);
        c.horizontal[k] = ld(&cp->horizontal[k]);
        c.vertical[k] = ld(&cp->vertical[k]);
        c.u[k] = ld(&cp->u[k]);
        c.v[k] = ld(&cp->v[k]);
    }
    c.time0 = ld(&cp->time0);
    c.time1 = ld(&cp->time1);
    c.lens_radius = ld(&cp->lens_radius);
    const bool pin = JPIN ? J.cam_pin != 0
                          : (c.lens_radius == 0.0 && c.origin[0] != 0.0 && c.origin[1] != 0.0 && c.origin[2] != 0.0);
    return camera_ray(c, u, v, rng, pin);
}

__device__ __forceinline__ void raygen(const job_t& J, const fresh_t& F, uint32_t k, uint32_t q) {
    uint32_t rng;
    const ray r = camera_sample(J, q, rng);
    F.ox[k] = r.o.x, F.oy[k] = r.o.y, F.oz[k] = r.o.z;
    F.dx[k] = r.d.x, F.dy[k] = r.d.y, F.dz[k] = r.d.z;
    F.tm[k] = r.t;
    F.rng[k] = rng;
    F.qid[k] = q;
}

// A path as the kernels see it: from the pool, or from staging when fresh.
struct path_in {
    ray r;
    uint32_t depth;
    bool fresh;
    uint32_t src;  // staging index (fresh) or pool slot
};

__device__ __forceinline__ path_in load_ray(const paths_t& P, const fresh_t& F, uint32_t i, uint32_t dw) {
    path_in x;
    x.fresh = (dw & kFresh) != 0;
    x.src = x.fresh ? (dw & ~kFresh) : i;
    // one load per field with a per-lane address: no divergence between
    // fresh and continuing paths
    x.r.o.x = *(x.fresh ? F.ox + x.src : P.ox + i);
    x.r.o.y = *(x.fresh ? F.oy + x.src : P.oy + i);
    x.r.o.z = *(x.fresh ? F.oz + x.src : P.oz + i);
    x.r.d.x = *(x.fresh ? F.dx + x.src : P.dx + i);
    x.r.d.y = *(x.fresh ? F.dy + x.src : P.dy + i);
    x.r.d.z = *(x.fresh ? F.dz + x.src : P.dz + i);
    x.r.t = *(x.fresh ? F.tm + x.src : P.tm + i);
    x.depth = dw;
    return x;
}

// Start a pass: slots [0, n0) empty (depth 0) for k_regen to fill.
__global__ __launch_bounds__(kBlock) void k_fill(paths_t P, ctrs_t* C, uint32_t n0) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n0) P.depth[i] = 0;
    if (i == 0) C->n = n0;
    if (i < kQShards) C->qshard[i].v = 0;
}

// rcp_hw of the image's width and height for camera_sample, once per render
// call, into the two doubles after the camera's device copy
__global__ void k_recips(double* out, int nx, int ny) {
    if (threadIdx.x == 0) out[0] = rcp_hw((double)nx), out[1] = rcp_hw((double)ny);
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
    const unsigned lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// block-wide exclusive prefix of a per-lane flag; returns this lane's rank and
// writes the block total to *total (all lanes).
__device__ __forceinline__ uint32_t block_rank(bool flag, uint32_t* s_wave, uint32_t& total) {
    const unsigned long long m = __ballot(flag);
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) s_wave[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) {
        const uint32_t c = s_wave[k];
        before += (k < (int)w) ? c : 0u;
        tot += c;
    }
    total = tot;
    return before + (uint32_t)__popcll(m & lanemask_lt());
}

// One world closest-hit query per live path.  The next path's ray is loaded
// while the current one is traversed (software pipelining of the HBM reads).
template <int F>
__global__ __launch_bounds__(kBlock) void k_intersect(scene S, paths_t P, fresh_t FR, double* __restrict__ ht,
                                                      int32_t* __restrict__ hid, ctrs_t* C) {
    __shared__ uint32_t s_cnt[kWaves];
    const uint32_t n = C->n;
    const uint32_t stride = gridDim.x * kBlock;
    uint32_t live = 0;
    uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    uint32_t dw = i < n ? P.depth[i] : 0u;
    path_in cur = load_ray(P, FR, i < n ? i : 0, dw);
    while (i < n) {
        const uint32_t nx = i + stride;
        const uint32_t ndw = nx < n ? P.depth[nx] : 0u;
        const path_in nxt = load_ray(P, FR, nx < n ? nx : i, ndw);
        if (dw != 0) {
            uint32_t rng = 0u;
            if (F & F_MEDIA) rng = cur.fresh ? FR.rng[cur.src] : P.rng[i];
            const hit_state h = world_closest<F>(S, cur.r, rng);
            if (F & F_MEDIA) {
                if (cur.fresh)
                    FR.rng[cur.src] = rng;
                else
                    P.rng[i] = rng;
            }
            ht[i] = h.t;
            hid[i] = h.prim;
            ++live;
        }
        i = nx;
        dw = ndw;
        cur = nxt;
    }
    // one 64-bit atomic per block for the segment counter
    for (int off = 32; off > 0; off >>= 1) live += __shfl_down(live, off, 64);
    if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = live;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int k = 0; k < kWaves; ++k) t += s_cnt[k];
        if (t) atomicAdd(&C->segments[blockIdx.x % 8].v, t);
    }
}

// Section profiler (profiling builds only: -DRTW_PROF).  Each lane charges
// the clock since its previous mark to the section it just finished; the
// per-lane sums land in g_prof and rtw_render_accumulate prints them.
enum { PS_LOOP, PS_LOAD, PS_TRAVERSE, PS_HIT, PS_SAMPLE, PS_PDF, PS_STORE, PS_N };
#ifdef RTW_PROF
__device__ unsigned long long g_prof[PS_N];
__device__ unsigned long long g_cls[2][8];  // [0] lanes per class, [1] waves with the class present
struct prof_t {
    uint64_t t;
    uint64_t acc[PS_N];
    uint32_t lanes[8] = {0, 0, 0, 0, 0, 0, 0, 0}, waves[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // segment class of this lane: 0 miss, 1+type material hit, 7 idle
    __device__ __forceinline__ void classify(int cls) {
        for (int k = 0; k < 8; ++k) {
            const unsigned long long m = __ballot(cls == k);
            lanes[k] += (uint32_t)__popcll(m);
            waves[k] += m ? 1u : 0u;
        }
    }
    __device__ prof_t() : t(clock64()) {
        for (int k = 0; k < PS_N; ++k) acc[k] = 0;
    }
    __device__ __forceinline__ void mark(int k) {
        const uint64_t now = clock64();
        acc[k] += now - t;
        t = now;
    }
    __device__ void flush() {
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < 8; ++k) {
                atomicAdd(&g_cls[0][k], (unsigned long long)lanes[k]);
                atomicAdd(&g_cls[1][k], (unsigned long long)waves[k]);
            }
        for (int k = 0; k < PS_N; ++k) {
            unsigned long long v = acc[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
            if ((threadIdx.x & 63) == 0) atomicAdd(&g_prof[k], v);
        }
    }
};
#elif defined(RTW_REGIONS)  // static attribution: region markers in the ISA
struct prof_t {
    __device__ __forceinline__ void classify(int) {}
    __device__ __forceinline__ void mark(int k) { asm volatile(";RTW_REGION %0" ::"i"(k)); }
    __device__ __forceinline__ void flush() {}
};
#else
struct prof_t {
    __device__ __forceinline__ void classify(int) {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush() {}
};
#endif

// Background of RayTracingWeekend.cpp:141-159.
__device__ __forceinline__ d3 background(const scene& S, const d3& dir) {
    if (S.background != RTW_BG_GRADIENT) return d3{0, 0, 0};
    const d3 u = normalize(dir);
    const double t = 0.5f * (u.y + 1.0);
    return d3{1.0, 1.0, 1.0} * (1.0 - t) + d3{0.5f, 0.7f, 1.0} * t;  // lerp, vec3.h:84-87
}

// A path between two color() calls: the ray of the next call, its engine,
// the depth argument of the next call and its sample id.  (The throughput,
// the product of the attenuation / pdf factors so far, is kept by the caller:
// the persistent kernel parks it in LDS, out of the register budget.)
struct path_st {
    ray r;
    uint32_t rng, depth, q;
};

// Outcome of one segment: the path continues with throughput *= f and the
// next call's ray, or ends with radiance thr * E, or ends with radiance 0.
enum { SEG_CONTINUE = 0, SEG_END = 1, SEG_END_ZERO = 2 };
constexpr uint32_t kDepthBits = 0x3fffffffu;  // a path's depth (bits above: reserved, zero)

// A sink receives the outcome inside the shading branch that produced it:
//   cont(f, next)   the path continues (throughput *= f, ray `next`)
//   end(E)          it ends with radiance thr * E
//   end_zero()      it ends with radiance 0
// seg_out keeps the outcome for the caller (wavefront kernels); the
// persistent kernels' sinks apply it on the spot (LDS throughput update,
// continuation ray into the path's slot, radiance store), so no value of a
// branch is live across the merge of the exec-masked branches, which run
// one after the other.
//   cont_mp(m, pdf, next)  (RTW_STRICT_RADIANCE, the lambertian bounce) the
//                   path continues with the factor m / pdf, m = attenuation
//                   * scattering_pdf, kept apart for the inside-out fold
struct seg_out {
    d3 w;      // f or E
    ray next;  // SEG_CONTINUE only
    RTW_D void cont(const d3& f, const ray& nr) { w = f, next = nr; }
    RTW_D void cont_mp(const d3& m, double pdf, const ray& nr) { cont(m / pdf, nr); }
    RTW_D void end(const d3& E) { w = E; }
    RTW_D void end_zero() {}
};
template <class C, class E, class Z>
struct fn_sink {  // a sink from three callables
    C c;
    E e;
    Z z;
    RTW_D void cont(const d3& f, const ray& nr) { c(f, nr); }
    RTW_D void cont_mp(const d3& m, double pdf, const ray& nr) { c(m / pdf, nr); }
    RTW_D void end(const d3& L) { e(L); }
    RTW_D void end_zero() { z(); }
};
template <class C, class E, class Z>
RTW_D fn_sink<C, E, Z> make_sink(C c, E e, Z z) { return fn_sink<C, E, Z>{c, e, z}; }
// ... and from four: cont_mp of its own (the strict build's k_persist)
template <class C, class M, class E, class Z>
struct fn_sink4 {
    C c;
    M cm;
    E e;
    Z z;
    RTW_D void cont(const d3& f, const ray& nr) { c(f, nr); }
    RTW_D void cont_mp(const d3& m, double pdf, const ray& nr) { cm(m, pdf, nr); }
    RTW_D void end(const d3& L) { e(L); }
    RTW_D void end_zero() { z(); }
};
template <class C, class M, class E, class Z>
RTW_D fn_sink4<C, M, E, Z> make_sink4(C c, M cm, E e, Z z) { return fn_sink4<C, M, E, Z>{c, cm, e, z}; }

// One segment of color() (RayTracingWeekend.cpp:52-159) for path x whose
// world hit is (t, prim); returns the outcome (SEG_*) after handing it to
// the sink.  x.r is only read; on SEG_CONTINUE x.rng and x.depth advance.
// The recursion's inside-out products are folded forward: the radiance of a
// path is thr * (last emitted / background), thr the product of the
// reference's per-bounce factors attenuation * scattering_pdf / pdf (or
// attenuation for specular scatter).
template <int M, bool STATIC = false, bool LIGHTS = false, bool BLACK = false, bool NOLIGHTS = false, class SINK>
__device__ __forceinline__ int shade_core(const scene& S, path_st& x, double t, int32_t prim, SINK& sk,
                                          prof_t& pf) {
    const ray r = x.r;
    uint32_t rng = x.rng;
    const uint32_t depth = x.depth;
    // the scattered branches' common tail: the next color() call has depth
    // depth - 1, and returns 0 when that is 0
    auto scatter = [&](const d3& f, const d3& p, const d3& dir) -> int {
        if (depth <= 1) {
            sk.end_zero();
            return SEG_END_ZERO;
        }
        sk.cont(f, ray{p, dir, r.t});
        x.rng = rng;
        x.depth = depth - 1;
        return SEG_CONTINUE;
    };
    if (prim == -1) {
        sk.end(BLACK ? d3{0, 0, 0} : background(S, r.d));
        return SEG_END;
    }
    d3 p, n;
    int mat;
    bool rect;
    hit_record<(M & SF_ISO) != 0, STATIC>(S, r, hit_state{t, prim, false}, p, n, mat, rect);
    if (!BLACK && S.render_type == RTW_RENDER_NORMAL) {  // :135-136
        sk.end(d3{0.5f, 0.5f, 0.5f} * (n + d3{1, 1, 1}));
        return SEG_END;
    }
    const rtw_material& m = S.materials[mat];
    pf.mark(PS_HIT);
    if (m.type == RTW_MAT_DIFFUSE_LIGHT) {  // material.h:232-244: no scatter
        if (!(dot(n, r.d) > 0)) {
            sk.end_zero();
            return SEG_END_ZERO;
        }
        sk.end(texture_value<M>(S, m.texture, p));
        return SEG_END;
    } else if ((M & SF_METAL) && m.type == RTW_MAT_METAL) {  // material.h:128-136
        const d3 reflected = reflect(normalize(r.d), n);
        const d3 dir = reflected + random_in_unit_sphere(rng) * m.fuzz;
        return scatter(ld3(m.albedo), p, dir);
    } else if ((M & SF_DIEL) && m.type == RTW_MAT_DIELECTRIC) {  // material.h:146-222
        d3 outward;
        double ni_over_nt, cosine;
        const double ri = m.ref_idx;
        if (dot(r.d, n) > 0) {
            outward = -n;
            ni_over_nt = ri;
            cosine = dot(r.d, n) / len(r.d);
            cosine = RTW_SQRT(1 - ri * ri * (1 - cosine * cosine));
        } else {
            outward = n;
            ni_over_nt = S.mat_aux[2 * mat];  // 1.0 / ri, host-computed
            cosine = -dot(r.d, n) / len(r.d);
        }
        const d3 reflected = reflect(r.d, n);
        d3 refracted{0, 0, 0};
        const double reflect_prob = refract(r.d, outward, ni_over_nt, refracted) ? schlick_r0(cosine, S.mat_aux[2 * mat + 1]) : 1.0;
        const d3 dir = (rnd01(rng) < reflect_prob) ? reflected : refracted;
        return scatter(d3{1.0, 1.0, 1.0}, p, dir);
    } else if ((M & SF_ISO) && m.type == RTW_MAT_ISOTROPIC) {  // material.h:257-262
        const d3 dir = random_in_unit_sphere(rng);
        return scatter(texture_value<M>(S, m.texture, p), p, dir);
    } else {  // lambertian material.h:81-119 + RayTracingWeekend.cpp:112-132
        // (RTW_RADIANCE_FAST: quantities that only scale radiance -- the
        // attenuation / pdf factor and the pdfs' magnitudes -- are formed with
        // fewer divisions than the reference's expressions; everything a
        // decision reads -- directions, t, the sign of pdf_val -- is the
        // reference's own arithmetic.  See RTW_RADIANCE_FAST below.)
        // onb::build_from_w(normal) (onb.h:32-38), built where it is used
        const surf_frame sf{n, prim, rect, true};
        pf.mark(PS_HIT);
        d3 dir;
        double pdf_val, cosine;
        if (LIGHTS || (!NOLIGHTS && S.n_lights > 0)) {  // mixture_pdf(cosine_pdf, hittable_pdf(lights)) pdf.h:55-79
            dir = mixture_generate(S, sf, p, rng);
            pf.mark(PS_SAMPLE);
            // both cosines before the light pdfs, so the normal and the frame
            // are dead while those run (the values are what the reference
            // computes after them)
            const d3 ud = normalize(dir);
            const double cw = dot(ud, frame_w(S, sf));
            cosine = dot(n, ud);  // material.h:115-119
            const double p0 = (cw <= 0) ? 0 : (RTW_RADIANCE_FAST ? cw * kInvPi : cw / kPi);
            pdf_val = 0.5 * p0 + 0.5 * lights_pdf_value<STATIC>(S, p, dir);
        } else {
            dir = local(frame_onb(S, sf), random_cosine_direction(rng));
            const d3 ud = normalize(dir);
            const double cw = dot(ud, frame_w(S, sf));
            cosine = dot(n, ud);  // material.h:115-119
            pdf_val = (cw <= 0) ? 0 : (RTW_RADIANCE_FAST ? cw * kInvPi : cw / kPi);
        }
        if (pdf_val <= 0.0) {  // :126-127 returns emitted (= 0)
            sk.end_zero();
            return SEG_END_ZERO;
        }
        pf.mark(PS_PDF);
        // attenuation = texture value (material.h:98), read only now: it
        // draws nothing, and a late read keeps it out of the busiest registers
#if RTW_RADIANCE_FAST
        // attenuation * scattering_pdf / pdf_val as one scalar quotient
        const double w = cosine < 0 ? 0 : rad_div(cosine, kPi * pdf_val);
        return scatter(texture_value<M>(S, m.texture, p) * w, p, dir);
#elif RTW_STRICT_RADIANCE
        // the reference's ((attenuation * scattering_pdf) * color) / pdf_val
        // (RayTracingWeekend.cpp:129-132): m and pdf_val go to the path's
        // factor log; the fold applies them around the returned color
        const double spdf = cosine < 0 ? 0 : cosine / kPi;
        if (depth <= 1) {
            sk.end_zero();
            return SEG_END_ZERO;
        }
        sk.cont_mp(texture_value<M>(S, m.texture, p) * spdf, pdf_val, ray{p, dir, r.t});
        x.rng = rng;
        x.depth = depth - 1;
        return SEG_CONTINUE;
#else
        const double spdf = cosine < 0 ? 0 : cosine / kPi;
        return scatter((texture_value<M>(S, m.texture, p) * spdf) / pdf_val, p, dir);
#endif
    }
}

// The wavefront form: path x (read from pool slot i or, fresh, from staging)
// -> shade_core -> continuation written back to slot i (no longer fresh).
template <int M>
__device__ __forceinline__ bool shade_one(const scene& S, const job_t& J, const paths_t& P, const fresh_t& FR,
                                          uint32_t i, const path_in& x, uint32_t rng, double t, int32_t prim, d3& L,
                                          uint32_t& q, prof_t& pf) {
    path_st s;
    s.r = x.r;
    s.rng = rng;
    s.depth = x.fresh ? (uint32_t)J.max_depth : x.depth;
    s.q = x.fresh ? FR.qid[x.src] : P.qid[i];
    q = s.q;
    seg_out so;
    const int out = shade_core<M>(S, s, t, prim, so, pf);
    const d3 w = so.w;
    const ray nr = so.next;
    const d3 thr = x.fresh ? d3{1.0, 1.0, 1.0} : d3{P.tr[i], P.tg[i], P.tb[i]};
    if (out == SEG_END) {
        L = thr * w;
        return true;
    }
    if (out == SEG_END_ZERO) {
        L = thr * 0.0;  // (NaN / inf throughputs give NaN, as the reference's products do)
        return true;
    }
    const d3 nt = thr * w;
    P.ox[i] = nr.o.x, P.oy[i] = nr.o.y, P.oz[i] = nr.o.z;
    P.dx[i] = nr.d.x, P.dy[i] = nr.d.y, P.dz[i] = nr.d.z;
    P.tm[i] = nr.t;
    P.tr[i] = nt.x, P.tg[i] = nt.y, P.tb[i] = nt.z;
    P.rng[i] = s.rng;
    P.depth[i] = s.depth;
    P.qid[i] = s.q;
    return false;
}

// Re-point a scene's shading arrays into an LDS copy of its prefix.
__device__ __forceinline__ scene lds_scene(const scene& S, const char* base, const char* lds) {
    scene L = S;
    auto rb = [&](const void* p) -> const void* { return p ? (const void*)(lds + ((const char*)p - base)) : nullptr; };
    L.prims = (const rtw_prim*)rb(S.prims);
    L.entries = (const dev_entry*)rb(S.entries);
    L.ops = (const dev_op*)rb(S.ops);
    L.materials = (const rtw_material*)rb(S.materials);
    L.textures = (const rtw_texture*)rb(S.textures);
    L.lights = (const rtw_light*)rb(S.lights);
    L.ranvec = (const double*)rb(S.ranvec);
    L.perm = (const int32_t*)rb(S.perm);
    L.media = (const int32_t*)rb(S.media);
    L.prim_onb = (const double*)rb(S.prim_onb);
    L.mat_aux = (const double*)rb(S.mat_aux);
    return L;
}

// Shade every live path; a path that ends stores its radiance in its sample's
// slot of the radiance buffer (one 24-byte record) and empties its pool slot.
// With LDS, a small scene's shading data (prims .. media, `bytes` from `base`)
// is staged in LDS once per block: the dependent chain hit -> primitive ->
// entry -> material -> texture is then LDS latency, not L2 latency.
template <int M, bool LDS>
__global__ __launch_bounds__(kBlock) void k_shade(scene S, job_t J, paths_t P, fresh_t FR,
                                                  const double* __restrict__ ht, const int32_t* __restrict__ hid,
                                                  ctrs_t* C, const char* base, uint32_t bytes) {
    extern __shared__ __attribute__((aligned(16))) char s_scene[];
    if (LDS) {
        const uint4* src = reinterpret_cast<const uint4*>(base);
        uint4* dst = reinterpret_cast<uint4*>(s_scene);
        for (uint32_t k = threadIdx.x; k < bytes / 16; k += kBlock) dst[k] = src[k];
        __syncthreads();
    }
    const scene SS = LDS ? lds_scene(S, base, s_scene) : S;
    const uint32_t n = C->n;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const uint32_t dw = P.depth[i];
        if (dw == 0) continue;
        d3 L;
        uint32_t q;
        const path_in x = load_ray(P, FR, i, dw);
        const uint32_t rng = x.fresh ? FR.rng[x.src] : P.rng[i];
        prof_t pf;
        if (shade_one<M>(SS, J, P, FR, i, x, rng, ht[i], hid[i], L, q, pf)) {
            double* o = J.L + 3 * (size_t)q;
            store_record(o, L.x, L.y, L.z);
            P.depth[i] = 0;
        }
    }
}

// Fused segment: traversal + shading of each live path in one pass over the
// pool (the ray is read once; no hit records go through HBM).  Same results
// as k_intersect followed by k_shade.
#ifdef RTW_SEG_WAVES  // occupancy experiments: cap registers for N waves per SIMD
#define RTW_SEG_ATTR __attribute__((amdgpu_waves_per_eu(RTW_SEG_WAVES)))
#else
#define RTW_SEG_ATTR
#endif
template <int F, int M, bool LDS>
__global__ __launch_bounds__(kBlock) RTW_SEG_ATTR void k_segment(scene S, job_t J, paths_t P, fresh_t FR, ctrs_t* C,
                                                    const char* base, uint32_t bytes) {
    extern __shared__ __attribute__((aligned(16))) char s_scene[];
    __shared__ uint32_t s_cnt[kWaves];
    if (LDS) {
        const uint4* src = reinterpret_cast<const uint4*>(base);
        uint4* dst = reinterpret_cast<uint4*>(s_scene);
        for (uint32_t k = threadIdx.x; k < bytes / 16; k += kBlock) dst[k] = src[k];
        __syncthreads();
    }
    const scene SS = LDS ? lds_scene(S, base, s_scene) : S;
    const uint32_t n = C->n;
    uint32_t live = 0;
    prof_t pf;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const uint32_t dw = P.depth[i];
        if (dw == 0) continue;
        pf.mark(PS_LOOP);
        const path_in x = load_ray(P, FR, i, dw);
        uint32_t rng = x.fresh ? FR.rng[x.src] : P.rng[i];
        pf.mark(PS_LOAD);
        const hit_state h = world_closest<F>(S, x.r, rng);
        pf.mark(PS_TRAVERSE);
        ++live;
        d3 L;
        uint32_t q;
        if (shade_one<M>(SS, J, P, FR, i, x, rng, h.t, h.prim, L, q, pf)) {
            double* o = J.L + 3 * (size_t)q;
            store_record(o, L.x, L.y, L.z);
            P.depth[i] = 0;
        }
        pf.mark(PS_STORE);
    }
    pf.flush();
    for (int off = 32; off > 0; off >>= 1) live += __shfl_down(live, off, 64);
    if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = live;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int k = 0; k < kWaves; ++k) t += s_cnt[k];
        if (t) atomicAdd(&C->segments[blockIdx.x % 8].v, t);
    }
}

// Persistent form: every lane keeps its path in registers and runs it to the
// end, then takes the next camera sample -- one launch per pass, no path
// state through HBM, no regeneration or compaction launches.
//
// Camera rays are made in batches of 64, one per lane (ray-gen never runs
// for just the few lanes whose paths ended this iteration): a wave reserves
// 64 consecutive sample ids of its queue shard with ONE atomic (neighbouring
// ids are neighbouring pixels; other shards are stolen from once its own is
// dry), every lane generates one ray into the wave's LDS buffer, and idle
// lanes pop rays from that buffer.  A wave exits when the queue is exhausted,
// its buffer is empty and its last path has ended.
// Camera samples a wave generates at once into its batch: 64, lane-full ray
// generation.
constexpr int kPBatch = 64;
// PIN (F_PIN): the origins are the camera's, read from the camera where a
// sample is popped instead of stored per entry -- 24 B x 64 per wave less LDS
// (24 KB per 1 024-thread workgroup), which the BVH node packet takes.
template <int NB, bool PIN = false>
struct ray_batch_t {  // one wave's buffer of generated camera samples (LDS)
    double ox[PIN ? 1 : NB], oy[PIN ? 1 : NB], oz[PIN ? 1 : NB];
    double dx[NB], dy[NB], dz[NB], tm[NB];
    uint32_t rng[NB], q[NB];
};

// the camera's origin (F_PIN batches), scalar loads through an opaque
// pointer as in camera_sample
__device__ __forceinline__ d3 camera_origin(const job_t& J) {
    const rtw_camera_desc* cp = J.cam;
    asm volatile("" : "+s"(cp));
    return d3{ld(&cp->origin[0]), ld(&cp->origin[1]), ld(&cp->origin[2])};
}
// F_PIN applies to a render whose camera makes every ray at its origin: no
// lens, no zero origin coordinate, and finite u, v (a non-finite u or v --
// vup parallel to the view direction makes u = unit_vector(0) = NaN -- gives
// the reference a NaN offset and NaN rays, camera.h:36-50)
inline bool camera_is_pinhole(const rtw_camera_desc& c) {
    bool uv = true;
    for (int k = 0; k < 3; ++k) uv = uv && std::isfinite(c.u[k]) && std::isfinite(c.v[k]);
    return c.lens_radius == 0.0 && c.origin[0] != 0.0 && c.origin[1] != 0.0 && c.origin[2] != 0.0 && uv;
}

// Occupancy: left alone the compiler gives k_persist 160-230 VGPRs (2-3
// waves per SIMD).  Capping at 128 (4 waves) costs some spilled registers and
// wins: 2 638 -> 2 980 Msamples/s on Cornell (5 waves spilled too much then).
// The scene-specialised list kernels (F_BLACK: Cornell; F_YSPH with the
// Book-1 material set: random_balls) are lean enough for 5 waves (96 VGPRs):
// Cornell +4.5 %, random_balls flat +6.8 %; the BVH and all-feature kernels
// lose 7-24 % at 5 and keep 4.
#ifdef RTW_SEG_WAVES
#define RTW_PERSIST_WAVES(F, M) RTW_SEG_WAVES
#else
#define RTW_PERSIST_WAVES(F, M)                                                                        \
    ((((F) & F_BLACK) && !((F) & (F_MEDIA | F_WBVH | F_GBVH))) || (((F) & F_YSPH) && (M) != SF_ALL) ? 5 : 4)
#endif
// The persistent kernels' one argument.
struct persist_args {
    scene S;
    job_t J;
    ctrs_t* C;
    const char* base;  // the scene allocation; its shading prefix is staged in LDS
    uint32_t bytes;    // bytes of that prefix
    uint32_t lds_nodes;      // BVH node packet: the top nodes staged in LDS (k_persist, LST)
    uint32_t lds_nodes_off;  // its byte offset in the dynamic LDS (after the prefix)
};

// The persistent kernels' argument, re-read from the kernarg segment (scalar
// loads through the scalar cache) by each phase of a loop iteration that
// uses it.  Read once, every scene / job field a persistent loop touches is
// hoisted into registers held across the whole loop -- some 80 SGPRs, far
// past the 106 a wave has, so they spill into VGPR lanes and push the paths'
// own registers out to scratch.  The opaque copy of the segment pointer stops
// that hoisting: each phase loads what it uses and lets it go.
__device__ __forceinline__ const persist_args& args_now() {
    cptr<persist_args> p = (cptr<persist_args>)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const persist_args*)p;
}

// LST: BVH traversal stacks in LDS (one column per lane) instead of scratch.
// The loop-carried ray stays in registers: every form that parked it in LDS
// (the whole ray with lane-direct camera samples, or its origin beside
// smaller batches) took that LDS from the node packet or the batches and
// measured slower than the spills it removed (EXPERIMENTS.md).
template <int F, int M, bool LDS, bool LST = false>
__global__ __launch_bounds__(kPBlock) __attribute__((amdgpu_waves_per_eu(RTW_PERSIST_WAVES(F, M))))
void k_persist(persist_args) {
    constexpr int NB = kPBatch;
    constexpr bool PIN = (F & F_PIN) != 0;
    extern __shared__ __attribute__((aligned(16))) char s_scene[];
    __shared__ uint32_t s_cnt[kPWaves];
    __shared__ ray_batch_t<NB, PIN> s_batch[kPWaves];
    __shared__ double s_thr[3][kPBlock];  // each lane's path throughput
    __shared__ uint16_t s_stack[LST ? kLdsStack : 1][kPBlock];
    __shared__ uint32_t s_q[kPBlock];     // each lane's sample id
    if (LDS) {
        const persist_args& A = args_now();
        const uint4* src = reinterpret_cast<const uint4*>(A.base);
        uint4* dst = reinterpret_cast<uint4*>(s_scene);
        for (uint32_t k = threadIdx.x; k < A.bytes / 16; k += kPBlock) dst[k] = src[k];
    }
    if (LST) {  // the BVH node packet (the top levels of every tree)
        const persist_args& A = args_now();
        const uint4* src = reinterpret_cast<const uint4*>(A.S.nodes);
        uint4* dst = reinterpret_cast<uint4*>(s_scene + A.lds_nodes_off);
        constexpr uint32_t kNode16 = (uint32_t)(sizeof(node_store) / 16);
        for (uint32_t k = threadIdx.x; k < A.lds_nodes * kNode16; k += kPBlock) dst[k] = src[k];
    }
    if (LDS || LST) __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const int own = blockIdx.x % kQShards;
    path_st x;
    x.depth = 0;
    bool open = true;      // wave-uniform: the queue may still hold samples
    uint32_t bl = 0, bh = 0;  // wave-uniform: unread batch entries [bl, bh)
    uint32_t segs = 0;
    prof_t pf;
    for (;;) {
        // lane-dependent LDS addresses (batch, throughput, sample id, stack
        // columns) are formed from an opaque copy of the thread index where
        // they are used: left to itself the compiler hoists one VGPR per
        // array out of the loop (C5's kernel: 65 of them)
        uint32_t tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const uint32_t ln = tid & 63;
        {
            // (the wave's batch too: formed once per kernel, its per-array
            // addresses were held in 15 VGPRs across the whole loop)
            ray_batch_t<NB, PIN>& B = s_batch[tid >> 6];
            for (int round = 0; round < 2; ++round) {
                const unsigned long long m = __ballot(x.depth == 0);
                if (!m) break;
                if (bl == bh) {
                    if (!open) break;
                    const persist_args& A = args_now();
                    const job_t& J = A.J;
                    ctrs_t* const C = A.C;
                    // reserve up to NB ids, own shard first
                    uint32_t left = NB, given = 0, q = 0;
                    bool got = false;
                    for (int a = 0; a < kQShards && left; ++a) {
                        const int sh = (own + a) % kQShards;
                        const unsigned long long lim = shard_limit(sh, J.total);
                        unsigned long long b = ~0ull;
                        if (ln == 0) {
                            const bool dry = a > 0 && __hip_atomic_load(&C->qshard[sh].v, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_AGENT) >= lim;
                            if (!dry) b = atomicAdd(&C->qshard[sh].v, (unsigned long long)left);
                        }
                        b = __shfl(b, 0, 64);
                        if (b == ~0ull || b >= lim) continue;
                        const uint32_t ok = (uint32_t)min((unsigned long long)left, lim - b);
                        if (ln >= given && ln < given + ok) {
                            q = (uint32_t)shard_sample(sh, b + (ln - given));
                            got = true;
                        }
                        given += ok;
                        left -= ok;
                    }
                    if (left) open = false;
                    if (got) {  // (lanes >= NB get no id)
                        uint32_t rng;
                        const ray r = camera_sample<false>(J, q, rng);
                        if constexpr (!PIN) B.ox[ln] = r.o.x, B.oy[ln] = r.o.y, B.oz[ln] = r.o.z;
                        B.dx[ln] = r.d.x, B.dy[ln] = r.d.y, B.dz[ln] = r.d.z;
                        B.tm[ln] = r.t;
                        B.rng[ln] = rng;
                        B.q[ln] = q;
                    }
                    bl = 0;
                    bh = given;
                    if (!bh) break;
                    __builtin_amdgcn_wave_barrier();
                }
                const uint32_t rank = (uint32_t)__popcll(m & lanemask_lt());
                const uint32_t avail = bh - bl;
                if (x.depth == 0 && rank < avail) {
                    const uint32_t k = bl + rank;
                    const d3 o = PIN ? camera_origin(args_now().J) : d3{B.ox[k], B.oy[k], B.oz[k]};
                    x.r = ray{o, d3{B.dx[k], B.dy[k], B.dz[k]}, B.tm[k]};
                    x.rng = B.rng[k];
                    s_q[tid] = B.q[k];
                    s_thr[0][tid] = 1.0, s_thr[1][tid] = 1.0, s_thr[2][tid] = 1.0;
                    x.depth = (uint32_t)args_now().J.max_depth;
                }
                bl += min((uint32_t)__popcll(m), avail);
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (!__any(x.depth != 0)) break;
        pf.mark(PS_LOAD);
        if (x.depth != 0) {
            const persist_args& A = args_now();
            scene S = A.S;
            hit_state h;
            if constexpr (LST) {
                S.lnodes = reinterpret_cast<const node_store*>(s_scene + A.lds_nodes_off);
                S.n_lnodes = (int32_t)A.lds_nodes;
                lds_stack stk{&s_stack[0][tid]};
                h = world_closest<F>(S, x.r, x.rng, stk);
            } else {
                h = world_closest<F>(S, x.r, x.rng);
            }
            pf.mark(PS_TRAVERSE);
            ++segs;
            const persist_args& A2 = args_now();
            const scene SS = LDS ? lds_scene(A2.S, A2.base, s_scene) : A2.S;
#ifdef RTW_PROF
            pf.classify(h.prim == -1 ? 0
                        : 1 + SS.materials[h.prim <= -2 ? SS.entries[-h.prim - 2].phase_material
                                                        : SS.prims[h.prim].material].type);
#endif
            // the outcome is applied inside the branch that produced it
            uint32_t me = tid;
            auto radiance = [&](const d3& L) {
                double* o = A2.J.L + 3 * (size_t)s_q[me];
                store_record(o, L.x, L.y, L.z);
            };
            ray nr;
#if RTW_STRICT_RADIANCE
            // the path's factors in its thread's log, folded inside-out at its
            // end: c = E, then c = (m_k * c) / pdf_k for k = last .. 0 -- the
            // returns of the recursive color() (RayTracingWeekend.cpp:107,
            // 129-132; emitted of a scattering material is 0 and 0 + c == c),
            // specular bounces logged with pdf 1 (x / 1 == x)
            const uint32_t kb = (uint32_t)A2.J.max_depth - x.depth;  // this segment's bounce
            const size_t gth = (size_t)blockIdx.x * kPBlock + tid;
            double* const flog = A2.J.flog;
            const size_t nth = A2.J.flog_threads;
            auto log_factor = [&](const d3& m, double pdf, const ray& r) {
                double* e = flog + 4 * ((size_t)kb * nth + gth);
                e[0] = m.x, e[1] = m.y, e[2] = m.z, e[3] = pdf;
                nr = r;
            };
            auto fold = [&](d3 c) {
                for (int k = (int)kb - 1; k >= 0; --k) {
                    const double* e = flog + 4 * ((size_t)k * nth + gth);
                    c = (d3{e[0], e[1], e[2]} * c) / e[3];
                }
                radiance(c);
            };
            auto sk = make_sink4([&](const d3& f, const ray& r) { log_factor(f, 1.0, r); },
                                 [&](const d3& m, double pdf, const ray& r) { log_factor(m, pdf, r); },
                                 [&](const d3& E) { fold(E); }, [&]() { fold(d3{0.0, 0.0, 0.0}); });
#else
            auto sk = make_sink(
                [&](const d3& f, const ray& r) {
                    s_thr[0][me] *= f.x, s_thr[1][me] *= f.y, s_thr[2][me] *= f.z;
                    nr = r;
                },
                [&](const d3& E) { radiance(d3{s_thr[0][me], s_thr[1][me], s_thr[2][me]} * E); },
                [&]() {
                    // thr * 0, not 0: the reference multiplies its factors into
                    // the 0 color() returns, so a non-finite throughput gives NaN
                    const double z = in_place<0>();
                    radiance(d3{s_thr[0][me], s_thr[1][me], s_thr[2][me]} * z);
                });
#endif
            const int out = shade_core<M, (F & F_STATIC) != 0, (F & F_LIGHTS) != 0, (F & F_BLACK) != 0,
                                       (F & F_NOLIGHTS) != 0>(SS, x, h.t, h.prim, sk, pf);
            if (out != SEG_CONTINUE)
                x.depth = 0;
            else
                x.r = nr;
            pf.mark(PS_STORE);
        }
    }
    pf.flush();
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_down(segs, off, 64);
    if (lane == 0) s_cnt[threadIdx.x >> 6] = segs;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int k = 0; k < kPWaves; ++k) t += s_cnt[k];
        if (t) atomicAdd(&args_now().C->segments[blockIdx.x % 8].v, t);
    }
}

// Persistent form with material regrouping.  A wave pays for every shading
// branch one of its lanes takes; on Cornell about half the lanes shade
// lambertian, 30 % dielectric, 20 % emit or miss, and every wave carries all
// of them.  Here, after each traversal, the block's 256 paths are sorted by
// what their hit needs (lambertian, dielectric, metal, isotropic, emitter,
// miss, idle) with a counting sort over wave ballots and moved through LDS
// to the lane of their rank, so most waves run one branch.  Idle lanes end
// up together at the top of the block: they take fresh camera samples
// there, so ray generation also runs nearly lane-full.
// The keys' order is the order of the sorted block: material order, the
// path-ending keys (emitter, miss) last.  The paths that end are the lanes
// that take camera samples next: they sit together at the block's top,
// beside the idle ones, so ray generation runs lane-full in one or two waves.
// (Cheap keys between the expensive ones measured T -7 %, and sorting
// lambertian hits on their mixture choice T -1 %: EXPERIMENTS.md.)
enum { K_LAMB = 0, K_DIEL, K_METAL, K_ISO, K_EMIT, K_MISS, K_IDLE, K_N };

// Ray generation threshold: a wave takes camera samples only when at least
// this many of its lanes are idle.  After shading a few lambertian paths per
// wave end (pdf <= 0, depth), and a wave would run a whole camera_sample
// (~150 VALU) for one to three lanes; with fewer than K idle lanes the slots
// wait one iteration, are sorted to the block's top with the other idle
// records (K_IDLE) and refill there, lane-full.  A block always ends with
// every wave fully idle, so the queue still drains.  Measured (1 MI355X,
// A/B, profiles/r03/ab_refill_min.log): K = 8 T +0.45 %, C2 +0.8 %; K = 24
// T +0.2 %, C2 -0.7 %.
#ifndef RTW_REFILL_MIN
#define RTW_REFILL_MIN 8
#endif
// Paths regrouped together (one workgroup).  (128 or 512 measured T -15 % /
// -13 %, EXPERIMENTS.md.)
constexpr int kSortBlock = 256;
constexpr int kSortWaves = kSortBlock / 64;
// The counting sort's block prefix from a key-major
// count table s_kc[key][wave] (kKeySlots x 4; slots of keys the scene cannot
// produce stay zero): lane k < 8 of every wave reads key k's four per-wave
// counts in one 16-B LDS read and forms their total and the count in the
// waves before its own; an exclusive scan of the totals over lanes 0..7
// (three DPP row shifts) adds the paths of every key before k; each lane
// fetches its own key's base with one ds_bpermute.  The plain form has every
// lane read all 4 x K_N counts and sum them under selects (~67 VALU per
// wave-iteration on T); measured T +3.0 %, T fp32 +4.8 %
// (profiles/r05/ab_r5l_sort_dpp.log).
constexpr int kKeySlots = 8;
__device__ __forceinline__ uint32_t sort_base_dpp(const uint32_t (*s_kc)[4], uint32_t lane, uint32_t wave, int key,
                                                  int k_idle, uint32_t& idle_total) {
    const uint4 c = *reinterpret_cast<const uint4*>(s_kc[lane & (kKeySlots - 1)]);
    const uint32_t tot = c.x + c.y + c.z + c.w;
    const uint32_t before = (wave > 0 ? c.x : 0u) + (wave > 1 ? c.y : 0u) + (wave > 2 ? c.z : 0u);
    uint32_t incl = tot;  // inclusive scan over lanes 0..7 (row_shr:1, 2, 4; lanes without a source add 0)
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x111, 0xF, 0xF, true);
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x112, 0xF, 0xF, true);
    incl += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x114, 0xF, 0xF, true);
    const uint32_t base = incl - tot + before;
    idle_total = (uint32_t)__builtin_amdgcn_readlane((int)tot, k_idle);
    return (uint32_t)__builtin_amdgcn_ds_bpermute(key << 2, (int)base);
}
static_assert(kSortWaves == 4 && K_N <= kKeySlots, "sort_base_dpp: 256-thread sort blocks, at most 8 keys");
template <int F, int M, bool LDS>
__global__ __launch_bounds__(kSortBlock) __attribute__((amdgpu_waves_per_eu(RTW_PERSIST_WAVES(F, M))))
void k_persist_sort(persist_args) {
    extern __shared__ __attribute__((aligned(16))) char s_scene[];
    __shared__ __attribute__((aligned(16))) uint32_t s_kc[kKeySlots][kSortWaves];  // per key, lanes per wave
    if (threadIdx.x < kKeySlots * kSortWaves) (&s_kc[0][0])[threadIdx.x] = 0u;  // (before the barrier below)
    __shared__ uint32_t s_seg[kSortWaves];
    // the exchange: one path per slot (SoA)
    __shared__ double x_o[3][kSortBlock], x_d[3][kSortBlock], x_tm[kSortBlock], x_t[kSortBlock];
    __shared__ int32_t x_prim[kSortBlock];
    __shared__ uint32_t x_rng[kSortBlock], x_depth[kSortBlock], x_q[kSortBlock], x_home[kSortBlock];
    // the record's ray in slot `s`
    auto ray_at = [&](uint32_t s) {
        return ray{d3{x_o[0][s], x_o[1][s], x_o[2][s]}, d3{x_d[0][s], x_d[1][s], x_d[2][s]},
                   (F & F_STATIC) ? 0.0 : x_tm[s]};
    };
    auto put_ray = [&](uint32_t s, const ray& r) {
        x_o[0][s] = r.o.x, x_o[1][s] = r.o.y, x_o[2][s] = r.o.z;
        x_d[0][s] = r.d.x, x_d[1][s] = r.d.y, x_d[2][s] = r.d.z;
        if constexpr (!(F & F_STATIC)) x_tm[s] = r.t;
    };
    // Path throughputs stay put: each path record (live or idle) owns one
    // home slot of s_thr and carries its index through the exchange, so the
    // throughput is read and written only where shading uses it and is never
    // held in registers across traversal and sort.  A lane whose path ended
    // keeps the record's slot for the camera sample it takes next.
    __shared__ double s_thr[3][kSortBlock];
    // Between iterations a lane's path record sits in its own exchange slot
    // (ray, home index, sample id at [tid]); only the engine and the depth
    // are loop-carried registers.  A loop-carried ray would hold 12 VGPRs
    // through every shading branch (exec-masked branches run one after the
    // other, so a value live into any of them is live across all) -- that
    // is what pushed this kernel past 96 VGPRs into scratch.
    x_home[threadIdx.x] = threadIdx.x;
    if (LDS) {
        const persist_args& A = args_now();
        const uint4* src = reinterpret_cast<const uint4*>(A.base);
        uint4* dst = reinterpret_cast<uint4*>(s_scene);
        for (uint32_t k = threadIdx.x; k < A.bytes / 16; k += kSortBlock) dst[k] = src[k];
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int own = blockIdx.x % kQShards;
    path_st x;
    x.depth = 0;
    bool open = true;  // wave-uniform: the queue may still hold samples
    uint32_t segs = 0;
    prof_t pk;  // section profiler (RTW_PROF builds): refill, traverse, sort, exchange, shade
    for (;;) {
        // 1. idle lanes take new camera samples (one reservation per wave)
        {
            const bool idle = x.depth == 0;
            const unsigned long long m = __ballot(idle);
            if (open && __popcll(m) >= RTW_REFILL_MIN) {
                const persist_args& A = args_now();
                const job_t& J = A.J;
                ctrs_t* const C = A.C;
                const uint32_t want = (uint32_t)__popcll(m);
                const uint32_t rank = (uint32_t)__popcll(m & lanemask_lt());
                uint32_t left = want, given = 0, q = 0;
                bool got = false;
                for (int a = 0; a < kQShards && left; ++a) {
                    const int sh = (own + a) % kQShards;
                    const unsigned long long lim = shard_limit(sh, J.total);
                    unsigned long long b = ~0ull;
                    if (lane == 0) {
                        const bool dry = a > 0 && __hip_atomic_load(&C->qshard[sh].v, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT) >= lim;
                        if (!dry) b = atomicAdd(&C->qshard[sh].v, (unsigned long long)left);
                    }
                    b = __shfl(b, 0, 64);
                    if (b == ~0ull || b >= lim) continue;
                    const uint32_t ok = (uint32_t)min((unsigned long long)left, lim - b);
                    if (idle && rank >= given && rank < given + ok) {
                        q = (uint32_t)shard_sample(sh, b + (rank - given));
                        got = true;
                    }
                    given += ok;
                    left -= ok;
                }
                if (left) open = false;
                if (got) {
                    const ray r = camera_sample(J, q, x.rng);
                    const uint32_t me = threadIdx.x;
                    const uint32_t home = x_home[me];
                    put_ray(me, r);  // (F_STATIC: the time is never read)
                    x_q[me] = q;
                    x.depth = (uint32_t)J.max_depth;
                    s_thr[0][home] = 1.0, s_thr[1][home] = 1.0, s_thr[2][home] = 1.0;
                }
            }
        }
        pk.mark(PS_LOAD);
        // 2. traversal
        double th = 0.0;
        int32_t hp = -1;
        int key = K_IDLE;
        if (x.depth != 0) {
            const uint32_t me = threadIdx.x;
            x.r = ray_at(me);
            const persist_args& A = args_now();
            const scene SS = LDS ? lds_scene(A.S, A.base, s_scene) : A.S;
            const hit_state h = world_closest<F>(A.S, x.r, x.rng);
            ++segs;
            th = h.t;
            hp = h.prim;
            if (hp == -1) {
                key = K_MISS;
            } else {
                const int mat = hp <= -2 ? SS.entries[-hp - 2].phase_material : SS.prims[hp].material;
                const int ty = SS.materials[mat].type;
                key = ty == RTW_MAT_LAMBERTIAN ? K_LAMB
                      : ty == RTW_MAT_DIELECTRIC ? K_DIEL
                      : ty == RTW_MAT_METAL ? K_METAL
                      : ty == RTW_MAT_ISOTROPIC ? K_ISO
                                                : K_EMIT;
            }
        }
        pk.mark(PS_TRAVERSE);
        // 3. counting sort of the block's paths by key (the record's home and
        // sample id are read from the lane's own slot before the barrier that
        // precedes the exchange's writes)
        const uint32_t my_home = x_home[threadIdx.x], my_q = x_q[threadIdx.x];
        uint32_t rank_in_wave = 0;
        // keys the scene's material set cannot produce are skipped (their
        // counts stay 0; keep s_kc's slots zero for the prefix below)
        constexpr auto key_used = [](int k) {
            return !((k == K_METAL && !(M & SF_METAL)) || (k == K_ISO && !(M & SF_ISO)));
        };
#pragma unroll
        for (int k = 0; k < K_N; ++k) {
            if (!key_used(k)) continue;
            const unsigned long long m = __ballot(key == k);
            if (key == k) rank_in_wave = (uint32_t)__popcll(m & lanemask_lt());
            if (lane == 0) s_kc[k][wave] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        uint32_t idle_total;
        const uint32_t dst = rank_in_wave + sort_base_dpp(s_kc, lane, wave, key, K_IDLE, idle_total);
        if (idle_total == kSortBlock) break;  // block-uniform: nothing left to trace or take
        pk.mark(PS_HIT);
        // 4. move every path to the slot of its rank (an idle record's ray
        // is garbage and stays behind)
        if (x.depth != 0) put_ray(dst, x.r);
        x_home[dst] = my_home;
        x_t[dst] = th;
        x_prim[dst] = hp;
        x_rng[dst] = x.rng;
        x_depth[dst] = x.depth;
        x_q[dst] = my_q;
        __syncthreads();
        // (opaque, so the exchange's per-lane LDS addresses are formed here
        // from one register, not hoisted out of the loop one per array)
        uint32_t me = threadIdx.x;
        asm volatile("" : "+v"(me));
        x.rng = x_rng[me];
        x.depth = x_depth[me];
        pk.mark(PS_SAMPLE);
        // 5. shading, now mostly one branch per wave
        if (x.depth != 0) {
            x.r = ray_at(me);
            const persist_args& A = args_now();
            const scene SS = LDS ? lds_scene(A.S, A.base, s_scene) : A.S;
            prof_t pf;
            // the outcome is applied inside the branch that produced it
            auto radiance = [&](const d3& L) {
                double* o = A.J.L + 3 * (size_t)x_q[me];
                store_record(o, L.x, L.y, L.z);
            };
            auto sk = make_sink(
                [&](const d3& f, const ray& nr) {
                    const uint32_t home = x_home[me];
                    s_thr[0][home] *= f.x, s_thr[1][home] *= f.y, s_thr[2][home] *= f.z;
                    // the continuation ray waits in the lane's own slot
                    put_ray(me, nr);
                },
                [&](const d3& E) {
                    const uint32_t home = x_home[me];
                    radiance(d3{s_thr[0][home], s_thr[1][home], s_thr[2][home]} * E);
                },
                [&]() {
                    // thr * 0 (k_persist's reason: NaN / inf throughputs give NaN)
                    const uint32_t home = x_home[me];
                    const double z = in_place<0>();
                    radiance(d3{s_thr[0][home], s_thr[1][home], s_thr[2][home]} * z);
                });
            const int out = shade_core<M, (F & F_STATIC) != 0, (F & F_LIGHTS) != 0, (F & F_BLACK) != 0,
                                       (F & F_NOLIGHTS) != 0>(SS, x, x_t[me], x_prim[me], sk, pf);
            if (out != SEG_CONTINUE) x.depth = 0;
        }
        pk.mark(PS_STORE);
    }
    pk.flush();
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_down(segs, off, 64);
    if (lane == 0) s_seg[wave] = segs;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int k = 0; k < kSortWaves; ++k) t += s_seg[k];
        if (t) atomicAdd(&args_now().C->segments[blockIdx.x % 8].v, t);
    }
}

// ----------------------------------------------------------------------
// fp32 fast mode (RTW_PRECISION_FP32, rtw_fast.h): the persistent form with
// every lane's path in registers -- ray, throughput, engine, depth, sample
// id -- and camera samples taken by idle lanes (one queue reservation per
// wave).  Waves run independently (no block barrier in the loop), so a wave
// leaves as soon as the queue is dry and its last path has ended.
// The fast mode's per-sample radiance record: 12 B of fp32 (k_reduce<float>
// sums it in double in sample order, as it sums fp64 records).
__device__ __forceinline__ void store_record_f32(double* L, uint32_t q, float x, float y, float z) {
    float* o = reinterpret_cast<float*>(L) + 3 * (size_t)q;
    store_record(o, x, y, z);
}

struct fast_args {
    rtwf::fscene S;
    job_t J;
    ctrs_t* C;
    rtwf::cam32 cam;
    uint32_t lds_nodes;  // k_fast<.., LST>: BVH node packet (the top nodes) in dynamic LDS
    // k_fast_sort<.., LDS>: each fscene array's byte offset in the LDS copy of
    // the shading prefix, ~0u for one outside it (host-computed: a range test of
    // every pointer at every use, two 64-bit compares, becomes one 32-bit test)
    uint32_t lds_off[9];
};

// fast_args re-read from the kernarg segment by each phase that uses it
// (args_now's reason: hoisted whole, the scene and job fields fill the
// SGPRs and spill into VGPR lanes)
__device__ __forceinline__ const fast_args& fast_args_now() {
    cptr<fast_args> p = (cptr<fast_args>)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const fast_args*)p;
}

// fp32 kernels for scenes without a noise texture (F bit, fast kernels only):
// the marble texture compiled out of shading (rtw_fast.h texture_value)
constexpr int FF_NONOISE = 1 << 12;

// Waves per SIMD of k_fast.  With the node packet, 8 waves in two
// 1 024-thread workgroups per CU (each with a ~48 KB packet) beat 6 waves in
// two 768-thread ones (~56 KB packets, no spills) although the kernel then
// spills ~17 VGPRs: C3 fp32 4 710 vs 4 386, C5 fp32 806 vs 728 Msamples/s;
// one 1 024-thread workgroup at 6 waves (16 waves per CU) 3 350 / 536; 384
// threads at 6 waves 3 602 / 556; no packet at 6 waves (round 3 before it)
// 3 553 / 645 (1 MI355X, A/B, profiles/r03/ab_fp32_packet.log).
#ifndef RTW_FAST_BVH_WAVES
#define RTW_FAST_BVH_WAVES 8
#endif
// The path -- ray, throughput, engine, depth, sample id -- is in registers.
// (Throughput and sample id in LDS home slots halve the media kernel's spill
// stores but take a third of its node packet: -1 %, EXPERIMENTS.md.)
template <int F, bool LST>
__global__ __launch_bounds__(rtwf::fast_block(F)) __attribute__((amdgpu_waves_per_eu(RTW_FAST_BVH_WAVES)))
void k_fast(fast_args) {
    using namespace rtwf;
    constexpr bool NOISE = (F & FF_NONOISE) == 0;
    constexpr int kFB = fast_block(F);
    constexpr int kFW = kFB / 64;
    extern __shared__ __attribute__((aligned(16))) char s_nodes[];
    __shared__ uint16_t s_stack[LST ? fast_stack(F) : 1][kFB];
    __shared__ uint32_t s_cnt[kFW];
    if (LST) {  // the BVH node packet (the top levels of every tree)
        const fast_args& A = fast_args_now();
        const uint4* src = reinterpret_cast<const uint4*>(A.S.nodes);
        uint4* dst = reinterpret_cast<uint4*>(s_nodes);
        for (uint32_t k = threadIdx.x; k < A.lds_nodes * (uint32_t)(sizeof(node_store) / 16); k += kFB)
            dst[k] = src[k];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63;
    const int own = blockIdx.x % kQShards;
    fray r{f3{0, 0, 0}, f3{0, 0, 1}, 0};
    f3 thr{1, 1, 1};
    uint32_t rng = 0, depth = 0, q = 0, segs = 0;
    bool open = true;  // wave-uniform: the queue may still hold samples
    for (;;) {
        // idle lanes take new camera samples (RayTracingWeekend.cpp:227-231)
        const bool idle = depth == 0;
        const unsigned long long m = __ballot(idle);
        if (open && m) {
            const fast_args& A = fast_args_now();
            const uint32_t want = (uint32_t)__popcll(m);
            const uint32_t rank = (uint32_t)__popcll(m & lanemask_lt());
            uint32_t left = want, given = 0, nq = 0;
            bool got = false;
            for (int a = 0; a < kQShards && left; ++a) {
                const int sh = (own + a) % kQShards;
                const unsigned long long lim = shard_limit(sh, A.J.total);
                unsigned long long b = ~0ull;
                if (lane == 0) {
                    const bool dry = a > 0 && __hip_atomic_load(&A.C->qshard[sh].v, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT) >= lim;
                    if (!dry) b = atomicAdd(&A.C->qshard[sh].v, (unsigned long long)left);
                }
                b = __shfl(b, 0, 64);
                if (b == ~0ull || b >= lim) continue;
                const uint32_t ok = (uint32_t)min((unsigned long long)left, lim - b);
                if (idle && rank >= given && rank < given + ok) {
                    nq = (uint32_t)shard_sample(sh, b + (rank - given));
                    got = true;
                }
                given += ok;
                left -= ok;
            }
            if (left) open = false;
            if (got) {
                int i, j, sm;
                sample_coords(A.J, nq, i, j, sm);
                rng = path_seed(A.J.seed_mix, (uint32_t)(j * A.J.nx + i), (uint32_t)sm);
                const float u = ((float)i + u01(rng)) * rcp((float)A.J.nx);
                const float v = ((float)j + u01(rng)) * rcp((float)A.J.ny);
                r = camera_ray(A.cam, u, v, rng);
                thr = f3{1, 1, 1};
                q = nq;
                depth = (uint32_t)A.J.max_depth;
            }
        }
        if (!__any(depth != 0)) break;
        if (depth == 0) continue;
        fhit h;
        if constexpr (LST) {
            lds_stackf_t<kFB, fast_stack(F)> stk{&s_stack[0][threadIdx.x]};
            const fast_args& A = fast_args_now();
            fscene S = A.S;
            S.lnodes = reinterpret_cast<const node_store*>(s_nodes);
            S.n_lnodes = (int32_t)A.lds_nodes;
            h = world_closest<F>(S, r, rng, stk);
        } else {
            priv_stackf stk;
            h = world_closest<F>(fast_args_now().S, r, rng, stk);
        }
        ++segs;
        // one segment of color() (RayTracingWeekend.cpp:52-159)
        const seg_f sg = shade<NOISE>(fast_args_now().S, r, h, rng, depth);
        bool end = !sg.cont;
        f3 L{0, 0, 0};
        if (sg.cont) {
            thr = thr * sg.w;
            r = sg.next;
            --depth;
        } else {
            L = thr * sg.w;
        }
        if (end) {
            store_record_f32(fast_args_now().J.L, q, L.x, L.y, L.z);
            depth = 0;
        }
    }
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_down(segs, off, 64);
    if (lane == 0) s_cnt[threadIdx.x >> 6] = segs;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int k = 0; k < kFW; ++k) t += s_cnt[k];
        if (t) atomicAdd(&fast_args_now().C->segments[blockIdx.x % 8].v, t);
    }
}

// k_fast_sort re-points its scene with the host's offsets
// (fast_args::lds_off) instead of range-testing every pointer at every use --
// two 64-bit compares, a subtract and selects per pointer, twice per
// iteration, on the scalar unit, which the fp32 kernel's issue shares with
// ~840 VALU per wave-segment (~680 SALU).  Measured (1 MI355X, A/B,
// profiles/r05/ab_r5t_fast_lds_off.log; bit-identical, parity_r5t.log):
// T fp32 8 654 vs 8 075 Msamples/s (+7.2 %), T fp64 +-0.  (The same offsets
// for k_persist_sort's lds_scene, whose rebase has no range test, added
// SALU and VALU there: not used.)
__device__ __forceinline__ rtwf::fscene lds_fscene_off(const rtwf::fscene& S, const uint32_t* off, const char* lds) {
    rtwf::fscene L = S;
    auto rb = [&](const void* p, uint32_t o) -> const void* { return o != ~0u ? (const void*)(lds + o) : p; };
    L.prims = (const rtwf::prim32*)rb(S.prims, off[0]);
    L.entries = (const rtwf::ent32*)rb(S.entries, off[1]);
    L.ops = (const rtwf::op32*)rb(S.ops, off[2]);
    L.materials = (const rtwf::mat32*)rb(S.materials, off[3]);
    L.textures = (const rtwf::tex32*)rb(S.textures, off[4]);
    L.lights = (const rtw_light*)rb(S.lights, off[5]);
    L.ranvec = (const float*)rb(S.ranvec, off[6]);
    L.perm = (const int32_t*)rb(S.perm, off[7]);
    L.frames = (const float*)rb(S.frames, off[8]);
    return L;
}

// fp32 fast mode with material regrouping (list scenes, as k_persist_sort
// for fp64): after each traversal the block's 256 paths are counting-sorted
// by what their hit needs and moved through LDS to the lane of their rank,
// so most waves run one shading branch; idle lanes gather at the top and take
// camera samples there.  Paths wait between iterations in their lane's LDS
// slot; throughputs stay in home slots.  LDS: the fp32 scene (when it fits)
// for shading, traversal reads the scene through the scalar cache.
#ifndef RTW_FAST_WAVES
#define RTW_FAST_WAVES 7  // T fp32: 5 601 (4 waves), 6 465 (5), 7 000 (6), 7 136 (7), 6 462 (8): profiles/r03/ab_fp32_sort_waves.log, ab_fp32_sort_waves7.log
#endif
template <int F, bool LDS>
__global__ __launch_bounds__(kSortBlock) __attribute__((amdgpu_waves_per_eu(RTW_FAST_WAVES)))
void k_fast_sort(fast_args, const char* base, uint32_t bytes) {
    using namespace rtwf;
    constexpr bool NOISE = (F & FF_NONOISE) == 0;
    extern __shared__ __attribute__((aligned(16))) char s_scene[];
    static_assert(FK_N <= kKeySlots, "sort_base_dpp: at most 8 keys");
    __shared__ __attribute__((aligned(16))) uint32_t s_kc[kKeySlots][kSortWaves];  // per key, lanes per wave
    if (threadIdx.x < kKeySlots * kSortWaves) (&s_kc[0][0])[threadIdx.x] = 0u;  // (before the barrier below)
    __shared__ uint32_t s_seg[kSortWaves];
    __shared__ float x_o[3][kSortBlock], x_d[3][kSortBlock], x_tm[kSortBlock], x_t[kSortBlock];
    __shared__ int32_t x_prim[kSortBlock];
    __shared__ uint32_t x_rng[kSortBlock], x_depth[kSortBlock], x_q[kSortBlock], x_home[kSortBlock];
    __shared__ float s_thr[3][kSortBlock];
    x_home[threadIdx.x] = threadIdx.x;
    if (LDS) {
        const uint4* src = reinterpret_cast<const uint4*>(base);
        uint4* dst = reinterpret_cast<uint4*>(s_scene);
        for (uint32_t k = threadIdx.x; k < bytes / 16; k += kSortBlock) dst[k] = src[k];
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int own = blockIdx.x % kQShards;
    uint32_t rng = 0, depth = 0, segs = 0;
    bool open = true;  // wave-uniform: the queue may still hold samples
    for (;;) {
        const uint32_t me = threadIdx.x;
        // 1. idle lanes take new camera samples (one reservation per wave)
        {
            const bool idle = depth == 0;
            const unsigned long long m = __ballot(idle);
            if (open && m) {
                const fast_args& A = fast_args_now();
                const uint32_t rank = (uint32_t)__popcll(m & lanemask_lt());
                uint32_t left = (uint32_t)__popcll(m), given = 0, q = 0;
                bool got = false;
                for (int a = 0; a < kQShards && left; ++a) {
                    const int sh = (own + a) % kQShards;
                    const unsigned long long lim = shard_limit(sh, A.J.total);
                    unsigned long long b = ~0ull;
                    if (lane == 0) {
                        const bool dry = a > 0 && __hip_atomic_load(&A.C->qshard[sh].v, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT) >= lim;
                        if (!dry) b = atomicAdd(&A.C->qshard[sh].v, (unsigned long long)left);
                    }
                    b = __shfl(b, 0, 64);
                    if (b == ~0ull || b >= lim) continue;
                    const uint32_t ok = (uint32_t)min((unsigned long long)left, lim - b);
                    if (idle && rank >= given && rank < given + ok) {
                        q = (uint32_t)shard_sample(sh, b + (rank - given));
                        got = true;
                    }
                    given += ok;
                    left -= ok;
                }
                if (left) open = false;
                if (got) {
                    int i, j, sm;
                    sample_coords(A.J, q, i, j, sm);
                    rng = path_seed(A.J.seed_mix, (uint32_t)(j * A.J.nx + i), (uint32_t)sm);
                    const float u = ((float)i + u01(rng)) * rcp((float)A.J.nx);
                    const float v = ((float)j + u01(rng)) * rcp((float)A.J.ny);
                    const fray r = camera_ray(A.cam, u, v, rng);
                    x_o[0][me] = r.o.x, x_o[1][me] = r.o.y, x_o[2][me] = r.o.z;
                    x_d[0][me] = r.d.x, x_d[1][me] = r.d.y, x_d[2][me] = r.d.z;
                    x_tm[me] = r.t;
                    x_q[me] = q;
                    depth = (uint32_t)A.J.max_depth;
                    const uint32_t home = x_home[me];
                    s_thr[0][home] = 1.0f, s_thr[1][home] = 1.0f, s_thr[2][home] = 1.0f;
                }
            }
        }
        // 2. traversal
        fhit h{0.0f, -1, false};
        int key = FK_IDLE;
        fray r;
        if (depth != 0) {
            r = fray{f3{x_o[0][me], x_o[1][me], x_o[2][me]}, f3{x_d[0][me], x_d[1][me], x_d[2][me]}, x_tm[me]};
            priv_stackf stk;
            h = world_closest<F>(fast_args_now().S, r, rng, stk);
            ++segs;
            const fast_args& A = fast_args_now();
            key = hit_key(LDS ? lds_fscene_off(A.S, A.lds_off, s_scene) : A.S, h);
        }
        // 3. counting sort of the block's paths by key
        const uint32_t my_home = x_home[me], my_q = x_q[me];
        uint32_t rank_in_wave = 0;
#pragma unroll
        for (int k = 0; k < FK_N; ++k) {
            const unsigned long long m = __ballot(key == k);
            if (key == k) rank_in_wave = (uint32_t)__popcll(m & lanemask_lt());
            if (lane == 0) s_kc[k][wave] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        uint32_t idle_total;
        const uint32_t dst = rank_in_wave + sort_base_dpp(s_kc, lane, wave, key, FK_IDLE, idle_total);
        if (idle_total == kSortBlock) break;  // block-uniform: nothing left to trace or take
        // 4. move every path to the slot of its rank
        if (depth != 0) {
            x_o[0][dst] = r.o.x, x_o[1][dst] = r.o.y, x_o[2][dst] = r.o.z;
            x_d[0][dst] = r.d.x, x_d[1][dst] = r.d.y, x_d[2][dst] = r.d.z;
            x_tm[dst] = r.t;
        }
        x_home[dst] = my_home;
        x_t[dst] = h.t;
        x_prim[dst] = h.prim;
        x_rng[dst] = rng;
        x_depth[dst] = depth;
        x_q[dst] = my_q;
        __syncthreads();
        rng = x_rng[me];
        depth = x_depth[me];
        // 5. shading, now mostly one branch per wave
        if (depth != 0) {
            const fray rr{f3{x_o[0][me], x_o[1][me], x_o[2][me]}, f3{x_d[0][me], x_d[1][me], x_d[2][me]}, x_tm[me]};
            const fhit hh{x_t[me], x_prim[me], false};
            const fast_args& A = fast_args_now();
            const seg_f sg = shade<NOISE>(LDS ? lds_fscene_off(A.S, A.lds_off, s_scene) : A.S, rr, hh, rng, depth);
            const uint32_t home = x_home[me];
            const f3 thr{s_thr[0][home], s_thr[1][home], s_thr[2][home]};
            if (sg.cont) {
                s_thr[0][home] = thr.x * sg.w.x, s_thr[1][home] = thr.y * sg.w.y, s_thr[2][home] = thr.z * sg.w.z;
                x_o[0][me] = sg.next.o.x, x_o[1][me] = sg.next.o.y, x_o[2][me] = sg.next.o.z;
                x_d[0][me] = sg.next.d.x, x_d[1][me] = sg.next.d.y, x_d[2][me] = sg.next.d.z;
                --depth;
            } else {
                store_record_f32(A.J.L, x_q[me], thr.x * sg.w.x, thr.y * sg.w.y, thr.z * sg.w.z);
                depth = 0;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_down(segs, off, 64);
    if (lane == 0) s_seg[wave] = segs;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int k = 0; k < kSortWaves; ++k) t += s_seg[k];
        if (t) atomicAdd(&fast_args_now().C->segments[blockIdx.x % 8].v, t);
    }
}

// Block-wide exclusive prefix sum of one value per thread (blockDim = kBlock).
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t* s_wave, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += y;
    }
    if (lane == 63) s_wave[w] = incl;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) {
        const uint32_t c = s_wave[k];
        before += (k < (int)w) ? c : 0u;
        tot += c;
    }
    total = tot;
    return before + incl - v;
}

// Refill empty pool slots with new camera samples.  Block b owns the slot
// range [lo, lo + kRegenSlots): its empty slots are ranked with a block prefix
// sum into an LDS list (stream compaction), ONE atomic on queue shard
// b % kQShards reserves that many sample ids, ray-gen runs densely over the
// list and writes the rays DENSELY to staging entries lo, lo+1, ...; each empty
// slot only receives its 4-byte fresh marker.  (Scattered 8-byte stores into
// pool lines that have left L2 cost a memory-side read-modify-write each:
// measured 52 us vs 5 us per launch for 13 scattered arrays vs 3.)
constexpr uint32_t kRegenSlots = 1024;

__global__ __launch_bounds__(kBlock) void k_regen(job_t J, paths_t P, fresh_t FR, ctrs_t* C) {
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_list[kRegenSlots];
    const uint32_t n = C->n;
    const uint32_t lo = blockIdx.x * kRegenSlots;
    if (lo >= n) return;
    const uint32_t hi = min(n, lo + kRegenSlots);
    constexpr int kPer = kRegenSlots / kBlock;
    bool need[kPer];
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t i = lo + threadIdx.x + k * kBlock;
        need[k] = i < hi && P.depth[i] == 0;
        mine += need[k];
    }
    uint32_t total;
    uint32_t off = block_scan(mine, s_wave, total);
    if (total == 0) return;
#pragma unroll
    for (int k = 0; k < kPer; ++k)
        if (need[k]) s_list[off++] = lo + threadIdx.x + k * kBlock;
    // Reserve sample ids: own shard first, then the others while it is dry,
    // so every shard drains whatever the number of blocks.
    __shared__ uint32_t s_got[kQShards];
    __shared__ unsigned long long s_first[kQShards];
    if (threadIdx.x == 0) {
        uint32_t left = total;
        const int own = blockIdx.x % kQShards;
        for (int a = 0; a < kQShards; ++a) {
            const int sh = (own + a) % kQShards;
            s_got[a] = 0;
            if (left == 0) continue;
            const unsigned long long lim = shard_limit(sh, J.total);
            if (a > 0) {  // stealing: skip dry shards without an atomic
                const unsigned long long cur =
                    __hip_atomic_load(&C->qshard[sh].v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (cur >= lim) continue;
            }
            const unsigned long long b = atomicAdd(&C->qshard[sh].v, (unsigned long long)left);
            const uint32_t ok = b >= lim ? 0u : (uint32_t)min((unsigned long long)left, lim - b);
            s_first[a] = b;
            s_got[a] = ok;
            left -= ok;
        }
    }
    __syncthreads();
    const int own = blockIdx.x % kQShards;
    for (uint32_t e = threadIdx.x; e < total; e += kBlock) {
        uint32_t k = e;
        for (int a = 0; a < kQShards; ++a) {
            if (k < s_got[a]) {
                const int sh = (own + a) % kQShards;
                raygen(J, FR, lo + e, (uint32_t)shard_sample(sh, s_first[a] + k));
                P.depth[s_list[e]] = kFresh | (lo + e);
                break;
            }
            k -= s_got[a];
        }
    }
}

// true once every queue shard has handed out all of its samples
inline bool queue_drained(const ctrs_t& c, uint32_t total) {
    for (int s = 0; s < kQShards; ++s)
        if (c.qshard[s].v < shard_limit(s, total)) return false;
    return true;
}

// Tail-phase stream compaction of live slots (depth != 0) from A into B
// (fresh markers move with their slot; staging is not rewritten in the tail).
__global__ __launch_bounds__(kBlock) void k_compact(paths_t A, paths_t B, ctrs_t* C) {
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_base;
    const uint32_t n = C->n;
    for (uint32_t b = blockIdx.x * kBlock; b < n; b += gridDim.x * kBlock) {
        const uint32_t i = b + threadIdx.x;
        const bool live = i < n && A.depth[i] != 0;
        uint32_t total;
        const uint32_t rank = block_rank(live, s_wave, total);
        if (total) {
            if (threadIdx.x == 0) s_base = atomicAdd(&C->n_out, total);
            __syncthreads();
            if (live) {
                const uint32_t o = s_base + rank;
                B.ox[o] = A.ox[i], B.oy[o] = A.oy[i], B.oz[o] = A.oz[i];
                B.dx[o] = A.dx[i], B.dy[o] = A.dy[i], B.dz[o] = A.dz[i];
                B.tm[o] = A.tm[i];
                B.tr[o] = A.tr[i], B.tg[o] = A.tg[i], B.tb[o] = A.tb[i];
                B.rng[o] = A.rng[i], B.depth[o] = A.depth[i], B.qid[o] = A.qid[i];
            }
        }
        __syncthreads();
    }
}

__global__ void k_commit(ctrs_t* C) {
    C->n = C->n_out;
    C->n_out = 0;
}

// running[pix] += sample s of pix for s = 0..S-1 in order (RayTracingWeekend.cpp:235-239)
// Records are doubles (fp64 mode) or floats (the fp32 fast mode's radiance
// is single precision: 12 B records, converted exactly to double here and
// summed in the same order, so its sums are unchanged).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_reduce(const T* __restrict__ L, uint32_t npix, uint32_t spp,
                                                   double* __restrict__ run) {
    for (uint32_t p = blockIdx.x * kBlock + threadIdx.x; p < npix; p += gridDim.x * kBlock) {
        double r = run[3 * p], g = run[3 * p + 1], bl = run[3 * p + 2];
        for (uint32_t s = 0; s < spp; ++s) {
            const T* x = L + 3 * ((size_t)s * npix + p);
            r = r + (double)x[0];
            g = g + (double)x[1];
            bl = bl + (double)x[2];
        }
        run[3 * p] = r, run[3 * p + 1] = g, run[3 * p + 2] = bl;
    }
}
// k_reduce's grid for npix pixels
unsigned reduce_grid(uint64_t npix) {
    return (unsigned)std::min<uint64_t>((npix + kBlock - 1) / kBlock, 4096);
}

// accum[(j*nx+i)*3+c] += run[(k*nx+i)*3+c], j = row_begin + k*row_step
__global__ __launch_bounds__(kBlock) void k_emit(const double* __restrict__ run, uint32_t npix, int nx, int row_begin,
                                                 int row_step, double* __restrict__ accum) {
    for (uint32_t p = blockIdx.x * kBlock + threadIdx.x; p < npix; p += gridDim.x * kBlock) {
        const uint32_t k = p / (uint32_t)nx, i = p - k * (uint32_t)nx;
        const size_t o = ((size_t)(row_begin + (int)k * row_step) * nx + i) * 3;
        accum[o] += run[3 * p];
        accum[o + 1] += run[3 * p + 1];
        accum[o + 2] += run[3 * p + 2];
    }
}

// canvas = min(sqrt(accum / spp), 1) (RayTracingWeekend.cpp:241-244)
__global__ __launch_bounds__(kBlock) void k_finalize(const double* __restrict__ accum, size_t n, double spp,
                                                     double* __restrict__ canvas) {
    for (size_t k = blockIdx.x * (size_t)kBlock + threadIdx.x; k < n; k += (size_t)gridDim.x * kBlock) {
        const double s = __builtin_sqrt(accum[k] / spp);
        canvas[k] = (1.0 < s) ? 1.0 : s;
    }
}

// ======================================================================
// host side
// ======================================================================
#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess)                                                                  \
            return rtw_fail(RTW_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_));      \
    } while (0)

uint64_t host_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct dev_buf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t n) {
        if (n <= bytes) return RTW_OK;
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, n) != hipSuccess) return rtw_fail(RTW_ERR_OOM, "hipMalloc of " + std::to_string(n) + " bytes failed");
        bytes = n;
        return RTW_OK;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct handle_t {
    int device = 0;
    hipStream_t stream = nullptr;
    scene S{};
    bool media = false;
    int features = 0;    // F_MEDIA | F_WBVH | F_GBVH of the uploaded scene
    bool ysph = false;   // its world list holds y-sphere runs (F_YSPH kernels)
    int n_runs = 0, n_ysph_runs = 0, n_plain_runs = 0;  // world-list run layout (rtw_scene_query)
    bool movers = true;  // it holds moving spheres (else F_STATIC kernels)
    int shade_mask = 0;  // SF_* material / texture set of the uploaded scene
    const char* scene_base = nullptr;
    uint32_t shade_bytes = 0;  // bytes of the shading prefix of scene_mem
    dev_buf scene_mem;
    dev_buf scene32;  // fp32 mirror of the scene (fast mode, rtw_fast.h)
    rtwf::fscene F32{};
    uint32_t f32_bytes = 0;  // bytes of scene32 fp32 shading reads
    dev_buf pool[2];  // path SoA, ping-pong for compaction
    dev_buf fresh;    // staging of new camera rays (fresh_t)
    dev_buf hits;
    dev_buf radiance; // per-sample planes of one pass
    dev_buf run;      // per-pixel running sums
    dev_buf flog;     // RTW_STRICT_RADIANCE: per-thread factor logs (job_t::flog)
    dev_buf accum;    // device accum when the caller passes a host pointer
    dev_buf ctrs;
    dev_buf camera;                // device copy of the call's camera
    rtw_camera_desc cam_host{};    // its source (lives until the copy ran)
    ctrs_t* host_ctrs = nullptr;  // pinned
    uint32_t pool_cap = 0;
    int grid = 2048;
    int cus = 256;
    int stack_need = 0;  // deepest BVH stack a traversal of this scene can use
    int group_depth = 0;  // depth of its deepest group BVH
    // BVH boxes of moving spheres cover the desc camera's shutter only
    bool bvh_motion = false;
    double shutter0 = 0.0, shutter1 = 0.0;
    bool desc_pin = false;  // the desc's own camera is a pinhole (F_PIN kernels; rtw_scene_query)
    std::vector<hipEvent_t> events;
};

paths_t carve_paths(void* base, uint32_t cap) {
    char* p = static_cast<char*>(base);
    paths_t P;
    double** d[] = {&P.ox, &P.oy, &P.oz, &P.dx, &P.dy, &P.dz, &P.tm, &P.tr, &P.tg, &P.tb};
    for (double** x : d) {
        *x = reinterpret_cast<double*>(p);
        p += (size_t)cap * 8;
    }
    uint32_t** u[] = {&P.rng, &P.depth, &P.qid};
    for (uint32_t** x : u) {
        *x = reinterpret_cast<uint32_t*>(p);
        p += (size_t)cap * 4;
    }
    return P;
}
size_t paths_bytes(uint32_t cap) { return (size_t)cap * (10 * 8 + 3 * 4); }

fresh_t carve_fresh(void* base, uint32_t cap) {
    char* p = static_cast<char*>(base);
    fresh_t F;
    double** d[] = {&F.ox, &F.oy, &F.oz, &F.dx, &F.dy, &F.dz, &F.tm};
    for (double** x : d) {
        *x = reinterpret_cast<double*>(p);
        p += (size_t)cap * 8;
    }
    F.rng = reinterpret_cast<uint32_t*>(p);
    F.qid = F.rng + cap;
    return F;
}
size_t fresh_bytes(uint32_t cap) { return (size_t)cap * (7 * 8 + 2 * 4); }

int upload_scene(handle_t* h, const rtw_scene_desc* d) {
    // one allocation, 256-byte aligned sub-arrays
    // The media walk (scene::media, world_closest with F_MEDIA): the visit
    // program (rtw_scene_desc::visits) without its deterministic replays --
    // a second walk over an object with no random draws re-accepts only an
    // exact tie -- or, without a program, the world's two walks the same way:
    // every entry, then the media again.
    std::vector<int32_t> media;
    bool has_media = false;
    for (int e = 0; e < d->n_entries; ++e) has_media |= d->entries[e].kind == RTW_ENTRY_MEDIUM;
    if (has_media) {
        if (d->n_visits > 0) {
            for (int k = 0; k < d->n_visits; ++k) {
                const int e = d->visits[k] & RTW_VISIT_ENTRY;
                if (!(d->visits[k] & RTW_VISIT_REPLAY) || d->entries[e].kind == RTW_ENTRY_MEDIUM) media.push_back(e);
            }
        } else {
            for (int e = 0; e < d->n_entries; ++e) media.push_back(e);
            for (int e = 0; e < d->n_entries; ++e)
                if (d->entries[e].kind == RTW_ENTRY_MEDIUM) media.push_back(e);
        }
    }
    struct part {
        const void* src;
        size_t bytes;
        size_t off;
    };
    // World-space onb of every rect primitive's normal: rect_normal, the
    // prim's own flip, then its entry's ops outward -- hit_record's normal
    // path (rtw_device.h) -- and onb_from_w, all with the device's expressions.
    std::vector<double> frames((size_t)d->n_prims * 9, 0.0);
    for (int pi = 0; pi < d->n_prims; ++pi) {
        const rtw_prim& q = d->prims[pi];
        if (q.type < RTW_PRIM_RECT_XY || q.entry < 0) continue;
        d3 n = rect_normal(q.type);
        if (q.flip & 1) n = -n;
        const rtw_entry& e = d->entries[q.entry];
        for (int k = RTW_MAX_OPS - 1; k >= 0; --k) {
            if (k >= e.n_ops) continue;
            if (e.op[k] == RTW_OP_ROTATE_Y) {
                const double s = e.op_param[k][0], c = e.op_param[k][1];
                const d3 n0 = n;
                n.x = c * n0.x + s * n0.z;
                n.z = -s * n0.x + c * n0.z;
            } else if (e.op[k] == RTW_OP_FLIP) {
                n = -n;
            }
        }
        const onb b = onb_from_w(n);
        double* f = frames.data() + 9 * (size_t)pi;
        f[0] = b.u.x, f[1] = b.u.y, f[2] = b.u.z;
        f[3] = b.v.x, f[4] = b.v.y, f[5] = b.v.z;
        f[6] = b.w.x, f[7] = b.w.y, f[8] = b.w.z;
    }
    // per material: 1/ref_idx and schlick's r0^2 (material.h:158, :46-47)
    std::vector<double> mat_aux((size_t)d->n_materials * 2, 0.0);
    for (int k = 0; k < d->n_materials; ++k) {
        const double ri = d->materials[k].ref_idx;
        double r0 = (1 - ri) / (1 + ri);
        r0 = r0 * r0;
        mat_aux[2 * k] = 1.0 / ri;
        mat_aux[2 * k + 1] = r0;
    }
    // Device copy of the prims: sphere records rewritten as rtw_device.h
    // (DP_MOVING_COMMON) describes -- radius^2, center1 - center0, time1 -
    // time0 precomputed with the reference's expressions -- and the moving
    // spheres sharing the first mover's interval tagged so traversal computes
    // their time fraction once per ray.
    std::vector<rtw_prim> dprims(d->prims, d->prims + d->n_prims);
    bool mv_common = false;
    double mv_t0 = 0.0, mv_den = 1.0;
    for (rtw_prim& q : dprims) {
        if (!is_sphere(q.type)) continue;
        q.p[9] = q.p[3] * q.p[3];
        if (q.type != RTW_PRIM_MOVING_SPHERE) continue;
        for (int k = 0; k < 3; ++k) q.p[4 + k] = q.p[4 + k] - q.p[k];
        q.p[8] = q.p[8] - q.p[7];
        // the shared fraction must stay finite: (time - t0) is at most ~2^129
        // in magnitude (light pdf rays carry time FLT_MAX)
        const bool finite_frac = std::isfinite(q.p[7]) && std::isfinite(q.p[8]) && std::fabs(q.p[8]) >= 1e-200;
        if (!finite_frac) continue;
        if (!mv_common) {
            mv_common = true;
            mv_t0 = q.p[7];
            mv_den = q.p[8];
        }
        if (std::memcmp(&q.p[7], &mv_t0, 8) != 0 || std::memcmp(&q.p[8], &mv_den, 8) != 0) continue;
        // y-only mover: x and z stay center0's exactly when dc is +-0 and
        // center0's component is nonzero (x + +-0 == x for x != 0)
        const bool y_only = q.p[4] == 0.0 && q.p[6] == 0.0 && q.p[0] != 0.0 && q.p[2] != 0.0;
        q.type = y_only ? DP_MOVING_COMMON_Y : DP_MOVING_COMMON;
    }
    // World list runs: consecutive plain entries (one group, no BVH, no op
    // that moves the ray -- flip_normals only turns the normal, which
    // hit_record applies from the prim's entry) scan their contiguous prims
    // as one run.  (Cornell: the flipped walls join the plain ones.)
    auto ray_plain = [](const rtw_entry& E) {
        if (E.kind != RTW_ENTRY_GROUP || E.bvh_root >= 0) return false;
        for (int k = 0; k < E.n_ops; ++k)
            if (E.op[k] != RTW_OP_FLIP) return false;
        return true;
    };
    std::vector<world_run> runs;
    std::vector<int32_t> entry_movers(std::max(d->n_entries, 1), 0);
    for (int e = 0; e < d->n_entries; ++e) {
        const rtw_entry& E = d->entries[e];
        for (int i = E.first_prim; i < E.first_prim + E.n_prims; ++i)
            entry_movers[e] |= dprims[i].type >= DP_MOVING_COMMON ? 1 : 0;
        const bool plain = ray_plain(E);
        if (plain && !runs.empty() && runs.back().entry < 0 &&
            runs.back().first_prim + runs.back().n_prims == E.first_prim) {
            runs.back().n_prims += E.n_prims;
            runs.back().movers |= entry_movers[e];
            continue;
        }
        runs.push_back(world_run{plain ? WORLD_RUN_PLAIN : e, E.first_prim, E.n_prims, entry_movers[e]});
    }
    // plain runs of y-only spheres -> ysphere_scan (static ones get dy = 0)
    for (world_run& R : runs) {
        if (R.entry != WORLD_RUN_PLAIN || R.n_prims < 2) continue;
        bool all = true;
        for (int i = R.first_prim; i < R.first_prim + R.n_prims && all; ++i)
            all = dprims[i].type == DP_MOVING_COMMON_Y || (dprims[i].type == RTW_PRIM_SPHERE && dprims[i].p[1] != 0.0);
        if (!all) continue;
        R.entry = WORLD_RUN_YSPHERES;
        for (int i = R.first_prim; i < R.first_prim + R.n_prims; ++i)
            if (dprims[i].type == RTW_PRIM_SPHERE) dprims[i].p[5] = 0.0;
    }
    // ysphere_scan's fp32 prefilter records (rtw_device.h): spheres of
    // y-sphere runs whose centre (incl. motion) is within 2^8 and radius
    // within 2^4 are filtered, others (the random_balls ground, r = 1000)
    // carry r^2 = +inf and always take the fp64 test; the maxima over the
    // filtered ones bound the prefilter's rounding error
    // (the records of a run are interleaved pairwise, spheres
    // first + 2p and first + 2p + 1 sharing the 16 floats at 8 (first + 2p),
    // component c of member s at 2c + s; the last sphere of a run of odd
    // length keeps the plain record {cx, cy, cz, dy, rr} in its own 8 floats,
    // so every record stays inside its run's slots; kYsAhead + 2 spare
    // records at the end, slack for the unpacked form's prefetch ring)
    std::vector<float> ysph(8 * (std::max<size_t>(dprims.size(), 1) + kYsAhead + 2), 0.0f);
    float ysb[5] = {0, 0, 0, 0, 0};  // |cx|, |cy|, |dy|, |cz|, r^2 maxima
    auto up = [](double v) {  // fp32 value >= v
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, INFINITY);
        return f;
    };
    for (const world_run& R : runs) {
        if (R.entry != WORLD_RUN_YSPHERES) continue;
        for (int i = R.first_prim; i < R.first_prim + R.n_prims; ++i) {
            const rtw_prim& q = dprims[i];
            const int k = i - R.first_prim;
            const bool lone = k == R.n_prims - 1 && (k & 1) == 0;
            float* const rec = ysph.data() + 8 * (size_t)(R.first_prim + (k & ~1)) + (k & 1);
            auto f = [rec, lone](int c) -> float& { return rec[lone ? c : 2 * c]; };
            const double dy = q.type == DP_MOVING_COMMON_Y ? q.p[5] : 0.0;
            f(0) = (float)q.p[0], f(1) = (float)q.p[1], f(2) = (float)q.p[2], f(3) = (float)dy;
            const bool small = std::fabs(q.p[0]) <= 256 && std::fabs(q.p[1]) <= 256 && std::fabs(dy) <= 256 &&
                               std::fabs(q.p[2]) <= 256 && std::fabs(q.p[3]) <= 16;
            if (!small) {
                f(4) = INFINITY;
                continue;
            }
            f(4) = (float)q.p[9];
            ysb[0] = std::max(ysb[0], up(std::fabs(q.p[0])));
            ysb[1] = std::max(ysb[1], up(std::fabs(q.p[1])));
            ysb[2] = std::max(ysb[2], up(std::fabs(dy)));
            ysb[3] = std::max(ysb[3], up(std::fabs(q.p[2])));
            ysb[4] = std::max(ysb[4], up(q.p[9]));
        }
    }
    // World-BVH leaves reference entries; a plain one-prim entry's item is
    // replaced by ~prim so the walk tests the prim without reading the entry.
    std::vector<int32_t> ditems(d->bvh_items, d->bvh_items + d->n_bvh_items);
    std::vector<char> world_node(d->n_bvh_nodes, 0);  // (the fp32 nodes' inline world leaves)
    if (d->world_bvh_root >= 0) {
        std::vector<int> todo{d->world_bvh_root};
        while (!todo.empty()) {
            const rtw_bvh_node& N = d->bvh_nodes[todo.back()];
            world_node[todo.back()] = 1;
            todo.pop_back();
            if (N.count == 0) {
                todo.push_back(N.left);
                todo.push_back(N.right);
                continue;
            }
            for (int k = N.left; k < N.left + N.count; ++k) {
                if (ditems[k] < 0 || ditems[k] >= d->n_entries)
                    return rtw_fail(RTW_ERR_INVALID, "world bvh item out of range");
                const rtw_entry& E = d->entries[ditems[k]];
                if (ray_plain(E) && E.n_prims == 1)
                    ditems[k] = ~E.first_prim;
            }
        }
    }
    // Box items' planes (scene::boxes): one 64-B record per box item,
    // {x0, x1, y0, y1, z0, z1, first rect (int)}, packed densely (the 400
    // ground boxes of Book 2 in 25 KB), when every box item's six rects are
    // the hittable_list box's (+z, -z, +y, -y, +x, -x: XY at z1 and z0, XZ at
    // y1 and y0, YZ at x1 and x0, each with the box's other two ranges) to
    // the last bit.  The device items then read RTW_ITEM_BOX | record (the
    // fp32 copy likewise, fscene::boxes); otherwise no table, and the walks
    // read the rects of RTW_ITEM_BOX | first rect.
    // (RTW_BOX_TABLE=0 at upload: no table, for tests of the rect path)
    const char* box_env = std::getenv("RTW_BOX_TABLE");
    const bool box_table = !(box_env && *box_env && std::atoi(box_env) == 0);
    auto box_planes = [&](auto get, int i, auto* out) {  // get(prim, k) = p[k]; false if not a box
        if (i < 0 || i + 6 > (int)dprims.size()) return false;
        const int ty[6] = {RTW_PRIM_RECT_XY, RTW_PRIM_RECT_XY, RTW_PRIM_RECT_XZ,
                           RTW_PRIM_RECT_XZ, RTW_PRIM_RECT_YZ, RTW_PRIM_RECT_YZ};
        for (int j = 0; j < 6; ++j)
            if (dprims[i + j].type != ty[j]) return false;
        const auto x0 = get(i + 5, 4), x1 = get(i + 4, 4), y0 = get(i + 3, 4), y1 = get(i + 2, 4);
        const auto z0 = get(i + 1, 4), z1 = get(i, 4);
        const decltype(x0) want[6][4] = {{x0, x1, y0, y1}, {x0, x1, y0, y1}, {x0, x1, z0, z1},
                                         {x0, x1, z0, z1}, {y0, y1, z0, z1}, {y0, y1, z0, z1}};
        for (int j = 0; j < 6; ++j)
            for (int k = 0; k < 4; ++k)
                if (!(get(i + j, k) == want[j][k])) return false;
        out[0] = x0, out[1] = x1, out[2] = y0, out[3] = y1, out[4] = z0, out[5] = z1;
        int32_t f = i;
        std::memcpy(out + 6, &f, sizeof f);  // the first rect, in the record's seventh slot
        return true;
    };
    std::vector<int> box_firsts;  // record -> first rect
    std::vector<double> boxes64;
    {
        std::vector<int> slot_items;  // item slots of box items
        for (size_t k = 0; k < ditems.size(); ++k)
            if (box_table && ditems[k] >= 0 && (ditems[k] & RTW_ITEM_BOX)) slot_items.push_back((int)k);
        std::map<int, int> rec_of;
        bool ok = true;
        for (int k : slot_items) {
            const int i = ditems[k] & RTW_ITEM_INDEX;
            if (rec_of.count(i)) continue;
            rec_of[i] = (int)box_firsts.size();
            box_firsts.push_back(i);
        }
        boxes64.assign(8 * box_firsts.size(), 0.0);
        for (size_t b = 0; b < box_firsts.size() && ok; ++b)
            ok = box_planes([&](int q, int k) { return dprims[q].p[k]; }, box_firsts[b], boxes64.data() + 8 * b);
        if (!ok) {
            boxes64.clear();
            box_firsts.clear();
        } else {
            for (int k : slot_items) ditems[k] = RTW_ITEM_BOX | rec_of[ditems[k] & RTW_ITEM_INDEX];
        }
    }
    // Inner BVH nodes: the axis along which their children's centres differ
    // most, and whether the left child is the upper one (push_children).
    std::vector<rtw_bvh_node> dnodes(d->bvh_nodes, d->bvh_nodes + d->n_bvh_nodes);
    for (rtw_bvh_node& N : dnodes) {
        N.pad = 0;
        if (N.count > 0) continue;
        const rtw_bvh_node& L = d->bvh_nodes[N.left];
        const rtw_bvh_node& R = d->bvh_nodes[N.right];
        int ax = 0;
        double best = -1.0;
        for (int k = 0; k < 3; ++k) {
            const double gap = std::fabs((R.bmin[k] + R.bmax[k]) - (L.bmin[k] + L.bmax[k]));
            if (gap > best) best = gap, ax = k;
        }
        const bool left_upper = (L.bmin[ax] + L.bmax[ax]) > (R.bmin[ax] + R.bmax[ax]);
        N.pad = ax | (left_upper ? 4 : 0);
    }
    // fp32 device nodes (rtw_device.h bvh_node32): bounds rounded outward;
    // a BVH whose bounds are not finite within 2^90 is not used at all (the
    // flat list gives the same image)
    std::vector<bvh_node32> dnodes32(dnodes.size());
    // The fp32 kernels' copy of the nodes: a one-item leaf holds its item
    // (entry, ~prim, prim or box) in a instead of its index into the item
    // array (b = -1), and a two-item group leaf holds both (a, and b =
    // INT_MIN | second; b in [-16, -2] stays an index and a count), so the
    // fp32 walks (rtw_fast.h) reach the prims with one dependent load less
    // per leaf.  Measured (1 MI355X, A/B; bit-identical): C3 fp32 +1.9 %
    // (profiles/r06/ab_r6r_C3f.log, parity_r6r_inl2.log), C5 fp32 +0.5 % for
    // the group pairs (ab_r6t_C5f.log, parity_r6t_pair.log).  The fp64 walks
    // keep the shared form: inline leaves there measured C3 -0.7 %
    // (ab_r6r_C3.log).
    std::vector<bvh_node32> dnodes32f(dnodes.size());
    double bvh_bound = 0.0;
    bool bvh_ok = dnodes.size() < (1u << 28);
    for (size_t k = 0; k < dnodes.size(); ++k) {
        const rtw_bvh_node& N = dnodes[k];
        bvh_node32& M = dnodes32[k];
        for (int j = 0; j < 3; ++j) {
            bvh_ok = bvh_ok && std::isfinite(N.bmin[j]) && std::isfinite(N.bmax[j]) &&
                     std::fabs(N.bmin[j]) <= 0x1p90 && std::fabs(N.bmax[j]) <= 0x1p90;
            float lo = (float)N.bmin[j], hi = (float)N.bmax[j];
            if ((double)lo > N.bmin[j]) lo = std::nextafter(lo, -INFINITY);
            if ((double)hi < N.bmax[j]) hi = std::nextafter(hi, INFINITY);
            M.lo[j] = lo, M.hi[j] = hi;
            bvh_bound = std::max(bvh_bound, std::max(std::fabs((double)lo), std::fabs((double)hi)));
        }
        M.a = N.left;
        M.b = N.count > 0 ? -N.count : (N.right | (N.pad << 28));
        dnodes32f[k] = M;
        if (N.count == 1) dnodes32f[k].a = ditems[N.left];
        // a group leaf's two items (prims or boxes: >= 0) in a and b's low bits
        if (!world_node[k] && N.count == 2 && ditems[N.left] >= 0 && ditems[N.left + 1] >= 0 &&
            ditems[N.left + 1] < 0x7fffffef) {
            dnodes32f[k].a = ditems[N.left];
            dnodes32f[k].b = (int32_t)(0x80000000u | (uint32_t)ditems[N.left + 1]);
        }
    }
    // Breadth-first numbering from all roots together (the world BVH's, then
    // every group's, in entry order): nodes [0, k) are then the top levels of
    // every tree, the node packet the persistent BVH kernels stage in LDS.
    std::vector<rtw_entry> dentries(d->entries, d->entries + d->n_entries);
    int world_root = d->world_bvh_root;
    if (!dnodes32.empty()) {
        std::vector<int> order, newid(dnodes32.size(), -1);
        order.reserve(dnodes32.size());
        auto enqueue = [&](int n) {
            if (n >= 0 && newid[n] < 0) newid[n] = (int)order.size(), order.push_back(n);
        };
        enqueue(world_root);
        for (const rtw_entry& E : dentries) enqueue(E.bvh_root);
        for (size_t q = 0; q < order.size(); ++q) {
            const rtw_bvh_node& N = dnodes[order[q]];
            if (N.count == 0) enqueue(N.left), enqueue(N.right);
        }
        for (size_t n = 0; n < dnodes32.size(); ++n) enqueue((int)n);  // unreachable nodes keep a slot
        auto renumber = [&](std::vector<bvh_node32>& nodes) {
            std::vector<bvh_node32> bfs(nodes.size());
            for (size_t n = 0; n < nodes.size(); ++n) {
                bvh_node32 M = nodes[n];
                if (M.b >= 0) {  // inner: renumber both children, keep the split bits
                    M.a = newid[M.a];
                    M.b = newid[M.b & 0x0fffffff] | (M.b & ~0x0fffffff);
                }
                bfs[newid[n]] = M;
            }
            nodes.swap(bfs);
        };
        renumber(dnodes32);
        renumber(dnodes32f);
        if (world_root >= 0) world_root = newid[world_root];
        for (rtw_entry& E : dentries)
            if (E.bvh_root >= 0) E.bvh_root = newid[E.bvh_root];
    }
    // device entries (dev_entry) and their op pool
    std::vector<dev_entry> dev_entries(std::max<size_t>(dentries.size(), 1));
    std::vector<dev_op> dev_ops;
    for (size_t e = 0; e < dentries.size(); ++e) {
        const rtw_entry& E = dentries[e];
        dev_entry& D = dev_entries[e];
        std::memset(&D, 0, sizeof D);
        D.kind = E.kind, D.first_prim = E.first_prim, D.n_prims = E.n_prims, D.n_ops = E.n_ops;
        D.first_op = (int32_t)dev_ops.size();
        D.phase_material = E.phase_material, D.bvh_root = E.bvh_root, D.n_outer_ops = E.n_outer_ops;
        D.movers = entry_movers[e];
        // the reference's -(1 / density), once per upload (a correctly
        // rounded division and a negation, as on the device)
        D.neg_inv_density = E.kind == RTW_ENTRY_MEDIUM ? -(1.0 / E.density) : 0.0;
        for (int k = 0; k < E.n_ops; ++k) {
            dev_op o;
            std::memset(&o, 0, sizeof o);
            o.type = E.op[k];
            for (int j = 0; j < 3; ++j) o.p[j] = E.op_param[k][j];
            dev_ops.push_back(o);
        }
    }
    std::vector<part> parts = {
        // parts 0..10 are what shading reads; they come first so a small
        // scene's shading data is one contiguous prefix the shade kernel can
        // stage in LDS
        {dprims.data(), sizeof(rtw_prim) * dprims.size(), 0},
        {dev_entries.data(), sizeof(dev_entry) * (size_t)d->n_entries, 0},
        {d->materials, sizeof(rtw_material) * d->n_materials, 0},
        {d->textures, sizeof(rtw_texture) * d->n_textures, 0},
        {d->lights, sizeof(rtw_light) * d->n_lights, 0},
        {d->has_perlin ? d->perlin_ranvec : nullptr, d->has_perlin ? sizeof(double) * 768 : 0, 0},
        {d->has_perlin ? d->perlin_perm : nullptr, d->has_perlin ? sizeof(int32_t) * 768 : 0, 0},
        {media.data(), sizeof(int32_t) * media.size(), 0},
        {frames.data(), sizeof(double) * frames.size(), 0},
        {mat_aux.data(), sizeof(double) * mat_aux.size(), 0},
        {dev_ops.data(), sizeof(dev_op) * dev_ops.size(), 0},
        {dnodes32.data(), sizeof(bvh_node32) * dnodes32.size(), 0},
        {ditems.data(), sizeof(int32_t) * ditems.size(), 0},
        {runs.data(), sizeof(world_run) * runs.size(), 0},
        {ysph.data(), sizeof(float) * ysph.size(), 0},
        {boxes64.data(), sizeof(double) * boxes64.size(), 0},
    };
    size_t total = 0;
    for (auto& p : parts) {
        p.off = total;
        total += (p.bytes + 255) & ~size_t(255);
    }
    int rc = h->scene_mem.ensure(std::max<size_t>(total, 256));
    if (rc) return rc;
    std::vector<char> staging(std::max<size_t>(total, 256), 0);
    for (auto& p : parts)
        if (p.bytes && p.src) std::memcpy(staging.data() + p.off, p.src, p.bytes);
    HIPCHK(hipMemcpy(h->scene_mem.p, staging.data(), staging.size(), hipMemcpyHostToDevice));
    char* base = static_cast<char*>(h->scene_mem.p);
    auto at = [&](int k) { return parts[k].bytes ? (void*)(base + parts[k].off) : nullptr; };
    scene& S = h->S;
    S.prims = (const rtw_prim*)at(0);
    S.entries = (const dev_entry*)at(1);
    S.materials = (const rtw_material*)at(2);
    S.textures = (const rtw_texture*)at(3);
    S.lights = (const rtw_light*)at(4);
    S.ranvec = (const double*)at(5);
    S.perm = (const int32_t*)at(6);
    S.media = (const int32_t*)at(7);
    S.prim_onb = (const double*)at(8);
    S.mat_aux = (const double*)at(9);
    S.ops = (const dev_op*)at(10);
    S.nodes = (const node_store*)at(11);
    S.bvh_bound = bvh_bound;
    S.items = (const int32_t*)at(12);
    S.runs = (const world_run*)at(13);
    S.ysph = (const float*)at(14);
    S.boxes = (const double*)at(15);
    S.ysb_cx = ysb[0], S.ysb_cy = ysb[1], S.ysb_dy = ysb[2], S.ysb_cz = ysb[3], S.ysb_r2 = ysb[4];
    S.n_runs = (int32_t)runs.size();
    S.mv_common = mv_common ? 1 : 0;
    S.mv_t0 = mv_t0;
    S.mv_den = mv_den;
    // walk_quot (rtw_device.h): every prim coordinate and radius within 2^40,
    // every mover on the common interval
    {
        bool bounded = true;
        auto in = [&](double v) { return std::isfinite(v) && std::fabs(v) <= 0x1p40; };
        for (const rtw_prim& q : dprims) {
            if (q.type == RTW_PRIM_MOVING_SPHERE) bounded = false;
            const int np = is_sphere(q.type) ? (q.type == RTW_PRIM_SPHERE ? 4 : 7) : 5;
            for (int k = 0; k < np; ++k) bounded = bounded && in(q.p[k]);
        }
        S.fast_div = bounded ? 1 : 0;
    }
    h->shade_bytes = (uint32_t)parts[11].off;  // the shading prefix
    h->scene_base = base;
    S.n_entries = d->n_entries;
    S.n_lights = d->n_lights;
    S.light_weight = d->n_lights > 0 ? 1.0 / (double)d->n_lights : 0.0;
    S.world_bvh_root = bvh_ok ? world_root : -1;
    S.n_nodes = bvh_ok ? (int32_t)dnodes32.size() : 0;
    S.render_type = d->render_type;
    S.background = d->background;
    S.n_media = (int32_t)media.size();
    S.has_media = has_media ? 1 : 0;
    h->media = has_media;
    h->features = (h->media ? F_MEDIA : 0) | (bvh_ok && d->world_bvh_root >= 0 ? F_WBVH : 0);
    h->ysph = false;
    for (const world_run& R : runs) h->ysph = h->ysph || R.entry == WORLD_RUN_YSPHERES;
    h->n_runs = (int)runs.size();
    h->n_ysph_runs = h->n_plain_runs = 0;
    for (const world_run& R : runs) {
        h->n_ysph_runs += R.entry == WORLD_RUN_YSPHERES;
        h->n_plain_runs += R.entry == WORLD_RUN_PLAIN;
    }
    h->movers = false;
    for (int k = 0; k < d->n_prims; ++k) h->movers = h->movers || d->prims[k].type == RTW_PRIM_MOVING_SPHERE;
    for (int e = 0; e < d->n_entries; ++e)
        if (bvh_ok && d->entries[e].bvh_root >= 0) h->features |= F_GBVH;
    int m = 0;
    for (int k = 0; k < d->n_materials; ++k) {
        const int t = d->materials[k].type;
        m |= t == RTW_MAT_METAL ? SF_METAL : t == RTW_MAT_DIELECTRIC ? SF_DIEL : t == RTW_MAT_ISOTROPIC ? SF_ISO : 0;
    }
    for (int k = 0; k < d->n_textures; ++k) {
        const int t = d->textures[k].type;
        m |= t == RTW_TEX_NOISE ? SF_NOISE : t == RTW_TEX_CHECKER ? SF_CHECKER : 0;
    }
    h->shade_mask = m;
    // BVH stack depth: a walk pushes two children per inner node and pops
    // one, so it holds at most depth + 1 entries; a group BVH inside a world
    // leaf stacks on top of the world walk
    auto depth = [&](int root) {
        int best = 0;
        std::vector<std::pair<int, int>> todo{{root, 1}};
        while (!todo.empty()) {
            const auto [n, dd] = todo.back();
            todo.pop_back();
            best = std::max(best, dd);
            const rtw_bvh_node& N = d->bvh_nodes[n];
            if (N.count == 0) todo.push_back({N.left, dd + 1}), todo.push_back({N.right, dd + 1});
        }
        return best;
    };
    int group_depth = 0;
    for (int e = 0; e < d->n_entries; ++e)
        if (d->entries[e].bvh_root >= 0) group_depth = std::max(group_depth, depth(d->entries[e].bvh_root));
    const int world_depth = d->world_bvh_root >= 0 ? depth(d->world_bvh_root) : 0;
    h->stack_need = world_depth + group_depth + 2;
    // A walk from an empty stack that pops one node and pushes both children
    // of an inner one holds at most D entries for a tree of depth D (the
    // entry at stack position j has depth >= j + 1: true for the root at 0,
    // and an inner node of depth k popped from position k' <= k - 1 puts
    // depth-(k + 1) children at k' and k' + 1).  The fp32 media kernel's
    // group walks are such walks (launch_fast).
    h->group_depth = group_depth;
    bool movers = false;
    for (int k = 0; k < d->n_prims; ++k) movers |= d->prims[k].type == RTW_PRIM_MOVING_SPHERE;
    h->desc_pin = camera_is_pinhole(d->camera);
    h->bvh_motion = movers && d->n_bvh_nodes > 0;
    h->shutter0 = std::min(d->camera.time0, d->camera.time1);
    h->shutter1 = std::max(d->camera.time0, d->camera.time1);
    if (h->stack_need > kStack)
        return rtw_fail(RTW_ERR_UNSUPPORTED, "BVH too deep for the traversal stack (" + std::to_string(h->stack_need) +
                                                 " > " + std::to_string(kStack) + " entries)");

    // fp32 mirror for the fast mode (rtw_fast.h): prims, entries, ops,
    // materials, textures, Perlin vectors and rect frames in single
    // precision; BVH nodes / items, world runs, the media walk and the lights
    // are the arrays above
    {
        using namespace rtwf;
        std::vector<prim32> p32(std::max(d->n_prims, 1));
        for (int i = 0; i < d->n_prims; ++i) {
            const rtw_prim& q = d->prims[i];
            prim32& o = p32[i];
            std::memset(&o, 0, sizeof o);
            o.type = q.type, o.material = q.material, o.flip = q.flip, o.entry = q.entry;
            for (int k = 0; k < 10; ++k) o.p[k] = (float)q.p[k];
            if (is_sphere(q.type)) {
                o.p[9] = (float)(q.p[3] * q.p[3]);
                if (q.type == RTW_PRIM_MOVING_SPHERE) {
                    for (int k = 0; k < 3; ++k) o.p[4 + k] = (float)(q.p[4 + k] - q.p[k]);
                    o.p[7] = (float)q.p[7];
                    o.p[8] = (float)(1.0 / (q.p[8] - q.p[7]));
                }
            }
        }
        std::vector<ent32> e32(std::max(d->n_entries, 1));
        for (int e = 0; e < d->n_entries; ++e) {
            const dev_entry& D = dev_entries[e];
            ent32& o = e32[e];
            std::memset(&o, 0, sizeof o);
            o.kind = D.kind, o.first_prim = D.first_prim, o.n_prims = D.n_prims, o.n_ops = D.n_ops;
            o.first_op = D.first_op, o.phase_material = D.phase_material;
            o.bvh_root = bvh_ok ? D.bvh_root : -1;
            o.n_outer_ops = D.n_outer_ops;
            o.neg_inv_density = (float)D.neg_inv_density;
        }
        std::vector<op32> o32(std::max<size_t>(dev_ops.size(), 1));
        for (size_t k = 0; k < dev_ops.size(); ++k) {
            o32[k].type = dev_ops[k].type;
            for (int j = 0; j < 3; ++j) o32[k].p[j] = (float)dev_ops[k].p[j];
        }
        std::vector<mat32> m32(std::max(d->n_materials, 1));
        for (int k = 0; k < d->n_materials; ++k) {
            const rtw_material& M = d->materials[k];
            mat32& o = m32[k];
            std::memset(&o, 0, sizeof o);
            o.type = M.type, o.texture = M.texture;
            for (int j = 0; j < 3; ++j) o.albedo[j] = (float)M.albedo[j];
            o.fuzz = (float)M.fuzz, o.ref_idx = (float)M.ref_idx;
            o.inv_ref_idx = (float)mat_aux[2 * k], o.r0 = (float)mat_aux[2 * k + 1];
        }
        std::vector<tex32> t32(std::max(d->n_textures, 1));
        for (int k = 0; k < d->n_textures; ++k) {
            const rtw_texture& T = d->textures[k];
            tex32& o = t32[k];
            std::memset(&o, 0, sizeof o);
            o.type = T.type, o.odd = T.odd, o.even = T.even, o.scale = (float)T.scale;
            for (int j = 0; j < 3; ++j) o.color[j] = (float)T.color[j];
        }
        std::vector<float> boxes32(8 * box_firsts.size(), 0.0f);  // the same records in fp32 (fscene::boxes)
        for (size_t b = 0; b < box_firsts.size(); ++b)
            if (!box_planes([&](int q, int k) { return p32[q].p[k]; }, box_firsts[b], boxes32.data() + 8 * b))
                return rtw_fail(RTW_ERR_INVALID, "box planes: fp32 rects differ from the fp64 ones");
        std::vector<float> rv32(d->has_perlin ? 768 : 0), fr32(frames.size());
        for (size_t k = 0; k < rv32.size(); ++k) rv32[k] = (float)d->perlin_ranvec[k];
        for (size_t k = 0; k < frames.size(); ++k) fr32[k] = (float)frames[k];
        // everything fp32 shading reads, in one allocation: the prefix the
        // regrouping kernel stages in LDS (k_fast_sort)
        std::vector<part> p2 = {
            {p32.data(), sizeof(prim32) * p32.size(), 0},
            {e32.data(), sizeof(ent32) * e32.size(), 0},
            {o32.data(), sizeof(op32) * o32.size(), 0},
            {m32.data(), sizeof(mat32) * m32.size(), 0},
            {t32.data(), sizeof(tex32) * t32.size(), 0},
            {rv32.data(), sizeof(float) * rv32.size(), 0},
            {fr32.data(), sizeof(float) * fr32.size(), 0},
            {d->lights, sizeof(rtw_light) * d->n_lights, 0},
            {d->has_perlin ? d->perlin_perm : nullptr, d->has_perlin ? sizeof(int32_t) * 768 : 0, 0},
            // (after the staged prefix)
            {dnodes32f.data(), sizeof(bvh_node32) * dnodes32f.size(), 0},
            {boxes32.data(), sizeof(float) * boxes32.size(), 0},
        };
        size_t tot = 0;
        for (auto& x : p2) {
            x.off = tot;
            tot += (x.bytes + 255) & ~size_t(255);
        }
        if ((rc = h->scene32.ensure(std::max<size_t>(tot, 256)))) return rc;
        std::vector<char> st2(std::max<size_t>(tot, 256), 0);
        for (auto& x : p2)
            if (x.bytes && x.src) std::memcpy(st2.data() + x.off, x.src, x.bytes);
        HIPCHK(hipMemcpy(h->scene32.p, st2.data(), st2.size(), hipMemcpyHostToDevice));
        char* b2 = static_cast<char*>(h->scene32.p);
        fscene& F = h->F32;
        F.prims = (const prim32*)(b2 + p2[0].off);
        F.entries = (const ent32*)(b2 + p2[1].off);
        F.ops = (const op32*)(b2 + p2[2].off);
        F.materials = (const mat32*)(b2 + p2[3].off);
        F.textures = (const tex32*)(b2 + p2[4].off);
        F.ranvec = p2[5].bytes ? (const float*)(b2 + p2[5].off) : nullptr;
        F.frames = (const float*)(b2 + p2[6].off);
        F.lights = p2[7].bytes ? (const rtw_light*)(b2 + p2[7].off) : nullptr;
        F.perm = p2[8].bytes ? (const int32_t*)(b2 + p2[8].off) : nullptr;
        h->f32_bytes = (uint32_t)(p2[8].off + p2[8].bytes);
        F.nodes = S.nodes ? (const node_store*)(b2 + p2[9].off) : nullptr;
        F.boxes = p2[10].bytes ? (const float*)(b2 + p2[10].off) : nullptr;
        F.items = S.items;
        F.runs = S.runs;
        F.media = S.media;
        F.ysph = S.ysph;
        F.mv_t0 = (float)S.mv_t0;
        F.mv_inv_den = (float)(1.0 / S.mv_den);
        F.light_weight = (float)S.light_weight;
        F.n_lights = S.n_lights;
        F.world_bvh_root = S.world_bvh_root;
        F.render_type = S.render_type;
        F.background = S.background;
        F.n_media = S.n_media;
        F.n_runs = S.n_runs;
        F.n_nodes = S.n_nodes;
    }
    return RTW_OK;
}

// Shade kernels are instantiated for a few material/texture sets; a scene
// runs the smallest instantiated superset of its own set.
constexpr int SF_NOCHECKER = SF_ALL & ~SF_CHECKER;  // the Book-2 set: noise, metal, glass, media
constexpr int kShadeMasks[] = {SF_DIEL, SF_METAL | SF_DIEL, SF_NOISE, SF_NOCHECKER, SF_ALL};

constexpr uint32_t kShadeLdsMax = 40 * 1024;

int pick_shade_mask(int mask) {
    for (int cand : kShadeMasks)
        if ((mask & ~cand) == 0) return cand;
    return SF_ALL;
}

// Kernel names as rocprofv3 demangles them ("k_persist_sort<112, 8, true>"),
// for rtw_scene_query and the bench's PMC bookkeeping.
std::string kname(const char* k, int f, int m, int lds = -1, int lst = -1) {
    std::string s = std::string(k) + "<" + std::to_string(f);
    if (m >= 0) s += ", " + std::to_string(m);
    if (lds >= 0) s += lds ? ", true" : ", false";
    if (lst >= 0) s += lst ? ", true" : ", false";
    return s + ">";
}

// Fused traversal + shading for the common scene shapes; returns false when
// no fused instantiation covers (features, material set), and the caller
// then runs the split k_intersect / k_shade pair.  probe: only report (and
// name the kernel in *name when given).
bool launch_segment(bool probe, int f, int mask, int grid, hipStream_t st, const scene& S, const job_t& J,
                    const paths_t& A, const fresh_t& FR, ctrs_t* C, const char* base, uint32_t bytes,
                    std::string* name = nullptr) {
    const int pick = pick_shade_mask(mask);
    const bool lds = bytes <= kShadeLdsMax;
    const size_t shm = lds ? bytes : 0;
#define RTW_SEG(FF, MM, LL)                                                                                    \
    if (f == (FF) && pick == (MM) && lds == (LL)) {                                                          \
        if (name) *name = kname("k_segment", FF, MM, LL);                                                    \
        if (!probe)                                                                                           \
            hipLaunchKernelGGL((k_segment<FF, MM, LL>), dim3(grid), dim3(kBlock), shm, st, S, J, A, FR, C, base, bytes); \
        return true;                                                                                         \
    }
#ifndef RTW_SUBSET
    RTW_SEG(0, SF_DIEL, true)
    RTW_SEG(0, SF_METAL | SF_DIEL, true)
    RTW_SEG(0, SF_ALL, true)
    RTW_SEG(0, SF_ALL, false)
    RTW_SEG(F_WBVH, SF_ALL, false)
    RTW_SEG(F_WBVH, SF_ALL, true)
#endif
#undef RTW_SEG
    return false;
}

// Resident workgroups per CU of kernel `fn` at `block` threads and `shm`
// bytes of dynamic LDS on the current device: one occupancy query per
// (kernel, block, LDS bytes, device), cached.  rtw_render_multi renders from
// one host thread per device at once, so the cache is guarded.  Returns 0
// when the block does not fit at all and -1 when the query itself fails (not
// cached): the packet probes and the LDS guard read -1 as "does not fit", only
// grid sizing (grid_blocks) falls back to 2 workgroups per CU.
int blocks_per_cu(const void* fn, int block, size_t shm) {
    static std::mutex mu;
    static std::map<std::tuple<const void*, int, size_t, int>, int> cache;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    const auto key = std::make_tuple(fn, block, shm, dev);
    {
        std::lock_guard<std::mutex> g(mu);
        const auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, block, shm) != hipSuccess) return -1;
    nb = std::max(nb, 0);
    std::lock_guard<std::mutex> g(mu);
    cache[key] = nb;
    return nb;
}

// Grid of a persistent launch: resident workgroups per CU x CUs; a failed
// occupancy query assumes 2 per CU, a block that does not fit still gets 1
// per CU (the LDS guards in the launchers refuse those before this).
int grid_blocks(const void* fn, int block, size_t shm, int cus) {
    const int nb = blocks_per_cu(fn, block, shm);
    return (nb < 0 ? 2 : std::max(1, nb)) * cus;
}

// Persistent kernel for the same instantiation set.  The grid is the number
// of blocks that can be resident at once, so every block starts immediately.
template <int FF, int MM, bool LL, bool LST>
int persist_grid(size_t shm, int cus) {
    return grid_blocks(reinterpret_cast<const void*>(&k_persist<FF, MM, LL, LST>), kPBlock, shm, cus);
}

template <int FF, int MM, bool LL>
int persist_sort_grid(size_t shm, int cus) {
    return grid_blocks(reinterpret_cast<const void*>(&k_persist_sort<FF, MM, LL>), kSortBlock, shm, cus);
}

// The persistent kernels: material-regrouping k_persist_sort for list
// traversal, plain k_persist under a BVH (measured, 1 MI355X: Cornell +14 %,
// random_balls flat +12 %, Book-2 flat +37 % with regrouping; random_balls
// BVH -8 %, Book-2 BVH -2 %: divergent BVH walks dominate there and the
// per-iteration block barriers cost).  RTW_SORT=0/1 forces either (A/B, tests).
bool sort_forced(bool& value) {
    const char* e = std::getenv("RTW_SORT");
    if (!(e && *e)) return false;
    value = std::atoi(e) != 0;
    return true;
}

// BVH node packet of a k_persist<.., LST> launch: the most top nodes (BFS
// numbering, rtw_scene_upload) that fit in LDS beside the kernel's own
// arrays and the shading prefix without costing a workgroup per CU
// (occupancy query per candidate size).  RTW_LDS_NODES=<n> caps it (0 = off:
// A/B).  The node count of the last launch or probe is kept for
// rtw_scene_query.
thread_local uint32_t g_node_packet = 0;
constexpr size_t kPacketNodeBytes = sizeof(node_store);
template <int FF, int MM, bool LL>
uint32_t node_packet(size_t shm, int n_nodes) {
    const char* e = std::getenv("RTW_LDS_NODES");
    uint32_t cap = (e && *e) ? (uint32_t)std::max(0, std::atoi(e)) : 4096u;
    cap = std::min<uint32_t>(cap, (uint32_t)std::max(0, n_nodes));
    if (!cap) return 0;
    const void* fn = reinterpret_cast<const void*>(&k_persist<FF, MM, LL, true>);
    const int base = blocks_per_cu(fn, kPBlock, shm);
    if (base <= 0) return 0;
    const size_t off = (shm + 15) & ~size_t(15);
    uint32_t best = 0;
    for (uint32_t k = 32; k <= cap + 31; k += 32) {
        const uint32_t kk = std::min(k, cap);
        if (blocks_per_cu(fn, kPBlock, off + kk * kPacketNodeBytes) < base) break;
        best = kk;
        if (kk == cap) break;
    }
    return best;
}

// The strict build's factor log holds J.flog_threads threads' paths, indexed
// by global thread id (a path never leaves its thread in k_persist): its grid
// is capped to fit whatever the occupancy query says (a persistent kernel
// drains the sample queue with any grid).
inline int strict_grid(int grid, const job_t& J) {
#if RTW_STRICT_RADIANCE
    return std::max(1, std::min(grid, (int)(J.flog_threads / (uint32_t)kPBlock)));
#else
    return grid;
#endif
}
template <int FF, int MM, bool LL>
void launch_pk(bool probe, std::string* name, int cus, size_t shm, hipStream_t st, const scene& S, const job_t& J,
               ctrs_t* C, const char* base, uint32_t bytes, int stack_need) {
    g_node_packet = 0;
    static const bool sorted = [] {
        bool v;
        // (the strict build folds each path's factors in k_persist)
        return !RTW_STRICT_RADIANCE && (sort_forced(v) ? v : (FF & (F_WBVH | F_GBVH)) == 0);
    }();
    if (sorted) {
        if (name) *name = kname("k_persist_sort", FF, MM, LL);
        if (!probe)
            hipLaunchKernelGGL((k_persist_sort<FF, MM, LL>), dim3(persist_sort_grid<FF, MM, LL>(shm, cus)),
                               dim3(kSortBlock), shm, st, persist_args{S, J, C, base, bytes});
    } else if ((FF & (F_WBVH | F_GBVH)) && stack_need <= kLdsStack &&
               S.n_nodes < 65536) {  // 16-bit LDS stacks
        if (name) *name = kname("k_persist", FF, MM, LL, true);
        uint32_t packet = node_packet<FF, MM, LL>(shm, S.n_nodes);
        const uint32_t off = (uint32_t)((shm + 15) & ~size_t(15));
        // a launch whose LDS does not fit would fault: no packet then
        if (packet && blocks_per_cu(reinterpret_cast<const void*>(&k_persist<FF, MM, LL, true>), kPBlock,
                                    off + packet * kPacketNodeBytes) <= 0)
            packet = 0;
        g_node_packet = packet;
        const size_t shm2 = packet ? off + packet * kPacketNodeBytes : shm;
        if (!probe)
            hipLaunchKernelGGL((k_persist<FF, MM, LL, true>), dim3(strict_grid(persist_grid<FF, MM, LL, true>(shm, cus), J)),
                               dim3(kPBlock), shm2, st, persist_args{S, J, C, base, bytes, packet, off});
    } else {
        if (name) *name = kname("k_persist", FF, MM, LL, false);
        if (!probe)
            hipLaunchKernelGGL((k_persist<FF, MM, LL, false>), dim3(strict_grid(persist_grid<FF, MM, LL, false>(shm, cus), J)),
                               dim3(kPBlock), shm, st, persist_args{S, J, C, base, bytes});
    }
}

bool launch_persist(bool probe, int f, int mask, int cus, hipStream_t st, const scene& S, const job_t& J, ctrs_t* C,
                    const char* base, uint32_t bytes, int stack_need = kStack, bool ysph = false,
                    bool static_scene = false, bool lights = false, bool black = false, bool pin = false,
                    std::string* name = nullptr) {
    if (ysph && !(f & (F_WBVH | F_MEDIA))) f |= F_YSPH;  // world runs are walked: y-sphere scans
    const int pick = pick_shade_mask(mask);
    // specialised kernels only
    const int fs = f | (static_scene ? F_STATIC : 0) | (lights ? F_LIGHTS : F_NOLIGHTS) | (black ? F_BLACK : 0);
    const bool lds = bytes <= kShadeLdsMax;
    const size_t shm = lds ? bytes : 0;
    // the BVH kernels' pinhole forms (F_PIN: camera batches without
    // origins, a larger node packet) for renders whose camera allows it
    if (pin) {
#define RTW_PIN(FF, MM, LL)                                                                    \
        if ((fs | F_PIN) == (FF) && pick == (MM) && lds == (LL)) {                             \
            launch_pk<FF, MM, LL>(probe, name, cus, shm, st, S, J, C, base, bytes, stack_need); \
            return true;                                                                       \
        }
        // Measured (1 MI355X, A/B, profiles/r04/ab_pin_quad_boxrcp.log): C5
        // slice 656.1 vs 644.8 Msamples/s (the packet then holds all 1 668 of
        // Book 2's nodes); C3 2 918 vs 2 933 (its 969 nodes fit already): the
        // Book-2 kernel only.
#ifndef RTW_SUBSET
        RTW_PIN(F_MEDIA | F_GBVH | F_LIGHTS | F_BLACK | F_PIN, SF_NOCHECKER, false)
#endif
#undef RTW_PIN
    }
#define RTW_PER(FF, MM, LL)                                                                     \
    if ((f == (FF) || fs == (FF)) && pick == (MM) && lds == (LL)) {                           \
        launch_pk<FF, MM, LL>(probe, name, cus, shm, st, S, J, C, base, bytes, stack_need);   \
        return true;                                                                          \
    }
    // specialised: small list scenes whose shading data fit in LDS, and the
    // lambertian / metal / dielectric sets of the Book-1 scene, flat or BVH
#ifndef RTW_SUBSET
    RTW_PER(F_STATIC | F_LIGHTS | F_BLACK, SF_DIEL, true)
    RTW_PER(F_STATIC | F_LIGHTS, SF_DIEL, true)
    RTW_PER(0, SF_DIEL, true)
    RTW_PER(0, SF_METAL | SF_DIEL, true)
    RTW_PER(0, SF_ALL, true)
    RTW_PER(0, SF_METAL | SF_DIEL, false)
    RTW_PER(F_YSPH | F_NOLIGHTS, SF_METAL | SF_DIEL, false)
    RTW_PER(F_YSPH, SF_METAL | SF_DIEL, false)
    RTW_PER(F_WBVH | F_NOLIGHTS, SF_METAL | SF_DIEL, false)
    RTW_PER(F_WBVH, SF_METAL | SF_DIEL, false)
    // media scenes without checker textures (Book 2): the checker's sines
    // and texture recursion compiled out halves the kernel's SGPR spills
    RTW_PER(F_MEDIA | F_GBVH | F_LIGHTS | F_BLACK, SF_NOCHECKER, false)
    RTW_PER(F_MEDIA | F_GBVH, SF_NOCHECKER, false)
    RTW_PER(F_MEDIA, SF_NOCHECKER, false)
#else
    // experiment builds (scripts/ru_kernel.sh): one persistent kernel only
    RTW_PER(RTW_SUBSET_F, RTW_SUBSET_M, RTW_SUBSET_L)
#endif
#undef RTW_PER
    // general: every material / texture, scene read through the caches, one
    // instantiation per traversal feature set (a world BVH never holds media)
#define RTW_PER(FF)                                                                          \
    if (f == (FF)) {                                                                       \
        launch_pk<FF, SF_ALL, false>(probe, name, cus, 0, st, S, J, C, base, bytes, stack_need); \
        return true;                                                                       \
    }
#ifndef RTW_SUBSET
    RTW_PER(0)
    RTW_PER(F_YSPH)
    RTW_PER(F_MEDIA)
    RTW_PER(F_WBVH)
    RTW_PER(F_GBVH)
    RTW_PER(F_YSPH | F_GBVH)
    RTW_PER(F_MEDIA | F_GBVH)
    RTW_PER(F_WBVH | F_GBVH)
#endif
#undef RTW_PER
    return false;
}

// BVH node packet of a k_fast<.., LST> launch: the most top nodes that fit
// in LDS beside the stacks without costing a workgroup per CU (node_packet's
// rule; RTW_LDS_NODES caps it, 0 = off).
uint32_t fast_node_packet(const void* fn, int n_nodes, int block) {
    const char* e = std::getenv("RTW_LDS_NODES");
    uint32_t cap = (e && *e) ? (uint32_t)std::max(0, std::atoi(e)) : 4096u;
    cap = std::min<uint32_t>(cap, (uint32_t)std::max(0, n_nodes));
    if (!cap) return 0;
    const int base = blocks_per_cu(fn, block, 0);
    if (base <= 0) return 0;
    uint32_t best = 0;
    for (uint32_t k = 32; k <= cap + 31; k += 32) {
        const uint32_t kk = std::min(k, cap);
        if (blocks_per_cu(fn, block, kk * sizeof(node_store)) < base) break;
        best = kk;
        if (kk == cap) break;
    }
    return best;
}

// The fp32 fast-mode kernel of a scene: one instantiation per traversal
// feature set, LDS stacks when the deepest walk fits them.  grid = resident
// blocks (occupancy query, cached).  probe: name it only.
template <int FF, bool LST>
void launch_fast_t(bool probe, std::string* name, int cus, hipStream_t st, const fast_args& A) {
    if (name) *name = kname("k_fast", FF, -1, LST ? 1 : 0);
    if (probe) return;
    const void* fn = reinterpret_cast<const void*>(&k_fast<FF, LST>);
    fast_args a = A;
    constexpr int blk = rtwf::fast_block(FF);
    a.lds_nodes = LST ? fast_node_packet(fn, A.S.n_nodes, blk) : 0u;
    const size_t shm = (size_t)a.lds_nodes * sizeof(node_store);
    const int grid = grid_blocks(fn, blk, shm, cus);
    hipLaunchKernelGGL((k_fast<FF, LST>), dim3(grid), dim3(blk), shm, st, a);
}
template <int FF, bool LL>
void launch_fast_sort_t(bool probe, std::string* name, int cus, hipStream_t st, const fast_args& A,
                        const char* base, uint32_t bytes) {
    if (name) *name = kname("k_fast_sort", FF, -1, LL ? 1 : 0);
    if (probe) return;
    const size_t shm = LL ? bytes : 0;
    const int grid = grid_blocks(reinterpret_cast<const void*>(&k_fast_sort<FF, LL>), kSortBlock, shm, cus);
    fast_args a = A;  // the arrays' offsets in the LDS copy (lds_fscene_off)
    const void* ptrs[9] = {A.S.prims, A.S.entries, A.S.ops, A.S.materials, A.S.textures,
                           A.S.lights, A.S.ranvec, A.S.perm, A.S.frames};
    for (int k = 0; k < 9; ++k) {
        const char* c = static_cast<const char*>(ptrs[k]);
        a.lds_off[k] = (c && base && c >= base && c < base + bytes) ? (uint32_t)(c - base) : ~0u;
    }
    hipLaunchKernelGGL((k_fast_sort<FF, LL>), dim3(grid), dim3(kSortBlock), shm, st, a, base, bytes);
}
// RTW_FAST_SORT=0: list scenes take k_fast too (A/B)
bool fast_sort_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("RTW_FAST_SORT");
        return !(e && *e && std::atoi(e) == 0);
    }();
    return on;
}
// the stack a persistent fp64 launch with LDS stacks needs
int lst_stack_need(const handle_t* h) { return h->stack_need; }
void launch_fast(bool probe, const handle_t* h, hipStream_t st, const fast_args& A, std::string* name = nullptr) {
    const int f = h->features & (F_MEDIA | F_WBVH | F_GBVH);
#ifdef RTW_SUBSET_FAST  // experiment builds (scripts/ru_kernel.sh): the list scenes' fp32 kernel only
#ifdef RTW_SUBSET_FAST_F  // ... or one BVH kernel k_fast<RTW_SUBSET_FAST_F, true>
    launch_fast_t<RTW_SUBSET_FAST_F, true>(probe, name, h->cus, st, A);
#else
    launch_fast_sort_t<FF_NONOISE, true>(probe, name, h->cus, st, A, static_cast<const char*>(h->scene32.p),
                                         h->f32_bytes);
    launch_fast_t<F_WBVH | FF_NONOISE, true>(probe, name, h->cus, st, A);
#endif
#else
    if ((f & (F_WBVH | F_GBVH)) == 0 && fast_sort_enabled()) {  // list scenes: regrouping kernel
        const char* base = static_cast<const char*>(h->scene32.p);
        const bool lds = h->f32_bytes <= kShadeLdsMax;
        if (f == 0 && !(h->shade_mask & SF_NOISE))  // Cornell, random_balls: no marble texture
            lds ? launch_fast_sort_t<FF_NONOISE, true>(probe, name, h->cus, st, A, base, h->f32_bytes)
                : launch_fast_sort_t<FF_NONOISE, false>(probe, name, h->cus, st, A, base, h->f32_bytes);
        else if (f == F_MEDIA)
            lds ? launch_fast_sort_t<F_MEDIA, true>(probe, name, h->cus, st, A, base, h->f32_bytes)
                : launch_fast_sort_t<F_MEDIA, false>(probe, name, h->cus, st, A, base, h->f32_bytes);
        else
            lds ? launch_fast_sort_t<0, true>(probe, name, h->cus, st, A, base, h->f32_bytes)
                : launch_fast_sort_t<0, false>(probe, name, h->cus, st, A, base, h->f32_bytes);
        return;
    }
    // (media scenes have no world BVH: their walks are group walks from an
    // empty stack, group_depth entries deep)
    const int need = (f & F_MEDIA) ? h->group_depth : h->stack_need;
    const bool lst = (f & (F_WBVH | F_GBVH)) && need <= rtwf::fast_stack(f) && h->S.n_nodes < 65536;
    if (f == F_WBVH && lst && !(h->shade_mask & SF_NOISE)) {  // random_balls + BVH: no marble texture
        launch_fast_t<F_WBVH | FF_NONOISE, true>(probe, name, h->cus, st, A);
        return;
    }
    switch (f * 2 + (lst ? 1 : 0)) {
#define RTW_FAST(FF, LL) \
    case (FF) * 2 + (LL ? 1 : 0): launch_fast_t<FF, LL>(probe, name, h->cus, st, A); break;
        RTW_FAST(0, false)
        RTW_FAST(F_MEDIA, false)
        RTW_FAST(F_GBVH, false)
        RTW_FAST(F_GBVH, true)
        RTW_FAST(F_WBVH, false)
        RTW_FAST(F_WBVH, true)
        RTW_FAST(F_WBVH | F_GBVH, false)
        RTW_FAST(F_WBVH | F_GBVH, true)
        RTW_FAST(F_MEDIA | F_GBVH, false)
        RTW_FAST(F_MEDIA | F_GBVH, true)
#undef RTW_FAST
    default:
        launch_fast_t<F_MEDIA | F_GBVH, false>(probe, name, h->cus, st, A);
    }
#endif
}

void launch_shade(int mask, int grid, hipStream_t st, const scene& S, const job_t& J, const paths_t& A,
                  const fresh_t& F, const double* ht, const int32_t* hid, ctrs_t* C, const char* base, uint32_t bytes) {
    const int pick = pick_shade_mask(mask);
    const bool lds = bytes <= kShadeLdsMax;
    const size_t shm = lds ? bytes : 0;
    switch (pick * 2 + (lds ? 1 : 0)) {
#define RTW_CASE(M, LDS)                                                                                   \
    case M * 2 + (LDS ? 1 : 0):                                                                            \
        hipLaunchKernelGGL((k_shade<M, LDS>), dim3(grid), dim3(kBlock), shm, st, S, J, A, F, ht, hid, C, base, bytes); \
        break;
#ifndef RTW_SUBSET
        RTW_CASE(SF_DIEL, true)
        RTW_CASE(SF_DIEL, false)
        RTW_CASE(SF_METAL | SF_DIEL, true)
        RTW_CASE(SF_METAL | SF_DIEL, false)
        RTW_CASE(SF_NOISE, true)
        RTW_CASE(SF_NOISE, false)
        RTW_CASE(SF_ALL, true)
#endif
#undef RTW_CASE
    default:
        hipLaunchKernelGGL((k_shade<SF_ALL, false>), dim3(grid), dim3(kBlock), 0, st, S, J, A, F, ht, hid, C, base, bytes);
    }
}

// one traversal kernel per scene-feature combination (a world BVH never
// coexists with media: validate_desc)
void launch_intersect(int f, int grid, hipStream_t st, const scene& S, const paths_t& A, const fresh_t& FR,
                      double* ht, int32_t* hid,
                      ctrs_t* C) {
    switch (f) {
#define RTW_CASE(F)                                                                               \
    case F:                                                                                       \
        hipLaunchKernelGGL(k_intersect<F>, dim3(grid), dim3(kBlock), 0, st, S, A, FR, ht, hid, C); \
        break;
#ifndef RTW_SUBSET
        RTW_CASE(0)
        RTW_CASE(F_MEDIA)
        RTW_CASE(F_WBVH)
        RTW_CASE(F_GBVH)
        RTW_CASE(F_MEDIA | F_GBVH)
        RTW_CASE(F_WBVH | F_GBVH)
#endif
#undef RTW_CASE
    default:
        hipLaunchKernelGGL(k_intersect<F_MEDIA | F_GBVH>, dim3(grid), dim3(kBlock), 0, st, S, A, FR, ht, hid, C);
    }
}


hipEvent_t event_at(handle_t* h, size_t k) {
    while (h->events.size() <= k) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        h->events.push_back(e);
    }
    return h->events[k];
}

size_t pass_budget_samples() {
    if (const char* s = std::getenv("RTW_PASS_SAMPLES")) {
        const long long v = std::atoll(s);
        if (v > 0) return (size_t)v;
    }
    return size_t(1) << 30;  // 24 GiB of per-sample radiance records per pass (T: one pass)
}

// The traversal kernel a render of `h` launches under the current
// environment (RTW_MODE / RTW_SPLIT / RTW_SORT), named as rocprofv3 does.
std::string render_kernel_name(const handle_t* h) {
    std::string name;
    const job_t J{};
    const char* mode_env = std::getenv("RTW_MODE");
    const bool wavefront = mode_env && std::string(mode_env) == "wavefront";
    if (!wavefront && launch_persist(true, h->features, h->shade_mask, 0, nullptr, h->S, J, nullptr, h->scene_base,
                                     h->shade_bytes, lst_stack_need(h), h->ysph, !h->movers, h->S.n_lights > 0,
                                     h->S.background != RTW_BG_GRADIENT && h->S.render_type != RTW_RENDER_NORMAL,
                                     h->desc_pin, &name))
        return name;
    const char* split_env = std::getenv("RTW_SPLIT");
    const paths_t A{};
    const fresh_t FR{};
    if (!(split_env && std::atoi(split_env) != 0) &&
        launch_segment(true, h->features, h->shade_mask, 0, nullptr, h->S, J, A, FR, nullptr, h->scene_base,
                       h->shade_bytes, &name))
        return name;
    return kname("k_intersect", h->features, -1);
}

// PPM channel bytes (RayTracingWeekend.cpp:266-270): int(255.99f * c) as
// x86 converts (truncation; NaN / out of range -> INT_MIN, cvttsd2si).
__global__ __launch_bounds__(kBlock) void k_quantize(const double* __restrict__ canvas, size_t n,
                                                     int32_t* __restrict__ out) {
    for (size_t k = blockIdx.x * (size_t)kBlock + threadIdx.x; k < n; k += (size_t)gridDim.x * kBlock) {
        const double x = (double)255.99f * canvas[k];
        out[k] = (x == x && x < 2147483648.0 && x > -2147483649.0) ? (int32_t)x : (int32_t)0x80000000u;
    }
}

// dst += src (rtw_render_multi's final add into a device accumulator)
__global__ __launch_bounds__(kBlock) void k_add(double* __restrict__ dst, const double* __restrict__ src, size_t n) {
    for (size_t k = blockIdx.x * (size_t)kBlock + threadIdx.x; k < n; k += (size_t)gridDim.x * kBlock)
        dst[k] += src[k];
}

unsigned grid_for(size_t n) { return (unsigned)std::max<size_t>(1, std::min<size_t>((n + kBlock - 1) / kBlock, 8192)); }

}  // namespace

#ifndef RTW_BUILD_ID
#define RTW_BUILD_ID "unknown"
#endif
extern "C" const char* rtw_build_id(void) { return RTW_BUILD_ID; }

extern "C" int rtw_scene_query(void* handle, rtw_scene_info* out) {
    const handle_t* h = static_cast<const handle_t*>(handle);
    if (!h || !out) return rtw_fail(RTW_ERR_INVALID, "rtw_scene_query: null argument");
    std::memset(out, 0, sizeof *out);
    out->device = h->device;
    out->n_world_runs = h->n_runs;
    out->n_ysphere_runs = h->n_ysph_runs;
    out->n_plain_runs = h->n_plain_runs;
    out->features = h->features;
    out->shade_mask = h->shade_mask;
    out->shade_lds_bytes = h->shade_bytes <= kShadeLdsMax ? (int32_t)h->shade_bytes : 0;
    HIPCHK(hipSetDevice(h->device));  // occupancy queries of the probe
    g_node_packet = 0;
    const std::string k = render_kernel_name(h);
    out->bvh_lds_nodes = (int32_t)g_node_packet;  // set by the probe (launch_pk)
    std::snprintf(out->kernel, sizeof out->kernel, "%s", k.c_str());
    std::snprintf(out->build_id, sizeof out->build_id, "%s", RTW_BUILD_ID);
    std::string kf;
    launch_fast(true, h, nullptr, fast_args{}, &kf);
    std::snprintf(out->kernel_fast, sizeof out->kernel_fast, "%s", kf.c_str());
    return RTW_OK;
}

extern "C" int rtw_quantize_canvas_device(void* handle, const double* canvas, int nx, int ny, int32_t* out) {
    handle_t* h = static_cast<handle_t*>(handle);
    if (!h || !canvas || !out || nx <= 0 || ny <= 0)
        return rtw_fail(RTW_ERR_INVALID, "rtw_quantize_canvas_device: bad argument");
    HIPCHK(hipSetDevice(h->device));
    const size_t n = (size_t)nx * (size_t)ny * 3;
    hipLaunchKernelGGL(k_quantize, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, canvas, n, out);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(h->stream));
    return RTW_OK;
}

// internal (rtw_host_util.h): the device of a handle, and dst += src on it
int rtw_handle_device(void* handle) { return handle ? static_cast<handle_t*>(handle)->device : -1; }

int rtw_handle_add_device(void* handle, double* dst, const double* src, size_t n) {
    handle_t* h = static_cast<handle_t*>(handle);
    HIPCHK(hipSetDevice(h->device));
    hipLaunchKernelGGL(k_add, dim3(grid_for(n)), dim3(kBlock), 0, h->stream, dst, src, n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(h->stream));
    return RTW_OK;
}

// A device accumulator must be memory the scene's GPU can address: device
// memory of that GPU (hipMalloc, torch's caching and expandable-segment
// allocators) or managed memory (hipMallocManaged: any GPU).  Host memory,
// pinned host memory and unknown pointers are refused (a host pointer is
// passed with accum_on_device = 0 instead).
int rtw_check_device_ptr(const void* p, int device, const char* what, bool allow_managed) {
    hipPointerAttribute_t a;
    std::memset(&a, 0, sizeof a);
    if (hipPointerGetAttributes(&a, p) != hipSuccess ||
        (a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged)) {
        (void)hipGetLastError();  // clear the sticky error of a failed query
        return rtw_fail(RTW_ERR_INVALID, std::string(what) + ": accum_on_device is set but the accumulator is not "
                                                              "device or managed memory");
    }
    if (a.type == hipMemoryTypeManaged && !allow_managed)
        return rtw_fail(RTW_ERR_UNSUPPORTED, std::string(what) + ": a managed-memory accumulator is supported with "
                                                                  "one GPU only (the cross-device write is unverified)");
    if (a.type == hipMemoryTypeDevice && a.device != device)
        return rtw_fail(RTW_ERR_INVALID, std::string(what) + ": the device accumulator lives on device " +
                                             std::to_string(a.device) + ", the scene on device " +
                                             std::to_string(device));
    return RTW_OK;
}

extern "C" int rtw_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" int rtw_scene_upload(int device, const rtw_scene_desc* desc, void** out_handle) {
    if (!out_handle) return rtw_fail(RTW_ERR_INVALID, "rtw_scene_upload: null out_handle");
    *out_handle = nullptr;
    int rc = validate_desc(desc);
    if (rc) return rc;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return rtw_fail(RTW_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return rtw_fail(RTW_ERR_INVALID, "device index out of range");
    HIPCHK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return rtw_fail(RTW_ERR_NO_DEVICE, std::string("device is ") + prop.gcnArchName + ", this build targets gfx950");
    handle_t* h = new handle_t;
    h->device = device;
    h->grid = prop.multiProcessorCount * 8;
    h->cus = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return rtw_fail(RTW_ERR_HIP, "hipStreamCreate failed");
    }
    rc = upload_scene(h, desc);
    if (!rc) rc = h->ctrs.ensure(sizeof(ctrs_t));
    if (!rc && hipHostMalloc((void**)&h->host_ctrs, sizeof(ctrs_t) * 64, hipHostMallocDefault) != hipSuccess)
        rc = rtw_fail(RTW_ERR_OOM, "hipHostMalloc failed");
    if (rc) {
        rtw_scene_free(h);
        return rc;
    }
    *out_handle = h;
    return RTW_OK;
}

extern "C" void rtw_scene_free(void* handle) {
    handle_t* h = static_cast<handle_t*>(handle);
    if (!h) return;
    hipSetDevice(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    h->scene_mem.release();
    h->scene32.release();
    h->pool[0].release();
    h->pool[1].release();
    h->fresh.release();
    h->hits.release();
    h->radiance.release();
    h->run.release();
    h->flog.release();
    h->accum.release();
    h->ctrs.release();
    h->camera.release();
    if (h->host_ctrs) hipHostFree(h->host_ctrs);
    for (hipEvent_t e : h->events) hipEventDestroy(e);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;
}

extern "C" int rtw_finalize_canvas_device(void* handle, const double* accum, int nx, int ny, int spp,
                                          double* canvas) {
    handle_t* h = static_cast<handle_t*>(handle);
    if (!h || !accum || !canvas || nx <= 0 || ny <= 0 || spp <= 0)
        return rtw_fail(RTW_ERR_INVALID, "rtw_finalize_canvas_device: bad argument");
    HIPCHK(hipSetDevice(h->device));
    const size_t n = (size_t)nx * (size_t)ny * 3;
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)std::min<size_t>((n + kBlock - 1) / kBlock, 8192)), dim3(kBlock), 0,
                       h->stream, accum, n, (double)spp, canvas);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(h->stream));
    return RTW_OK;
}

extern "C" int rtw_render_accumulate(void* handle, const rtw_camera_desc* camera, const rtw_render_params* prm,
                                     double* accum_rgb, rtw_stats* out_stats) {
    handle_t* h = static_cast<handle_t*>(handle);
    if (!h || !camera || !prm || !accum_rgb) return rtw_fail(RTW_ERR_INVALID, "rtw_render_accumulate: null argument");
    const rtw_render_params& R = *prm;
    if (R.nx <= 0 || R.ny <= 0 || R.spp <= 0 || R.spp_begin < 0 || R.spp_begin > R.spp || R.spp_count < 0)
        return rtw_fail(RTW_ERR_INVALID, "rtw_render_accumulate: bad image / sample parameters");
    const int spp_count = R.spp_count ? R.spp_count : R.spp - R.spp_begin;
    if (R.spp_begin + (long long)spp_count > R.spp) return rtw_fail(RTW_ERR_INVALID, "sample range exceeds spp");
    if (R.precision != RTW_PRECISION_FP64 && R.precision != RTW_PRECISION_FP32)
        return rtw_fail(RTW_ERR_INVALID, "rtw_render_accumulate: unknown precision");
    const int row_step = R.row_step > 0 ? R.row_step : 1;
    if (R.row_begin < 0 || R.row_begin >= R.ny) return rtw_fail(RTW_ERR_INVALID, "row_begin out of range");
    const int n_rows = (R.ny - R.row_begin + row_step - 1) / row_step;
    const uint64_t npix = (uint64_t)n_rows * (uint64_t)R.nx;
    if ((uint64_t)R.nx * R.ny >= (1ull << 32) || npix >= (1ull << 31))
        return rtw_fail(RTW_ERR_INVALID, "image too large for 32-bit pixel ids");
    if (h->bvh_motion && (std::min(camera->time0, camera->time1) < h->shutter0 ||
                          std::max(camera->time0, camera->time1) > h->shutter1))
        return rtw_fail(RTW_ERR_INVALID,
                        "rtw_render_accumulate: camera shutter outside the one the scene's BVH was built for "
                        "(moving spheres); flatten the scene with this camera");
    HIPCHK(hipSetDevice(h->device));
    if (R.accum_on_device)
        if (int rc = rtw_check_device_ptr(accum_rgb, h->device, "rtw_render_accumulate")) return rc;
    hipStream_t st = h->stream;

    rtw_stats stats;
    std::memset(&stats, 0, sizeof stats);
    if (spp_count == 0 || R.max_depth <= 0) {
        // color() with depth <= 0 returns 0 (RayTracingWeekend.cpp:47-48):
        // every sample adds zero radiance, the accumulator is unchanged.
        stats.samples = (uint64_t)spp_count * npix;
        if (out_stats) *out_stats = stats;
        return RTW_OK;
    }

    // execution form: persistent (paths in registers, one launch per pass)
    // unless RTW_MODE=wavefront or no persistent instantiation covers the
    // scene (a probe: nothing is launched); the strict build refuses the
    // other forms here, before any allocation or launch
    const char* mode_env = std::getenv("RTW_MODE");
    // fp32 fast mode: its own persistent kernel (rtw_fast.h), same passes,
    // radiance records and ordered per-pixel reduction
    const bool fast = R.precision == RTW_PRECISION_FP32;
    const bool pin = camera_is_pinhole(*camera);
    bool persistent;
    {
        job_t J0{};
        persistent = fast || (!(mode_env && std::string(mode_env) == "wavefront") &&
                              launch_persist(true, h->features, h->shade_mask, 0, st, h->S, J0, nullptr,
                                             h->scene_base, h->shade_bytes, lst_stack_need(h), h->ysph, !h->movers,
                                             h->S.n_lights > 0,
                                             h->S.background != RTW_BG_GRADIENT &&
                                                 h->S.render_type != RTW_RENDER_NORMAL,
                                             pin));
    }
    if (RTW_STRICT_RADIANCE && !persistent)
        return rtw_fail(RTW_ERR_UNSUPPORTED, "the strict-radiance build renders with the persistent kernel only "
                                             "(RTW_MODE=wavefront or a scene without a persistent instantiation)");

    // pool and pass sizing
    uint32_t pool = R.wavefront_paths > 0 ? (uint32_t)R.wavefront_paths : (1u << 21);
    const size_t budget = pass_budget_samples();
    uint64_t pass_spp = std::max<uint64_t>(1, std::min<uint64_t>(spp_count, budget / npix));
    pass_spp = std::min<uint64_t>(pass_spp, ((1ull << 32) - 1) / npix);
    const uint64_t pass_samples = pass_spp * npix;
    pool = (uint32_t)std::min<uint64_t>(pool, pass_samples);
    pool = std::max<uint32_t>(pool, 1);

    int rc;
    if ((rc = h->pool[0].ensure(paths_bytes(pool)))) return rc;
    if ((rc = h->pool[1].ensure(paths_bytes(pool)))) return rc;
    if ((rc = h->fresh.ensure(fresh_bytes(pool)))) return rc;
    if ((rc = h->hits.ensure((size_t)pool * 12))) return rc;
    if ((rc = h->radiance.ensure(pass_samples * 24))) return rc;
    if ((rc = h->run.ensure(npix * 24))) return rc;
    paths_t A = carve_paths(h->pool[0].p, pool), B = carve_paths(h->pool[1].p, pool);
    const fresh_t FR = carve_fresh(h->fresh.p, pool);
    double* ht = static_cast<double*>(h->hits.p);
    int32_t* hid = reinterpret_cast<int32_t*>(static_cast<char*>(h->hits.p) + (size_t)pool * 8);
    ctrs_t* C = static_cast<ctrs_t*>(h->ctrs.p);
    double* run = static_cast<double*>(h->run.p);
    HIPCHK(hipMemsetAsync(run, 0, npix * 24, st));
    HIPCHK(hipMemsetAsync(C, 0, sizeof(ctrs_t), st));

    job_t J;
    h->cam_host = *camera;
    // camera_sample<false>'s pinhole test reads lens_radius and the origin; a
    // lens-less camera whose u or v is not finite gets lens_radius NaN in the
    // device copy: rd = NaN * p, so its offset is NaN as the reference's
    // u * rd.x + v * rd.y is (the same all-NaN rays, the same draws), and the
    // shortcut does not apply
    {
        bool uv = true;
        for (int k = 0; k < 3; ++k) uv = uv && std::isfinite(camera->u[k]) && std::isfinite(camera->v[k]);
        if (!uv && h->cam_host.lens_radius == 0.0) h->cam_host.lens_radius = __builtin_nan("");
    }
    if ((rc = h->camera.ensure(sizeof(rtw_camera_desc) + 2 * sizeof(double)))) return rc;
    HIPCHK(hipMemcpyAsync(h->camera.p, &h->cam_host, sizeof(rtw_camera_desc), hipMemcpyHostToDevice, st));
    J.cam = static_cast<const rtw_camera_desc*>(h->camera.p);
    hipLaunchKernelGGL(k_recips, dim3(1), dim3(64), 0, st,
                       reinterpret_cast<double*>(static_cast<char*>(h->camera.p) + sizeof(rtw_camera_desc)), R.nx, R.ny);
    HIPCHK(hipGetLastError());
    J.seed_mix = host_splitmix64(R.seed);
    J.cam_pin = pin ? 1u : 0u;
    J.npix = (uint32_t)npix;
    J.nx = R.nx, J.ny = R.ny, J.row_begin = R.row_begin, J.row_step = row_step;
    J.div_npix = rtwd::udiv_magic(J.npix);
    J.div_nx = rtwd::udiv_magic((uint32_t)R.nx);
    J.max_depth = R.max_depth;
    J.L = static_cast<double*>(h->radiance.p);
#if RTW_STRICT_RADIANCE
    // a factor log per thread of the largest resident grid (2 048 threads per
    // CU), one 32-B entry per bounce
    J.flog_threads = (uint32_t)h->cus * 2048u;
    if ((rc = h->flog.ensure((size_t)J.flog_threads * (size_t)R.max_depth * 32))) return rc;
    J.flog = static_cast<double*>(h->flog.p);
#endif

    const int grid = h->grid;
    const int regen_grid = (int)((pool + kRegenSlots - 1) / kRegenSlots);
    size_t ev = 0;
    std::vector<std::pair<size_t, size_t>> isect_ev, shade_ev;
    hipEvent_t ev_begin = event_at(h, ev++), ev_end = event_at(h, ev++);
    if (!ev_begin || !ev_end) return rtw_fail(RTW_ERR_HIP, "hipEventCreate failed");
    HIPCHK(hipEventRecord(ev_begin, st));
    // collect_kernel_times: 1 = events around each traversal launch (the
    // roofline kernel), 2 = also around each shade launch.  Every event pair
    // costs a few us of queue gap per iteration, so the default is neither.
    const bool timed = R.collect_kernel_times != 0;
    const bool timed_shade = R.collect_kernel_times >= 2;
    // traversal + shading fused into one kernel where an instantiation covers
    // the scene (RTW_SPLIT=1 forces the split pair, for tests and profiling)
    const char* split_env = std::getenv("RTW_SPLIT");
    const bool fused = !(split_env && std::atoi(split_env) != 0) &&
                       launch_segment(true, h->features, h->shade_mask, 0, st, h->S, J, A, FR, C, h->scene_base,
                                      h->shade_bytes);
    const int check_every = 4;
    fast_args FA{};
    if (fast) {
        FA.S = h->F32;
        FA.C = C;
        const rtw_camera_desc& c = *camera;
        for (int k = 0; k < 3; ++k) {
            FA.cam.origin[k] = (float)c.origin[k], FA.cam.lower_left[k] = (float)c.lower_left[k];
            FA.cam.horizontal[k] = (float)c.horizontal[k], FA.cam.vertical[k] = (float)c.vertical[k];
            FA.cam.u[k] = (float)c.u[k], FA.cam.v[k] = (float)c.v[k];
        }
        FA.cam.time0 = (float)c.time0, FA.cam.dtime = (float)(c.time1 - c.time0);
        FA.cam.lens_radius = (float)c.lens_radius;
    }
    for (uint64_t done = 0; done < (uint64_t)spp_count; done += pass_spp) {
        const uint32_t S_pass = (uint32_t)std::min<uint64_t>(pass_spp, spp_count - done);
        J.total = (uint32_t)(S_pass * npix);
        J.spp_pass = S_pass;
        J.div_spp = rtwd::udiv_magic(S_pass);
        J.s_begin = R.spp_begin + (int)done;
        const uint32_t n0 = std::min<uint32_t>(pool, J.total);
        if (persistent) {
            hipLaunchKernelGGL(k_fill, dim3(1), dim3(kBlock), 0, st, A, C, 0u);  // reset the queue
            size_t e0 = 0, e1 = 0;
            if (timed) {
                e0 = ev++, e1 = ev++;
                if (!event_at(h, e1)) return rtw_fail(RTW_ERR_HIP, "hipEventCreate failed");
                HIPCHK(hipEventRecord(h->events[e0], st));
            }
            if (fast) {
                FA.J = J;
                launch_fast(false, h, st, FA);
            } else {
                launch_persist(false, h->features, h->shade_mask, h->cus, st, h->S, J, C, h->scene_base,
                               h->shade_bytes, lst_stack_need(h), h->ysph, !h->movers, h->S.n_lights > 0,
                               h->S.background != RTW_BG_GRADIENT && h->S.render_type != RTW_RENDER_NORMAL, pin);
            }
            HIPCHK(hipGetLastError());
            if (timed) {
                HIPCHK(hipEventRecord(h->events[e1], st));
                isect_ev.push_back({e0, e1});
            }
            stats.launches_intersect++;
            stats.iterations++;
            if (fast)
                hipLaunchKernelGGL(k_reduce<float>, dim3(reduce_grid(npix)), dim3(kBlock), 0, st,
                                   reinterpret_cast<const float*>(J.L), (uint32_t)npix, S_pass, run);
            else
                hipLaunchKernelGGL(k_reduce<double>, dim3(reduce_grid(npix)), dim3(kBlock), 0, st, J.L,
                                   (uint32_t)npix, S_pass, run);
            HIPCHK(hipGetLastError());
            stats.samples += J.total;
            continue;
        }
        hipLaunchKernelGGL(k_fill, dim3((n0 + kBlock - 1) / kBlock), dim3(kBlock), 0, st, A, C, n0);
        hipLaunchKernelGGL(k_regen, dim3(regen_grid), dim3(kBlock), 0, st, J, A, FR, C);
        HIPCHK(hipGetLastError());
        bool tail = false;
        std::vector<size_t> checks;  // event slots of status copies, with their copy index
        // every iteration retires >= 1 live segment; a pass needs at most
        // total * max_depth / pool + max_depth iterations plus the lag of the
        // status snapshots -- far beyond that the pool is not draining: fail
        const uint64_t cap = (uint64_t)J.total * (uint64_t)R.max_depth / n0 + 4ull * R.max_depth + 64;
        for (uint64_t it = 0;; ++it) {
            if (it > cap) return rtw_fail(RTW_ERR_HIP, "wavefront did not drain (internal error)");
            {
                size_t e0 = 0, e1 = 0;
                if (fused) {
                    if (timed) {
                        e0 = ev++, e1 = ev++;
                        if (!event_at(h, e1)) return rtw_fail(RTW_ERR_HIP, "hipEventCreate failed");
                        HIPCHK(hipEventRecord(h->events[e0], st));
                    }
                    launch_segment(false, h->features, h->shade_mask, grid, st, h->S, J, A, FR, C, h->scene_base,
                                   h->shade_bytes);
                    if (timed) {
                        HIPCHK(hipEventRecord(h->events[e1], st));
                        isect_ev.push_back({e0, e1});
                    }
                } else {
                if (timed) {
                    e0 = ev++, e1 = ev++;
                    if (!event_at(h, e1)) return rtw_fail(RTW_ERR_HIP, "hipEventCreate failed");
                    HIPCHK(hipEventRecord(h->events[e0], st));
                }
                launch_intersect(h->features, grid, st, h->S, A, FR, ht, hid, C);
                if (timed) {
                    HIPCHK(hipEventRecord(h->events[e1], st));
                    isect_ev.push_back({e0, e1});
                }
                if (timed_shade) {
                    e0 = ev++, e1 = ev++;
                    if (!event_at(h, e1)) return rtw_fail(RTW_ERR_HIP, "hipEventCreate failed");
                    HIPCHK(hipEventRecord(h->events[e0], st));
                }
                launch_shade(h->shade_mask, grid, st, h->S, J, A, FR, ht, hid, C, h->scene_base, h->shade_bytes);
                if (timed_shade) {
                    HIPCHK(hipEventRecord(h->events[e1], st));
                    shade_ev.push_back({e0, e1});
                }
                }
                if (!tail) hipLaunchKernelGGL(k_regen, dim3(regen_grid), dim3(kBlock), 0, st, J, A, FR, C);
                HIPCHK(hipGetLastError());
                stats.launches_intersect++;
                stats.iterations++;
                if (tail) {
                    hipLaunchKernelGGL(k_compact, dim3(grid), dim3(kBlock), 0, st, A, B, C);
                    hipLaunchKernelGGL(k_commit, dim3(1), dim3(1), 0, st, C);
                    HIPCHK(hipGetLastError());
                    std::swap(A, B);
                }
            }
            if (it % check_every == check_every - 1) {
                // status snapshot; decide from the previous snapshot so the GPU
                // keeps `check_every` iterations of queued work
                const size_t slot = checks.size() % 64;
                HIPCHK(hipMemcpyAsync(&h->host_ctrs[slot], C, sizeof(ctrs_t), hipMemcpyDeviceToHost, st));
                const size_t e = ev++;
                if (!event_at(h, e)) return rtw_fail(RTW_ERR_HIP, "hipEventCreate failed");
                HIPCHK(hipEventRecord(h->events[e], st));
                checks.push_back(e);
                const size_t idx = checks.size() >= 2 ? checks.size() - 2 : 0;
                HIPCHK(hipEventSynchronize(h->events[checks[idx]]));
                const ctrs_t snap = h->host_ctrs[idx % 64];
                if (queue_drained(snap, J.total)) tail = true;
                if (tail && snap.n == 0) break;
            }
        }
        hipLaunchKernelGGL(k_reduce<double>, dim3(reduce_grid(npix)), dim3(kBlock), 0, st,
                           J.L, (uint32_t)npix, S_pass, run);  // the wavefront form is fp64 only
        HIPCHK(hipGetLastError());
        stats.samples += J.total;
    }

    // accum += run
    double* acc_dev = accum_rgb;
    const size_t img_bytes = (size_t)R.nx * R.ny * 24;
    if (!R.accum_on_device) {
        if ((rc = h->accum.ensure(img_bytes))) return rc;
        acc_dev = static_cast<double*>(h->accum.p);
        HIPCHK(hipMemcpyAsync(acc_dev, accum_rgb, img_bytes, hipMemcpyHostToDevice, st));
    }
    hipLaunchKernelGGL(k_emit, dim3(std::min<uint64_t>((npix + kBlock - 1) / kBlock, 4096)), dim3(kBlock), 0, st, run,
                       (uint32_t)npix, R.nx, R.row_begin, row_step, acc_dev);
    HIPCHK(hipGetLastError());
    if (!R.accum_on_device) HIPCHK(hipMemcpyAsync(accum_rgb, acc_dev, img_bytes, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&h->host_ctrs[63], C, sizeof(ctrs_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(ev_end, st));
    HIPCHK(hipStreamSynchronize(st));

    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, ev_begin, ev_end));
    stats.ms_total = ms;
    for (int k = 0; k < 8; ++k) stats.segments += h->host_ctrs[63].segments[k].v;
    for (auto& p : isect_ev) {
        HIPCHK(hipEventElapsedTime(&ms, h->events[p.first], h->events[p.second]));
        stats.ms_intersect += ms;
    }
    for (auto& p : shade_ev) {
        HIPCHK(hipEventElapsedTime(&ms, h->events[p.first], h->events[p.second]));
        stats.ms_shade += ms;
    }
#ifdef RTW_PROF_WALK
    {
        static unsigned long long w[32][64];
        HIPCHK(hipMemcpyFromSymbol(w, HIP_SYMBOL(g_walk), sizeof w));
        std::fprintf(stderr, "[rtw walk] sampled clock by media-walk position:");
        for (int k = 0; k < 32; ++k) {
            unsigned long long t = 0;
            for (int l = 0; l < 64; ++l) t += w[k][l];
            if (t) std::fprintf(stderr, " %d:%llu", k, t);
        }
        std::fprintf(stderr, "\n");
    }
#endif
#ifdef RTW_PROF
    {
        unsigned long long pr[PS_N];
        HIPCHK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_prof), sizeof pr));
        static const char* names[PS_N] = {"loop", "load", "traverse", "hit+material", "sample", "pdf", "store"};
        double tot = 0;
        for (int k = 0; k < PS_N; ++k) tot += (double)pr[k];
        std::fprintf(stderr, "[rtw prof] lane-cycles per segment:");
        for (int k = 0; k < PS_N; ++k)
            std::fprintf(stderr, " %s %.0f (%.1f%%)", names[k], (double)pr[k] / std::max<double>(1, stats.segments),
                         100.0 * pr[k] / std::max(1.0, tot));
        std::fprintf(stderr, "\n");
        std::memset(pr, 0, sizeof pr);
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), pr, sizeof pr));
        unsigned long long cl[2][8];
        HIPCHK(hipMemcpyFromSymbol(cl, HIP_SYMBOL(g_cls), sizeof cl));
        static const char* cn[8] = {"miss", "lambertian", "metal", "dielectric", "light", "isotropic", "-", "idle"};
        std::fprintf(stderr, "[rtw prof] segment classes (lane share / share of wave-iterations where present):");
        double lt = 0, wt = 0;
        for (int k = 0; k < 8; ++k) lt += (double)cl[0][k];
        wt = (double)(cl[1][0] + 0);  // every wave-iteration has some class; use max as the iteration count
        for (int k = 0; k < 8; ++k) wt = std::max(wt, (double)cl[1][k]);
        unsigned long long it = 0;
        for (int k = 0; k < 8; ++k) it = std::max(it, cl[1][k]);
        std::fprintf(stderr, " (wave-iterations >= %llu)", it);
        for (int k = 0; k < 8; ++k)
            if (cl[0][k]) std::fprintf(stderr, " %s %.3f/%.3f", cn[k], cl[0][k] / lt, cl[1][k] / wt);
        std::fprintf(stderr, "\n");
        std::memset(cl, 0, sizeof cl);
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_cls), cl, sizeof cl));
    }
#endif
    // algorithmic traversal bytes: 56 B ray in +
    // 12 B hit out per world query, whatever the execution form (k_persist
    // keeps both in registers; k_segment / k_intersect stream them)
    // (fp32 fast mode: 7 x 4 B ray in, 4 + 4 B hit out = 36 B)
    stats.bytes_intersect = (fast ? 36.0 : 68.0) * (double)stats.segments;
    if (out_stats) *out_stats = stats;
    return RTW_OK;
}
