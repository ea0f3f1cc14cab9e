// slab_check.hip — on the card: the BVH kernels' fp32 slab test
// (rtw_device.h make_slab_ray / slab32 with t_lo32 / t_hi32) never culls a
// box the real-arithmetic slab test keeps.  Each case is a ray, a t range
// and an fp32 box placed on or near the ray (a random point of the ray, a
// box around it, then shifted so the ray passes inside, on or just outside
// an edge or corner, by 2^-4 ... 2^-48 of the box size).  The reference is
// the slab test in fp64 (errors ~2^-52 relative); a case whose fp64 margin
// tn <= tf exceeds 2^-36 of the magnitudes is a real hit, and slab32 must
// keep it.  Classes: scene-sized rays and boxes; magnitudes over the whole
// range the walks allow (|o| up to 2^40, direction components 2^-60 ...
// 2^60); direction components exactly 0 with origins on box planes; the
// media walks' t range (t_min = -DBL_MAX) and closest-hit bounds at the
// box's own entry / exit t.  Test tool (tests/test_slab32.py).
//
//   slab_check <log2 cases per class>  prints "class <k> misses <n> of <m> (real hits <h>, grazing <g>)"
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "rtw_device.h"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP error %s\n", hipGetErrorString(e)); return 2; } } while (0)

using namespace rtwd;

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ double u01(unsigned long long r) { return (double)(r >> 11) * 0x1p-53; }
__device__ __forceinline__ double pm1(unsigned long long r) { return 2.0 * u01(r) - 1.0; }
// random double with |v| in [2^elo, 2^ehi), random mantissa and sign
__device__ __forceinline__ double rnd_exp(unsigned long long r, int elo, int ehi) {
    const int e = elo + (int)((r >> 53) % (unsigned long long)(ehi - elo));
    const unsigned long long bits = ((unsigned long long)(e + 1023) << 52) | (r & 0xFFFFFFFFFFFFFull);
    double v;
    memcpy(&v, &bits, 8);
    return ((r >> 52) & 1) ? -v : v;
}
// the next representable value up / down (finite arguments)
__device__ __forceinline__ float next_upf(float f) {
    if (f == 0.0f) return 0x1p-149f;
    int b;
    memcpy(&b, &f, 4);
    b += f > 0 ? 1 : -1;
    memcpy(&f, &b, 4);
    return f;
}
__device__ __forceinline__ float next_downf(float f) { return -next_upf(-f); }
__device__ __forceinline__ double next_up(double f) {
    if (f == 0.0) return 0x1p-1074;
    long long b;
    memcpy(&b, &f, 8);
    b += f > 0 ? 1 : -1;
    memcpy(&f, &b, 8);
    return f;
}
__device__ __forceinline__ double next_down(double f) { return -next_up(-f); }
// fp32 bounds rounded outward from fp64 (as rtw_scene_upload does)
__device__ __forceinline__ float down(double x) {
    float f = (float)x;
    if ((double)f > x) f = next_downf(f);
    return f;
}
__device__ __forceinline__ float up(double x) {
    float f = (float)x;
    if ((double)f < x) f = next_upf(f);
    return f;
}

// real-arithmetic slab test in fp64 over [tmin, tmax]: returns the margin
// tf - tn (negative: miss) and its scale
__device__ void ref_slab(const double lo[3], const double hi[3], const double o[3], const double d[3], double tmin,
                         double tmax, double& margin, double& scale, bool& ok) {
    double tn = tmin, tf = tmax;
    ok = true;
    scale = 0.0;
    for (int k = 0; k < 3; ++k) {
        if (d[k] == 0.0) {  // parallel: inside the slab or not at all
            if (o[k] < lo[k] || o[k] > hi[k]) ok = false;
            if (o[k] == lo[k] || o[k] == hi[k]) scale = __builtin_inf();  // on a plane: grazing
            continue;
        }
        const double a = (lo[k] - o[k]) / d[k], b = (hi[k] - o[k]) / d[k];
        tn = __builtin_fmax(tn, __builtin_fmin(a, b));
        tf = __builtin_fmin(tf, __builtin_fmax(a, b));
        scale = __builtin_fmax(scale, __builtin_fmax(__builtin_fabs(a), __builtin_fabs(b)));
    }
    margin = tf - tn;
    if (!ok) margin = -1.0;
}

__global__ void k_check(int cls, unsigned long long n, unsigned long long* out) {
    unsigned long long misses = 0, hits = 0, grazing = 0;
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        unsigned long long r = mix(i * 16 + (unsigned long long)cls * 0x100000000000ull);
        auto nx = [&]() { r = mix(r); return r; };
        double o[3], d[3];
        double scene_size;
        if (cls == 0 || cls == 3) {  // scene-sized
            scene_size = 1000.0;
            for (int k = 0; k < 3; ++k) o[k] = pm1(nx()) * 1000.0, d[k] = pm1(nx());
        } else if (cls == 1) {  // the whole range the walks allow
            scene_size = __builtin_ldexp(1.0, (int)(nx() % 40));
            for (int k = 0; k < 3; ++k) o[k] = pm1(nx()) * scene_size, d[k] = rnd_exp(nx(), -60, 60);
        } else {  // exact zeros in the direction
            scene_size = 500.0;
            for (int k = 0; k < 3; ++k) o[k] = pm1(nx()) * 500.0, d[k] = pm1(nx());
            const int z = (int)(nx() % 3);
            d[z] = (nx() & 1) ? 0.0 : -0.0;
            if (nx() & 1) d[(z + 1) % 3] = 0.0;
        }
        // a box around a point of the ray (t in [0, 2 size / |d|]), shifted
        // by a random tangent offset along each axis
        double dd = 0.0;
        for (int k = 0; k < 3; ++k) dd = __builtin_fmax(dd, __builtin_fabs(d[k]));
        const double tp = u01(nx()) * 2.0 * scene_size / dd;
        double lo[3], hi[3];
        const double ext = scene_size * __builtin_ldexp(u01(nx()) + 0.01, -(int)(nx() % 12));
        for (int k = 0; k < 3; ++k) {
            const double p = o[k] + tp * d[k];
            const double e0 = ext * u01(nx()), e1 = ext * u01(nx());
            lo[k] = p - e0, hi[k] = p + e1;
        }
        // move one or two faces onto the ray's point +- 2^-s of the box size
        const int s = 4 + (int)(nx() % 45);
        for (int j = 0; j < 2; ++j) {
            const int k = (int)(nx() % 3);
            const double p = o[k] + tp * d[k];
            const double off = pm1(nx()) * __builtin_ldexp(ext, -s);
            if (nx() & 1) lo[k] = p + off; else hi[k] = p + off;
            if (lo[k] > hi[k]) { const double t = lo[k]; lo[k] = hi[k]; hi[k] = t; }
        }
        if (cls == 2 && (nx() & 1)) {  // origin exactly on a box plane of a zero-direction axis
            for (int k = 0; k < 3; ++k)
                if (d[k] == 0.0) o[k] = (nx() & 1) ? lo[k] : hi[k];
        }
        bvh_node32 nd;
        double flo[3], fhi[3];
        float B = 0.0f;
        for (int k = 0; k < 3; ++k) {
            nd.lo[k] = down(lo[k]), nd.hi[k] = up(hi[k]);
            flo[k] = nd.lo[k], fhi[k] = nd.hi[k];
            B = __builtin_fmaxf(B, __builtin_fmaxf(__builtin_fabsf(nd.lo[k]), __builtin_fabsf(nd.hi[k])));
        }
        nd.a = 0, nd.b = -1;
        // the t range: a world walk's [0.001, closest], or a media probe's
        // [-DBL_MAX, ...]; class 3 puts the closest hit on the box's own
        // entry / exit t (+- a few ulps)
        double tmin = (cls == 3 && (nx() & 1)) ? -kDblMax : 0.001;
        double tmax = (nx() & 3) ? kDblMax : u01(nx()) * 4.0 * scene_size / dd;
        if (cls == 3) {
            double m, sc;
            bool okr;
            ref_slab(flo, fhi, o, d, -kDblMax, kDblMax, m, sc, okr);
            double te = 0.0, tx = 0.0;  // entry / exit
            double tn = -kDblMax, tf = kDblMax;
            for (int k = 0; k < 3; ++k) {
                if (d[k] == 0.0) continue;
                const double a = (flo[k] - o[k]) / d[k], b = (fhi[k] - o[k]) / d[k];
                tn = __builtin_fmax(tn, __builtin_fmin(a, b));
                tf = __builtin_fmin(tf, __builtin_fmax(a, b));
            }
            te = tn, tx = tf;
            const int ulps = (int)(nx() % 9) - 4;
            double edge = (nx() & 1) ? te : tx;
            for (int u = 0; u < (ulps < 0 ? -ulps : ulps); ++u)
                edge = ulps < 0 ? next_down(edge) : next_up(edge);
            if (nx() & 1) tmax = edge; else tmin = edge;
            if (!(tmin <= tmax)) { const double t = tmin; tmin = tmax; tmax = t; }
        }
        double margin, scale;
        bool okr;
        ref_slab(flo, fhi, o, d, tmin, tmax, margin, scale, okr);
        const double mag = __builtin_fmax(scale, __builtin_fmax(__builtin_fabs(tmin < -1e300 ? 0.0 : tmin),
                                                               __builtin_fabs(tmax > 1e300 ? 0.0 : tmax)));
        const bool real_hit = okr && margin > 0x1p-36 * mag && __builtin_isfinite(mag);
        const bool near = okr && !real_hit && margin > -0x1p-36 * mag;
        scene S = {};
        S.bvh_bound = B;
        const ray rr{d3{o[0], o[1], o[2]}, d3{d[0], d[1], d[2]}, 0.0};
        const slab_ray sr = make_slab_ray(S, rr);
        const bool got = slab32(nd, sr, t_lo32(tmin), t_hi32(tmax));
        hits += real_hit;
        grazing += near;
        misses += real_hit && !got;
    }
    if (misses) atomicAdd(&out[0], misses);
    atomicAdd(&out[1], hits);
    atomicAdd(&out[2], grazing);
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? std::atoi(argv[1]) : 26;
    const unsigned long long n = 1ull << lg;
    unsigned long long* dev;
    CHK(hipMalloc(&dev, 3 * sizeof(unsigned long long)));
    int fails = 0;
    for (int cls = 0; cls < 4; ++cls) {
        CHK(hipMemset(dev, 0, 3 * sizeof(unsigned long long)));
        hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, 0, cls, n, dev);
        CHK(hipGetLastError());
        unsigned long long h[3] = {0, 0, 0};
        CHK(hipMemcpy(h, dev, sizeof h, hipMemcpyDeviceToHost));
        std::printf("class %d misses %llu of %llu (real hits %llu, grazing %llu)\n", cls, h[0], n, h[1], h[2]);
        fails += h[0] != 0 || h[1] < n / 64;
    }
    CHK(hipFree(dev));
    return fails ? 1 : 0;
}
