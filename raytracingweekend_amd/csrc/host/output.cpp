// output.cpp — canvas finalisation, PPM writer, error state, seeding.
#include <cmath>
#include <cstdio>
#include <string>
#include "rtw_host_util.h"

namespace {
thread_local std::string g_last_error;
}

int rtw_fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

extern "C" const char* rtw_last_error(void) { return g_last_error.c_str(); }

extern "C" int rtw_abi_version(void) { return RTW_ABI_VERSION; }

// RayTracingWeekend.cpp:241-244: col = sum / spp (a true division, the double
// broadcast to vec3), then std::min(sqrt(c), 1.0) — std::min returns its
// first argument unless the second compares smaller, so a NaN passes through.
extern "C" void rtw_finalize_canvas(const double* accum, int nx, int ny, int spp, double* canvas) {
    const size_t n = (size_t)nx * (size_t)ny * 3;
    const double d = static_cast<double>(spp);
    for (size_t k = 0; k < n; ++k) {
        const double s = std::sqrt(accum[k] / d);
        canvas[k] = (1.0 < s) ? 1.0 : s;
    }
}

// RayTracingWeekend.cpp:252-276: ASCII P3, rows written top (j = ny-1) to
// bottom, each channel int(255.99f * c) — 255.99f widened to double.
extern "C" int rtw_write_ppm(const char* path, const double* canvas, int nx, int ny) {
    if (!path || !canvas || nx <= 0 || ny <= 0) return rtw_fail(RTW_ERR_INVALID, "rtw_write_ppm: bad argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return rtw_fail(RTW_ERR_INVALID, std::string("rtw_write_ppm: cannot open ") + path);
    std::fprintf(f, "P3\n%d %d\n255\n", nx, ny);
    const double k = (double)255.99f;
    for (int j = ny - 1; j >= 0; --j) {
        for (int i = 0; i < nx; ++i) {
            const double* c = canvas + ((size_t)j * nx + i) * 3;
            int q[3];
            for (int a = 0; a < 3; ++a) {
                const double x = k * c[a];
                // int(NaN) / out-of-range is INT_MIN on x86 (cvttsd2si); keep that
                q[a] = (x == x && x < 2147483648.0 && x > -2147483649.0) ? (int)x : (int)0x80000000u;
            }
            std::fprintf(f, "%d %d %d\n", q[0], q[1], q[2]);
        }
    }
    const bool ok = std::fclose(f) == 0;
    return ok ? RTW_OK : rtw_fail(RTW_ERR_INVALID, "rtw_write_ppm: write failed");
}

// The same file from channels already quantized on the device
// (rtw_quantize_canvas_device): rows ny-1..0, "r g b\n".
extern "C" int rtw_write_ppm_quantized(const char* path, const int32_t* rgb, int nx, int ny) {
    if (!path || !rgb || nx <= 0 || ny <= 0) return rtw_fail(RTW_ERR_INVALID, "rtw_write_ppm_quantized: bad argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return rtw_fail(RTW_ERR_INVALID, std::string("rtw_write_ppm_quantized: cannot open ") + path);
    std::fprintf(f, "P3\n%d %d\n255\n", nx, ny);
    for (int j = ny - 1; j >= 0; --j)
        for (int i = 0; i < nx; ++i) {
            const int32_t* q = rgb + ((size_t)j * nx + i) * 3;
            std::fprintf(f, "%d %d %d\n", q[0], q[1], q[2]);
        }
    const bool ok = std::fclose(f) == 0;
    return ok ? RTW_OK : rtw_fail(RTW_ERR_INVALID, "rtw_write_ppm_quantized: write failed");
}

static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

extern "C" uint32_t rtw_path_seed(uint64_t seed, uint32_t pixel, uint32_t s) {
    const uint64_t key = ((uint64_t)s << 32) ^ (uint64_t)pixel;
    return (uint32_t)(1u + splitmix64(splitmix64(seed) ^ key) % 2147483646ull);
}
