// rtw_render — the host program of the reference (RayTracingWeekend.cpp:195-289)
// on the MI355X path: build a scene with the hittable API, flatten it, run the
// per-pixel render loop on the GPU through the C ABI, gamma + clamp, write the
// P3 PPM, report Trace/Write milliseconds.
//
//   rtw_render [--scene cornell_box] [--nx 400] [--ny 400] [--spp 64]
//              [--depth 100] [--seed 0] [--bvh] [--device 0] [--gpus 1]
//              [--precision fp64|fp32] [--out out.ppm]
//
// --precision fp64 (default) is the parity mode (the reference's double
// arithmetic on every path decision); fp32 the fast mode (single precision,
// statistical parity only; rtw_render_params.precision).
//
// --gpus N renders on devices device .. device+N-1 from this one process
// (rtw_render_multi: one host thread per GPU, RCCL reduce to the first).
//
// Defaults are the reference's compile-time constants (RayTracingWeekend.cpp:32-43,
// scene typedef :201).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "rtw/scene.h"
#include "rtw_gpu.h"

int main(int argc, char** argv) {
    std::string scene_name = "cornell_box", out = "1.ppm";
    int nx = 400, ny = 400, spp = 64, depth = 100, device = 0, bvh = 0, gpus = 1, precision = RTW_PRECISION_FP64;
    unsigned long long seed = 0;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "missing value for %s\n", a.c_str());
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "--scene") scene_name = next();
        else if (a == "--nx") nx = std::atoi(next());
        else if (a == "--ny") ny = std::atoi(next());
        else if (a == "--spp") spp = std::atoi(next());
        else if (a == "--depth") depth = std::atoi(next());
        else if (a == "--seed") seed = std::strtoull(next(), nullptr, 10);
        else if (a == "--device") device = std::atoi(next());
        else if (a == "--gpus") gpus = std::atoi(next());
        else if (a == "--out") out = next();
        else if (a == "--bvh") bvh = 1;
        else if (a == "--precision") {
            const std::string v = next();
            if (v == "fp64") precision = RTW_PRECISION_FP64;
            else if (v == "fp32") precision = RTW_PRECISION_FP32;
            else {
                std::fprintf(stderr, "--precision %s: expected fp64 or fp32\n", v.c_str());
                return 2;
            }
        }
        else {
            std::fprintf(stderr, "unknown argument %s\n", a.c_str());
            return 2;
        }
    }

    auto sc = make_builtin_scene(scene_name, nx * 1.0 / ny);  // RayTracingWeekend.cpp:204
    if (!sc) {
        std::fprintf(stderr, "unknown scene %s\n", scene_name.c_str());
        return 2;
    }
    rtw_scene_desc* desc = nullptr;
    if (rtw_flatten_scene(*sc, bvh, &desc) != RTW_OK) {
        std::fprintf(stderr, "flatten: %s\n", rtw_last_error());
        return 1;
    }
    if (gpus < 1 || device < 0 || device + gpus > rtw_device_count()) {
        std::fprintf(stderr, "--device %d --gpus %d: only %d devices visible\n", device, gpus, rtw_device_count());
        return 2;
    }
    std::vector<void*> h(gpus, nullptr);
    for (int g = 0; g < gpus; ++g)
        if (rtw_scene_upload(device + g, desc, &h[g]) != RTW_OK) {
            std::fprintf(stderr, "upload: %s\n", rtw_last_error());
            return 1;
        }
    const rtw_camera_desc cam = sc->GetCamera().desc();
    rtw_render_params p;
    std::memset(&p, 0, sizeof p);
    p.nx = nx, p.ny = ny, p.spp = spp, p.max_depth = depth, p.seed = seed, p.row_step = 1;
    p.precision = precision;
    std::vector<double> accum((size_t)nx * ny * 3, 0.0), canvas(accum.size());
    rtw_stats st;
    auto t0 = std::chrono::high_resolution_clock::now();
    const int rc = gpus == 1 ? rtw_render_accumulate(h[0], &cam, &p, accum.data(), &st)
                             : rtw_render_multi(gpus, h.data(), &cam, &p, accum.data(), &st);
    if (rc != RTW_OK) {
        std::fprintf(stderr, "render: %s\n", rtw_last_error());
        return 1;
    }
    rtw_finalize_canvas(accum.data(), nx, ny, spp, canvas.data());
    auto t1 = std::chrono::high_resolution_clock::now();
    if (rtw_write_ppm(out.c_str(), canvas.data(), nx, ny) != RTW_OK) {
        std::fprintf(stderr, "write: %s\n", rtw_last_error());
        return 1;
    }
    auto t2 = std::chrono::high_resolution_clock::now();
    using ms = std::chrono::milliseconds;
    std::printf("Trace: %lldms\n", (long long)std::chrono::duration_cast<ms>(t1 - t0).count());
    std::printf("Write: %lldms\n", (long long)std::chrono::duration_cast<ms>(t2 - t1).count());
    std::printf("Msamples/s: %.3f  segments/sample: %.4f\n",
                (double)st.samples / (std::chrono::duration<double>(t1 - t0).count() * 1e6),
                (double)st.segments / (double)st.samples);
    for (void* x : h) rtw_scene_free(x);
    if (gpus > 1) rtw_release_communicators();
    rtw_scene_desc_free(desc);
    return 0;
}
