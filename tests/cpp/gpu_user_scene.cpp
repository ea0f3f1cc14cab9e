// GPU parity for a user scene that exercises what the built-in scenes leave
// out (compiled and run by tests/test_gpu_parity.py on the GPU box):
// checker texture (texture.h:38-49), a marble texture whose sine argument
// crosses 2^19 (texture.h:57-68), metal with fuzz (material.h:128-136),
// hollow glass (negative radius, sphere.h:71-77), nested translate/rotate_y/
// flip_normals, a moving sphere, a constant medium, lights of all three
// kinds (xz_rect, sphere, and a box = hittable default pdf), gradient
// background -- built with the host scene API, flattened with and without
// BVHs, rendered through the C ABI and by the oracle (test infrastructure),
// and compared: per-channel canvas <= 1e-4 and equal traversal counts.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>
#include "rtw/scene.h"
#include "rtw_gpu.h"
#include "../../oracle/rtw_oracle.h"

class user_scene : public scene {
public:
    explicit user_scene(double aspect) : scene() {
        auto tex = [](double r, double g, double b) { return std::make_shared<constant_texture>(vec3(r, g, b)); };
        auto white = std::make_shared<lambertian>(tex(0.73, 0.73, 0.73));
        std::shared_ptr<texture> odd = tex(0.2, 0.3, 0.1), even = tex(0.9, 0.9, 0.9);
        auto checker = std::make_shared<lambertian>(std::make_shared<checker_texture>(odd, even));
        auto light = std::make_shared<diffuse_light>(tex(7.0, 7.0, 7.0));
        auto glass = std::make_shared<dielectric>(1.5);
        auto fuzzy = std::make_shared<metal>(vec3(0.8, 0.6, 0.2), 0.3);
        auto mirror = std::make_shared<metal>(vec3(0.9, 0.9, 0.9), 0.0);

        auto lamp = std::make_shared<xz_rect>(-1.0, 1.0, -1.0, 1.0, 4.0, light);
        Add(std::make_shared<flip_normals>(lamp));
        lights->objects.push_back(lamp);
        Add(std::make_shared<sphere>(vec3(0, -1000, 0), 1000, checker));  // checker ground
        auto ball = std::make_shared<sphere>(vec3(0, 1, 0), 1.0, glass);
        Add(ball);
        Add(std::make_shared<sphere>(vec3(0, 1, 0), -0.9, glass));  // hollow glass shell
        lights->objects.push_back(ball);
        Add(std::make_shared<sphere>(vec3(-2.2, 0.7, 0.5), 0.7, fuzzy));
        // marble with a huge scale: sin(scale * p.z + 10 turb) runs both the
        // device's sin_wide (|x| <= 2^19) and its ocml fallback beyond
        Add(std::make_shared<sphere>(vec3(1.2, 0.5, -1.0), 0.5,
                                     std::make_shared<lambertian>(std::make_shared<noise_texture>(1.0e6))));
        Add(std::make_shared<translate>(
            std::make_shared<rotate_y>(
                std::make_shared<translate>(std::make_shared<box>(vec3(0, 0, 0), vec3(1, 2, 1), mirror),
                                            vec3(-0.5, 0, -0.5)),
                30.0),
            vec3(2.2, 0, 0.3)));
        auto smoke_box = std::make_shared<box>(vec3(-3.5, 0, -2), vec3(-2.5, 1, -1), white);
        Add(std::make_shared<constant_medium>(
            smoke_box, 0.5, std::make_shared<isotropic>(tex(0.8, 0.8, 0.9))));
        lights->objects.push_back(std::make_shared<box>(vec3(5, 0, 5), vec3(6, 1, 6), white));  // default pdf
        moving_sphere* ms = new moving_sphere(vec3(1.0, 0.3, 2.0), 0.3, white);
        movement_linear mv;
        mv.center1 = vec3(1.0, 0.6, 2.0);
        ms->set_movement(mv);
        Add(std::shared_ptr<hittable>(ms));
        cam = camera(vec3(0.0, 2.5, 8.0), vec3(0.0, 0.8, 0.0), vec3(0.0, 1.0, 0.0), 35.0, aspect, 0.05, 8.0,
                     0.0, 1.0);
        background_type = BackgroundType::Gradient;
    }
};

// Every motion class and world-run form the upload derives (rtw_device.h,
// DP_MOVING_COMMON*, WORLD_RUN_*): a run of y-only movers and static spheres
// (ysphere_scan), a run broken by a static sphere at y == 0, x-movers, a
// y-mover at x == 0 (general common mover), movers on a second interval
// (their own division), a translated group holding a mover, and a moving
// sphere among the lights (its pdf ray carries time FLT_MAX).
class motion_scene : public scene {
public:
    explicit motion_scene(double aspect) : scene() {
        auto tex = [](double r, double g, double b) { return std::make_shared<constant_texture>(vec3(r, g, b)); };
        auto white = std::make_shared<lambertian>(tex(0.73, 0.73, 0.73));
        auto red = std::make_shared<lambertian>(tex(0.65, 0.05, 0.05));
        auto light = std::make_shared<diffuse_light>(tex(6.0, 6.0, 6.0));
        auto glass = std::make_shared<dielectric>(1.5);
        auto mover = [&](vec3 c0, vec3 c1, double r, std::shared_ptr<material> m, double t0, double t1) {
            moving_sphere* ms = new moving_sphere(c0, r, m);
            movement_linear mv;
            mv.center1 = c1;
            mv.time0 = t0;
            mv.time1 = t1;
            ms->set_movement(mv);
            return std::shared_ptr<hittable>(ms);
        };
        // run 1: y-only movers and static spheres off y == 0 -> ysphere_scan
        Add(std::make_shared<sphere>(vec3(0.5, -1000, 0.25), 1000, white));
        for (int k = 0; k < 6; ++k)
            Add(mover(vec3(-2.5 + k, 0.3, 1.5), vec3(-2.5 + k, 0.3 + 0.1 * k, 1.5), 0.3, k & 1 ? red : white, 0.0, 1.0));
        Add(std::make_shared<sphere>(vec3(1.7, 0.4, -0.6), 0.4, glass));
        // a ninth sphere: the run's length is odd, so ysphere_scan's packed
        // pairs end with a lone sphere filtered from its plain record
        Add(std::make_shared<sphere>(vec3(-1.2, 0.2, 0.6), 0.2, red));
        // a light between the runs: translated (by zero, which moves nothing)
        // so that it is not a plain entry -- a flip alone folds into the prim
        // and would merge run 1, the lamp and run 2 into one mixed run
        auto lamp = std::make_shared<xz_rect>(-1.0, 1.0, -1.0, 1.0, 4.0, light);
        Add(std::make_shared<translate>(std::make_shared<flip_normals>(lamp), vec3(0.0, 0.0, 0.0)));
        lights->objects.push_back(lamp);
        // run 2: a static sphere at y == 0, an x-mover, a y-mover at x == 0,
        // movers on another interval
        Add(std::make_shared<sphere>(vec3(-1.8, 0.0, -1.2), 0.35, red));
        Add(mover(vec3(-0.8, 0.35, -1.4), vec3(-0.5, 0.35, -1.4), 0.35, white, 0.0, 1.0));
        Add(mover(vec3(0.0, 0.3, -2.0), vec3(0.0, 0.7, -2.0), 0.3, red, 0.0, 1.0));
        Add(mover(vec3(0.9, 0.3, -2.2), vec3(0.9, 0.9, -2.2), 0.3, white, 0.2, 0.7));
        Add(mover(vec3(2.0, 0.5, -1.0), vec3(2.3, 0.5, -1.3), 0.3, glass, 0.2, 0.7));
        // a translated group holding a mover
        Add(std::make_shared<translate>(mover(vec3(0, 0.25, 0), vec3(0, 0.55, 0), 0.25, red, 0.0, 1.0),
                                        vec3(-0.6, 0.0, 2.4)));
        // a moving sphere light (not in the world list)
        lights->objects.push_back(mover(vec3(2.5, 3.0, 2.0), vec3(2.5, 3.2, 2.0), 0.5, light, 0.0, 1.0));
        cam = camera(vec3(0.0, 2.0, 7.0), vec3(0.0, 0.5, 0.0), vec3(0.0, 1.0, 0.0), 40.0, aspect, 0.0, 7.0,
                     0.0, 1.0);
        background_type = BackgroundType::Gradient;
    }
};

static int check_scene(const scene& us, const char* name, int nx, int ny, int spp, int depth, uint64_t seed,
                       int min_ysphere_runs = 0) {
    int failures = 0;
    for (int bvh = 0; bvh <= 1; ++bvh) {
        rtw_scene_desc* d = nullptr;
        if (rtw_flatten_scene(us, bvh, &d) != RTW_OK) {
            std::printf("flatten failed: %s\n", rtw_last_error());
            return 1;
        }
        void* h = nullptr;
        if (rtw_scene_upload(0, d, &h) != RTW_OK) {
            std::printf("upload failed: %s\n", rtw_last_error());
            return 1;
        }
        rtw_scene_info info;
        if (rtw_scene_query(h, &info) != RTW_OK) {
            std::printf("query failed: %s\n", rtw_last_error());
            return 1;
        }
        if (!bvh && info.n_ysphere_runs < min_ysphere_runs) {
            std::printf("%s: %d y-sphere runs, expected >= %d (run layout %d runs, %d plain)\n", name,
                        info.n_ysphere_runs, min_ysphere_runs, info.n_world_runs, info.n_plain_runs);
            ++failures;
        }
        const rtw_camera_desc cam = us.GetCamera().desc();
        rtw_render_params p;
        std::memset(&p, 0, sizeof p);
        p.nx = nx, p.ny = ny, p.spp = spp, p.max_depth = depth, p.seed = seed, p.row_step = 1;
        std::vector<double> gpu((size_t)nx * ny * 3, 0.0), ref(gpu.size(), 0.0), cg(gpu.size()), cr(gpu.size());
        rtw_stats st;
        if (rtw_render_accumulate(h, &cam, &p, gpu.data(), &st) != RTW_OK) {
            std::printf("render failed: %s\n", rtw_last_error());
            return 1;
        }
        uint64_t seg = 0;
        if (rtw_oracle_render(d, &cam, nx, ny, 0, ny, 0, spp, depth, seed, 0, ref.data(), &seg) != 0) {
            std::printf("oracle failed\n");
            return 1;
        }
        rtw_finalize_canvas(gpu.data(), nx, ny, spp, cg.data());
        rtw_finalize_canvas(ref.data(), nx, ny, spp, cr.data());
        double md = 0;
        for (size_t k = 0; k < cg.size(); ++k) md = std::fmax(md, std::fabs(cg[k] - cr[k]));
        const bool ok = md <= 1e-4 && st.segments == seg && std::isfinite(md);
        std::printf("%s bvh=%d max|diff|=%.3e segments gpu=%llu oracle=%llu %s\n", name, bvh, md,
                    (unsigned long long)st.segments, (unsigned long long)seg, ok ? "ok" : "MISMATCH");
        failures += !ok;
        rtw_scene_free(h);
        rtw_scene_desc_free(d);
    }
    return failures;
}

int main() {
    const int nx = 64, ny = 48, spp = 8, depth = 50;
    int failures = 0;
    {
        user_scene us(nx * 1.0 / ny);
        failures += check_scene(us, "user", nx, ny, spp, depth, 9);
    }
    {
        motion_scene ms(nx * 1.0 / ny);
        failures += check_scene(ms, "motion", nx, ny, spp, depth, 11, 1);
    }
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
    return failures ? 1 : 0;
}
