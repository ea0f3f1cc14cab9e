// scenes.cpp — the reference's scenes, rebuilt with the host scene API.
//
// Each constructor produces the same objects, in the same list order, with the
// same fp64 constants (float literals widened exactly as the reference's are)
// as Scene/scene.h.  Tests compare the flattened result field by field with a
// dump of the reference's own scene graph (tests/golden/scene_*.json).
#include <cmath>
#include <random>
#include "rtw/scene.h"

namespace {
using tex_ptr = std::shared_ptr<texture>;
using mat_ptr = std::shared_ptr<material>;

tex_ptr solid(double r, double g, double b) { return std::make_shared<constant_texture>(vec3(r, g, b)); }
mat_ptr diffuse(double r, double g, double b) { return std::make_shared<lambertian>(solid(r, g, b)); }

camera look(const vec3& from, const vec3& at, double vfov, double aspect, double aperture, double focus) {
    return camera(from, at, vec3(0.0, 1.0, 0.0), vfov, aspect, aperture, focus, 0.0, 1.0);
}
}  // namespace

// Scene/scene.h:42-70 — Perlin ground, Perlin ball, a light ball and a light
// quad; no explicit light list (so no light sampling).
light_sample::light_sample(double aspect) {
    tex_ptr marble = std::make_shared<noise_texture>(4.0);
    tex_ptr four = solid(4, 4, 4);
    std::vector<std::shared_ptr<hittable>> objs = {
        std::make_shared<sphere>(vec3(0, -1000, 0), 1000.0, std::make_shared<lambertian>(marble)),
        std::make_shared<sphere>(vec3(0, 2, 0), 2.0, std::make_shared<lambertian>(marble)),
        std::make_shared<sphere>(vec3(0, 7, 0), 2.0, std::make_shared<diffuse_light>(four)),
        std::make_shared<xy_rect>(3.0, 5.0, 1.0, 3.0, -2.0, std::make_shared<diffuse_light>(four)),
    };
    world = hittable_list(objs);
    const vec3 from(24, 5, 5), at(0, 3, 0);
    cam = look(from, at, 20.0, aspect, 0.2f, (from - at).length());
}

// Scene/scene.h:72-96 — the Book 1 material test (hollow glass via r < 0).
dielectric_scene::dielectric_scene(double aspect) {
    Add(std::make_shared<sphere>(vec3(0, 0, -1), 0.5f, diffuse(0.1f, 0.2f, 0.5f)));
    Add(std::make_shared<sphere>(vec3(0, -100.5f, -1), 100.0, diffuse(0.8f, 0.8f, 0.0)));
    Add(std::make_shared<sphere>(vec3(1, 0, -1), 0.5f, std::make_shared<metal>(vec3(0.8f, 0.6f, 0.2f), 0.0)));
    Add(std::make_shared<sphere>(vec3(-1, 0, -1), 0.5f, std::make_shared<dielectric>(1.5f)));
    Add(std::make_shared<sphere>(vec3(-1, 0, -1), -0.45f, std::make_shared<dielectric>(1.5f)));
    cam = look(vec3(0, 0, 0), vec3(0, 0, -1), 120.0, aspect, 0.0, 10.0);
}

// Scene/scene.h:98-174 — Book 1's cover: a 22x22 grid of jittered small
// balls (moving lambertian / metal / glass) and three big ones.  The layout
// comes from one default-seeded minstd_rand, drawn in the reference's order;
// the reference computes `vec3 center(a + 0.9f*U, 0.2f, b + 0.9f*U)` and g++
// evaluates those arguments right to left, so the z jitter is drawn first.
random_balls_scene::random_balls_scene(double aspect) {
    std::uniform_real_distribution<double> U;
    std::minstd_rand eng;

    Add(std::make_shared<sphere>(vec3(0, -1000, 0), 1000.0, diffuse(0.5f, 0.5f, 0.5f)));

    const vec3 keep_clear(4.0, 0.2f, 0.0);
    for (int a = -11; a < 11; ++a) {
        for (int b = -11; b < 11; ++b) {
            const double pick = U(eng);
            const double jz = U(eng);
            const double jx = U(eng);
            const vec3 c(a + 0.9f * jx, 0.2f, b + 0.9f * jz);
            if (!((c - keep_clear).length() > 0.9f)) continue;

            if (pick < 0.8f) {
                vec3 albedo;
                albedo.r = U(eng) * U(eng);
                albedo.g = U(eng) * U(eng);
                albedo.b = U(eng) * U(eng);
                auto ball = std::make_shared<moving_sphere>(c, 0.2f,
                    std::make_shared<lambertian>(std::make_shared<constant_texture>(albedo)));
                movement_linear path;
                path.center1 = c + vec3(0.0, 0.5f * U(eng), 0.0);
                path.time0 = 0.0;
                path.time1 = 1.0;
                ball->set_movement(path);
                Add(ball);
            } else if (pick < 0.95) {
                vec3 albedo;
                albedo.r = 0.5f * (1 + U(eng));
                albedo.g = 0.5f * (1 + U(eng));
                albedo.b = 0.5f * (1 + U(eng));
                const double fuzz = 0.5f * U(eng);
                Add(std::make_shared<sphere>(c, 0.2f, std::make_shared<metal>(albedo, fuzz)));
            } else {
                const double glass = 1.5f;
                Add(std::make_shared<sphere>(c, 0.2f, std::make_shared<dielectric>(glass)));
            }
        }
    }

    Add(std::make_shared<sphere>(vec3(0, 1, 0), 1.0, std::make_shared<dielectric>(1.5f)));
    Add(std::make_shared<sphere>(vec3(-4, 1, 0), 1.0, diffuse(0.4f, 0.2f, 0.1f)));
    Add(std::make_shared<sphere>(vec3(4, 1, 0), 1.0, std::make_shared<metal>(vec3(0.7f, 0.6f, 0.5f), 0.0)));

    cam = look(vec3(13, 2, 3), vec3(0, 0, 0), 20.0, aspect, 0.0, 10.0);
}

// Scene/scene.h:176-250 — Cornell box, glass-sphere variant (the `#if 1`
// block at :453-459): light quad, five walls, glass ball, tall rotated box.
// lights = { light quad, glass ball } drive the mixture-pdf sampling.
cornell_box_scene::cornell_box_scene(double aspect) {
    auto red = diffuse(0.65f, 0.05f, 0.05f);
    auto white = diffuse(0.73f, 0.73f, 0.73f);
    auto green = diffuse(0.12f, 0.45f, 0.15f);
    auto light = std::make_shared<diffuse_light>(solid(15.0, 15.0, 15.0));

    std::vector<std::shared_ptr<hittable>> objs;
    auto lamp = std::make_shared<xz_rect>(213.0, 343.0, 227.0, 332.0, 554.0, light);
    objs.push_back(lamp);
    lights->objects.push_back(lamp);

    const double L = 555.0;
    objs.push_back(std::make_shared<flip_normals>(std::make_shared<yz_rect>(0.0, L, 0.0, L, L, green)));
    objs.push_back(std::make_shared<yz_rect>(0.0, L, 0.0, L, 0.0, red));
    objs.push_back(std::make_shared<flip_normals>(std::make_shared<xz_rect>(0.0, L, 0.0, L, L, white)));
    objs.push_back(std::make_shared<xz_rect>(0.0, L, 0.0, L, 0.0, white));
    objs.push_back(std::make_shared<flip_normals>(std::make_shared<xy_rect>(0.0, L, 0.0, L, L, white)));

    auto ball = std::make_shared<sphere>(vec3(190, 90, 190), 90, std::make_shared<dielectric>(1.5));
    objs.push_back(ball);
    lights->objects.push_back(ball);

    auto tall = std::make_shared<box>(vec3(0.0, 0.0, 0.0), vec3(165.0, 330.0, 165.0), white);
    objs.push_back(std::make_shared<translate>(std::make_shared<rotate_y>(tall, 15.0), vec3(265.0, 0.0, 295.0)));

    world = hittable_list(objs);
    cam = look(vec3(278.0, 278.0, -800.0), vec3(278.0, 278.0, 0.0), 40.0, aspect, 0.0, 10.0);
    background_type = BackgroundType::Black;
}

// Book 2 "The Next Week" final scene.  Not in the reference;
// composed from the reference's classes, as oracle/ref_harness.cpp does:
// 20x20 ground boxes, a light quad, a moving ball, glass and metal balls, a
// blue smoke ball inside a glass ball, global thin fog, a constant-colour
// ball where the book maps earth.jpg, a Perlin marble ball, and 1000 small
// balls in a rotated, translated cluster.  Random layout from one
// default-seeded minstd_rand, drawn in the order written below.
book2_final_scene::book2_final_scene(double aspect) {
    std::uniform_real_distribution<double> U;
    std::minstd_rand eng;
    auto between = [&](double lo, double hi) { return lo + (hi - lo) * U(eng); };

    auto ground = diffuse(0.48, 0.83, 0.53);
    std::vector<std::shared_ptr<hittable>> boxes1;
    for (int i = 0; i < 20; ++i) {
        for (int j = 0; j < 20; ++j) {
            const double w = 100.0;
            const double x0 = -1000.0 + i * w, z0 = -1000.0 + j * w;
            const double y1 = between(1, 101);
            boxes1.push_back(std::make_shared<box>(vec3(x0, 0.0, z0), vec3(x0 + w, y1, z0 + w), ground));
        }
    }
    Add(std::make_shared<hittable_list>(boxes1));

    auto lamp = std::make_shared<xz_rect>(123.0, 423.0, 147.0, 412.0, 554.0,
                                          std::make_shared<diffuse_light>(solid(7, 7, 7)));
    Add(lamp);
    lights->objects.push_back(lamp);

    const vec3 c0(400, 400, 200);
    auto mover = std::make_shared<moving_sphere>(c0, 50.0, diffuse(0.7, 0.3, 0.1));
    movement_linear path;
    path.center1 = c0 + vec3(30, 0, 0);
    path.time0 = 0.0;
    path.time1 = 1.0;
    mover->set_movement(path);
    Add(mover);

    Add(std::make_shared<sphere>(vec3(260, 150, 45), 50.0, std::make_shared<dielectric>(1.5)));
    Add(std::make_shared<sphere>(vec3(0, 150, 145), 50.0, std::make_shared<metal>(vec3(0.8, 0.8, 0.9), 1.0)));

    auto shell = std::make_shared<sphere>(vec3(360, 150, 145), 70.0, std::make_shared<dielectric>(1.5));
    Add(shell);
    Add(std::make_shared<constant_medium>(shell, 0.2, std::make_shared<isotropic>(solid(0.2, 0.4, 0.9))));
    auto fog = std::make_shared<sphere>(vec3(0, 0, 0), 5000.0, std::make_shared<dielectric>(1.5));
    Add(std::make_shared<constant_medium>(fog, 0.0001, std::make_shared<isotropic>(solid(1, 1, 1))));

    Add(std::make_shared<sphere>(vec3(400, 200, 400), 100.0, diffuse(0.2, 0.3, 0.6)));
    Add(std::make_shared<sphere>(vec3(220, 280, 300), 80.0,
                                 std::make_shared<lambertian>(std::make_shared<noise_texture>(0.1))));

    auto white = diffuse(0.73, 0.73, 0.73);
    std::vector<std::shared_ptr<hittable>> cluster;
    for (int k = 0; k < 1000; ++k) {
        const double z = between(0, 165);
        const double y = between(0, 165);
        const double x = between(0, 165);
        cluster.push_back(std::make_shared<sphere>(vec3(x, y, z), 10.0, white));
    }
    Add(std::make_shared<translate>(std::make_shared<rotate_y>(std::make_shared<hittable_list>(cluster), 15.0),
                                    vec3(-100, 270, 395)));

    cam = look(vec3(478, 278, -600), vec3(278, 278, 0), 40.0, aspect, 0.0, 10.0);
    background_type = BackgroundType::Black;
}

// A test scene for arbitrary nesting (not in the reference; composed the
// same way in oracle/ref_harness.cpp from the reference's classes): the
// Cornell room, then instanced boxes inside a list, a flip over a list
// holding a transformed rect, a medium inside a nested list, a medium inside
// a translated list, lists two deep under rotate_y / translate, and a flip
// over a list holding a bare and a translated rect.  "nested_plain" drops
// the media (world runs instead of the media walk).
nested_scene::nested_scene(double aspect, bool media) {
    auto red = diffuse(0.65f, 0.05f, 0.05f);
    auto white = diffuse(0.73f, 0.73f, 0.73f);
    auto green = diffuse(0.12f, 0.45f, 0.15f);
    auto light = std::make_shared<diffuse_light>(solid(15.0, 15.0, 15.0));
    auto glass = std::make_shared<dielectric>(1.5);
    using list = std::vector<std::shared_ptr<hittable>>;
    auto L_ = [](list v) { return std::make_shared<hittable_list>(v); };

    auto lamp = std::make_shared<xz_rect>(213.0, 343.0, 227.0, 332.0, 554.0, light);
    Add(lamp);
    lights->objects.push_back(lamp);
    const double W = 555.0;
    Add(std::make_shared<flip_normals>(std::make_shared<yz_rect>(0.0, W, 0.0, W, W, green)));
    Add(std::make_shared<yz_rect>(0.0, W, 0.0, W, 0.0, red));
    Add(std::make_shared<flip_normals>(std::make_shared<xz_rect>(0.0, W, 0.0, W, W, white)));
    Add(std::make_shared<xz_rect>(0.0, W, 0.0, W, 0.0, white));
    Add(std::make_shared<flip_normals>(std::make_shared<xy_rect>(0.0, W, 0.0, W, W, white)));
    // instanced boxes in a list
    Add(L_({std::make_shared<translate>(
                std::make_shared<rotate_y>(std::make_shared<box>(vec3(0, 0, 0), vec3(80, 80, 80), white), 30.0),
                vec3(60, 0, 350)),
            std::make_shared<translate>(std::make_shared<box>(vec3(0, 0, 0), vec3(60, 120, 60), red),
                                        vec3(420, 0, 380)),
            std::make_shared<rotate_y>(
                std::make_shared<translate>(std::make_shared<box>(vec3(0, 0, 0), vec3(50, 50, 50), green),
                                            vec3(300, 0, 100)),
                -10.0)}));
    // a flip over a list holding a transformed rect
    Add(std::make_shared<flip_normals>(
        L_({std::make_shared<translate>(std::make_shared<xy_rect>(0.0, 100.0, 0.0, 100.0, 0.0, white),
                                        vec3(230, 300, 500))})));
    // a medium inside a nested list (a glass ball full of fog)
    auto ball = std::make_shared<sphere>(vec3(150, 60, 150), 60.0, glass);
    lights->objects.push_back(ball);
    if (media)
        Add(L_({ball,
                std::make_shared<constant_medium>(std::make_shared<sphere>(vec3(150, 60, 150), 55.0, glass), 0.02,
                                                  std::make_shared<isotropic>(solid(0.9, 0.9, 0.9))),
                std::make_shared<translate>(std::make_shared<box>(vec3(0, 0, 0), vec3(40, 40, 40), white),
                                            vec3(60, 0, 60))}));
    else
        Add(L_({ball, std::make_shared<translate>(std::make_shared<box>(vec3(0, 0, 0), vec3(40, 40, 40), white),
                                                  vec3(60, 0, 60))}));
    // a medium inside a translated list
    if (media)
    Add(std::make_shared<translate>(
        L_({std::make_shared<constant_medium>(
                std::make_shared<rotate_y>(std::make_shared<box>(vec3(0, 0, 0), vec3(100, 100, 100), white), 20.0),
                0.01, std::make_shared<isotropic>(solid(0.2, 0.4, 0.9))),
            std::make_shared<sphere>(vec3(50, 150, 50), 30.0,
                                     std::make_shared<metal>(vec3(0.8, 0.85, 0.88), 0.1))}),
        vec3(350, 0, 150)));
    // lists two deep under transforms
    Add(L_({L_({std::make_shared<translate>(std::make_shared<sphere>(vec3(0, 0, 0), 40.0, white),
                                            vec3(400, 300, 300))}),
            std::make_shared<rotate_y>(
                L_({std::make_shared<translate>(std::make_shared<box>(vec3(0, 0, 0), vec3(50, 50, 50), red),
                                                vec3(100, 350, 250))}),
                20.0)}));
    // a flip over a list of a bare rect and a translated one (the bare rect
    // becomes an entry whose only op is the flip)
    Add(std::make_shared<flip_normals>(
        L_({std::make_shared<xz_rect>(400.0, 500.0, 50.0, 150.0, 500.0, white),
            std::make_shared<translate>(std::make_shared<xz_rect>(0.0, 100.0, 0.0, 100.0, 0.0, green),
                                        vec3(50, 520, 400))})));
    cam = look(vec3(278.0, 278.0, -800.0), vec3(278.0, 278.0, 0.0), 40.0, aspect, 0.0, 10.0);
    background_type = BackgroundType::Black;
}

std::unique_ptr<scene> make_builtin_scene(const std::string& name, double aspect) {
    if (name == "nested") return std::make_unique<nested_scene>(aspect);
    if (name == "nested_plain") return std::make_unique<nested_scene>(aspect, false);
    if (name == "cornell_box") return std::make_unique<cornell_box_scene>(aspect);
    if (name == "random_balls") return std::make_unique<random_balls_scene>(aspect);
    if (name == "dielectric") return std::make_unique<dielectric_scene>(aspect);
    if (name == "light_sample") return std::make_unique<light_sample>(aspect);
    if (name == "book2_final") return std::make_unique<book2_final_scene>(aspect);
    return nullptr;
}
