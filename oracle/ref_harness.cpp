// ref_harness.cpp — TEST INFRASTRUCTURE ONLY (oracle/_ref).
//
// Compiles the reference's own headers, where they lie under
// /root/reference/RayTracingWeekend, with g++ (recipe: oracle/Makefile), and
// drives them to produce golden vectors for this repository's parity tests.
// Nothing here is linked into, or called by, the product library.
//
// What is the reference's and what is not:
//   * hittable/material/pdf/texture/noise/camera/scene classes: the
//     reference's code, unmodified (#include'd from /root/reference).
//   * RayTracingWeekend.cpp itself cannot be compiled here: it includes the
//     MSVC-only <ppl.h> and <crtdbg.h>, which this image lacks, and we do not
//     write stand-ins for them.  Its integrator color() (RayTracingWeekend.cpp:
//     45-160) and the body of its render loop (:227-241) are therefore
//     restated below, line for line in behaviour, calling the reference
//     classes; the ppl parallel_for over rows becomes an OpenMP loop.
//   * Randomness: every std::minstd_rand is redirected to the per-path stream
//     of oracle/rng_inject.h (see there).
//   * book2_final: Book 2's final scene is not in the reference
//     (SURVEY.md A.8); it is composed here from the reference classes, with a
//     flat hittable_list where the book uses the (broken, unused) bvh_node
//     (hittable.h:41-140) and a constant texture where the book
//     uses image_texture(earth.jpg) (no image loader exists in the reference).
//
// Commands (all output to stdout unless a path is given):
//   scene  <name> <aspect>                  JSON dump of the scene graph
//   render <name> <nx> <ny> <spp> <depth> <seed> <threads> <out.bin>
//          writes nx*ny*3 doubles: per-pixel radiance SUM over spp samples
//   bench  <name> <nx> <ny> <spp> <depth> <seed> <threads> [row_stride]
//          times render() over every row_stride-th row (default: all rows)
//   perlin                                  Perlin tables + noise/turb samples
#include "rng_inject.h"

#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <chrono>
#include <map>
#include <string>
#include <vector>
#include <algorithm>
#include <iostream>
#include <limits>
#include <memory>
#include <math.h>
#include <omp.h>

#define private public  // read perlin's static tables for the fixture dump
#include "vec3.h"
#include "onb.h"
#include "ray.h"
#include "pdf.h"
#include "sphere.h"
#include "hittable_list.h"
#include "camera.h"
#include "material.h"
#include "utility.h"
#include "Scene/scene.h"
#undef private

// ---------------------------------------------------------------------------
// Book 2 "The Next Week" final scene, composed from the reference classes.
// ---------------------------------------------------------------------------
class book2_final_scene : public scene {
public:
    book2_final_scene(double aspect) : scene() {
        std::uniform_real_distribution<double> uniform;
        std::minstd_rand engine;
        auto rnd = [&](double a, double b) { return a + (b - a) * uniform(engine); };

        auto ground = std::make_shared<lambertian>(std::make_shared<constant_texture>(vec3(0.48, 0.83, 0.53)));
        std::vector<std::shared_ptr<hittable>> boxes1;
        const int boxes_per_side = 20;
        for (int i = 0; i < boxes_per_side; i++) {
            for (int j = 0; j < boxes_per_side; j++) {
                double w = 100.0;
                double x0 = -1000.0 + i * w;
                double z0 = -1000.0 + j * w;
                double y0 = 0.0;
                double x1 = x0 + w;
                double y1 = rnd(1, 101);
                double z1 = z0 + w;
                boxes1.push_back(std::make_shared<box>(vec3(x0, y0, z0), vec3(x1, y1, z1), ground));
            }
        }
        Add(std::make_shared<hittable_list>(boxes1));

        auto light = std::make_shared<diffuse_light>(std::make_shared<constant_texture>(vec3(7, 7, 7)));
        auto light_rect = std::make_shared<xz_rect>(123.0, 423.0, 147.0, 412.0, 554.0, light);
        Add(light_rect);
        lights->objects.push_back(light_rect);

        vec3 center1(400, 400, 200);
        vec3 center2 = center1 + vec3(30, 0, 0);
        auto ms = std::make_shared<moving_sphere>(center1, 50.0,
            std::make_shared<lambertian>(std::make_shared<constant_texture>(vec3(0.7, 0.3, 0.1))));
        movement_linear m;
        m.center1 = center2;
        m.time0 = 0.0;
        m.time1 = 1.0;
        ms->set_movement(m);
        Add(ms);

        Add(std::make_shared<sphere>(vec3(260, 150, 45), 50.0, std::make_shared<dielectric>(1.5)));
        Add(std::make_shared<sphere>(vec3(0, 150, 145), 50.0, std::make_shared<metal>(vec3(0.8, 0.8, 0.9), 1.0)));

        auto boundary = std::make_shared<sphere>(vec3(360, 150, 145), 70.0, std::make_shared<dielectric>(1.5));
        Add(boundary);
        Add(std::make_shared<constant_medium>(boundary, 0.2,
            std::make_shared<isotropic>(std::make_shared<constant_texture>(vec3(0.2, 0.4, 0.9)))));
        auto boundary2 = std::make_shared<sphere>(vec3(0, 0, 0), 5000.0, std::make_shared<dielectric>(1.5));
        Add(std::make_shared<constant_medium>(boundary2, 0.0001,
            std::make_shared<isotropic>(std::make_shared<constant_texture>(vec3(1, 1, 1)))));

        // earth: image_texture in the book -> constant texture here
        Add(std::make_shared<sphere>(vec3(400, 200, 400), 100.0,
            std::make_shared<lambertian>(std::make_shared<constant_texture>(vec3(0.2, 0.3, 0.6)))));
        Add(std::make_shared<sphere>(vec3(220, 280, 300), 80.0,
            std::make_shared<lambertian>(std::make_shared<noise_texture>(0.1))));

        auto white = std::make_shared<lambertian>(std::make_shared<constant_texture>(vec3(0.73, 0.73, 0.73)));
        std::vector<std::shared_ptr<hittable>> boxes2;
        for (int j = 0; j < 1000; j++) {
            double z = rnd(0, 165);
            double y = rnd(0, 165);
            double x = rnd(0, 165);
            boxes2.push_back(std::make_shared<sphere>(vec3(x, y, z), 10.0, white));
        }
        Add(std::make_shared<translate>(
            std::make_shared<rotate_y>(std::make_shared<hittable_list>(boxes2), 15.0),
            vec3(-100, 270, 395)));

        auto lookfrom = vec3(478, 278, -600);
        auto lookat = vec3(278, 278, 0);
        this->cam = camera(lookfrom, lookat, vec3(0.0, 1.0, 0.0), 40.0, aspect, 0.0, 10.0, 0.0, 1.0);
        this->background_type = BackgroundType::Black;
    }
};

// ---------------------------------------------------------------------------
// Arbitrary-nesting test scene (ours; raytracingweekend_amd/csrc/host/
// scenes.cpp builds the same with the library's host API): the Cornell room,
// instanced boxes inside a list, a flip over a list holding a transformed
// rect, a medium inside a nested list, a medium inside a translated list,
// lists two deep under rotate_y / translate.
// ---------------------------------------------------------------------------
class nested_scene : public scene {
public:
    nested_scene(double aspect, bool media = true) : scene() {
        auto solid = [](double r, double g, double b) { return std::make_shared<constant_texture>(vec3(r, g, b)); };
        auto red = std::make_shared<lambertian>(solid(0.65f, 0.05f, 0.05f));
        auto white = std::make_shared<lambertian>(solid(0.73f, 0.73f, 0.73f));
        auto green = std::make_shared<lambertian>(solid(0.12f, 0.45f, 0.15f));
        auto light = std::make_shared<diffuse_light>(solid(15.0, 15.0, 15.0));
        auto glass = std::make_shared<dielectric>(1.5);
        typedef std::vector<std::shared_ptr<hittable>> objs;
        auto L_ = [](objs v) { return std::make_shared<hittable_list>(v); };

        auto lamp = std::make_shared<xz_rect>(213.0, 343.0, 227.0, 332.0, 554.0, light);
        Add(lamp);
        lights->objects.push_back(lamp);
        const double W = 555.0;
        Add(std::make_shared<flip_normals>(std::make_shared<yz_rect>(0.0, W, 0.0, W, W, green)));
        Add(std::make_shared<yz_rect>(0.0, W, 0.0, W, 0.0, red));
        Add(std::make_shared<flip_normals>(std::make_shared<xz_rect>(0.0, W, 0.0, W, W, white)));
        Add(std::make_shared<xz_rect>(0.0, W, 0.0, W, 0.0, white));
        Add(std::make_shared<flip_normals>(std::make_shared<xy_rect>(0.0, W, 0.0, W, W, white)));
        Add(L_({std::make_shared<translate>(
                    std::make_shared<rotate_y>(std::make_shared<box>(vec3(0, 0, 0), vec3(80, 80, 80), white), 30.0),
                    vec3(60, 0, 350)),
                std::make_shared<translate>(std::make_shared<box>(vec3(0, 0, 0), vec3(60, 120, 60), red),
                                            vec3(420, 0, 380)),
                std::make_shared<rotate_y>(
                    std::make_shared<translate>(std::make_shared<box>(vec3(0, 0, 0), vec3(50, 50, 50), green),
                                                vec3(300, 0, 100)),
                    -10.0)}));
        Add(std::make_shared<flip_normals>(
            L_({std::make_shared<translate>(std::make_shared<xy_rect>(0.0, 100.0, 0.0, 100.0, 0.0, white),
                                            vec3(230, 300, 500))})));
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
        if (media)
        Add(std::make_shared<translate>(
            L_({std::make_shared<constant_medium>(
                    std::make_shared<rotate_y>(std::make_shared<box>(vec3(0, 0, 0), vec3(100, 100, 100), white),
                                               20.0),
                    0.01, std::make_shared<isotropic>(solid(0.2, 0.4, 0.9))),
                std::make_shared<sphere>(vec3(50, 150, 50), 30.0,
                                         std::make_shared<metal>(vec3(0.8, 0.85, 0.88), 0.1))}),
            vec3(350, 0, 150)));
        Add(L_({L_({std::make_shared<translate>(std::make_shared<sphere>(vec3(0, 0, 0), 40.0, white),
                                                vec3(400, 300, 300))}),
                std::make_shared<rotate_y>(
                    L_({std::make_shared<translate>(std::make_shared<box>(vec3(0, 0, 0), vec3(50, 50, 50), red),
                                                    vec3(100, 350, 250))}),
                    20.0)}));
        Add(std::make_shared<flip_normals>(
            L_({std::make_shared<xz_rect>(400.0, 500.0, 50.0, 150.0, 500.0, white),
                std::make_shared<translate>(std::make_shared<xz_rect>(0.0, 100.0, 0.0, 100.0, 0.0, green),
                                            vec3(50, 520, 400))})));
        this->cam = camera(vec3(278.0, 278.0, -800.0), vec3(278.0, 278.0, 0.0), vec3(0.0, 1.0, 0.0), 40.0, aspect,
                           0.0, 10.0, 0.0, 1.0);
        this->background_type = BackgroundType::Black;
    }
};

static scene* make_scene(const std::string& name, double aspect) {
    if (name == "nested") return new nested_scene(aspect);
    if (name == "nested_plain") return new nested_scene(aspect, false);
    if (name == "cornell_box") return new cornell_box_scene(aspect);
    if (name == "random_balls") return new random_balls_scene(aspect);
    if (name == "dielectric") return new dielectric_scene(aspect);
    if (name == "light_sample") return new light_sample(aspect);
    if (name == "book2_final") return new book2_final_scene(aspect);
    fprintf(stderr, "unknown scene %s\n", name.c_str());
    exit(2);
}

// ---------------------------------------------------------------------------
// Integrator: restatement of RayTracingWeekend.cpp:45-160 over the reference
// classes.  g_segments counts world hit queries (one per call with depth > 0).
// ---------------------------------------------------------------------------
static thread_local uint64_t g_segments = 0;

static vec3 color(const ray& r, const scene* s, int depth) {
    if (depth <= 0) return vec3(0.0);  // :47-48
    hit_record rec;
    ++g_segments;
    if (s->GetWorld().hit(r, 0.001f, std::numeric_limits<double>::max(), rec)) {  // :52
        switch (s->GetRenderType()) {
        case RenderType::Shaded: {
            vec3 emitted = rec.mat_ptr->emitted(r, rec, rec.u, rec.v, rec.p);  // :58
            scatter_record srec;
            if (!rec.mat_ptr->scatter(r, rec, srec)) return emitted;  // :62-63
            std::shared_ptr<pdf> material_pdf = srec.pdf_ptr;  // :112
            if (material_pdf == nullptr)                       // :114-115
                return srec.attenuation * color(srec.scattered_ray_without_pdf, s, depth - 1);
            std::shared_ptr<pdf> p = material_pdf;             // :117-121
            if (s->GetLights() != nullptr && !s->GetLights()->objects.empty())
                p = std::make_shared<mixture_pdf>(material_pdf, std::make_shared<hittable_pdf>(s->GetLights(), rec.p));
            ray scattered = ray(rec.p, p->generate(), r.time());  // :123
            double pdf_val = p->value(scattered.direction());     // :124
            if (pdf_val <= 0.0) return emitted;                   // :126-127
            return emitted + srec.attenuation * rec.mat_ptr->scattering_pdf(r, rec, scattered) *
                                 color(scattered, s, depth - 1) / pdf_val;  // :129-132
        }
        case RenderType::Normal:
            return 0.5f * (rec.normal + 1);  // :135-136
        default:
            return vec3(0, 0, 0);
        }
    }
    switch (s->GetBackgroundType()) {  // :143-158
    case BackgroundType::Gradient: {
        vec3 unit_direction = normalize(r.direction());
        double t = 0.5f * (unit_direction.y + 1.0);
        return lerp(vec3(0.5f, 0.7f, 1.0), vec3(1.0, 1.0, 1.0), t);
    }
    case BackgroundType::Black:
    default:
        return vec3(0, 0, 0);
    }
}

// Force the lazy, racy Perlin initialisation (noise.h:91-94) to happen with
// no path key active, i.e. from default-seeded engines as in the reference.
static void init_perlin() {
    noise_texture nt(1.0);
    (void)nt.value(0, 0, vec3(0.5, 0.5, 0.5));
}

// Render loop body of RayTracingWeekend.cpp:214-241 (without the gamma step,
// which the tests apply to the returned sums exactly as :241-244 does).
// row_stride > 1 renders rows 0, row_stride, 2*row_stride, ... only (a bounded
// sample of a large image for the bench's CPU baseline); other rows stay 0.
static void render(scene* sc, int nx, int ny, int spp, int depth, uint64_t seed, int threads,
                   std::vector<double>& sums, uint64_t& segments, int row_stride = 1) {
    init_perlin();
    camera& cam = sc->GetCamera();
    sums.assign((size_t)nx * ny * 3, 0.0);
    uint64_t seg_total = 0;
    omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : seg_total)
    for (int j = 0; j < ny; j += row_stride) {
        g_segments = 0;
        std::uniform_real_distribution<double> uniform;
        std::minstd_rand engine;  // -> per-path stream while a key is active
        for (int i = 0; i < nx; i++) {
            vec3 sum(0, 0, 0);
            const uint32_t pixel = (uint32_t)(j * nx + i);
            for (int s = 0; s < spp; s++) {
                rtw_inject_begin(seed, pixel, (uint32_t)s);
                double u = double(i + uniform(engine)) / double(nx);  // :227
                double v = double(j + uniform(engine)) / double(ny);  // :228
                ray r = cam.get_ray(u, v);                            // :231
                vec3 c = color(r, sc, depth);                         // :232
                rtw_inject_end();
                sum += c;                                             // :235-239
            }
            double* o = &sums[((size_t)j * nx + i) * 3];
            o[0] = sum.x;
            o[1] = sum.y;
            o[2] = sum.z;
        }
        seg_total += g_segments;
    }
    segments = seg_total;
}

// ---------------------------------------------------------------------------
// scene dump
// ---------------------------------------------------------------------------
struct dumper {
    std::map<const material*, int> mats;
    std::map<const texture*, int> texs;
    std::vector<std::string> mat_json, tex_json;

    static std::string d(double x) {
        char b[64];
        snprintf(b, sizeof b, "%.17g", x);
        return b;
    }
    static std::string v3(const vec3& v) { return "[" + d(v.x) + "," + d(v.y) + "," + d(v.z) + "]"; }

    int tex(const texture* t) {
        auto it = texs.find(t);
        if (it != texs.end()) return it->second;
        std::string j;
        if (auto c = dynamic_cast<const constant_texture*>(t)) {
            j = "{\"type\":\"constant\",\"color\":" + v3(c->color) + "}";
        } else if (auto n = dynamic_cast<const noise_texture*>(t)) {
            j = "{\"type\":\"noise\",\"scale\":" + d(n->scale) + "}";
        } else if (auto ch = dynamic_cast<const checker_texture*>(t)) {
            int o = tex(ch->odd.get()), e = tex(ch->even.get());
            j = "{\"type\":\"checker\",\"odd\":" + std::to_string(o) + ",\"even\":" + std::to_string(e) + "}";
        } else {
            j = "{\"type\":\"unknown\"}";
        }
        int id = (int)tex_json.size();
        texs[t] = id;
        tex_json.push_back(j);
        return id;
    }

    int mat(const material* m) {
        auto it = mats.find(m);
        if (it != mats.end()) return it->second;
        std::string j;
        if (auto l = dynamic_cast<const lambertian*>(m)) {
            j = "{\"type\":\"lambertian\",\"texture\":" + std::to_string(tex(l->albedo.get())) + "}";
        } else if (auto me = dynamic_cast<const metal*>(m)) {
            j = "{\"type\":\"metal\",\"albedo\":" + v3(me->albedo) + ",\"fuzz\":" + d(me->fuzz) + "}";
        } else if (auto di = dynamic_cast<const dielectric*>(m)) {
            j = "{\"type\":\"dielectric\",\"ref_idx\":" + d(di->ref_idx) + "}";
        } else if (auto dl = dynamic_cast<const diffuse_light*>(m)) {
            j = "{\"type\":\"diffuse_light\",\"texture\":" + std::to_string(tex(dl->emit.get())) + "}";
        } else if (auto is = dynamic_cast<const isotropic*>(m)) {
            j = "{\"type\":\"isotropic\",\"texture\":" + std::to_string(tex(is->albedo.get())) + "}";
        } else {
            j = "{\"type\":\"unknown\"}";
        }
        int id = (int)mat_json.size();
        mats[m] = id;
        mat_json.push_back(j);
        return id;
    }

    std::string obj(const hittable* h) {
        if (auto l = dynamic_cast<const hittable_list*>(h)) {
            std::string j = "{\"type\":\"list\",\"objects\":[";
            for (size_t i = 0; i < l->objects.size(); i++) j += (i ? "," : "") + obj(l->objects[i].get());
            return j + "]}";
        }
        if (auto b = dynamic_cast<const box*>(h)) {
            return "{\"type\":\"box\",\"pmin\":" + v3(b->pmin) + ",\"pmax\":" + v3(b->pmax) +
                   ",\"list\":" + obj(&b->list_ptr) + "}";
        }
        if (auto r = dynamic_cast<const xy_rect*>(h)) {
            return "{\"type\":\"xy_rect\",\"p\":[" + d(r->x0) + "," + d(r->x1) + "," + d(r->y0) + "," + d(r->y1) +
                   "," + d(r->k) + "],\"mat\":" + std::to_string(mat(r->mp.get())) + "}";
        }
        if (auto r = dynamic_cast<const xz_rect*>(h)) {
            return "{\"type\":\"xz_rect\",\"p\":[" + d(r->x0) + "," + d(r->x1) + "," + d(r->z0) + "," + d(r->z1) +
                   "," + d(r->k) + "],\"mat\":" + std::to_string(mat(r->mp.get())) + "}";
        }
        if (auto r = dynamic_cast<const yz_rect*>(h)) {
            return "{\"type\":\"yz_rect\",\"p\":[" + d(r->y0) + "," + d(r->y1) + "," + d(r->z0) + "," + d(r->z1) +
                   "," + d(r->k) + "],\"mat\":" + std::to_string(mat(r->mp.get())) + "}";
        }
        if (auto f = dynamic_cast<const flip_normals*>(h)) {
            return "{\"type\":\"flip\",\"ptr\":" + obj(f->ptr.get()) + "}";
        }
        if (auto t = dynamic_cast<const translate*>(h)) {
            return "{\"type\":\"translate\",\"offset\":" + v3(t->offset) + ",\"ptr\":" + obj(t->ptr.get()) + "}";
        }
        if (auto ro = dynamic_cast<const rotate_y*>(h)) {
            return "{\"type\":\"rotate_y\",\"sin\":" + d(ro->sin_theta) + ",\"cos\":" + d(ro->cos_theta) +
                   ",\"hasbox\":" + (ro->hasbox ? "true" : "false") + ",\"bmin\":" + v3(ro->bbox._min) +
                   ",\"bmax\":" + v3(ro->bbox._max) + ",\"ptr\":" + obj(ro->ptr.get()) + "}";
        }
        if (auto cm = dynamic_cast<const constant_medium*>(h)) {
            return "{\"type\":\"constant_medium\",\"density\":" + d(cm->density) +
                   ",\"mat\":" + std::to_string(mat(cm->mp.get())) + ",\"boundary\":" + obj(cm->boundary.get()) + "}";
        }
        if (auto s = dynamic_cast<const sphere*>(h)) {
            return "{\"type\":\"sphere\",\"center\":" + v3(s->center) + ",\"radius\":" + d(s->radius) +
                   ",\"mat\":" + std::to_string(mat(s->mat.get())) + "}";
        }
        if (auto s = dynamic_cast<const moving_sphere*>(h)) {
            return "{\"type\":\"moving_sphere\",\"center\":" + v3(s->center) + ",\"radius\":" + d(s->radius) +
                   ",\"center1\":" + v3(s->movement.center1) + ",\"time0\":" + d(s->movement.time0) +
                   ",\"time1\":" + d(s->movement.time1) + ",\"mat\":" + std::to_string(mat(s->mat.get())) + "}";
        }
        return "{\"type\":\"unknown\"}";
    }
};

static void dump_scene(scene* sc) {
    dumper dp;
    std::string world = dp.obj(&sc->GetWorld());
    std::string lights = sc->GetLights() ? dp.obj(sc->GetLights().get()) : "null";
    const camera& c = sc->GetCamera();
    printf("{\"world\":%s,\n\"lights\":%s,\n", world.c_str(), lights.c_str());
    printf("\"materials\":[");
    for (size_t i = 0; i < dp.mat_json.size(); i++) printf("%s%s", i ? "," : "", dp.mat_json[i].c_str());
    printf("],\n\"textures\":[");
    for (size_t i = 0; i < dp.tex_json.size(); i++) printf("%s%s", i ? "," : "", dp.tex_json[i].c_str());
    printf("],\n\"camera\":{\"origin\":%s,\"lower_left\":%s,\"horizontal\":%s,\"vertical\":%s,"
           "\"u\":%s,\"v\":%s,\"w\":%s,\"time0\":%s,\"time1\":%s,\"lens_radius\":%s},\n",
           dumper::v3(c.origin).c_str(), dumper::v3(c.lower_left_corner).c_str(), dumper::v3(c.horizontal).c_str(),
           dumper::v3(c.vertical).c_str(), dumper::v3(c.u).c_str(), dumper::v3(c.v).c_str(),
           dumper::v3(c.w).c_str(), dumper::d(c.time0).c_str(), dumper::d(c.time1).c_str(),
           dumper::d(c.lens_radius).c_str());
    printf("\"render_type\":\"%s\",\"background\":\"%s\"}\n",
           sc->GetRenderType() == RenderType::Shaded ? "shaded" : "normal",
           sc->GetBackgroundType() == BackgroundType::Gradient ? "gradient" : "black");
}

static void dump_perlin() {
    init_perlin();
    printf("{\"ranvec\":[");
    for (int i = 0; i < 256; i++)
        printf("%s%s", i ? "," : "", dumper::v3(perlin::ranvec[i]).c_str());
    printf("],\n\"ranfloat\":[");
    for (int i = 0; i < 256; i++) printf("%s%.17g", i ? "," : "", perlin::ranfloat[i]);
    const int* perms[3] = {perlin::perm_x, perlin::perm_y, perlin::perm_z};
    const char* names[3] = {"perm_x", "perm_y", "perm_z"};
    for (int a = 0; a < 3; a++) {
        printf("],\n\"%s\":[", names[a]);
        for (int i = 0; i < 256; i++) printf("%s%d", i ? "," : "", perms[a][i]);
    }
    // known-answer samples of noise(), turb() and noise_texture::value
    printf("],\n\"samples\":[");
    std::minstd_rand eng;  // inactive -> plain minstd_rand, deterministic points
    std::uniform_real_distribution<double> U;
    perlin pn;
    noise_texture nt(0.1);
    for (int k = 0; k < 64; k++) {
        double x = -300.0 + 600.0 * U(eng);
        double y = -300.0 + 600.0 * U(eng);
        double z = -300.0 + 600.0 * U(eng);
        if (k < 8) { x *= 0.01; y *= 0.01; z *= 0.01; }
        vec3 p(x, y, z);
        vec3 tv = nt.value(0, 0, p);
        printf("%s{\"p\":%s,\"noise\":%.17g,\"turb\":%.17g,\"tex\":%s}", k ? "," : "", dumper::v3(p).c_str(),
               pn.noise(p), pn.turb(p), dumper::v3(tv).c_str());
    }
    printf("]}\n");
}

// The reference's output step for a rendered image, RayTracingWeekend.cpp:
// 235-244 (average, gamma 2, clamp into the canvas) and 252-276 (P3 header,
// rows ny-1..0, int(255.99f * c) per channel, streamed with operator<<),
// over the per-pixel sums of render().
static int write_ppm_reference(const char* path, const std::vector<double>& sums, int nx, int ny, int spp) {
    std::vector<vec3> canvas(nx * ny);
    for (int j = 0; j < ny; j++)
        for (int i = 0; i < nx; i++) {
            const double* o = &sums[((size_t)j * nx + i) * 3];
            vec3 sum(o[0], o[1], o[2]);
            vec3 col = sum / static_cast<double>(spp);
            col = vec3(std::min(sqrt(col.x), 1.0), std::min(sqrt(col.y), 1.0), std::min(sqrt(col.z), 1.0));
            canvas[j * nx + i] = col;
        }
    std::ofstream out(path, std::ios::binary);
    if (!out) return 3;
    out << "P3\n" << nx << " " << ny << "\n255\n";
    for (int j = ny - 1; j >= 0; j--)
        for (int i = 0; i < nx; i++) {
            vec3 col = canvas[j * nx + i];
            int ir = int(255.99f * col.r);
            int ig = int(255.99f * col.g);
            int ib = int(255.99f * col.b);
            out << ir << " " << ig << " " << ib << "\n";
        }
    return out.good() ? 0 : 3;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s scene|render|bench|perlin|ppm ...\n", argv[0]);
        return 2;
    }
    std::string cmd = argv[1];
    if (cmd == "scene" && argc == 4) {
        scene* sc = make_scene(argv[2], atof(argv[3]));
        dump_scene(sc);
        return 0;
    }
    if (cmd == "perlin") {
        dump_perlin();
        return 0;
    }
    if ((cmd == "render" && argc == 10) || (cmd == "bench" && (argc == 9 || argc == 10)) ||
        (cmd == "ppm" && argc == 10)) {
        std::string name = argv[2];
        int nx = atoi(argv[3]), ny = atoi(argv[4]), spp = atoi(argv[5]), depth = atoi(argv[6]);
        uint64_t seed = strtoull(argv[7], nullptr, 10);
        int threads = atoi(argv[8]);
        int row_stride = (cmd == "bench" && argc == 10) ? std::max(1, atoi(argv[9])) : 1;
        scene* sc = make_scene(name, nx * 1.0 / ny);  // RayTracingWeekend.cpp:204
        std::vector<double> sums;
        uint64_t segments = 0;
        auto t0 = std::chrono::steady_clock::now();
        render(sc, nx, ny, spp, depth, seed, threads, sums, segments, row_stride);
        auto t1 = std::chrono::steady_clock::now();
        double sec = std::chrono::duration<double>(t1 - t0).count();
        double samples = (double)nx * ((ny + row_stride - 1) / row_stride) * spp;
        printf("{\"seconds\":%.6f,\"samples\":%.0f,\"segments\":%llu,\"msamples_per_s\":%.6f,\"threads\":%d}\n", sec,
               samples, (unsigned long long)segments, samples / sec / 1e6, threads);
        if (cmd == "ppm") return write_ppm_reference(argv[9], sums, nx, ny, spp);
        if (cmd == "render") {
            FILE* f = fopen(argv[9], "wb");
            if (!f) return 3;
            fwrite(sums.data(), sizeof(double), sums.size(), f);
            fclose(f);
        }
        return 0;
    }
    fprintf(stderr, "bad arguments\n");
    return 2;
}
