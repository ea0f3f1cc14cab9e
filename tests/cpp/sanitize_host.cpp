// sanitize_host.cpp — the host library's CPU-side code under ASan / UBSan
// (SURVEY.md §5), built by tests/test_sanitizers.py with g++
// -fsanitize=address,undefined from the host sources (flatten, scene API,
// scenes, desc validation, output) and the oracle's C restatement:
//   1. every built-in scene (and user graphs of every nesting form the
//      flattener takes apart) flattened flat and with BVHs, validated, freed;
//   2. the same descs corrupted field by field -- counts, indices, kinds,
//      ops, BVH links, visit program, null arrays -- and handed to
//      validate_desc, which must refuse or accept them without touching
//      memory it does not own;
//   3. refused graphs (a bvh_node over a medium, unknown subclasses, nulls);
//   4. the oracle rendering each valid desc, finalize, the PPM writer;
//   5. the header API's evaluating half (hit / scatter / get_ray / pdfs) over
//      a few paths of every scene.
// Prints "OK (<n> checks)" on success; any sanitizer report aborts.
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <string>
#include <vector>
#include <unistd.h>

#include "flatten.h"
#include "rtw_host_util.h"
#include "scene.h"
#include "../../oracle/rtw_oracle.h"

namespace {

int g_checks = 0;
#define CHECK(c)                                                                 \
    do {                                                                         \
        ++g_checks;                                                              \
        if (!(c)) {                                                              \
            std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

// A deep, owned copy of a desc whose fields can be corrupted freely.
struct owned_desc {
    rtw_scene_desc d;
    std::vector<rtw_prim> prims;
    std::vector<rtw_entry> entries;
    std::vector<rtw_material> materials;
    std::vector<rtw_texture> textures;
    std::vector<rtw_light> lights;
    std::vector<rtw_bvh_node> nodes;
    std::vector<int32_t> items, visits, perm;
    std::vector<double> ranvec;

    explicit owned_desc(const rtw_scene_desc& s) : d(s) {
        prims.assign(s.prims, s.prims + s.n_prims);
        entries.assign(s.entries, s.entries + s.n_entries);
        materials.assign(s.materials, s.materials + s.n_materials);
        textures.assign(s.textures, s.textures + s.n_textures);
        lights.assign(s.lights, s.lights + s.n_lights);
        nodes.assign(s.bvh_nodes, s.bvh_nodes + s.n_bvh_nodes);
        items.assign(s.bvh_items, s.bvh_items + s.n_bvh_items);
        visits.assign(s.visits, s.visits + s.n_visits);
        if (s.has_perlin) {
            perm.assign(s.perlin_perm, s.perlin_perm + 3 * 256);
            ranvec.assign(s.perlin_ranvec, s.perlin_ranvec + 3 * 256);
        }
        relink();
    }
    void relink() {
        d.prims = prims.data();
        d.entries = entries.data();
        d.materials = materials.data();
        d.textures = textures.data();
        d.lights = lights.data();
        d.bvh_nodes = nodes.data();
        d.bvh_items = items.data();
        d.visits = visits.data();
        d.perlin_perm = perm.empty() ? nullptr : perm.data();
        d.perlin_ranvec = ranvec.empty() ? nullptr : ranvec.data();
    }
};

int32_t nasty(std::mt19937& g, int32_t n) {
    const int32_t pick[] = {-2, -1, 0, 1, n - 1, n, n + 1, 2 * n + 7, INT_MAX, INT_MIN, INT_MAX - 3,
                            (int32_t)(RTW_ITEM_BOX | 3), (int32_t)(RTW_VISIT_REPLAY | 1)};
    return pick[g() % (sizeof pick / sizeof pick[0])];
}

// Corrupt one integer field of a copy of `src` and validate it.
void fuzz_validate(const rtw_scene_desc& src, std::mt19937& g, int rounds) {
    for (int r = 0; r < rounds; ++r) {
        owned_desc o(src);
        rtw_scene_desc& d = o.d;
        const int what = (int)(g() % 22);
        auto any = [&](int n) { return n > 0 ? (int)(g() % n) : 0; };
        switch (what) {
        case 0: d.n_prims = nasty(g, d.n_prims); break;
        case 1: d.n_entries = nasty(g, d.n_entries); break;
        case 2: d.n_materials = nasty(g, d.n_materials); break;
        case 3: d.n_textures = nasty(g, d.n_textures); break;
        case 4: d.n_lights = nasty(g, d.n_lights); break;
        case 5: d.n_bvh_nodes = nasty(g, d.n_bvh_nodes); break;
        case 6: d.n_bvh_items = nasty(g, d.n_bvh_items); break;
        case 7: d.n_visits = nasty(g, d.n_visits); break;
        case 8: d.world_bvh_root = nasty(g, d.n_bvh_nodes); break;
        case 9: if (!o.entries.empty()) o.entries[any(d.n_entries)].first_prim = nasty(g, d.n_prims); break;
        case 10: if (!o.entries.empty()) o.entries[any(d.n_entries)].n_prims = nasty(g, d.n_prims); break;
        case 11: if (!o.entries.empty()) o.entries[any(d.n_entries)].n_ops = nasty(g, RTW_MAX_OPS); break;
        case 12: if (!o.entries.empty()) o.entries[any(d.n_entries)].bvh_root = nasty(g, d.n_bvh_nodes); break;
        case 13: if (!o.entries.empty()) o.entries[any(d.n_entries)].kind = nasty(g, 2); break;
        case 14: if (!o.prims.empty()) o.prims[any(d.n_prims)].material = nasty(g, d.n_materials); break;
        case 15: if (!o.prims.empty()) o.prims[any(d.n_prims)].entry = nasty(g, d.n_entries); break;
        case 16: if (!o.materials.empty()) o.materials[any(d.n_materials)].texture = nasty(g, d.n_textures); break;
        case 17: if (!o.lights.empty()) o.lights[any(d.n_lights)].prim = nasty(g, d.n_prims); break;
        case 18:
            if (!o.nodes.empty()) {
                rtw_bvh_node& n = o.nodes[any(d.n_bvh_nodes)];
                (g() & 1 ? n.left : (g() & 1 ? n.right : n.count)) = nasty(g, d.n_bvh_nodes);
            }
            break;
        case 19: if (!o.items.empty()) o.items[any(d.n_bvh_items)] = nasty(g, d.n_prims); break;
        case 20: if (!o.visits.empty()) o.visits[any(d.n_visits)] = nasty(g, d.n_entries); break;
        case 21: {  // a null array behind a nonzero count
            const int k = any(4);
            if (k == 0) d.prims = nullptr; else if (k == 1) d.entries = nullptr; else if (k == 2) d.bvh_nodes = nullptr;
            else d.bvh_items = nullptr;
            break;
        }
        }
        // A count is the caller's promise about its array's length, which no
        // validator can check; so a corrupted count comes with an array that
        // long (zero-filled), and the nulled array of case 21 stays null.
        const int cap = 1 << 16;
        const int counts[] = {d.n_prims, d.n_entries, d.n_materials, d.n_textures, d.n_lights,
                              d.n_bvh_nodes, d.n_bvh_items, d.n_visits};
        bool sane = true;
        for (int c : counts) sane = sane && c <= cap;
        if (!sane) continue;
        const bool null_prims = what == 21 && !d.prims, null_entries = what == 21 && !d.entries;
        const bool null_nodes = what == 21 && !d.bvh_nodes, null_items = what == 21 && !d.bvh_items;
        auto grow = [](auto& v, int n) { if (n > (int)v.size()) v.resize(n); };
        grow(o.prims, d.n_prims);
        grow(o.entries, d.n_entries);
        grow(o.materials, d.n_materials);
        grow(o.textures, d.n_textures);
        grow(o.lights, d.n_lights);
        grow(o.nodes, d.n_bvh_nodes);
        grow(o.items, d.n_bvh_items);
        grow(o.visits, d.n_visits);
        o.relink();
        if (null_prims) d.prims = nullptr;
        if (null_entries) d.entries = nullptr;
        if (null_nodes) d.bvh_nodes = nullptr;
        if (null_items) d.bvh_items = nullptr;
        const int rc = validate_desc(&d);
        CHECK(rc == RTW_OK || rc == RTW_ERR_INVALID || rc == RTW_ERR_UNSUPPORTED);
    }
}

// RayTracingWeekend.cpp:45-160 over the header API (as tests/cpp/host_render.cpp)
vec3 color(const ray& r, const scene& s, int depth) {
    if (depth <= 0) return vec3(0.0);
    hit_record rec;
    if (!s.GetWorld().hit(r, 0.001f, std::numeric_limits<double>::max(), rec)) {
        if (s.GetBackgroundType() != BackgroundType::Gradient) return vec3(0, 0, 0);
        const vec3 u = normalize(r.direction());
        return lerp(vec3(0.5f, 0.7f, 1.0), vec3(1.0, 1.0, 1.0), 0.5f * (u.y + 1.0));
    }
    const vec3 emitted = rec.mat_ptr->emitted(r, rec, rec.u, rec.v, rec.p);
    scatter_record srec;
    if (!rec.mat_ptr->scatter(r, rec, srec)) return emitted;
    if (!srec.pdf_ptr) return srec.attenuation * color(srec.scattered_ray_without_pdf, s, depth - 1);
    std::shared_ptr<pdf> p = srec.pdf_ptr;
    if (s.GetLights() && !s.GetLights()->objects.empty())
        p = std::make_shared<mixture_pdf>(srec.pdf_ptr, std::make_shared<hittable_pdf>(s.GetLights(), rec.p));
    const ray scattered(rec.p, p->generate(), r.time());
    const double pv = p->value(scattered.direction());
    if (pv <= 0.0) return emitted;
    return emitted + srec.attenuation * rec.mat_ptr->scattering_pdf(r, rec, scattered) * color(scattered, s, depth - 1) / pv;
}

}  // namespace

int main() {
    std::mt19937 g(12345);
    const char* names[] = {"cornell_box", "random_balls", "dielectric", "light_sample", "book2_final", "nested",
                           "nested_plain"};
    char ppm[] = "/tmp/rtw_sanitize_XXXXXX";
    const int fd = mkstemp(ppm);
    CHECK(fd >= 0);
    close(fd);
    for (const char* name : names) {
        for (int bvh = 0; bvh < 2; ++bvh) {
            rtw_scene_desc* d = nullptr;
            CHECK(rtw_scene_builtin(name, 1.5, bvh, &d) == RTW_OK && d);
            CHECK(validate_desc(d) == RTW_OK);
            // the oracle over the valid desc, then finalize + PPM
            const int nx = 12, ny = 8;
            std::vector<double> sums(nx * ny * 3, 0.0), canvas(nx * ny * 3);
            uint64_t seg = 0;
            CHECK(rtw_oracle_render(d, &d->camera, nx, ny, 0, ny, 0, 2, 10, 7, 1, sums.data(), &seg) == 0);
            CHECK(seg > 0);
            rtw_finalize_canvas(sums.data(), nx, ny, 2, canvas.data());
            CHECK(rtw_write_ppm(ppm, canvas.data(), nx, ny) == RTW_OK);
            fuzz_validate(*d, g, 3000);
            rtw_scene_desc_free(d);
        }
        // the evaluating header API over a few paths
        auto sc = make_builtin_scene(name, 1.5);
        CHECK(sc != nullptr);
        for (int s = 0; s < 16; ++s) {
            rtw::path_stream st(3, (uint32_t)s, 0);
            const ray r = sc->GetCamera().get_ray((s % 4 + 0.5) / 4, (s / 4 + 0.5) / 4);
            const vec3 c = color(r, *sc, 20);
            CHECK(c.x == c.x && c.y == c.y && c.z == c.z);
        }
    }
    // refused graphs
    {
        rtw_scene_desc* d = nullptr;
        CHECK(rtw_scene_builtin("no such scene", 1.0, 0, &d) != RTW_OK);
        CHECK(validate_desc(nullptr) == RTW_ERR_INVALID);
        auto mat = std::make_shared<isotropic>(std::make_shared<constant_texture>(vec3(1, 1, 1)));
        auto fog = std::make_shared<constant_medium>(
            std::make_shared<sphere>(vec3(0, 0, 0), 1.0, std::shared_ptr<material>()), 0.1, mat);
        hittable_list world;
        world.objects.push_back(std::make_shared<bvh_node>(std::vector<std::shared_ptr<hittable>>{fog, fog}, 0.0, 1.0));
        camera cam(vec3(0, 0, 5), vec3(0, 0, 0), vec3(0, 1, 0), 40, 1.0, 0.0, 5.0, 0.0, 1.0);
        CHECK(rtw_flatten_world(world, nullptr, cam, 0, 1, 1, &d) == RTW_ERR_UNSUPPORTED);
        hittable_list nulls;
        nulls.objects.push_back(nullptr);
        CHECK(rtw_flatten_world(nulls, nullptr, cam, 0, 1, 0, &d) != RTW_OK);
    }
    std::remove(ppm);
    std::printf("OK (%d checks)\n", g_checks);
    return 0;
}
