/*
 * rtw_gpu.h — C ABI of the MI355X path tracer (raytracingweekend_amd).
 *
 * This is the drop-in boundary for the per-pixel render loop of
 * silvesthu/RayTracingWeekend.  The reference has no plugin/FFI layer; its
 * seam is the triple `_for` loop body in
 *     RayTracingWeekend/RayTracingWeekend.cpp:211-250
 * (jitter -> camera::get_ray -> color() -> average -> gamma -> canvas) fed by
 * the scene accessors GetWorld/GetLights/GetCamera/GetRenderType/
 * GetBackgroundType (Scene/scene.h:24-31) and the compile-time constants
 * nx, ny, subPixelCount, max_depth (RayTracingWeekend.cpp:32-43).
 *
 * A host program (C/C++, or Python through ctypes) flattens its hittable
 * graph into an rtw_scene_desc, uploads it once, and calls
 * rtw_render_accumulate() where the reference ran the triple `_for`.
 * rtw_finalize_canvas() is RayTracingWeekend.cpp:241-244 and rtw_write_ppm()
 * is RayTracingWeekend.cpp:252-276.
 *
 * Conventions
 *   - plain C types only; every pointer/size pair is caller-owned unless a
 *     function returns a handle;
 *   - every int-returning call returns 0 on success and a negative
 *     rtw_status on failure; rtw_last_error() gives a thread-local message;
 *   - calls are thread-compatible: one render per scene handle at a time.
 *
 * Arithmetic is IEEE fp64 throughout (the reference computes in double,
 * vec3.h:35-44), unless a render asks for the fp32 fast mode
 * (rtw_render_params.precision = RTW_PRECISION_FP32: statistical parity
 * only).  Randomness: every camera sample owns one std::minstd_rand
 * stream (48271 * x mod 2^31-1, libstdc++ generate_canonical<double,53>, i.e.
 * two raw draws per double) seeded from (seed, pixel, sample) by
 * rtw_path_seed() below, so results do not depend on how samples are sharded
 * across threads, wavefronts or GPUs.
 */
#ifndef RTW_GPU_H
#define RTW_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTW_ABI_VERSION 3
/* Fixed by the ABI: it sizes rtw_entry (op / op_param).  A client built with
 * another value would lay entries out differently from this library. */
#define RTW_MAX_OPS 8

/* ------------------------------------------------------------------ */
/* status codes                                                        */
/* ------------------------------------------------------------------ */
typedef enum rtw_status {
    RTW_OK = 0,
    RTW_ERR_INVALID = -1,     /* bad argument / malformed scene            */
    RTW_ERR_HIP = -2,         /* a HIP runtime call failed                 */
    RTW_ERR_NO_DEVICE = -3,   /* no gfx950 device visible                  */
    RTW_ERR_OOM = -4,         /* device allocation failed                  */
    RTW_ERR_UNSUPPORTED = -5  /* scene uses a feature this build lacks     */
} rtw_status;

/* ------------------------------------------------------------------ */
/* flattened scene (produced on the host from the hittable graph)      */
/* ------------------------------------------------------------------ */

/* Leaf primitives.  hittable.h:142-267 (xy/xz/yz_rect), sphere.h:40-131. */
typedef enum rtw_prim_type {
    RTW_PRIM_SPHERE = 0,        /* p = cx cy cz r                                  */
    RTW_PRIM_MOVING_SPHERE = 1, /* p = c0x c0y c0z r c1x c1y c1z time0 time1       */
    RTW_PRIM_RECT_XY = 2,       /* p = x0 x1 y0 y1 k   (plane z = k, normal +z)    */
    RTW_PRIM_RECT_XZ = 3,       /* p = x0 x1 z0 z1 k   (plane y = k, normal +y)    */
    RTW_PRIM_RECT_YZ = 4        /* p = y0 y1 z0 z1 k   (plane x = k, normal +x)    */
} rtw_prim_type;

typedef struct rtw_prim {
    int32_t type;     /* rtw_prim_type                                          */
    int32_t material; /* index into materials                                   */
    int32_t flip;     /* flip_normals wrappers directly around this primitive   */
    int32_t entry;    /* owning entry (-1: only referenced as a light)          */
    double p[10];
} rtw_prim; /* 96 bytes */

/* Transform ops of an entry, applied outermost first on the way in and
 * innermost first on the way out (hittable.h:269-416). */
typedef enum rtw_op_type {
    RTW_OP_TRANSLATE = 1, /* param = offset xyz                  (translate)    */
    RTW_OP_ROTATE_Y = 2,  /* param = sin_theta cos_theta -       (rotate_y)     */
    RTW_OP_FLIP = 3       /* negate normal                       (flip_normals) */
} rtw_op_type;

typedef enum rtw_entry_kind {
    RTW_ENTRY_GROUP = 0,  /* closest hit over prims [first_prim, +n_prims)       */
    RTW_ENTRY_MEDIUM = 1  /* constant_medium (hittable.h:420-489) whose boundary
                             is the group described by the same fields          */
} rtw_entry_kind;

/* One element of the world hittable_list (hittable_list.h:5-62).  A bare
 * primitive is a group of one; box (hittable_list.h:65-114) is a group of six
 * rects; translate(rotate_y(box)) is a group of six with two ops. */
typedef struct rtw_entry {
    int32_t kind;           /* rtw_entry_kind                                  */
    int32_t first_prim;
    int32_t n_prims;
    int32_t n_ops;
    int32_t op[RTW_MAX_OPS];
    int32_t phase_material; /* MEDIUM: isotropic material index                */
    int32_t bvh_root;       /* -1: linear scan; else root node of a BVH whose
                               items are prim indices of this group           */
    int32_t n_outer_ops;    /* MEDIUM: ops [0, n_outer_ops) enclose the medium
                               (its distances are measured in their frame);
                               the rest belong to its boundary (GROUP: 0)    */
    int32_t pad;
    double op_param[RTW_MAX_OPS][3];
    double density;         /* MEDIUM                                          */
    double bounds[6];       /* AABB min xyz, max xyz (world space)             */
} rtw_entry; /* 312 bytes */

/* BVH node: internal when count == 0 (children left/right), leaf when
 * count > 0 (items bvh_items[left .. left+count)).  Items of a group BVH are
 * prim indices of the group, or RTW_ITEM_BOX | i for the six rects
 * [i, i+6) of one box (hittable_list.h:65-114: xy, xy, xz, xz, yz, yz in that
 * list order), tested together as one leaf object; items of the world BVH
 * are entry indices. */
#define RTW_ITEM_BOX 0x40000000
#define RTW_ITEM_INDEX 0x3fffffff
typedef struct rtw_bvh_node {
    double bmin[3];
    double bmax[3];
    int32_t left;
    int32_t right;
    int32_t count;
    int32_t pad;
} rtw_bvh_node; /* 64 bytes */

/* material.h:59-265 */
typedef enum rtw_material_type {
    RTW_MAT_LAMBERTIAN = 0,    /* texture                          */
    RTW_MAT_METAL = 1,         /* albedo, fuzz                     */
    RTW_MAT_DIELECTRIC = 2,    /* ref_idx                          */
    RTW_MAT_DIFFUSE_LIGHT = 3, /* texture (emit)                   */
    RTW_MAT_ISOTROPIC = 4      /* texture                          */
} rtw_material_type;

typedef struct rtw_material {
    int32_t type;
    int32_t texture;
    double albedo[3];
    double fuzz;
    double ref_idx;
} rtw_material; /* 48 bytes */

/* texture.h:10-71 */
typedef enum rtw_texture_type {
    RTW_TEX_CONSTANT = 0, /* color                                       */
    RTW_TEX_CHECKER = 1,  /* odd/even texture indices                    */
    RTW_TEX_NOISE = 2     /* scale; needs perlin tables in the desc      */
} rtw_texture_type;

typedef struct rtw_texture {
    int32_t type;
    int32_t odd;
    int32_t even;
    int32_t pad;
    double color[3];
    double scale;
} rtw_texture; /* 48 bytes */

/* Members of scene::lights (Scene/scene.h:269) as seen by hittable_pdf
 * (pdf.h:35-53): only xz_rect and sphere_base override pdf_value/random
 * (hittable.h:208-228, sphere.h:88-108); anything else uses the hittable
 * defaults pdf_value = 0, random = (1,0,0) (hittable.h:36-37). */
typedef enum rtw_light_kind {
    RTW_LIGHT_DEFAULT = 0,
    RTW_LIGHT_XZ_RECT = 1,
    RTW_LIGHT_SPHERE = 2    /* sphere or moving_sphere                    */
} rtw_light_kind;

typedef struct rtw_light {
    int32_t kind;
    int32_t prim; /* index into prims (ignored for RTW_LIGHT_DEFAULT) */
} rtw_light;

/* camera.h:13-34 after construction */
typedef struct rtw_camera_desc {
    double origin[3];
    double lower_left[3];
    double horizontal[3];
    double vertical[3];
    double u[3], v[3], w[3];
    double time0, time1;
    double lens_radius;
} rtw_camera_desc;

typedef enum rtw_render_type { RTW_RENDER_SHADED = 0, RTW_RENDER_NORMAL = 1 } rtw_render_type;
typedef enum rtw_background { RTW_BG_BLACK = 0, RTW_BG_GRADIENT = 1 } rtw_background;

typedef struct rtw_scene_desc {
    int32_t abi_version;  /* RTW_ABI_VERSION */
    int32_t render_type;  /* rtw_render_type  (Scene/scene.h:272) */
    int32_t background;   /* rtw_background   (Scene/scene.h:273) */
    int32_t n_prims;
    int32_t n_entries;
    int32_t n_materials;
    int32_t n_textures;
    int32_t n_lights;
    int32_t n_bvh_nodes;
    int32_t n_bvh_items;
    int32_t world_bvh_root; /* -1: linear scan of entries; else BVH over entry indices */
    int32_t has_perlin;
    const rtw_prim* prims;
    const rtw_entry* entries;
    const rtw_material* materials;
    const rtw_texture* textures;
    const rtw_light* lights;
    const rtw_bvh_node* bvh_nodes;
    const int32_t* bvh_items;
    const double* perlin_ranvec; /* 256*3 (noise.h:219) */
    const int32_t* perlin_perm;  /* 3*256 perm_x, perm_y, perm_z (noise.h:221-223) */
    rtw_camera_desc camera;
    /* Visit program of a scene with media (n_visits > 0): the entries in the
     * order the reference's world hit calls them -- hittable_list::hit walks
     * its objects twice (hittable_list.h:16-34), so every list that holds a
     * constant_medium appears twice, nested lists inside each walk.  Second-
     * walk visits carry RTW_VISIT_REPLAY; entry index = visit & RTW_VISIT_ENTRY.
     * n_visits == 0: the world's two walks over entries[0 .. n_entries). */
    const int32_t* visits;
    int32_t n_visits;
    int32_t pad;
} rtw_scene_desc;

#define RTW_VISIT_REPLAY 0x40000000
#define RTW_VISIT_ENTRY 0x3fffffff

/* ------------------------------------------------------------------ */
/* render                                                              */
/* ------------------------------------------------------------------ */
typedef struct rtw_render_params {
    int32_t nx, ny;        /* image size (RayTracingWeekend.cpp:35-36)              */
    int32_t spp;           /* total samples per pixel (subPixelCount, :33)          */
    int32_t max_depth;     /* color() recursion limit (:42)                         */
    uint64_t seed;         /* RNG seed, see rtw_path_seed                           */
    int32_t spp_begin;     /* this call renders samples [spp_begin, spp_begin+spp_count) */
    int32_t spp_count;     /* (sample-range sharding; 0 = all of [spp_begin, spp))  */
    int32_t row_begin;     /* ... of rows j = row_begin + k*row_step (pixel sharding) */
    int32_t row_step;      /* 0 or 1 = every row                                    */
    int32_t accum_on_device; /* 1: accum_rgb is device memory of this handle's GPU
                                (hipMalloc / torch allocators) or managed memory
                                (hipMallocManaged; rtw_render_multi over several
                                GPUs refuses it: RTW_ERR_UNSUPPORTED); anything
                                else: RTW_ERR_INVALID */
    int32_t collect_kernel_times; /* 1: hipEvents around traversal launches,    */
                                  /* 2: and shade launches (adds queue gaps)   */
    int32_t wavefront_paths; /* paths in flight (0 = library default)             */
    int32_t precision;     /* rtw_precision: RTW_PRECISION_FP64 (0) = parity with the
                              CPU renderer: every path decision (rays, hit
                              distances, comparisons, random draws) in the
                              reference's IEEE double arithmetic; the radiance-only
                              factors (lambertian weight, pdf quotients) with fewer
                              divisions, a few ulps off (the strict build,
                              -DRTW_STRICT_RADIANCE=1, librtw_strict.so: the
                              reference's own expressions, folded inside-out
                              as color() returns them);
                              RTW_PRECISION_FP32 (1) = fast mode, single precision
                              traversal and shading, statistical parity only     */
} rtw_render_params;

typedef enum rtw_precision {
    RTW_PRECISION_FP64 = 0,
    RTW_PRECISION_FP32 = 1
} rtw_precision;

typedef struct rtw_stats {
    uint64_t samples;        /* camera samples completed                          */
    uint64_t segments;       /* ray traversals (world hit queries), device-counted */
    uint64_t iterations;     /* wavefront iterations                              */
    uint64_t launches_intersect; /* traversal launches: k_persist (default: one
                                    per pass), k_segment (wavefront, fused
                                    traversal + shading) or k_intersect (split) */
    double ms_total;         /* wall time of the call (hipEvents, whole stream)   */
    double ms_intersect;     /* sum of those launches' durations (if collected)   */
    double ms_shade;         /* sum of k_shade durations (split pair, level 2)    */
    double ms_finalize;      /* per-pixel ordered reduction (not collected)       */
    double bytes_intersect;  /* algorithmic traversal bytes: 68 per segment (ray
                                56 B in, hit 12 B out)             */
} rtw_stats;

/* Number of visible HIP devices (0 if none). */
int rtw_device_count(void);

/* Upload a flattened scene to `device`; returns an opaque handle. */
int rtw_scene_upload(int device, const rtw_scene_desc* desc, void** out_handle);

/* Render the samples selected by `params` and ADD, per pixel, the sum of their
 * radiance (summed in increasing sample order, as RayTracingWeekend.cpp:235-239)
 * into accum_rgb[(j*nx + i)*3 + c].  j = 0 is the bottom row.
 * RTW_ERR_INVALID when the scene has a BVH and moving spheres and `camera`'s
 * shutter [time0, time1] is not inside the desc camera's (the BVH boxes of
 * moving spheres cover that shutter only). */
int rtw_render_accumulate(void* scene_handle, const rtw_camera_desc* camera,
                          const rtw_render_params* params, double* accum_rgb,
                          rtw_stats* out_stats);

/* canvas = min(sqrt(accum / spp), 1) per channel (RayTracingWeekend.cpp:241-244). */
void rtw_finalize_canvas(const double* accum_rgb, int nx, int ny, int spp, double* canvas_rgb);

/* The same on the GPU, for device buffers of the handle's device (stream
 * ordered after the handle's renders; returns when the canvas is written). */
int rtw_finalize_canvas_device(void* scene_handle, const double* accum_rgb_dev, int nx, int ny, int spp,
                               double* canvas_rgb_dev);

/* P3 PPM, rows ny-1..0, int(255.99f * c) (RayTracingWeekend.cpp:252-276). */
int rtw_write_ppm(const char* path, const double* canvas_rgb, int nx, int ny);

void rtw_scene_free(void* scene_handle);

/* ------------------------------------------------------------------ */
/* multi-GPU: one process, one host thread per device, RCCL reduce     */
/* ------------------------------------------------------------------ */

/* The render of rtw_render_accumulate on ngpus scene handles at once -- the
 * reference's triple `_for` (RayTracingWeekend.cpp:211-239) spread over the
 * GPUs of one node.  handles[g] are scenes uploaded (rtw_scene_upload) from
 * the same desc to ngpus DISTINCT devices.  The sample range [spp_begin,
 * spp_begin + spp_count) of `params` is split into ngpus contiguous shards
 * (shard g on handles[g]; SURVEY.md 8(e) sample sharding: every GPU sees the
 * same pixel-cost mix); each device sums its shard per pixel into a zeroed
 * buffer of its own, one grouped RCCL reduce (ncclSum over ncclFloat64)
 * brings the sums to handles[0]'s device, and the result is ADDED into
 * accum_root: a host pointer, or (params->accum_on_device) a device pointer
 * on handles[0]'s device.  Rows (row_begin / row_step) are as in
 * rtw_render_accumulate, on every device.  The reduce reorders the fp64
 * additions of a pixel's sample sums (~1e-16 relative); with ngpus = 1 the
 * result is bit-identical to rtw_render_accumulate.  out_stats: samples,
 * segments, launches and ms_intersect summed over the devices, ms_total = wall
 * time of the call.  The RCCL communicator of a device set is created on
 * first use (ncclCommInitAll) and cached until rtw_release_communicators. */
int rtw_render_multi(int ngpus, void* const* scene_handles, const rtw_camera_desc* camera,
                     const rtw_render_params* params, double* accum_root, rtw_stats* out_stats);

/* Destroy the cached RCCL communicators of rtw_render_multi. */
void rtw_release_communicators(void);

/* ------------------------------------------------------------------ */
/* introspection                                                       */
/* ------------------------------------------------------------------ */
typedef struct rtw_scene_info {
    int32_t device;
    int32_t n_world_runs;     /* world list as the list kernels walk it        */
    int32_t n_ysphere_runs;   /* ... runs scanned by the y-sphere scan         */
    int32_t n_plain_runs;     /* ... other runs of contiguous plain prims      */
    int32_t features;         /* traversal feature bits of the render kernel  */
    int32_t shade_mask;       /* material / texture set bits                  */
    int32_t shade_lds_bytes;  /* shading data staged in LDS per workgroup     */
    int32_t bvh_lds_nodes;    /* BVH nodes staged in LDS per workgroup        */
    char kernel[128];         /* traversal kernel a render of this handle
                                 launches now, e.g. "k_persist_sort<112, 8, true>"
                                 (RTW_MODE / RTW_SORT / RTW_SPLIT respected) */
    char build_id[48];        /* hash of the device code's sources and flags  */
    char kernel_fast[128];    /* traversal kernel of a precision = FP32 render,
                                 e.g. "k_fast<0, false>"                     */
} rtw_scene_info;

int rtw_scene_query(void* scene_handle, rtw_scene_info* out);

/* Hash of the device code's sources and compile flags (rtw_scene_info). */
const char* rtw_build_id(void);

/* ------------------------------------------------------------------ */
/* output on the device                                                */
/* ------------------------------------------------------------------ */

/* The PPM channel bytes of a device canvas, on the GPU:
 * out[(j*nx+i)*3+c] = int(255.99f * canvas[(j*nx+i)*3+c]) with x86's int()
 * (truncation; NaN / out of range -> INT_MIN), RayTracingWeekend.cpp:266-270.
 * canvas_dev, out_dev: device buffers of the handle's device. */
int rtw_quantize_canvas_device(void* scene_handle, const double* canvas_dev, int nx, int ny, int32_t* out_dev);

/* P3 PPM from quantized channels (rtw_quantize_canvas_device, copied to the
 * host): rows ny-1..0, "r g b\n" (RayTracingWeekend.cpp:257-276). */
int rtw_write_ppm_quantized(const char* path, const int32_t* rgb, int nx, int ny);

/* Thread-local message for the last failing call on this thread. */
const char* rtw_last_error(void);

/* Initial minstd_rand state of the stream owned by sample `s` of pixel
 * `pixel` (= j*nx + i):  1 + splitmix64(splitmix64(seed) ^ (s << 32 ^ pixel))
 * mod 2147483646. */
uint32_t rtw_path_seed(uint64_t seed, uint32_t pixel, uint32_t s);

/* ------------------------------------------------------------------ */
/* host-side scene construction (the reference's Scene/scene.h)        */
/* ------------------------------------------------------------------ */

/* Build one of the reference scenes with the host C++ hittable API and
 * flatten it.  names: "cornell_box", "random_balls", "dielectric",
 * "light_sample", "book2_final".  `aspect` = nx/ny (Scene/scene.h ctor arg).
 * `use_bvh` builds BVHs over the world / large groups.  The returned desc is
 * owned by the library; free it with rtw_scene_desc_free. */
int rtw_scene_builtin(const char* name, double aspect, int use_bvh, rtw_scene_desc** out_desc);
void rtw_scene_desc_free(rtw_scene_desc* desc);

/* ABI version this library was built with (RTW_ABI_VERSION). */
int rtw_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* RTW_GPU_H */
