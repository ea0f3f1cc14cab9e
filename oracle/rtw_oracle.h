/*
 * rtw_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference renderer (silvesthu/RayTracingWeekend)
 * over the flattened scene of include/rtw_gpu.h.  Used by tests/ (parity
 * checker), __graft_entry__.smoke() and bench.py's cpu_baseline leg — never by
 * the product library.  It is recursive like the reference's color()
 * (RayTracingWeekend.cpp:45-160) and walks the world list twice like
 * hittable_list::hit (hittable_list.h:11-37), so its canvases are bit-identical
 * to those of the reference's own code driven by oracle/ref_harness.cpp
 * (pinned by tests/test_oracle.py against tests/golden/).
 */
#ifndef RTW_ORACLE_H
#define RTW_ORACLE_H
#include <stdint.h>
#include "rtw_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Render pixels of rows [row_begin, row_begin+row_count) (all columns) with
 * samples [spp_begin, spp_begin+spp_count); writes, per pixel, the radiance
 * SUM in increasing sample order to sums[(j*nx+i)*3+c] (other rows untouched).
 * threads <= 0: all OpenMP threads.  Returns 0, or -1 on a malformed scene. */
int rtw_oracle_render(const rtw_scene_desc* scene, const rtw_camera_desc* cam, int nx, int ny, int row_begin,
                      int row_count, int spp_begin, int spp_count, int max_depth, uint64_t seed, int threads,
                      double* sums, uint64_t* segments);

/* The same over rows row_begin + k*row_stride, k in [0, row_count): one
 * multithreaded call over a strided sample of the image (bench.py). */
int rtw_oracle_render_strided(const rtw_scene_desc* scene, const rtw_camera_desc* cam, int nx, int ny,
                              int row_begin, int row_stride, int row_count, int spp_begin, int spp_count,
                              int max_depth, uint64_t seed, int threads, double* sums, uint64_t* segments);

/* One path, with its segments recorded (origin, direction, time, hit t,
 * hit flag) for debugging parity: at most max_seg rows of 8 doubles. */
int rtw_oracle_trace(const rtw_scene_desc* scene, const rtw_camera_desc* cam, int nx, int ny, int i, int j, int s,
                     int max_depth, uint64_t seed, double* radiance3, double* seg_rows, int max_seg);

/* Known-answer helpers */
double rtw_oracle_canonical(uint32_t* state);          /* one generate_canonical<double,53> */
double rtw_oracle_noise(const rtw_scene_desc* scene, const double p[3]);
double rtw_oracle_turb(const rtw_scene_desc* scene, const double p[3]);
uint32_t rtw_oracle_path_seed(uint64_t seed, uint32_t pixel, uint32_t s);

#ifdef __cplusplus
}
#endif
#endif
