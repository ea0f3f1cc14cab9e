// camera.h surface of the host scene API (reference camera.h:8-73).
// The constructor derives the same basis, in the same fp64 operation order, as
// camera.h:13-34; get_ray (camera.h:36-50) runs on the device (ray-gen).
#pragma once
#include "ray.h"
#include "rtw_gpu.h"

class camera {
public:
    camera() {}
    camera(const vec3& lookfrom, const vec3& lookat, const vec3& vup, double vfov, double aspect, double aperture,
           double focus_dist, double t0, double t1);

    rtw_camera_desc desc() const;

    vec3 origin;
    vec3 lower_left_corner;
    vec3 horizontal;
    vec3 vertical;
    vec3 u, v, w;
    double time0 = 0.0, time1 = 0.0;
    double lens_radius = 0.0;
};
