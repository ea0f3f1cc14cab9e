// camera.h surface of the host scene API (reference camera.h:8-73).
// The constructor derives the same basis, in the same fp64 operation order, as
// camera.h:13-34; get_ray (camera.h:36-50) makes the thin-lens ray on the
// host with the reference's draws (renders make it on the device, ray-gen in
// rtw_kernels.hip, from the same formulas).
#pragma once
#include <random>
#include "ray.h"
#include "rtw_gpu.h"
#include "utility.h"

class camera {
public:
    camera() {}
    camera(const vec3& lookfrom, const vec3& lookat, const vec3& vup, double vfov, double aspect, double aperture,
           double focus_dist, double t0, double t1);

    rtw_camera_desc desc() const;

    // camera.h:36-50: a point of the lens (radius lens_radius) towards the
    // image-plane point (s, t), normalised direction, a time in [time0, time1)
    ray get_ray(double s, double t) {
        const vec3 rd = lens_radius * random_in_unit_disk();
        const vec3 offset = u * rd.x + v * rd.y;
        const double time = time0 + uniform(timeEngine) * (time1 - time0);
        const vec3 dir = lower_left_corner + s * horizontal + t * vertical - origin - offset;
        return ray(origin + offset, normalize(dir), time);
    }

    vec3 origin;
    vec3 lower_left_corner;
    vec3 horizontal;
    vec3 vertical;
    vec3 u, v, w;
    double time0 = 0.0, time1 = 0.0;
    double lens_radius = 0.0;

private:
    // camera.h:61-69: rejection sampling of the unit disk; g++ evaluates
    // vec3(U, U, 0) right to left, so the first draw of a try is y
    vec3 random_in_unit_disk() {
        vec3 p;
        do {
            const double py = uniform(rayEngine);
            const double px = uniform(rayEngine);
            p = 2.0 * vec3(px, py, 0) - vec3(1, 1, 0);
        } while (dot(p, p) >= 1.0);
        return p;
    }
    std::uniform_real_distribution<double> uniform;
    rtw::engine rayEngine;
    rtw::engine timeEngine;
};
