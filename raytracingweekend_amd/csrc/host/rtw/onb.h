// onb.h surface of the host scene API (reference onb.h:5-38): orthonormal
// basis from a normal.  The device builds the same frame with the same
// arithmetic (rtw_device.h onb_from_w; per-rect frames are built once on the
// host by the upload with this very code path's expressions).
#pragma once
#include <cmath>
#include "vec3.h"

class onb {
public:
    onb() {}

    vec3 operator[](int i) const { return axis[i]; }
    vec3 u() const { return axis[0]; }
    vec3 v() const { return axis[1]; }
    vec3 w() const { return axis[2]; }

    vec3 local(double a, double b, double c) const { return a * u() + b * v() + c * w(); }
    vec3 local(const vec3& a) const { return a.x * u() + a.y * v() + a.z * w(); }

    // onb.h:32-38
    void build_from_w(const vec3& n) {
        axis[2] = normalize(n);
        const vec3 a = (std::fabs(w().x) > 0.9) ? vec3(0, 1, 0) : vec3(1, 0, 0);
        axis[1] = normalize(cross(w(), a));
        axis[0] = cross(w(), v());
    }

    vec3 axis[3];
};
