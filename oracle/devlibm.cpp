// oracle/devlibm.cpp — TEST INFRASTRUCTURE ONLY.  The device's libm
// replacements (raytracingweekend_amd/csrc/rtw_math.h, compiled here for the
// host with the same unfused fp64 arithmetic) behind the C names the oracle's
// RTW_ORACLE_DEVLIBM build calls: librtw_oracle_devlibm.so is the checker of
// the strict-radiance GPU build (tests/test_gpu_strict.py), where every
// operation but these functions is the reference's.  Each mirrors the device
// call site, including the device's fallback outside the fast ranges.
#include <cmath>
#include "rtw_math.h"

extern "C" {
// the azimuth 2*pi*r1 of random_cosine_direction / random_to_sphere
// (utility.h:54-81; device: sincos_azimuth at rtw_device.h's samplers)
double rtw_devlibm_cos(double x) {
    double s, c;
    rtwd::sincos_azimuth(x, s, c);
    return c;
}
double rtw_devlibm_sin(double x) {
    double s, c;
    rtwd::sincos_azimuth(x, s, c);
    return s;
}
// texture sines (texture.h:45, :66; device: sin_tex)
double rtw_devlibm_sin_tex(double x) { return rtwd::sin_wide_ok(x) ? rtwd::sin_wide(x) : std::sin(x); }
// the media's free flight (hittable.h:450; device: log_dev)
double rtw_devlibm_log(double x) {
    return rtwd::log_pos_ok(x) ? rtwd::log_pos(x, [](int i) { return rtwd::kLogCoef[i]; }) : std::log(x);
}
// schlick's pow(x, 5) (material.h:44-49; device: schlick_r0)
double rtw_devlibm_pow5(double x) { return rtwd::pow5(x); }
}
