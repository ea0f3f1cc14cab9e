// vec3.h — host-side fp64 vector of the scene API.
// Same surface as the reference's vec3 (RayTracingWeekend/vec3.h:9-91): x/y/z
// aliased as r/g/b and e[], implicit broadcast from double, component-wise
// operators, dot/cross/normalize/clamp/lerp.  Used only to *describe* scenes
// and build cameras on the host; the device has its own fp64 math.
#pragma once
#include <cmath>
#include <algorithm>

class vec3 {
public:
    union {
        struct {
            union { double x; double r; };
            union { double y; double g; };
            union { double z; double b; };
        };
        double e[3];
    };

    vec3() : e{0.0, 0.0, 0.0} {}
    vec3(double t) : e{t, t, t} {}  // broadcast: lets `2.0 * v` mean vec3(2.0) * v
    vec3(double a, double b_, double c) : e{a, b_, c} {}

    const vec3& operator+() const { return *this; }
    vec3 operator-() const { return vec3(-x, -y, -z); }
    double operator[](int i) const { return e[i]; }
    double& operator[](int i) { return e[i]; }

    vec3& operator+=(const vec3& o) { x += o.x; y += o.y; z += o.z; return *this; }
    vec3& operator-=(const vec3& o) { x -= o.x; y -= o.y; z -= o.z; return *this; }
    vec3& operator*=(const vec3& o) { x *= o.x; y *= o.y; z *= o.z; return *this; }
    vec3& operator/=(const vec3& o) { x /= o.x; y /= o.y; z /= o.z; return *this; }
    vec3& operator*=(double t) { x *= t; y *= t; z *= t; return *this; }
    vec3& operator/=(double t) { x /= t; y /= t; z /= t; return *this; }

    double length_squared() const { return x * x + y * y + z * z; }
    double length() const { return std::sqrt(length_squared()); }
    void make_unit_vector();
};

inline vec3 operator+(vec3 a, const vec3& b) { return a += b; }
inline vec3 operator-(vec3 a, const vec3& b) { return a -= b; }
inline vec3 operator*(vec3 a, const vec3& b) { return a *= b; }
inline vec3 operator/(vec3 a, const vec3& b) { return a /= b; }

inline double dot(const vec3& a, const vec3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

inline vec3 cross(const vec3& a, const vec3& b) {
    const double cx = a.y * b.z - a.z * b.y;
    const double cy = -(a.x * b.z - a.z * b.x);
    const double cz = a.x * b.y - a.y * b.x;
    return vec3(cx, cy, cz);
}

inline vec3 normalize(vec3 v) {
    const double len = v.length();
    v /= len;
    return v;
}

inline void vec3::make_unit_vector() { *this = normalize(*this); }

template <typename T>
inline T clamp(const T& v, const T& lo, const T& hi) { return std::max(std::min(v, hi), lo); }

inline vec3 clamp(const vec3& v, const vec3& lo, const vec3& hi) {
    return vec3(clamp(v.x, lo.x, hi.x), clamp(v.y, lo.y, hi.y), clamp(v.z, lo.z, hi.z));
}

// lerp(from, to, t) = (1-t)*to + t*from — argument roles as in the reference.
inline vec3 lerp(vec3 from, vec3 to, double t) { return (1.0 - t) * to + t * from; }
