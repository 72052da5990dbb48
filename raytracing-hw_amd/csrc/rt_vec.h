// rt_vec.h — float vector arithmetic with the reference's exact evaluation order.
//
// Every helper restates one operator of src/utils/vector.h (packed vector3f/vector4f,
// component-wise, left to right, no FMA) so that host (g++) and device (hipcc, built with
// -ffp-contract=off) produce the reference's bits.  Notable orders kept on purpose:
//   dot/length accumulate from 0.f (vector.h:146-152, :365-370), so a -0 product becomes +0;
//   normal() multiplies by the reciprocal (vector.h:170-174), it does not divide;
//   a - b is a + (-b) (vector.h:326-328);  std::min/std::max select as (b < a ? b : a) /
//   (a < b ? b : a), which fixes the NaN behaviour.
#pragma once
#include <cmath>
#include "rt_libm.h"

namespace rtv {

struct V2 { float x, y; };
struct V3 { float x, y, z; };
struct V4 { float x, y, z, w; };

RT_HD float smin(float a, float b) { return (b < a) ? b : a; }   // std::min
RT_HD float smax(float a, float b) { return (a < b) ? b : a; }   // std::max

RT_HD float at(const V3 &v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
RT_HD void set(V3 &v, int i, float f) { if (i == 0) v.x = f; else if (i == 1) v.y = f; else v.z = f; }

RT_HD V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_HD V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
RT_HD V3 sub(V3 a, V3 b) { return add(a, neg(b)); }
RT_HD V3 mul(V3 v, float t) { return {v.x * t, v.y * t, v.z * t}; }   // vector3f * float and float * vector3f
RT_HD V3 mulv(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
RT_HD V3 divv(V3 a, V3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
RT_HD V3 addf(V3 v, float t) { return {v.x + t, v.y + t, v.z + t}; } // vector3f::add
RT_HD V3 vmin(V3 a, V3 b) { return {smin(a.x, b.x), smin(a.y, b.y), smin(a.z, b.z)}; }
RT_HD V3 vmax(V3 a, V3 b) { return {smax(a.x, b.x), smax(a.y, b.y), smax(a.z, b.z)}; }
RT_HD bool is_zero(V3 v) { return v.x == 0 && v.y == 0 && v.z == 0; }

RT_HD float dot(V3 a, V3 b) {
    float s = 0.f;
    s += a.x * b.x;
    s += a.y * b.y;
    s += a.z * b.z;
    return s;
}
RT_HD V3 cross(V3 a, V3 b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
RT_HD float length(V3 v) {
    float m = 0.f;
    m += v.x * v.x;
    m += v.y * v.y;
    m += v.z * v.z;
    return sqrtf(m);
}
RT_HD float length(V4 v) {
    float m = 0.f;
    m += v.x * v.x;
    m += v.y * v.y;
    m += v.z * v.z;
    m += v.w * v.w;
    return sqrtf(m);
}
RT_HD float length(V2 v) {
    float m = 0.f;
    m += v.x * v.x;
    m += v.y * v.y;
    return sqrtf(m);
}
RT_HD V3 normal(V3 v) {
    float m = length(v);
    m = 1.f / m;
    return {v.x * m, v.y * m, v.z * m};
}
RT_HD V4 normal(V4 v) {
    float m = length(v);
    m = 1.f / m;
    return {v.x * m, v.y * m, v.z * m, v.w * m};
}
RT_HD V3 reduce(V4 v) { return {v.x, v.y, v.z}; }
RT_HD V4 conj(V4 q) { return {-q.x, -q.y, -q.z, q.w}; }        // vector.h:221 operator*(vector4f)

// vector.h:380-387
RT_HD V3 rotate(V3 v, V4 q) {
    V3 u = reduce(q);
    float s = q.w;
    V3 a = mul(u, 2.f * dot(u, v));
    V3 b = mul(v, s * s - dot(u, u));
    V3 c = mul(cross(u, v), 2.f * s);
    return add(add(a, b), c);
}
// vector.h:454-458
RT_HD V4 quat_from_two_vectors(V3 u, V3 v) {
    V3 w = cross(u, v);
    return normal(V4{w.x, w.y, w.z, 1.f + dot(u, v)});
}

}  // namespace rtv
