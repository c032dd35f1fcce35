// hmath.h — host-side float math with glm 0.9.6 operation order (scene ingest only).
// Compiled with -ffp-contract=off so every product/sum is rounded where glm rounds it.
#pragma once

#include <cmath>

#include "pt/scene_structs.h"

namespace pth {

using v3 = pt_vec3;
using v2 = pt_vec2;
using v4 = pt_vec4;

inline v3 V3(float x, float y, float z) { return v3{x, y, z}; }
inline v4 V4(float x, float y, float z, float w) { return v4{x, y, z, w}; }
inline v3 operator+(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline v3 operator-(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline v3 operator-(v3 a) { return V3(-a.x, -a.y, -a.z); }
inline v3 operator*(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
inline v3 operator/(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
inline v2 operator-(v2 a, v2 b) { return v2{a.x - b.x, a.y - b.y}; }
inline v4 operator+(v4 a, v4 b) { return V4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
inline v4 operator-(v4 a, v4 b) { return V4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
inline v4 operator*(v4 a, v4 b) { return V4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
inline v4 operator*(v4 a, float s) { return V4(a.x * s, a.y * s, a.z * s, a.w * s); }
inline float dot(v3 a, v3 b) { float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return x + y + z; }
inline v3 cross(v3 x, v3 y) { return V3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y); }
inline float length(v3 v) { return std::sqrt(dot(v, v)); }
inline v3 normalize(v3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }
inline float gmin(float x, float y) { return x < y ? x : y; }
inline float gmax(float x, float y) { return x > y ? x : y; }
inline v3 vmin(v3 a, v3 b) { return V3(gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)); }
inline v3 vmax(v3 a, v3 b) { return V3(gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)); }
inline float comp(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

inline v4 col(const pt_mat4& m, int c) { return V4(m.m[c][0], m.m[c][1], m.m[c][2], m.m[c][3]); }
inline void setcol(pt_mat4& m, int c, v4 v) { m.m[c][0] = v.x; m.m[c][1] = v.y; m.m[c][2] = v.z; m.m[c][3] = v.w; }
inline pt_mat4 identity() {
    pt_mat4 m{};
    m.m[0][0] = m.m[1][1] = m.m[2][2] = m.m[3][3] = 1.0f;
    return m;
}
// mat4 * vec4: (m0*x + m1*y) + (m2*z + m3*w)  (type_mat4x4.inl)
inline v4 mul(const pt_mat4& m, v4 v) {
    return (col(m, 0) * v.x + col(m, 1) * v.y) + (col(m, 2) * v.z + col(m, 3) * v.w);
}
// mat4 * mat4: ((A0*b0 + A1*b1) + A2*b2) + A3*b3 per column
inline pt_mat4 mul(const pt_mat4& A, const pt_mat4& B) {
    pt_mat4 r;
    for (int j = 0; j < 4; ++j)
        setcol(r, j, col(A, 0) * B.m[j][0] + col(A, 1) * B.m[j][1] + col(A, 2) * B.m[j][2] + col(A, 3) * B.m[j][3]);
    return r;
}

}  // namespace pth
