// pt_device.h — device-side building blocks of the wavefront path tracer (gfx950).
//
// Everything here is a __device__ restatement of the reference's per-path math with the
// exact IEEE operation order of the reference (glm 0.9.6 semantics, see DESIGN.md "Numerics"),
// so that — compiled with -ffp-contract=off, IEEE division/sqrt and the shared pt_libm trig —
// each path is bit-identical to the CPU oracle's.  Reference citations are file:line in
// /root/reference/src.
//
// Data layout choices (MI355X-first, not the reference's AoS):
//   * scene constants (geoms, BVH nodes, hot triangles) are read through wave-uniform or
//     cache-resident loads; geoms are pre-reduced to the 3 affine rows of each matrix;
//   * a path in flight is 3 x float4 (origin|pixel, direction|bounces, throughput|-),
//     each float4 stream contiguous across paths so one wave moves 1 KiB per instruction.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "pt/pt_libm.h"
#include "pt/scene_structs.h"

typedef float v4f __attribute__((ext_vector_type(4)));   // native vector: one dwordx4 load

#define PT_DEV __device__ __forceinline__

// Measurement hooks: nothing in the product.  Tool builds (-DPT_TOOLS -I../tools) take their
// definitions from tools/pt_tool_hooks.h (section duplicates for VALU attribution, resource probes).
#ifdef PT_TOOLS
#include "pt_tool_hooks.h"
#else
#define PT_HOOK(...) ((void)0)
#endif

namespace ptd {

// utilities.h:13-20
constexpr float PI = 3.1415926535897932384626422832795028841971f;
constexpr float TWO_PI = 6.2831853071795864769252867665590057683943f;
constexpr float PI_OVER_FOUR = 0.78539816339744831f;
constexpr float PI_OVER_TWO = 1.57079632679489662f;
constexpr float INV_PI = 0.31830988618379067154f;
constexpr float BABY_EPSILON = 0.00001f;
constexpr float LARGER_EPSILON = 0.001f;
constexpr float FLT_MAX_ = 3.402823466e+38f;

// ------------------------------------------------------------------------------------------
// float3 with glm 0.9.6 semantics
// ------------------------------------------------------------------------------------------
struct f3 {
    float x, y, z;
};
PT_DEV f3 mk(float x, float y, float z) { return f3{x, y, z}; }
PT_DEV f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
PT_DEV f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
PT_DEV f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
PT_DEV f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
PT_DEV f3 operator*(float s, f3 a) { return f3{s * a.x, s * a.y, s * a.z}; }
PT_DEV f3 operator/(f3 a, float s) { return f3{a.x / s, a.y / s, a.z / s}; }
PT_DEV f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
// compute_dot<tvec3>: (x*y).x + .y + .z, left to right
PT_DEV float dot(f3 a, f3 b) {
    float px = a.x * b.x, py = a.y * b.y, pz = a.z * b.z;
    return px + py + pz;
}
PT_DEV f3 cross(f3 x, f3 y) {
    return f3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
PT_DEV float length(f3 v) { return __builtin_sqrtf(dot(v, v)); }
// normalize = x * (1 / sqrt(dot(x, x)))  (func_geometric.inl:158, func_exponential.inl:150-153)
PT_DEV f3 normalize(f3 v) { return v * (1.0f / __builtin_sqrtf(dot(v, v))); }
// The same normalize, bit for bit, cheaper for a v that is already (nearly) unit length.  When
// d = dot(v, v) lies within NU_ULPS floats of 1, both IEEE roundings (s = sqrt(d), then 1 / s)
// follow from d's bits alone:
//   d = 1 + k 2^-23 (0 <= k):  s = 1 + floor(k/2) 2^-23,  1/s = 1 - floor(k/2) 2^-23
//   d = 1 - k 2^-24 (1 <= k):  s = 1 - ceil(k/2) 2^-24,   1/s = 1 + ceil(ceil(k/2)/2) 2^-23
// (tests/test_unit_normalize.py checks every such d against IEEE sqrtf and division).  Any
// other d, NaN included, takes the IEEE sequence.
constexpr int NU_ULPS = 64;
PT_DEV float inv_sqrt_near1_bits(int k) {   // k = bits(d) - bits(1.0f), |k| <= NU_ULPS
    const int m = k >= 0 ? -2 * (k >> 1) : ((((1 - k) >> 1) + 1) >> 1);
    return __int_as_float(0x3f800000 + m);
}
PT_DEV f3 normalize_unit(f3 v) {
    const float d = dot(v, v);
    const int k = (int)__float_as_uint(d) - 0x3f800000;
    if (k >= -NU_ULPS && k <= NU_ULPS) return v * inv_sqrt_near1_bits(k);
    return v * (1.0f / __builtin_sqrtf(d));
}
PT_DEV f3 reflect(f3 I, f3 N) { return I - (N * dot(N, I)) * 2.0f; }
// glm 0.9.6 refract: NaN (not 0) on total internal reflection
PT_DEV f3 refract(f3 I, f3 N, float eta) {
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    f3 a = eta * I;
    f3 b = (eta * d + __builtin_sqrtf(k)) * N;
    return (a - b) * (float)(k >= 0.0f);
}
PT_DEV float gmin(float x, float y) { return x < y ? x : y; }
PT_DEV float gmax(float x, float y) { return x > y ? x : y; }
PT_DEV float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
PT_DEV f3 mix(f3 x, f3 y, float a) { return x + a * (y - x); }
PT_DEV float comp(f3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

// ------------------------------------------------------------------------------------------
// device scene records
// ------------------------------------------------------------------------------------------
// Affine part of a glm mat4: rows 0..2 of the 4 columns, column-major (m[c*3 + r]).
struct Aff {
    float m[12];
};
// glm mat4 * vec4, keeping the w term even when w == 0 (exact signed-zero behaviour):
// r[i] = (m0[i]*x + m1[i]*y) + (m2[i]*z + m3[i]*w)
PT_DEV f3 xform(const float* m, f3 v, float w) {
    float r0 = (m[0] * v.x + m[3] * v.y) + (m[6] * v.z + m[9] * w);
    float r1 = (m[1] * v.x + m[4] * v.y) + (m[7] * v.z + m[10] * w);
    float r2 = (m[2] * v.x + m[5] * v.y) + (m[8] * v.z + m[11] * w);
    return f3{r0, r1, r2};
}

// 192-byte geom: inverseTransform | transform | invTranspose (affine rows), a conservative
// world-space box (center, half extents incl. a safety margin) used only to SKIP exact tests
// that cannot change the result, + type + material
// The first 112 bytes are what the exact tests read (DevGeomHot): the fused kernel stages only
// that prefix in LDS, so a 44-geom table takes 4.9 KB instead of 8.4 KB of the block's LDS.
struct DevGeomHot {
    float inv[12];
    float fwd[12];
    int32_t type;
    int32_t materialid;
    int32_t away_axis;  // cubes: object axis of the smallest scale for the pre-test's "away" drop
                        // (see away_on_axis); -1: none (spheres, or matrices too large to bound)
    int32_t _pad0;
};
static_assert(sizeof(DevGeomHot) == 112, "DevGeomHot");
struct DevGeom {
    float inv[12];
    float fwd[12];
    int32_t type;
    int32_t materialid;
    int32_t away_axis;
    int32_t _pad0;
    float itr[12];
    float box_lo[3];    // conservative world box (outward-rounded, margin included)
    float box_hi[3];
    int32_t _pad[2];
};
static_assert(sizeof(DevGeom) == 192, "DevGeom");
static_assert(offsetof(DevGeom, itr) == sizeof(DevGeomHot), "DevGeomHot is DevGeom's prefix");
PT_DEV const DevGeomHot& hot(const DevGeom& g) { return *reinterpret_cast<const DevGeomHot*>(&g); }


// Per-geom record of the candidate pre-test (block_intersect / wave_intersect), 48 bytes read
// as 3 float4 with no branch between them: the conservative world box of cull_geom, and the
// inverse-matrix row of away_on_axis's axis (all zero, never "away", for spheres and for cubes
// without one).
struct DevCull {
    float lo[3], hi[3];
    float row[4];          // inv[a], inv[3 + a], inv[6 + a], inv[9 + a]
    int32_t has_row;       // 1: a cube with an away axis (row valid)
    float _pad;
};
static_assert(sizeof(DevCull) == 48, "DevCull");

// The "away" case of geom_test's cube (see the comment there), on ONE object axis a, with
// geom_test's own arithmetic for qo[a] and u[a] (xform row a).  True only when geom_test's slab
// test certainly returns -1: the object-space origin is outside slab a and the direction points away.  u[a]'s w term
// (m[9 + a] * 0 = +-0) is left out: it cannot change a nonzero u[a], and `u > 0` / `u < 0` are
// false for either zero.  geom_test also requires dot(u, u) < inf; the caller guarantees it
// (|rd| components <= 1e3 and |inv| entries <= 1e12, checked on the host).
PT_DEV bool away_on_axis(const DevGeomHot& g, int a, f3 ro, f3 rd) {
    const float* m = g.inv;
    const float qo = (m[a] * ro.x + m[3 + a] * ro.y) + (m[6 + a] * ro.z + m[9 + a] * 1.0f);
    const float u = (m[a] * rd.x + m[3 + a] * rd.y) + m[6 + a] * rd.z;
    return (qo > 0.5f && u > 0.0f) || (qo < -0.5f && u < 0.0f);
}

// 64-byte material: only what shading reads (sceneStructs.h:36-57)
struct DevMaterial {
    float color[3];
    float emittance;
    float hasReflective, hasRefractive, roughness, metallic;
    float ior;
    int32_t hasTexture;
    int32_t textureID;
    int32_t hasBumpMap;
    int32_t bumpID;
    float bumpScale;
    int32_t _pad[2];
};
static_assert(sizeof(DevMaterial) == 64, "DevMaterial");

// 32-byte BVH node: (min.xyz, a) (max.xyz, b); internal: a = left, b = right (<0: none);
// leaf (reference: triCount > 0 && start >= 0): a = start, b = -(triCount + 2)
struct DevNode {
    float4 lo;
    float4 hi;
};

// The two children of one internal BVH node, 64 bytes (VAR_BVH_FAST layout): popping a node
// costs ONE dependent record fetch that holds both child boxes and everything needed to push
// them.  ref >= 0 names the child's own pair record when ref < num_pairs, else the leaf
// ref - num_pairs, whose triangles sit in the 4-slot group hot4[4 * leaf ..]; leaves are numbered
// in the reference's visit order (push left, push right, pop: right subtree first), so a smaller
// hot4 index is an earlier triangle in the reference's DFS.  The cull constants are those of
// cull_threshold for s = max triangle edge below the child (x 1.01), precomputed per child.
struct DevPair {
    float4 l_lo;   // left box min.xyz  | left ref (int bits)
    float4 l_hi;   // left box max.xyz  | left cull constants (A | d, 16 bits each, pack_cull)
    float4 r_lo;   // right box min.xyz | right ref (int bits)
    float4 r_hi;   // right box max.xyz | right cull constants
};

// hot triangle record in leaf order (index k = node.start + i): 3 positions, 48 bytes
struct DevTriHot {
    float4 a;   // v0.xyz, v1.x
    float4 b;   // v1.yz, v2.xy
    float4 c;   // v2.z, triIndex (int bits), -, -
};

// cold triangle data, by reference triangle index (read once for the winner)
struct DevTriCold {
    float n0[3], n1[3], n2[3];   // vertex normals
    float uv0[2], uv1[2], uv2[2];
    float dpdu[3], dpdv[3];
    int32_t materialID;
    int32_t _pad;
};

// ------------------------------------------------------------------------------------------
// RNG: utilhash (intersections.h:13-22) + thrust::minstd_rand + uniform_real_distribution<float>
// ------------------------------------------------------------------------------------------
PT_DEV uint32_t utilhash(uint32_t a) {
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return a;
}
struct Rng {
    uint32_t x;
};
// makeSeededRandomEngine(iter, index, depth), pathtrace.cu:51-56
PT_DEV Rng rng_make(int iter, int index, int depth) {
    uint32_t h = utilhash(0x80000000u | ((uint32_t)depth << 22) | (uint32_t)iter) ^ utilhash((uint32_t)index);
    uint32_t x = h % 2147483647u;
    return Rng{x == 0u ? 1u : x};
}
// x <- 48271 * x mod (2^31 - 1), exact via the Mersenne fold
PT_DEV uint32_t rng_next(Rng& r) {
    uint64_t p = (uint64_t)r.x * 48271ull;
    uint32_t s = (uint32_t)(p & 0x7fffffffull) + (uint32_t)(p >> 31);
    if (s >= 2147483647u) s -= 2147483647u;
    r.x = s;
    return s;
}
// float(x - 1) / (1 + float(max - min)) == float(x - 1) * 2^-31 exactly
PT_DEV float u01(Rng& r) { return (float)(rng_next(r) - 1u) * 4.656612873077392578125e-10f; }

// ------------------------------------------------------------------------------------------
// primitives (intersections.cu)
// ------------------------------------------------------------------------------------------
// getPointOnRay, intersections.h:29-32
PT_DEV f3 point_on_ray(f3 o, f3 d, float t) { return o + (t - .0001f) * normalize_unit(d); }   // d: unit q.direction

// The slab distances' two divisions per axis share one divisor.  AMDGPU's IEEE float division is
// div_scale(b), div_scale(a), y = rcp(b) refined by one Newton step, q = a * y corrected twice by
// its residual (the second through div_fmas), then div_fixup.  Where neither div_scale scales nor
// div_fixup replaces the result, that is exactly div_rcp + div_with_rcp below, so the refined
// reciprocal can be computed once per axis: 3 + 2 x 5 operations instead of 2 x 10, and one
// quarter-rate rcp instead of two.  slab_div_ok certifies that range for all three axes:
// |qd| >= 2^-40 (no zero, denormal or huge-reciprocal divisor) and |qo| <= 2^40, so the numerators
// (+-0.5 - qo) are 0 or of magnitude >= 2^-25 (exact Sterbenz differences near +-0.5) and at most
// 2^40 + 0.5: the exponent gap stays below div_scale's 96, no quotient, reciprocal or residual
// leaves the normal range, and a zero numerator gives the IEEE zero (sign of qd) without the
// fixup.  Anything else (axis-aligned or NaN directions, far origins) takes the division.
PT_DEV bool slab_div_ok(f3 qo, f3 qd) {
    const float dmin = fminf(fminf(__builtin_fabsf(qd.x), __builtin_fabsf(qd.y)), __builtin_fabsf(qd.z));
    const float omax = fmaxf(fmaxf(__builtin_fabsf(qo.x), __builtin_fabsf(qo.y)), __builtin_fabsf(qo.z));
    return dmin >= 0x1p-40f && omax <= 0x1p40f;
}   // (fminf / fmaxf skip a NaN component; its distances are NaN either way, and only compared)
PT_DEV float div_rcp(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
}
PT_DEV float div_with_rcp(float a, float b, float y) {
    const float q0 = a * y;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-b, q0, a), y, q0);
    return __builtin_fmaf(__builtin_fmaf(-b, q1, a), y, q1);
}

// boxIntersectionTest (intersections.cu:3-57) and sphereIntersectionTest (intersections.cu:
// 59-109) as ONE routine: both start by taking the ray to object space (q.origin, normalized
// q.direction) and end with the world hit point's distance, so a wave whose lanes test a mix of
// cubes and spheres runs the shared prologue/epilogue once and diverges only in the middle.
// Every float operation and its order is the reference's.  Returns t (-1 on miss); `seed`
// receives what the winner's normal is derived from: the box's object-space face normal
// (tmin_n), or the sphere's object-space hit point.
PT_DEV float geom_test(const DevGeomHot& g, f3 ro, f3 rd, f3& seed) {
    const f3 qo = xform(g.inv, ro, 1.0f);
    const f3 u = xform(g.inv, rd, 0.0f);
    const float uu = dot(u, u);
    // A cube the ray leaves on some axis (object-space origin outside the slab, direction pointing
    // away: qo > .5, u > 0 or qo < -.5, u < 0) is always a miss below: both slab distances on
    // that axis are negative (|0.5 - qo| >= 2^-24, |qd| <= 1), so tmax < 0.  sign(qd) = sign(u)
    // because qd = u * s with s = 1/sqrt(uu) > 0 finite (uu < inf; u == +-0 underflow still gives
    // -inf distances).  The pre-test's away row (away_on_axis) drops such candidates on that
    // argument.  Round 2 also returned early here on it; the exact tests now see few such cubes
    // and the check's ~12 instructions per test cost more than the skipped tests: cornell -2.1 %,
    // khaslana -0.8 % without it (A/B, round 3), same bits.
    const f3 qd = u * (1.0f / __builtin_sqrtf(uu));      // normalize(u), func_geometric.inl:158
    bool hit;
    float tq;
    f3 s = mk(0.f, 0.f, 0.f);
    if (g.type == PT_CUBE) {
        float tmin = -1e38f, tmax = 1e38f;
        // the slab normals tmin_n / tmax_n are +-1 on one axis and +0 elsewhere (or all +0): carried
        // as a code (axis + 1) * sign, decoded to the same bits at the end -- 2 registers, not 6, at
        // the fused kernel's peak register pressure (this runs inside the exact-test exchange)
        int tmin_c = 0, tmax_c = 0;
        const bool shared_rcp = slab_div_ok(qo, qd);
#pragma unroll
        for (int xyz = 0; xyz < 3; ++xyz) {
            float qdx = comp(qd, xyz), qox = comp(qo, xyz);
            float t1, t2;
            if (shared_rcp) {
                const float y = div_rcp(qdx);
                t1 = div_with_rcp(-0.5f - qox, qdx, y);
                t2 = div_with_rcp(+0.5f - qox, qdx, y);
            } else {
                t1 = (-0.5f - qox) / qdx;
                t2 = (+0.5f - qox) / qdx;
            }
            float ta = gmin(t1, t2);
            float tb = gmax(t1, t2);
            const int nc = t2 < t1 ? xyz + 1 : -(xyz + 1);
            if (ta > 0 && ta > tmin) { tmin = ta; tmin_c = nc; }
            if (tb < tmax) { tmax = tb; tmax_c = nc; }
        }
        hit = tmax >= tmin && tmax > 0;
        if (tmin <= 0) { tmin = tmax; tmin_c = tmax_c; }
        tq = tmin;
        const float sg = tmin_c > 0 ? +1.0f : -1.0f;
        const int ax = (tmin_c < 0 ? -tmin_c : tmin_c) - 1;
        s = mk(ax == 0 ? sg : 0.f, ax == 1 ? sg : 0.f, ax == 2 ? sg : 0.f);
    } else {
        float vDotDirection = dot(qo, qd);
        float radicand = vDotDirection * vDotDirection - (dot(qo, qo) - 0.25f);   // powf(.5, 2) == .25
        float squareRoot = __builtin_sqrtf(radicand);
        float firstTerm = -vDotDirection;
        float t1 = firstTerm + squareRoot;
        float t2 = firstTerm - squareRoot;
        hit = !(radicand < 0) && !(t1 < 0 && t2 < 0);
        tq = (t1 > 0 && t2 > 0) ? gmin(t1, t2) : gmax(t1, t2);
    }
    if (!hit) return -1.0f;
    const f3 objp = point_on_ray(qo, qd, tq);
    const f3 p = xform(g.fwd, objp, 1.0f);
    seed = g.type == PT_CUBE ? s : objp;
    return length(ro - p);
}

// Moller-Trumbore, intersections.cu:112-145, from v0 and the two edges v1 - v0, v2 - v0 (float
// differences: the leaf records hold them precomputed with the same single rounding)
PT_DEV bool tri_test_e(f3 ro, f3 rd, f3 v0, f3 edge1, f3 edge2, float& tOut, float& uOut, float& vOut) {
    f3 pvec = cross(rd, edge2);
    float det = dot(edge1, pvec);
    if (__builtin_fabsf(det) < BABY_EPSILON) return false;
    float invDet = 1.0f / det;
    f3 tvec = ro - v0;
    float u = dot(tvec, pvec) * invDet;
    if (u < 0.0f || u > 1.0f) return false;
    f3 qvec = cross(tvec, edge1);
    float v = dot(rd, qvec) * invDet;
    if (v < 0.0f || (u + v) > 1.0f) return false;
    float t = dot(edge2, qvec) * invDet;
    if (t <= BABY_EPSILON) return false;
    tOut = t; uOut = u; vOut = v;
    return true;
}
PT_DEV bool tri_test(f3 ro, f3 rd, f3 v0, f3 v1, f3 v2, float& tOut, float& uOut, float& vOut) {
    return tri_test_e(ro, rd, v0, v1 - v0, v2 - v0, tOut, uOut, vOut);
}

// aabbIntersectionTest, intersections.cu:237-275
PT_DEV bool aabb_test(float4 lo, float4 hi, f3 ro, f3 rd) {
    float t_min = -FLT_MAX_, t_max = FLT_MAX_;
    const float bmin[3] = {lo.x, lo.y, lo.z};
    const float bmax[3] = {hi.x, hi.y, hi.z};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float dir = comp(rd, i), origin = comp(ro, i);
        if (__builtin_fabsf(dir) < 0.00001f) {
            if (origin < bmin[i] || origin > bmax[i]) return false;
        } else {
            float t1 = (bmin[i] - origin) / dir;
            float t2 = (bmax[i] - origin) / dir;
            if (t1 > t2) { float tmp = t1; t1 = t2; t2 = tmp; }
            if (t1 > t_min) t_min = t1;
            if (t2 < t_max) t_max = t2;
            if (t_min > t_max) return false;
        }
    }
    return t_max >= t_min && t_max > 0.f;
}

// ------------------------------------------------------------------------------------------
// BSDFs (interactions.h / interactions.cu)
// ------------------------------------------------------------------------------------------
struct M3 {
    f3 c0, c1, c2;   // columns
};
PT_DEV f3 mul(const M3& m, f3 v) {
    return f3{m.c0.x * v.x + m.c1.x * v.y + m.c2.x * v.z, m.c0.y * v.x + m.c1.y * v.y + m.c2.y * v.z,
              m.c0.z * v.x + m.c1.z * v.y + m.c2.z * v.z};
}
// transpose(M) * v
PT_DEV f3 mulT(const M3& m, f3 v) {
    return f3{m.c0.x * v.x + m.c0.y * v.y + m.c0.z * v.z, m.c1.x * v.x + m.c1.y * v.y + m.c1.z * v.z,
              m.c2.x * v.x + m.c2.y * v.y + m.c2.z * v.z};
}
// coordinateSystem + LocalToWorld, interactions.h:14-27
// Both branches as one sequence of the same operations (a wave whose lanes take different
// branches ran both: 2 square roots and 6 divisions): the branch picks the operands, one sqrt and
// two divisions follow, and the zero component 0 / s is +0 whenever s > 0 (s = +0 or NaN keeps
// the division, so 0/0 and NaN propagate exactly as in the reference).
PT_DEV M3 local_to_world(f3 n) {
    const bool xb = __builtin_fabsf(n.x) > __builtin_fabsf(n.y);
    const float p = xb ? n.x : n.y;
    const float s = __builtin_sqrtf(p * p + n.z * n.z);   // x: n.x n.x + n.z n.z; y: n.y n.y + n.z n.z
    const float q1 = (xb ? -n.z : n.z) / s;                // x: t.x = -n.z / s;  y: t.y = n.z / s
    const float q2 = (xb ? n.x : -n.y) / s;                // x: t.z = n.x / s;   y: t.z = -n.y / s
    const float z = s > 0.0f ? 0.0f : 0.0f / s;
    const f3 t = xb ? mk(q1, z, q2) : mk(z, q1, q2);
    return M3{t, cross(n, t), n};
}

// glm::vec2(u01(rng), u01(rng)): argument evaluation order is the compiler's (arg_order 0 =
// right-to-left as g++ does, 1 = left-to-right)
PT_DEV void u01_pair(Rng& r, int arg_order, float& x, float& y) {
    float a = u01(r);
    float b = u01(r);
    x = arg_order ? a : b;
    y = arg_order ? b : a;
}

// squareToDiskConcentric + squareToHemisphereCosine, interactions.cu:49-85
PT_DEV f3 hemisphere_cosine(float xi0, float xi1) {
    float x, y;
    if (xi0 == 0.f && xi1 == 0.f) {
        x = 0.f; y = 0.f;
    } else {
        // the two branches as one sequence (lanes of a wave take both at random: two divisions):
        // the branch only picks the operands of the one division
        float a = (2.f * xi0) - 1.f;
        float b = (2.f * xi1) - 1.f;
        const bool ab = (a * a) > (b * b);
        const float radius = 1.f * (ab ? a : b);
        const float r = (ab ? b : a) / (ab ? a : b);
        const float qr = PI_OVER_FOUR * r;
        const float theta = ab ? qr : PI_OVER_TWO - qr;
        float s, c;
        pt_sincosf(theta, &s, &c);
        PT_HOOK(DUP_SINCOS, theta, xi1);
        x = radius * c;
        y = radius * s;
    }
    float z = __builtin_sqrtf(gmax(0.f, 1.0f - (x * x) - (y * y)));
    return mk(x, y, z);
}

// x / PI correctly rounded, for x = 0 or x in [2^-24, 1] -- the cosine sample's z (the square root
// of (1 - x^2) - y^2 with x, y in [-1, 1]: 0 or at least 2^-24): one product with RN(1 / PI) and
// one residual correction (Markstein), 3 operations instead of the division's ~10 with a
// quarter-rate reciprocal.  tools/check_div_by_pi.c checks it against IEEE division for every
// float from 0 to 1 (and every non-negative normal float): identical bits; tests/test_libm.py runs it.
PT_DEV float div_by_pi(float x) {
    const float INV_PI_RN = 0.318309873342514038085938f;   // RN(1 / PI) = 0x1.45f306p-2
    const float q = x * INV_PI_RN;
    const float r = __builtin_fmaf(-PI, q, x);
    return __builtin_fmaf(r, INV_PI_RN, q);
}
// sampleFDiffuse, interactions.cu:92-108 (returns bsdf; pdf, wiW out)
PT_DEV f3 sample_diffuse(f3 albedo, f3 normal, f3& wiW, float& pdf, Rng& rng, int arg_order) {
    float xi0, xi1;
    u01_pair(rng, arg_order, xi0, xi1);
    f3 wi = hemisphere_cosine(xi0, xi1);
    M3 ws = local_to_world(normal);
    wiW = normalize_unit(mul(ws, wi));
    pdf = div_by_pi(wi.z);
    return albedo * INV_PI;
}

// sampleFSpecularTrans, interactions.cu:146-168
PT_DEV f3 sample_spec_trans(f3 albedo, f3 normal, f3 wo, float IOR, f3& wiW) {
    bool entering = dot(wo, normal) < 0.0f;
    float eta = entering ? (1.0f / IOR) : IOR;
    f3 outNormal = entering ? normal : -normal;
    wiW = refract(normalize_unit(wo), normalize_unit(outNormal), eta);
    if (length(wiW) < BABY_EPSILON) {
        wiW = reflect(wo, normal);
        return mk(0.f, 0.f, 0.f);
    }
    return albedo;
}

// FresnelDielectricEval, interactions.cu:173-194
PT_DEV float fresnel_dielectric(float cosThetaI, float IOR) {
    float etaI = 1.f, etaT = IOR;
    cosThetaI = gclamp(cosThetaI, -1.f, 1.f);
    if (cosThetaI > 0.f) { float tmp = etaI; etaI = etaT; etaT = tmp; }
    cosThetaI = __builtin_fabsf(cosThetaI);
    float sinThetaI = __builtin_sqrtf(gmax(0.f, 1.f - cosThetaI * cosThetaI));
    float sinThetaT = etaI / etaT * sinThetaI;
    float cosThetaT = __builtin_sqrtf(gmax(0.f, 1.f - sinThetaT * sinThetaT));
    float Rparl = ((etaT * cosThetaI) - (etaI * cosThetaT)) / ((etaT * cosThetaI) + (etaI * cosThetaT));
    float Rperp = ((etaI * cosThetaI) - (etaT * cosThetaT)) / ((etaI * cosThetaI) + (etaT * cosThetaT));
    return (Rparl * Rparl + Rperp * Rperp) * 0.5f;
}

// FresnelSchlick, interactions.cu:197-201
PT_DEV f3 fresnel_schlick(float cosTheta, f3 F0) {
    float p = pt_pow5f(1.0f - cosTheta);
    return mk(F0.x + (1.0f - F0.x) * p, F0.y + (1.0f - F0.y) * p, F0.z + (1.0f - F0.z) * p);
}

// sampleFGlass, interactions.cu:204-235
PT_DEV f3 sample_glass(f3 albedo, f3 normal, f3 wo, float IOR, f3& wiW, Rng& rng) {
    float random = u01(rng);
    float fresnel = fresnel_dielectric(dot(wo, normal), IOR);
    if (random < fresnel) {
        wiW = reflect(wo, normal);
        return albedo;
    }
    f3 T = sample_spec_trans(albedo, normal, wo, IOR, wiW);
    if (length(wiW) < BABY_EPSILON) {
        wiW = reflect(wo, normal);
        return albedo;
    }
    return T;
}

// microfacet trig helpers, interactions.h:106-167
PT_DEV float cos2t(f3 w) { return w.z * w.z; }
PT_DEV float sin2t(f3 w) { return gmax(0.f, 1.f - cos2t(w)); }
PT_DEV float tan2t(f3 w) { return sin2t(w) / cos2t(w); }
PT_DEV float sint(f3 w) { return __builtin_sqrtf(sin2t(w)); }
PT_DEV float tant(f3 w) { return sint(w) / w.z; }
PT_DEV float cosphi(f3 w) { float s = sint(w); return (s == 0) ? 0.f : gclamp(w.x / s, -1.f, 1.f); }
PT_DEV float sinphi(f3 w) { float s = sint(w); return (s == 0) ? 0.f : gclamp(w.y / s, -1.f, 1.f); }

// sampleWH, interactions.cu:238-264
PT_DEV f3 sample_wh(f3 wo, float roughness, Rng& rng, int arg_order) {
    float xi0, xi1;
    u01_pair(rng, arg_order, xi0, xi1);
    float phi = TWO_PI * xi1;
    float tanTheta2 = roughness * roughness * xi0 / (1.0f - xi0);
    float cosTheta = 1.0f / __builtin_sqrtf(1.0f + tanTheta2);
    float sinTheta = __builtin_sqrtf(gmax(0.f, 1.f - cosTheta * cosTheta));
    float s, c;
    pt_sincosf(phi, &s, &c);
    f3 wh = mk(sinTheta * c, sinTheta * s, cosTheta);
    if (!(wo.z * wh.z > 0)) wh = -wh;
    return wh;
}
// TrowbridgeReitzD, interactions.cu:266-283
PT_DEV float tr_d(f3 wh, float r) {
    float tan2Theta = tan2t(wh);
    if (__builtin_isinf(tan2Theta)) return 0.f;
    float cos4Theta = cos2t(wh) * cos2t(wh);
    float cp = cosphi(wh), sp = sinphi(wh);
    float e = ((cp * cp) / (r * r) + (sp * sp) / (r * r)) * tan2Theta;
    return 1.0f / (PI * r * r * cos4Theta * (1.0f + e) * (1.0f + e));
}
// lambda, interactions.cu:285-297
PT_DEV float tr_lambda(f3 w, float r) {
    float absTanTheta = __builtin_fabsf(tant(w));
    if (__builtin_isinf(absTanTheta)) return 0.f;
    float a = (r * absTanTheta) * (r * absTanTheta);
    return (-1.0f + __builtin_sqrtf(1.f + a)) / 2.0f;
}
// fMicrofacetRefl, interactions.cu:314-348
PT_DEV f3 f_microfacet(f3 albedo, f3 wo, f3 wi, float r, float metallic) {
    float cosThetaO = __builtin_fabsf(wo.z);
    float cosThetaI = __builtin_fabsf(wi.z);
    f3 wh = wi + wo;
    if (cosThetaI == 0 || cosThetaO == 0) return mk(0.f, 0.f, 0.f);
    if (wh.x == 0 && wh.y == 0 && wh.z == 0) return mk(0.f, 0.f, 0.f);
    wh = normalize(wh);
    f3 F0 = mix(mk(0.04f, 0.04f, 0.04f), albedo, metallic);
    f3 F = fresnel_schlick(dot(wi, wh), F0);
    float D = tr_d(wh, r);
    float G = 1.0f / (1.0f + tr_lambda(wo, r) + tr_lambda(wi, r));
    return (F * (D * G)) / (4.0f * cosThetaI * cosThetaO);
}
// sampleFMicrofacetRefl, interactions.cu:350-380
PT_DEV f3 sample_microfacet(f3 albedo, f3 normal, f3 wo, float r, float metallic, f3& wiW, float& pdf,
                            Rng& rng, int arg_order) {
    M3 l2w = local_to_world(normal);
    f3 wo_local = mulT(l2w, wo);
    f3 wh_local = sample_wh(wo_local, r, rng, arg_order);
    if (wh_local.z < 0.0f) wh_local = -wh_local;
    f3 wi_local = reflect(-wo_local, wh_local);
    wiW = normalize_unit(mul(l2w, wi_local));
    float dotWO_WH = gmax(dot(wo_local, wh_local), 1e-6f);
    pdf = (tr_d(wh_local, r) * __builtin_fabsf(wh_local.z)) / (4.0f * dotWO_WH);
    return f_microfacet(albedo, wo_local, wi_local, r, metallic);
}
// sampleFCookTorrance, interactions.cu:383-435
PT_DEV f3 sample_cook_torrance(f3 albedo, f3 normal, f3 woW, float r, float metallic, f3& wiW, float& out_pdf,
                               Rng& rng, int arg_order) {
    f3 F0 = mix(mk(0.04f, 0.04f, 0.04f), albedo, metallic);
    float cosTheta = gclamp(dot(normal, woW), 0.0f, 1.0f);
    f3 F = fresnel_schlick(cosTheta, F0);
    float Fprob = gclamp(gmax(F.x, gmax(F.y, F.z)), 0.0f, 1.0f);
    float choose = u01(rng);
    f3 bsdf;
    float pdf_spec = 0.0f, pdf_diff = 0.0f;
    bool spec = choose < Fprob;
    if (spec) bsdf = sample_microfacet(albedo, normal, woW, r, metallic, wiW, pdf_spec, rng, arg_order);
    else bsdf = sample_diffuse(albedo, normal, wiW, pdf_diff, rng, arg_order);
    out_pdf = Fprob * pdf_spec + (1.0f - Fprob) * pdf_diff;
    return spec ? bsdf * F : bsdf * (mk(1.0f, 1.0f, 1.0f) - F);
}

// ------------------------------------------------------------------------------------------
// scatterRay (interactions.cu:438-542) on a path held in registers
// ------------------------------------------------------------------------------------------
struct PathReg {
    f3 o, d, c;
    int pix;
    int rb;
    int slot;       // frame of the pass this path belongs to (iteration = pass iteration + slot)
};

PT_DEV void scatter(PathReg& p, f3 intersect, f3 normal, const DevMaterial& m, f3 mcolor, Rng& rng, int arg_order) {
    f3 wiW = mk(0.f, 0.f, 0.f), bsdf;
    float pdf = 1.0f;
    if (m.hasRefractive > 0.0f && m.hasReflective > 0.0f) {          // Glass
        bsdf = sample_glass(mcolor, normal, p.d, m.ior, wiW, rng);
        p.d = normalize_unit(wiW);
        p.o = intersect + p.d * LARGER_EPSILON;
        p.c = p.c * bsdf;
    } else if (m.hasReflective > 0.0f) {                              // Mirror
        wiW = reflect(p.d, normal);
        p.d = normalize_unit(wiW);
        p.o = intersect + normal * BABY_EPSILON;
        p.c = p.c * mcolor;
    } else if (m.hasRefractive > 0.0f) {                              // Transmissive
        bsdf = sample_spec_trans(mcolor, normal, p.d, m.ior, wiW);
        p.d = normalize_unit(wiW);
        p.o = intersect + p.d * LARGER_EPSILON;
        p.c = p.c * bsdf;
    } else if (m.roughness >= 0.0f && m.metallic >= 0.0f) {           // Microfacet
        f3 woW = -normalize_unit(p.d);
        bsdf = sample_cook_torrance(mcolor, normal, woW, m.roughness, m.metallic, wiW, pdf, rng, arg_order);
        p.d = normalize_unit(wiW);
        p.o = intersect + p.d * LARGER_EPSILON;
        float cosTheta = gmax(0.0f, dot(normal, wiW));
        if (pdf > 0.0f) p.c = p.c * ((bsdf * cosTheta) / pdf);
    } else {                                                          // Diffuse
        bsdf = sample_diffuse(mcolor, normal, wiW, pdf, rng, arg_order);
        p.d = normalize_unit(wiW);
        p.o = intersect + normal * BABY_EPSILON;
        float cosTheta = gmax(0.0f, dot(normal, wiW));
        p.c = p.c * ((bsdf * cosTheta) / pdf);
    }
    p.rb -= 1;
}

}  // namespace ptd
