/*
 * pt_oracle.c — plain-C (C11) restatement of the reference hot path.  TEST INFRASTRUCTURE.
 * See pt_oracle.h for what it may be used for and how far parity is pinned.
 *
 * Written for literal fidelity, not speed: every float expression keeps the reference's
 * operation order (glm 0.9.6 semantics restated below), compiled with -ffp-contract=off.
 * Each function cites the reference file:line it restates (paths relative to the
 * reference repository root).
 */
#include "pt_oracle.h"
#include "pt/pt_libm.h"
#include "pt/pt_texture.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* utilities.h:13-20 */
#define PI                3.1415926535897932384626422832795028841971f
#define TWO_PI            6.2831853071795864769252867665590057683943f
#define PI_OVER_FOUR      0.78539816339744831f
#define PI_OVER_TWO       1.57079632679489662f
#define INV_PI            0.31830988618379067154f
#define BABY_EPSILON      0.00001f
#define LARGER_EPSILON    0.001f

typedef pt_vec3 v3;
typedef pt_vec2 v2;
typedef pt_vec4 v4;

/* ------------------------------------------------------------------------------------------ */
/* glm 0.9.6 semantics (external/include/glm/detail/func_geometric.inl, func_common.inl,       */
/* type_vec3.inl, type_mat4x4.inl, type_mat3x3.inl)                                            */
/* ------------------------------------------------------------------------------------------ */
static inline v3 V3(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline v2 V2(float x, float y) { v2 r; r.x = x; r.y = y; return r; }
static inline v4 V4(float x, float y, float z, float w) { v4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
static inline v3 add3(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul3(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls3(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }   /* vec*s and s*vec */
static inline v3 divs3(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 div3(v3 a, v3 b) { return V3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline v3 neg3(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline v2 add2(v2 a, v2 b) { return V2(a.x + b.x, a.y + b.y); }
static inline v2 sub2(v2 a, v2 b) { return V2(a.x - b.x, a.y - b.y); }
static inline v2 muls2(v2 a, float s) { return V2(a.x * s, a.y * s); }
/* compute_dot<tvec3>: tmp = x*y; return tmp.x + tmp.y + tmp.z  (func_geometric.inl) */
static inline float dot3(v3 a, v3 b) { v3 t = mul3(a, b); return t.x + t.y + t.z; }
static inline v3 cross3(v3 x, v3 y) {
    return V3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
static inline float length3(v3 v) { return sqrtf(dot3(v, v)); }
/* normalize = x * inversesqrt(dot(x,x)), inversesqrt = 1/sqrt (func_exponential.inl:150-153) */
static inline v3 normalize3(v3 v) { return muls3(v, 1.0f / sqrtf(dot3(v, v))); }
/* reflect: I - N * dot(N, I) * 2 */
static inline v3 reflect3(v3 I, v3 N) { return sub3(I, muls3(muls3(N, dot3(N, I)), 2.0f)); }
/* refract: NaN (not zero) on total internal reflection because sqrt(k<0)*0 = NaN */
static inline v3 refract3(v3 I, v3 N, float eta) {
    float d = dot3(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    v3 a = muls3(I, eta);
    v3 b = muls3(N, eta * d + sqrtf(k));
    return muls3(sub3(a, b), (float)(k >= 0.0f));
}
static inline float gmin(float x, float y) { return x < y ? x : y; }   /* func_common.inl:409-414 */
static inline float gmax(float x, float y) { return x > y ? x : y; }   /* func_common.inl:430-435 */
static inline float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
static inline v3 vmin3(v3 a, v3 b) { return V3(gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)); }
static inline v3 vmax3(v3 a, v3 b) { return V3(gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)); }
/* mix(x, y, a) = x + a * (y - x) */
static inline v3 mix3(v3 x, v3 y, float a) { return add3(x, muls3(sub3(y, x), a)); }
static inline float comp3(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
static inline void setcomp3(v3* v, int i, float f) { if (i == 0) v->x = f; else if (i == 1) v->y = f; else v->z = f; }

/* mat4 * vec4 (type_mat4x4.inl:592-626): (m0*v0 + m1*v1) + (m2*v2 + m3*v3) per row */
static inline v4 mat4_mul_v4(const pt_mat4* m, v4 v) {
    float r[4];
    for (int i = 0; i < 4; ++i) {
        float a0 = m->m[0][i] * v.x + m->m[1][i] * v.y;
        float a1 = m->m[2][i] * v.z + m->m[3][i] * v.w;
        r[i] = a0 + a1;
    }
    return V4(r[0], r[1], r[2], r[3]);
}
/* intersections.h:37-40 multiplyMV */
static inline v3 multiplyMV(const pt_mat4* m, v4 v) { v4 r = mat4_mul_v4(m, v); return V3(r.x, r.y, r.z); }

/* mat3 with columns c0,c1,c2;  mat3 * v (type_mat3x3.inl:487-493) */
typedef struct { v3 c0, c1, c2; } mat3c;
static inline v3 mat3_mul_v3(const mat3c* m, v3 v) {
    return V3(m->c0.x * v.x + m->c1.x * v.y + m->c2.x * v.z,
              m->c0.y * v.x + m->c1.y * v.y + m->c2.y * v.z,
              m->c0.z * v.x + m->c1.z * v.y + m->c2.z * v.z);
}
static inline mat3c mat3_transpose(const mat3c* m) {
    mat3c t;
    t.c0 = V3(m->c0.x, m->c1.x, m->c2.x);
    t.c1 = V3(m->c0.y, m->c1.y, m->c2.y);
    t.c2 = V3(m->c0.z, m->c1.z, m->c2.z);
    return t;
}

void or_glm_normalize(const pt_vec3* v, pt_vec3* out) { *out = normalize3(*v); }
void or_glm_reflect(const pt_vec3* i, const pt_vec3* n, pt_vec3* out) { *out = reflect3(*i, *n); }
void or_glm_refract(const pt_vec3* i, const pt_vec3* n, float eta, pt_vec3* out) { *out = refract3(*i, *n, eta); }

/* ------------------------------------------------------------------------------------------ */
/* transcendental dispatch: glibc (trig_mode 0) or pt_libm (trig_mode 1)                      */
/* ------------------------------------------------------------------------------------------ */
static inline float t_cos(const or_options* o, float x) { return o->trig_mode ? pt_cosf(x) : cosf(x); }
static inline float t_sin(const or_options* o, float x) { return o->trig_mode ? pt_sinf(x) : sinf(x); }
static inline float t_pow5(const or_options* o, float x) { return o->trig_mode ? pt_pow5f(x) : powf(x, 5.0f); }

/* ------------------------------------------------------------------------------------------ */
/* RNG                                                                                         */
/* ------------------------------------------------------------------------------------------ */
/* intersections.h:13-22 */
uint32_t or_utilhash(uint32_t a) {
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return a;
}

/* thrust::minstd_rand = linear_congruential_engine<uint32_t, 48271, 0, 2147483647>
 * (rocThrust random/detail/linear_congruential_engine.inl seed(): x = s mod m, 0 -> 1). */
typedef struct { uint32_t x; } or_rng;

/* pathtrace.cu:51-56 makeSeededRandomEngine(iter, index, depth) */
static or_rng rng_make(int32_t iter, int32_t index, int32_t depth) {
    uint32_t key = 0x80000000u | ((uint32_t)depth << 22) | (uint32_t)iter;
    uint32_t h = or_utilhash(key) ^ or_utilhash((uint32_t)index);
    or_rng r;
    r.x = h % 2147483647u;
    if (r.x == 0u) r.x = 1u;
    return r;
}
static inline uint32_t rng_next(or_rng* r) {
    r->x = (uint32_t)(((uint64_t)r->x * 48271u) % 2147483647u);
    return r->x;
}
/* uniform_real_distribution<float>(0,1) (rocThrust uniform_real_distribution.inl:67-80) */
static inline float u01(or_rng* r) {
    float result = (float)(rng_next(r) - 1u);
    result /= (1.0f + (float)(2147483646u - 1u));
    return (result * (1.0f - 0.0f)) + 0.0f;
}
/* glm::vec2(u01(rng), u01(rng)): argument evaluation order is compiler-defined. */
static inline v2 u01_pair(const or_options* o, or_rng* r) {
    float a = u01(r);
    float b = u01(r);
    return o->arg_order ? V2(a, b) : V2(b, a);
}

void or_rng_draws(int32_t iter, int32_t index, int32_t depth, int32_t n, float* out) {
    or_rng r = rng_make(iter, index, depth);
    for (int i = 0; i < n; ++i) out[i] = u01(&r);
}

/* ------------------------------------------------------------------------------------------ */
/* intersections.cu                                                                            */
/* ------------------------------------------------------------------------------------------ */
/* intersections.h:29-32 */
static inline v3 getPointOnRay(v3 o, v3 d, float t) { return add3(o, muls3(normalize3(d), t - .0001f)); }

/* intersections.cu:3-57 */
float or_box_test(const pt_geom* box, const pt_ray* r, pt_vec3* intersectionPoint, pt_vec3* normal,
                  int32_t* outside) {
    v3 qo = multiplyMV(&box->inverseTransform, V4(r->origin.x, r->origin.y, r->origin.z, 1.0f));
    v3 qd = normalize3(multiplyMV(&box->inverseTransform, V4(r->direction.x, r->direction.y, r->direction.z, 0.0f)));
    float tmin = -1e38f, tmax = 1e38f;
    v3 tmin_n = V3(0, 0, 0), tmax_n = V3(0, 0, 0);
    for (int xyz = 0; xyz < 3; ++xyz) {
        float qdxyz = comp3(qd, xyz);
        float t1 = (-0.5f - comp3(qo, xyz)) / qdxyz;
        float t2 = (+0.5f - comp3(qo, xyz)) / qdxyz;
        float ta = gmin(t1, t2);
        float tb = gmax(t1, t2);
        v3 n = V3(0, 0, 0);
        setcomp3(&n, xyz, t2 < t1 ? +1.0f : -1.0f);
        if (ta > 0 && ta > tmin) { tmin = ta; tmin_n = n; }
        if (tb < tmax) { tmax = tb; tmax_n = n; }
    }
    if (tmax >= tmin && tmax > 0) {
        *outside = 1;
        if (tmin <= 0) { tmin = tmax; tmin_n = tmax_n; *outside = 0; }
        v3 p = getPointOnRay(qo, qd, tmin);
        *intersectionPoint = multiplyMV(&box->transform, V4(p.x, p.y, p.z, 1.0f));
        *normal = normalize3(multiplyMV(&box->invTranspose, V4(tmin_n.x, tmin_n.y, tmin_n.z, 0.0f)));
        return length3(sub3(r->origin, *intersectionPoint));
    }
    return -1;
}

/* intersections.cu:59-109 */
float or_sphere_test(const pt_geom* sphere, const pt_ray* r, pt_vec3* intersectionPoint, pt_vec3* normal,
                     int32_t* outside) {
    float radius = .5f;
    v3 ro = multiplyMV(&sphere->inverseTransform, V4(r->origin.x, r->origin.y, r->origin.z, 1.0f));
    v3 rd = normalize3(multiplyMV(&sphere->inverseTransform, V4(r->direction.x, r->direction.y, r->direction.z, 0.0f)));
    float vDotDirection = dot3(ro, rd);
    float radicand = vDotDirection * vDotDirection - (dot3(ro, ro) - powf(radius, 2));
    if (radicand < 0) return -1;
    float squareRoot = sqrtf(radicand);
    float firstTerm = -vDotDirection;
    float t1 = firstTerm + squareRoot;
    float t2 = firstTerm - squareRoot;
    float t = 0;
    if (t1 < 0 && t2 < 0) {
        return -1;
    } else if (t1 > 0 && t2 > 0) {
        t = gmin(t1, t2);
        *outside = 1;
    } else {
        t = gmax(t1, t2);
        *outside = 0;
    }
    v3 objp = getPointOnRay(ro, rd, t);
    *intersectionPoint = multiplyMV(&sphere->transform, V4(objp.x, objp.y, objp.z, 1.0f));
    *normal = normalize3(multiplyMV(&sphere->invTranspose, V4(objp.x, objp.y, objp.z, 0.0f)));
    return length3(sub3(r->origin, *intersectionPoint));
}

/* intersections.cu:112-145 (Moller-Trumbore) */
int32_t or_triangle_test(const pt_ray* r, const pt_vec3* v0, const pt_vec3* v1, const pt_vec3* v2,
                         float* tOut, float* uOut, float* vOut) {
    v3 edge1 = sub3(*v1, *v0);
    v3 edge2 = sub3(*v2, *v0);
    v3 pvec = cross3(r->direction, edge2);
    float det = dot3(edge1, pvec);
    if (fabsf(det) < BABY_EPSILON) return 0;
    float invDet = 1.0f / det;
    v3 tvec = sub3(r->origin, *v0);
    float u = dot3(tvec, pvec) * invDet;
    if (u < 0.0f || u > 1.0f) return 0;
    v3 qvec = cross3(tvec, edge1);
    float v = dot3(r->direction, qvec) * invDet;
    if (v < 0.0f || (u + v) > 1.0f) return 0;
    float t = dot3(edge2, qvec) * invDet;
    if (t <= BABY_EPSILON) return 0;
    *tOut = t; *uOut = u; *vOut = v;
    return 1;
}

/* intersections.cu:237-275 */
int32_t or_aabb_test(const pt_aabb* aabb, const pt_ray* ray) {
    float t_min = -FLT_MAX, t_max = FLT_MAX;
    for (int i = 0; i < 3; ++i) {
        float dir = comp3(ray->direction, i);
        float origin = comp3(ray->origin, i);
        float bmin = comp3(aabb->min, i), bmax = comp3(aabb->max, i);
        if (fabsf(dir) < 0.00001f) {
            if (origin < bmin || origin > bmax) return 0;
        } else {
            float t1 = (bmin - origin) / dir;
            float t2 = (bmax - origin) / dir;
            if (t1 > t2) { float tmp = t1; t1 = t2; t2 = tmp; }
            if (t1 > t_min) t_min = t1;
            if (t2 < t_max) t_max = t2;
            if (t_min > t_max) return 0;
        }
    }
    return t_max >= t_min && t_max > 0.f;
}

/* intersections.cu:148-234.  An empty BVH is "no hit" (the reference dereferences nodes[0]
 * of a zero-byte allocation there). */
static float bvh_test(const or_scene* s, const pt_ray* r, v3* intersectionPoint, v3* normal, int* outside,
                      int* materialID, v2* outUV, int* outTriIndex, v3* out_dpdu, v3* out_dpdv) {
    float t_hit = FLT_MAX;
    int hitAnything = 0;
    *outTriIndex = -1;
    if (s->num_bvh_nodes <= 0) return -1.f;
    int stack[64];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        int nodeIdx = stack[--sp];
        const pt_bvh_node* node = &s->bvh_nodes[nodeIdx];
        if (!or_aabb_test(&node->aabb, r)) continue;
        if (node->triCount > 0 && node->start >= 0) {
            for (int i = 0; i < node->triCount; i++) {
                int triIndex = s->tri_indices[node->start + i];
                const pt_triangle* tri = &s->triangles[triIndex];
                const pt_vertex* v0 = &tri->v1;
                const pt_vertex* v1 = &tri->v2;
                const pt_vertex* v2 = &tri->v3;
                float t, u, v;
                if (or_triangle_test(r, &v0->position, &v1->position, &v2->position, &t, &u, &v)) {
                    if (t < t_hit && t > 0.0f) {
                        hitAnything = 1;
                        t_hit = t;
                        *outTriIndex = triIndex;
                        *intersectionPoint = add3(r->origin, muls3(r->direction, t));
                        if (length3(v0->normal) < 1e-6f || length3(v1->normal) < 1e-6f || length3(v2->normal) < 1e-6f) {
                            *normal = normalize3(cross3(sub3(v1->position, v0->position), sub3(v2->position, v0->position)));
                        } else {
                            float w0 = 1 - u - v;
                            *normal = normalize3(add3(add3(muls3(v0->normal, w0), muls3(v1->normal, u)), muls3(v2->normal, v)));
                        }
                        float w0 = 1.0f - u - v;
                        *outUV = add2(add2(muls2(v0->uv, w0), muls2(v1->uv, u)), muls2(v2->uv, v));
                        *outside = dot3(r->direction, *normal) < 0.0f;
                        *materialID = tri->materialID;
                        *out_dpdu = tri->dpdu;
                        *out_dpdv = tri->dpdv;
                    }
                }
            }
        } else {
            if (node->left >= 0) stack[sp++] = node->left;
            if (node->right >= 0) stack[sp++] = node->right;
        }
    }
    return hitAnything ? t_hit : -1.f;
}

/* pathtrace.cu:298-448 computeIntersections, one path.  `out` must be zeroed first
 * (the reference memsets dev_intersections every bounce, pathtrace.cu:699). */
void or_compute_intersection(const or_scene* s, const or_options* o, const pt_path_segment* ps,
                             pt_shadeable_isect* out) {
    pt_ray ray = ps->ray;
    float t = 0;
    v3 intersect_point = V3(0, 0, 0), normal = V3(0, 0, 0);
    float t_min = FLT_MAX;
    int hit_geom_index = -1;
    int hit_material_id = -1;
    int outside = 1;
    v2 hitUV = V2(0, 0);
    int hitTriIndex = -1;
    v3 tmp_intersect = V3(0, 0, 0), tmp_normal = V3(0, 0, 0), tmp_dpdu = V3(0, 0, 0), tmp_dpdv = V3(0, 0, 0);
    for (int i = 0; i < s->num_geoms; i++) {
        const pt_geom* geom = &s->geoms[i];
        if (geom->type == PT_CUBE) t = or_box_test(geom, &ray, &tmp_intersect, &tmp_normal, &outside);
        else if (geom->type == PT_SPHERE) t = or_sphere_test(geom, &ray, &tmp_intersect, &tmp_normal, &outside);
        if (t > 0.0f && t_min > t) {
            t_min = t;
            hit_geom_index = geom->materialid;
            intersect_point = tmp_intersect;
            normal = tmp_normal;
            hitUV = V2(0, 0);
            hitTriIndex = -1;
            hit_material_id = hit_geom_index;
        }
    }
    if (o->bvh) {
        int material_id_bvh = -1;
        float t_bvh = bvh_test(s, &ray, &tmp_intersect, &tmp_normal, &outside, &material_id_bvh, &hitUV,
                               &hitTriIndex, &tmp_dpdu, &tmp_dpdv);
        if (t_bvh > 0.0f && t_bvh < t_min) {
            t_min = t_bvh;
            hit_geom_index = -2;
            intersect_point = tmp_intersect;
            normal = tmp_normal;
            hit_material_id = material_id_bvh;
        }
    }
    (void)intersect_point;
    (void)hitTriIndex;
    if (hit_geom_index == -1) {
        out->t = -1.0f;
    } else {
        if (dot3(ray.direction, normal) > 0.0f) normal = neg3(normal);
        out->t = t_min;
        out->materialId = (hit_geom_index == -2) ? hit_material_id : hit_geom_index;
        out->surfaceNormal = normal;
        if (hit_geom_index == -2) {
            out->uv = hitUV;
            out->dpdu = tmp_dpdu;
            out->dpdv = tmp_dpdv;
        } else {
            out->uv = V2(0, 0);
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* interactions.h / interactions.cu                                                            */
/* ------------------------------------------------------------------------------------------ */
/* interactions.h:14-20 */
static inline void coordinateSystem(v3 v1, v3* v2, v3* v3o) {
    if (fabsf(v1.x) > fabsf(v1.y))
        *v2 = divs3(V3(-v1.z, 0, v1.x), sqrtf(v1.x * v1.x + v1.z * v1.z));
    else
        *v2 = divs3(V3(0, v1.z, -v1.y), sqrtf(v1.y * v1.y + v1.z * v1.z));
    *v3o = cross3(v1, *v2);
}
/* interactions.h:22-32 */
static inline mat3c LocalToWorld(v3 nor) {
    v3 tan, bit;
    coordinateSystem(nor, &tan, &bit);
    mat3c m; m.c0 = tan; m.c1 = bit; m.c2 = nor;
    return m;
}
static inline mat3c WorldToLocal(v3 nor) { mat3c m = LocalToWorld(nor); return mat3_transpose(&m); }

/* interactions.cu:49-75 */
static v3 squareToDiskConcentric(const or_options* o, v2 xi) {
    float x, y;
    if (xi.x == 0.f && xi.y == 0.f) {
        x = 0.f; y = 0.f;
    } else {
        float theta = 0.f, radius = 1.f;
        float a = (2.f * xi.x) - 1.f;
        float b = (2.f * xi.y) - 1.f;
        if ((a * a) > (b * b)) {
            radius *= a;
            theta = PI_OVER_FOUR * (b / a);
        } else {
            radius *= b;
            theta = PI_OVER_TWO - (PI_OVER_FOUR * (a / b));
        }
        x = radius * t_cos(o, theta);
        y = radius * t_sin(o, theta);
    }
    return V3(x, y, 0.f);
}
/* interactions.cu:77-85 */
static v3 squareToHemisphereCosine(const or_options* o, v2 xi) {
    v3 disk = squareToDiskConcentric(o, xi);
    float z = sqrtf(gmax(0.f, 1.0f - (disk.x * disk.x) - (disk.y * disk.y)));
    return V3(disk.x, disk.y, z);
}
/* interactions.cu:92-108 */
static v3 sampleFDiffuse(const or_options* o, v3 albedo, v3 normal, v3* wiW, float* pdf, or_rng* rng) {
    v2 xi = u01_pair(o, rng);
    v3 wi = squareToHemisphereCosine(o, xi);
    mat3c ws = LocalToWorld(normal);
    *wiW = normalize3(mat3_mul_v3(&ws, wi));
    *pdf = wi.z / PI;
    return muls3(albedo, INV_PI);
}
/* interactions.cu:146-168 */
static v3 sampleFSpecularTrans(v3 albedo, v3 normal, v3 wo, float IOR, v3* wiW) {
    int entering = dot3(wo, normal) < 0.0f;
    float eta = entering ? (1.0f / IOR) : IOR;
    v3 outNormal = entering ? normal : neg3(normal);
    *wiW = refract3(normalize3(wo), normalize3(outNormal), eta);
    if (length3(*wiW) < BABY_EPSILON) {
        *wiW = reflect3(wo, normal);
        return V3(0.f, 0.f, 0.f);
    }
    return albedo;
}
/* interactions.cu:173-194 */
static float FresnelDielectricEval(float cosThetaI, float IOR) {
    float etaI = 1.f, etaT = IOR;
    cosThetaI = gclamp(cosThetaI, -1.f, 1.f);
    if (cosThetaI > 0.f) { float tmp = etaI; etaI = etaT; etaT = tmp; }
    cosThetaI = fabsf(cosThetaI);
    float sinThetaI = sqrtf(gmax(0.f, 1.f - cosThetaI * cosThetaI));
    float sinThetaT = etaI / etaT * sinThetaI;
    float cosThetaT = sqrtf(gmax(0.f, 1.f - sinThetaT * sinThetaT));
    float Rparl = ((etaT * cosThetaI) - (etaI * cosThetaT)) / ((etaT * cosThetaI) + (etaI * cosThetaT));
    float Rperp = ((etaI * cosThetaI) - (etaT * cosThetaT)) / ((etaI * cosThetaI) + (etaT * cosThetaT));
    return (Rparl * Rparl + Rperp * Rperp) * 0.5f;
}
/* interactions.cu:197-201 */
static v3 FresnelSchlick(const or_options* o, float cosTheta, v3 F0) {
    float p = t_pow5(o, 1.0f - cosTheta);
    return V3(F0.x + (1.0f - F0.x) * p, F0.y + (1.0f - F0.y) * p, F0.z + (1.0f - F0.z) * p);
}
/* interactions.cu:204-235 */
static v3 sampleFGlass(v3 albedo, v3 normal, v3 wo, float IOR, v3* wiW, or_rng* rng) {
    float random = u01(rng);
    float cosTheta = dot3(wo, normal);
    float fresnel = FresnelDielectricEval(cosTheta, IOR);
    if (random < fresnel) {
        *wiW = reflect3(wo, normal);
        return albedo;
    } else {
        v3 T = sampleFSpecularTrans(albedo, normal, wo, IOR, wiW);
        if (length3(*wiW) < BABY_EPSILON) {
            *wiW = reflect3(wo, normal);
            return albedo;
        }
        return T;
    }
}
/* interactions.h:106-167 trig helpers */
static inline float Cos2Theta(v3 w) { return w.z * w.z; }
static inline float Sin2Theta(v3 w) { return gmax(0.f, 1.f - Cos2Theta(w)); }
static inline float Tan2Theta(v3 w) { return Sin2Theta(w) / Cos2Theta(w); }
static inline float SinTheta(v3 w) { return sqrtf(Sin2Theta(w)); }
static inline float TanTheta(v3 w) { return SinTheta(w) / w.z; }
static inline float CosPhi(v3 w) { float st = SinTheta(w); return (st == 0) ? 0 : gclamp(w.x / st, -1.f, 1.f); }
static inline float SinPhi(v3 w) { float st = SinTheta(w); return (st == 0) ? 0 : gclamp(w.y / st, -1.f, 1.f); }
static inline float Cos2Phi(v3 w) { return CosPhi(w) * CosPhi(w); }
static inline float Sin2Phi(v3 w) { return SinPhi(w) * SinPhi(w); }

/* interactions.cu:238-264 */
static v3 sampleWH(const or_options* o, v3 wo, float roughness, or_rng* rng) {
    v2 xi = u01_pair(o, rng);
    float phi = TWO_PI * xi.y;
    float tanTheta2 = roughness * roughness * xi.x / (1.0f - xi.x);
    float cosTheta = 1 / sqrtf(1 + tanTheta2);
    float sinTheta = sqrtf(gmax(0.f, 1.f - cosTheta * cosTheta));
    v3 wh = V3(sinTheta * t_cos(o, phi), sinTheta * t_sin(o, phi), cosTheta);
    if (!(wo.z * wh.z > 0)) wh = neg3(wh);
    return wh;
}
/* interactions.cu:266-283 */
static float TrowbridgeReitzD(v3 wh, float roughness) {
    float tan2Theta = Tan2Theta(wh);
    if (isinf(tan2Theta)) return 0.f;
    float cos4Theta = Cos2Theta(wh) * Cos2Theta(wh);
    float e = (Cos2Phi(wh) / (roughness * roughness) + Sin2Phi(wh) / (roughness * roughness)) * tan2Theta;
    return 1 / (PI * roughness * roughness * cos4Theta * (1 + e) * (1 + e));
}
/* interactions.cu:285-297 (the unused `alpha` local has no effect and is not restated) */
static float lambda_(v3 w, float roughness) {
    float absTanTheta = fabsf(TanTheta(w));
    if (isinf(absTanTheta)) return 0.f;
    float alpha2Tan2Theta = (roughness * absTanTheta) * (roughness * absTanTheta);
    return (-1 + sqrtf(1.f + alpha2Tan2Theta)) / 2;
}
/* interactions.cu:299-305 */
static float TrowbridgeReitzG(v3 wo, v3 wi, float roughness) {
    return 1.0f / (1.0f + lambda_(wo, roughness) + lambda_(wi, roughness));
}
/* interactions.cu:307-312 */
static float TrowbridgeReitzPdf(v3 wo, v3 wh, float roughness) {
    (void)wo;
    return TrowbridgeReitzD(wh, roughness) * fabsf(wh.z);
}
/* interactions.cu:314-348 */
static v3 fMicrofacetRefl(const or_options* o, v3 albedo, v3 wo, v3 wi, float IOR, float roughness, float metallic) {
    (void)IOR;
    float cosThetaO = fabsf(wo.z);
    float cosThetaI = fabsf(wi.z);
    v3 wh = add3(wi, wo);
    if (cosThetaI == 0 || cosThetaO == 0) return V3(0.f, 0.f, 0.f);
    if (wh.x == 0 && wh.y == 0 && wh.z == 0) return V3(0.f, 0.f, 0.f);
    wh = normalize3(wh);
    float dielectricF0 = 0.04f;
    v3 F0 = mix3(V3(dielectricF0, dielectricF0, dielectricF0), albedo, metallic);
    v3 F = FresnelSchlick(o, dot3(wi, wh), F0);
    float D = TrowbridgeReitzD(wh, roughness);
    float G = TrowbridgeReitzG(wo, wi, roughness);
    return divs3(muls3(F, D * G), 4.0f * cosThetaI * cosThetaO);
}
/* interactions.cu:350-380 */
static v3 sampleFMicrofacetRefl(const or_options* o, v3 albedo, v3 normal, v3 wo, float IOR, float roughness,
                                float metallic, v3* wiW, float* pdf, or_rng* rng) {
    mat3c worldToLocal = WorldToLocal(normal);
    mat3c localToWorld = LocalToWorld(normal);
    v3 wo_local = mat3_mul_v3(&worldToLocal, wo);
    v3 wh_local = sampleWH(o, wo_local, roughness, rng);
    if (wh_local.z < 0.0f) wh_local = neg3(wh_local);
    v3 wi_local = reflect3(neg3(wo_local), wh_local);
    *wiW = normalize3(mat3_mul_v3(&localToWorld, wi_local));
    float dotWO_WH = gmax(dot3(wo_local, wh_local), 1e-6f);
    *pdf = TrowbridgeReitzPdf(wo_local, wh_local, roughness) / (4.0f * dotWO_WH);
    return fMicrofacetRefl(o, albedo, wo_local, wi_local, IOR, roughness, metallic);
}
/* interactions.cu:383-435 */
static v3 sampleFCookTorrance(const or_options* o, v3 albedo, v3 normal, v3 woW, float IOR, float roughness,
                              float metallic, v3* wiW, float* out_pdf, or_rng* rng) {
    float dielectricF0 = 0.04f;
    v3 F0 = mix3(V3(dielectricF0, dielectricF0, dielectricF0), albedo, metallic);
    float cosTheta = gclamp(dot3(normal, woW), 0.0f, 1.0f);
    v3 F = FresnelSchlick(o, cosTheta, F0);
    float Fprob = gclamp(gmax(F.x, gmax(F.y, F.z)), 0.0f, 1.0f);
    float choose = u01(rng);
    v3 bsdf = V3(0.0f, 0.0f, 0.0f);
    float pdf_spec = 0.0f, pdf_diff = 0.0f;
    if (choose < Fprob) {
        bsdf = sampleFMicrofacetRefl(o, albedo, normal, woW, IOR, roughness, metallic, wiW, &pdf_spec, rng);
        pdf_diff = 0.0f;
    } else {
        bsdf = sampleFDiffuse(o, albedo, normal, wiW, &pdf_diff, rng);
        pdf_spec = 0.0f;
    }
    *out_pdf = Fprob * pdf_spec + (1.0f - Fprob) * pdf_diff;
    if (choose < Fprob) bsdf = mul3(bsdf, F);
    else bsdf = mul3(bsdf, sub3(V3(1.0f, 1.0f, 1.0f), F));
    return bsdf;
}

/* interactions.cu:438-542 scatterRay (rng already seeded) */
static void scatter_rng(const or_options* o, pt_path_segment* ps, v3 intersect, v3 normal, const pt_material* m,
                        or_rng* rng) {
    v3 wiW = V3(0, 0, 0), bsdf;
    float pdf = 1.0f;
    v3 mcolor = m->color;
    if (m->hasRefractive > 0.0f && m->hasReflective > 0.0f) {                 /* Glass */
        bsdf = sampleFGlass(mcolor, normal, ps->ray.direction, m->indexOfRefraction, &wiW, rng);
        ps->ray.direction = normalize3(wiW);
        ps->ray.origin = add3(intersect, muls3(ps->ray.direction, LARGER_EPSILON));
        ps->color = mul3(ps->color, bsdf);
    } else if (m->hasReflective > 0.0f) {                                      /* Mirror */
        wiW = reflect3(ps->ray.direction, normal);
        bsdf = mcolor;
        ps->ray.direction = normalize3(wiW);
        ps->ray.origin = add3(intersect, muls3(normal, BABY_EPSILON));
        ps->color = mul3(ps->color, bsdf);
    } else if (m->hasRefractive > 0.0f) {                                      /* Transmissive */
        bsdf = sampleFSpecularTrans(mcolor, normal, ps->ray.direction, m->indexOfRefraction, &wiW);
        ps->ray.direction = normalize3(wiW);
        ps->ray.origin = add3(intersect, muls3(ps->ray.direction, LARGER_EPSILON));
        ps->color = mul3(ps->color, bsdf);
    } else if (m->roughness >= 0.0f && m->metallic >= 0.0f) {                  /* Microfacet */
        v3 woW = neg3(normalize3(ps->ray.direction));
        bsdf = sampleFCookTorrance(o, mcolor, normal, woW, m->indexOfRefraction, m->roughness, m->metallic,
                                   &wiW, &pdf, rng);
        ps->ray.direction = normalize3(wiW);
        ps->ray.origin = add3(intersect, muls3(ps->ray.direction, LARGER_EPSILON));
        float cosTheta = gmax(0.0f, dot3(normal, wiW));
        if (pdf > 0.0f) ps->color = mul3(ps->color, divs3(muls3(bsdf, cosTheta), pdf));
    } else {                                                                   /* Diffuse */
        bsdf = sampleFDiffuse(o, mcolor, normal, &wiW, &pdf, rng);
        ps->ray.direction = normalize3(wiW);
        ps->ray.origin = add3(intersect, muls3(normal, BABY_EPSILON));
        float cosTheta = gmax(0.0f, dot3(normal, wiW));
        ps->color = mul3(ps->color, divs3(muls3(bsdf, cosTheta), pdf));
    }
    ps->remainingBounces -= 1;
}

void or_scatter(const or_options* o, pt_path_segment* path, pt_vec3 intersect, pt_vec3 normal,
                const pt_material* m, int32_t iter) {
    or_rng rng = rng_make(iter, path->pixelIndex, path->remainingBounces);
    scatter_rng(o, path, intersect, normal, m, &rng);
}

/* pathtrace.cu:505-519 sampleTexture / sampleHeight: tex2D<float4>(texObjects[id], x, 1 - y)
 * through the framework's definition of CUDA's linear/wrap fetch (include/pt/pt_texture.h) */
static v3 sample_texture(const or_scene* s, int texID, v2 uv) {
    if (texID < 0 || texID >= s->num_textures) return V3(1.0f, 0.0f, 1.0f);
    const pt_texture* t = &s->textures[texID];
    float c[4];
    pt_tex2d((const uint32_t*)t->data, t->width, t->height, uv.x, 1.f - uv.y, c);
    return V3(c[0], c[1], c[2]);
}
static float sample_height(const or_scene* s, int texID, v2 uv) {
    if (texID < 0 || texID >= s->num_textures) return 0.0f;
    const pt_texture* t = &s->textures[texID];
    float c[4];
    pt_tex2d((const uint32_t*)t->data, t->width, t->height, uv.x, 1.f - uv.y, c);
    return c[0];
}

/* pathtrace.cu:521-621 kernShadeMaterialProper, one path */
void or_shade(const or_scene* s, const or_options* o, int32_t iter, const pt_shadeable_isect* isect,
              pt_path_segment* ps) {
    if (ps->remainingBounces <= 0) return;
    if (isect->t > 0.0f) {
        pt_material material = s->materials[isect->materialId];
        v3 materialColor = material.color;
        if (material.hasTexture) materialColor = sample_texture(s, material.textureID, isect->uv);
        material.color = materialColor;
        if (material.emittance > 0.0f) {
            ps->color = mul3(ps->color, muls3(materialColor, material.emittance));
            ps->remainingBounces = 0;
        } else {
            or_rng rng = rng_make(iter, ps->pixelIndex, ps->remainingBounces);
            v3 intersect = add3(ps->ray.origin, muls3(ps->ray.direction, isect->t));
            v3 ng = isect->surfaceNormal;
            v3 dpdu = isect->dpdu, dpdv = isect->dpdv;
            v2 uv = isect->uv;
            v3 shadingNormal = ng;
            /* :579-607; bumpID < num_textures always holds for ids loadTexture returns */
            if (material.hasBumpMap && material.bumpID >= 0 && material.bumpID < s->num_textures) {
                int bumpTexID = material.bumpID;
                int texWidth = s->textures[bumpTexID].width;
                int texHeight = s->textures[bumpTexID].height;
                float du = 1.0f / (float)texWidth;
                float dv = 1.0f / (float)texHeight;
                float h = sample_height(s, bumpTexID, uv);
                float hU = sample_height(s, bumpTexID, V2(uv.x + du, uv.y));
                float hV = sample_height(s, bumpTexID, V2(uv.x, uv.y + dv));
                float dhdu = (hU - h) / du;
                float dhdv = (hV - h) / dv;
                float scale = material.bumpScale;
                v3 dpdu_p = add3(dpdu, muls3(ng, scale * dhdu));     /* dpdu + scale * dhdu * ng */
                v3 dpdv_p = add3(dpdv, muls3(ng, scale * dhdv));
                shadingNormal = normalize3(cross3(dpdu_p, dpdv_p));
                if (dot3(shadingNormal, ng) < 0.0f) shadingNormal = neg3(shadingNormal);
            }
            scatter_rng(o, ps, intersect, shadingNormal, &material, &rng);
        }
    } else {
        ps->color = V3(0.0f, 0.0f, 0.0f);
        ps->remainingBounces = 0;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* camera rays: pathtrace.cu:231-237 sampleAperture, :247-292 generateRayFromCamera            */
/* ------------------------------------------------------------------------------------------ */
void or_generate_ray(const pt_camera* cam, int32_t iter, int32_t traceDepth, int32_t x, int32_t y,
                     const or_options* o, pt_path_segment* seg) {
    int index = x + (y * cam->resolution.x);
    or_rng rng = rng_make(iter, index, 0);
    float jitterX = u01(&rng);
    float jitterY = u01(&rng);
    float sx = (float)x + jitterX - (float)cam->resolution.x * 0.5f;
    float sy = (float)y + jitterY - (float)cam->resolution.y * 0.5f;
    v3 a = muls3(muls3(cam->right, cam->pixelLength.x), sx);
    v3 b = muls3(muls3(cam->up, cam->pixelLength.y), sy);
    v3 pixelPoint = sub3(sub3(cam->view, a), b);
    v3 rayDir = normalize3(pixelPoint);
    v3 focalPoint = add3(cam->position, muls3(rayDir, cam->focalDist));
    /* sampleAperture */
    float r = cam->aperture * sqrtf(u01(&rng));
    float theta = 2 * PI * u01(&rng);
    v3 apertureOffset = V3(r * t_cos(o, theta), r * t_sin(o, theta), 0.0f);
    seg->ray.origin = add3(cam->position, apertureOffset);
    seg->color = V3(1.f, 1.f, 1.f);
    seg->ray.direction = normalize3(sub3(focalPoint, seg->ray.origin));
    seg->pixelIndex = index;
    seg->remainingBounces = traceDepth;
}

/* pathtrace.cu:59-80 */
void or_image_to_pbo(const float* image, int32_t n, int32_t iter, pt_uchar4* pbo) {
    for (int i = 0; i < n; ++i) {
        int c[3];
        for (int k = 0; k < 3; ++k) {
            double d = (double)(image[3 * i + k] / (float)iter) * 255.0;
            int v = (d != d) ? 0 : (d >= 2147483647.0 ? 2147483647 : (d <= -2147483648.0 ? (-2147483647 - 1) : (int)d));
            c[k] = v < 0 ? 0 : (v > 255 ? 255 : v);   /* glm::clamp(int) = min(max(v,0),255) */
        }
        pbo[i].w = 0; pbo[i].x = (uint8_t)c[0]; pbo[i].y = (uint8_t)c[1]; pbo[i].z = (uint8_t)c[2];
    }
}

/* ------------------------------------------------------------------------------------------ */
/* stream_compaction/cpu.cu:20-92                                                              */
/* ------------------------------------------------------------------------------------------ */
void or_cpu_scan(int32_t n, int32_t* odata, const int32_t* idata) {
    if (n == 0) return;
    odata[0] = 0;
    for (int i = 1; i < n; i++) odata[i] = odata[i - 1] + idata[i - 1];
}
int32_t or_cpu_compact_without_scan(int32_t n, int32_t* odata, const int32_t* idata) {
    int counter = 0;
    for (int i = 0; i < n; i++) if (idata[i] != 0) odata[counter++] = idata[i];
    return counter;
}
int32_t or_cpu_compact_with_scan(int32_t n, int32_t* odata, const int32_t* idata) {
    if (n <= 0) return 0;
    int32_t* flag = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    int32_t* scanned = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    for (int i = 0; i < n; i++) flag[i] = (idata[i] != 0) ? 1 : 0;
    scanned[0] = 0;
    for (int i = 1; i < n; i++) scanned[i] = scanned[i - 1] + flag[i - 1];
    int counter = 0;
    for (int i = 0; i < n; i++) if (flag[i] == 1) { odata[scanned[i]] = idata[i]; counter++; }
    free(flag); free(scanned);
    return counter;
}

/* thrust::stable_partition(paths, paths + n, PathAlive) (pathtrace.cu:750-757) restated as
 * the cpu.cu flag -> exclusive scan -> scatter, for both halves (stable). */
static int stable_partition_alive(pt_path_segment* paths, pt_path_segment* tmp, int32_t* flag, int32_t* scan, int n) {
    for (int i = 0; i < n; i++) flag[i] = paths[i].remainingBounces > 0;   /* PathAlive, sceneStructs.h:137-142 */
    or_cpu_scan(n, scan, flag);
    int alive = n ? scan[n - 1] + flag[n - 1] : 0;
    for (int i = 0; i < n; i++) {
        int dst = flag[i] ? scan[i] : alive + (i - scan[i]);
        tmp[dst] = paths[i];
    }
    memcpy(paths, tmp, sizeof(pt_path_segment) * (size_t)n);
    return alive;
}

/* thrust::stable_sort_by_key(isects, isects + n, paths, CompareMat) (pathtrace.cu:730-735):
 * a stable counting sort on materialId (keys >= 0; misses carry 0 from the memset). */
static void stable_sort_by_material(pt_shadeable_isect* is, pt_path_segment* ps, pt_shadeable_isect* tis,
                                    pt_path_segment* tps, int n) {
    int maxk = 0;
    for (int i = 0; i < n; i++) if (is[i].materialId > maxk) maxk = is[i].materialId;
    int32_t* cnt = (int32_t*)calloc((size_t)maxk + 2, sizeof(int32_t));
    for (int i = 0; i < n; i++) cnt[is[i].materialId + 1]++;
    for (int k = 0; k <= maxk; k++) cnt[k + 1] += cnt[k];
    for (int i = 0; i < n; i++) {
        int d = cnt[is[i].materialId]++;
        tis[d] = is[i];
        tps[d] = ps[i];
    }
    memcpy(is, tis, sizeof(*is) * (size_t)n);
    memcpy(ps, tps, sizeof(*ps) * (size_t)n);
    free(cnt);
}

/* ------------------------------------------------------------------------------------------ */
/* pathtrace.cu:639-787 pathtrace()                                                            */
/* ------------------------------------------------------------------------------------------ */
int32_t or_pathtrace_dump(const or_scene* s, const or_options* o, int32_t iter, float* image, int32_t* live_counts,
                          pt_path_segment* dump) {
    const pt_camera* cam = &s->camera;
    const int traceDepth = s->trace_depth;
    const int pixelcount = cam->resolution.x * cam->resolution.y;
#ifdef _OPENMP
    if (o->num_threads > 0) omp_set_num_threads(o->num_threads);
#endif
    pt_path_segment* paths = (pt_path_segment*)malloc(sizeof(pt_path_segment) * (size_t)pixelcount);
    pt_path_segment* tmp = (pt_path_segment*)malloc(sizeof(pt_path_segment) * (size_t)pixelcount);
    pt_shadeable_isect* isects = (pt_shadeable_isect*)malloc(sizeof(pt_shadeable_isect) * (size_t)pixelcount);
    pt_shadeable_isect* tisects = (pt_shadeable_isect*)malloc(sizeof(pt_shadeable_isect) * (size_t)pixelcount);
    int32_t* flag = (int32_t*)malloc(sizeof(int32_t) * (size_t)pixelcount);
    int32_t* scan = (int32_t*)malloc(sizeof(int32_t) * (size_t)pixelcount);
    if (live_counts) for (int b = 0; b < traceDepth; ++b) live_counts[b] = -1;

#pragma omp parallel for schedule(static)
    for (int y = 0; y < cam->resolution.y; ++y)
        for (int x = 0; x < cam->resolution.x; ++x)
            or_generate_ray(cam, iter, traceDepth, x, y, o, &paths[x + y * cam->resolution.x]);

    int depth = 0;
    int num_paths = pixelcount;
    int done = 0;
    while (!done) {
        memset(isects, 0, sizeof(pt_shadeable_isect) * (size_t)pixelcount);
        if (live_counts && depth < traceDepth) live_counts[depth] = num_paths;
#pragma omp parallel for schedule(dynamic, 1024)
        for (int i = 0; i < num_paths; ++i) or_compute_intersection(s, o, &paths[i], &isects[i]);
        depth++;
        if (o->material_sort) stable_sort_by_material(isects, paths, tisects, tmp, num_paths);
#pragma omp parallel for schedule(dynamic, 1024)
        for (int i = 0; i < num_paths; ++i) or_shade(s, o, iter, &isects[i], &paths[i]);
        if (o->stream_compaction) num_paths = stable_partition_alive(paths, tmp, flag, scan, num_paths);
        if (dump && depth <= traceDepth)
            memcpy(dump + (size_t)(depth - 1) * (size_t)pixelcount, paths, sizeof(pt_path_segment) * (size_t)pixelcount);
        if (num_paths == 0) done = 1;
        if (depth >= traceDepth) done = 1;
    }
    /* finalGather, pathtrace.cu:624-633, over ALL pixelcount paths */
    for (int i = 0; i < pixelcount; ++i) {
        int p = paths[i].pixelIndex;
        image[3 * p + 0] += paths[i].color.x;
        image[3 * p + 1] += paths[i].color.y;
        image[3 * p + 2] += paths[i].color.z;
    }
    free(paths); free(tmp); free(isects); free(tisects); free(flag); free(scan);
    return depth;
}

int32_t or_pathtrace(const or_scene* s, const or_options* o, int32_t iter, float* image, int32_t* live_counts) {
    return or_pathtrace_dump(s, o, iter, image, live_counts, NULL);
}

/* ------------------------------------------------------------------------------------------ */
/* scene ingest helpers                                                                        */
/* ------------------------------------------------------------------------------------------ */
static void mat4_identity(pt_mat4* m) {
    memset(m, 0, sizeof(*m));
    m->m[0][0] = m->m[1][1] = m->m[2][2] = m->m[3][3] = 1.0f;
}
static inline v4 col4(const pt_mat4* m, int c) { return V4(m->m[c][0], m->m[c][1], m->m[c][2], m->m[c][3]); }
static inline void setcol4(pt_mat4* m, int c, v4 v) { m->m[c][0] = v.x; m->m[c][1] = v.y; m->m[c][2] = v.z; m->m[c][3] = v.w; }
static inline v4 add4(v4 a, v4 b) { return V4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
static inline v4 sub4(v4 a, v4 b) { return V4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
static inline v4 mul4(v4 a, v4 b) { return V4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
static inline v4 muls4(v4 a, float s) { return V4(a.x * s, a.y * s, a.z * s, a.w * s); }
static inline v4 divs4(v4 a, float s) { return V4(a.x / s, a.y / s, a.z / s, a.w / s); }

/* gtc/matrix_transform.inl translate: Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3] */
static void glm_translate(const pt_mat4* m, v3 v, pt_mat4* out) {
    *out = *m;
    v4 r = add4(add4(add4(muls4(col4(m, 0), v.x), muls4(col4(m, 1), v.y)), muls4(col4(m, 2), v.z)), col4(m, 3));
    setcol4(out, 3, r);
}
/* gtc/matrix_transform.inl rotate (angle in radians, glm 0.9.6) */
static void glm_rotate(const pt_mat4* m, float angle, v3 v, pt_mat4* out) {
    float a = angle;
    float c = cosf(a);
    float s = sinf(a);
    v3 axis = normalize3(v);
    v3 temp = muls3(axis, 1.0f - c);
    float R[3][3];
    R[0][0] = c + temp.x * axis.x;
    R[0][1] = 0 + temp.x * axis.y + s * axis.z;
    R[0][2] = 0 + temp.x * axis.z - s * axis.y;
    R[1][0] = 0 + temp.y * axis.x - s * axis.z;
    R[1][1] = c + temp.y * axis.y;
    R[1][2] = 0 + temp.y * axis.z + s * axis.x;
    R[2][0] = 0 + temp.z * axis.x + s * axis.y;
    R[2][1] = 0 + temp.z * axis.y - s * axis.x;
    R[2][2] = c + temp.z * axis.z;
    pt_mat4 res;
    for (int j = 0; j < 3; ++j)
        setcol4(&res, j, add4(add4(muls4(col4(m, 0), R[j][0]), muls4(col4(m, 1), R[j][1])), muls4(col4(m, 2), R[j][2])));
    setcol4(&res, 3, col4(m, 3));
    *out = res;
}
static void glm_scale(const pt_mat4* m, v3 v, pt_mat4* out) {
    pt_mat4 res;
    setcol4(&res, 0, muls4(col4(m, 0), v.x));
    setcol4(&res, 1, muls4(col4(m, 1), v.y));
    setcol4(&res, 2, muls4(col4(m, 2), v.z));
    setcol4(&res, 3, col4(m, 3));
    *out = res;
}
/* type_mat4x4.inl operator*(mat4, mat4) */
static void glm_mat4_mul(const pt_mat4* A, const pt_mat4* B, pt_mat4* out) {
    pt_mat4 res;
    for (int j = 0; j < 4; ++j) {
        v4 r = add4(add4(add4(muls4(col4(A, 0), B->m[j][0]), muls4(col4(A, 1), B->m[j][1])),
                         muls4(col4(A, 2), B->m[j][2])), muls4(col4(A, 3), B->m[j][3]));
        setcol4(&res, j, r);
    }
    *out = res;
}

/* utilities.cpp:85-93 */
void or_build_transform(pt_vec3 translation, pt_vec3 rotation, pt_vec3 scale, pt_mat4* out) {
    pt_mat4 I, T, R, Ry, Rz, S, TR;
    mat4_identity(&I);
    glm_translate(&I, translation, &T);
    glm_rotate(&I, rotation.x * (float)PI / 180, V3(1, 0, 0), &R);
    glm_rotate(&I, rotation.y * (float)PI / 180, V3(0, 1, 0), &Ry);
    pt_mat4 tmp;
    glm_mat4_mul(&R, &Ry, &tmp);
    glm_rotate(&I, rotation.z * (float)PI / 180, V3(0, 0, 1), &Rz);
    glm_mat4_mul(&tmp, &Rz, &R);
    glm_scale(&I, scale, &S);
    glm_mat4_mul(&T, &R, &TR);
    glm_mat4_mul(&TR, &S, out);
}

/* type_mat4x4.inl:37-92 detail::compute_inverse */
void or_mat4_inverse(const pt_mat4* mm, pt_mat4* out) {
    float (*m)[4] = (float (*)[4])mm->m;
    float Coef00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
    float Coef02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float Coef03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float Coef04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float Coef06 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float Coef07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float Coef08 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
    float Coef10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float Coef11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float Coef12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float Coef14 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float Coef15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float Coef16 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
    float Coef18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float Coef19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float Coef20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float Coef22 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
    float Coef23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    v4 Fac0 = V4(Coef00, Coef00, Coef02, Coef03);
    v4 Fac1 = V4(Coef04, Coef04, Coef06, Coef07);
    v4 Fac2 = V4(Coef08, Coef08, Coef10, Coef11);
    v4 Fac3 = V4(Coef12, Coef12, Coef14, Coef15);
    v4 Fac4 = V4(Coef16, Coef16, Coef18, Coef19);
    v4 Fac5 = V4(Coef20, Coef20, Coef22, Coef23);
    v4 Vec0 = V4(m[1][0], m[0][0], m[0][0], m[0][0]);
    v4 Vec1 = V4(m[1][1], m[0][1], m[0][1], m[0][1]);
    v4 Vec2 = V4(m[1][2], m[0][2], m[0][2], m[0][2]);
    v4 Vec3 = V4(m[1][3], m[0][3], m[0][3], m[0][3]);
    v4 Inv0 = add4(sub4(mul4(Vec1, Fac0), mul4(Vec2, Fac1)), mul4(Vec3, Fac2));
    v4 Inv1 = add4(sub4(mul4(Vec0, Fac0), mul4(Vec2, Fac3)), mul4(Vec3, Fac4));
    v4 Inv2 = add4(sub4(mul4(Vec0, Fac1), mul4(Vec1, Fac3)), mul4(Vec3, Fac5));
    v4 Inv3 = add4(sub4(mul4(Vec0, Fac2), mul4(Vec1, Fac4)), mul4(Vec2, Fac5));
    v4 SignA = V4(+1, -1, +1, -1);
    v4 SignB = V4(-1, +1, -1, +1);
    pt_mat4 Inverse;
    setcol4(&Inverse, 0, mul4(Inv0, SignA));
    setcol4(&Inverse, 1, mul4(Inv1, SignB));
    setcol4(&Inverse, 2, mul4(Inv2, SignA));
    setcol4(&Inverse, 3, mul4(Inv3, SignB));
    v4 Row0 = V4(Inverse.m[0][0], Inverse.m[1][0], Inverse.m[2][0], Inverse.m[3][0]);
    v4 Dot0 = mul4(col4(mm, 0), Row0);
    float Dot1 = (Dot0.x + Dot0.y) + (Dot0.z + Dot0.w);
    float OneOverDeterminant = 1.0f / Dot1;
    for (int c = 0; c < 4; ++c) setcol4(out, c, muls4(col4(&Inverse, c), OneOverDeterminant));
}

/* gtc/matrix_inverse.inl:95-147 inverseTranspose(mat4) */
void or_mat4_inverse_transpose(const pt_mat4* mm, pt_mat4* out) {
    float (*m)[4] = (float (*)[4])mm->m;
    float S00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
    float S01 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float S02 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
    float S03 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float S04 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
    float S05 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float S06 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float S07 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float S08 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float S09 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float S10 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float S11 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float S12 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
    float S13 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float S14 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float S15 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float S16 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float S17 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float S18 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    float I[4][4];
    I[0][0] = +(m[1][1] * S00 - m[1][2] * S01 + m[1][3] * S02);
    I[0][1] = -(m[1][0] * S00 - m[1][2] * S03 + m[1][3] * S04);
    I[0][2] = +(m[1][0] * S01 - m[1][1] * S03 + m[1][3] * S05);
    I[0][3] = -(m[1][0] * S02 - m[1][1] * S04 + m[1][2] * S05);
    I[1][0] = -(m[0][1] * S00 - m[0][2] * S01 + m[0][3] * S02);
    I[1][1] = +(m[0][0] * S00 - m[0][2] * S03 + m[0][3] * S04);
    I[1][2] = -(m[0][0] * S01 - m[0][1] * S03 + m[0][3] * S05);
    I[1][3] = +(m[0][0] * S02 - m[0][1] * S04 + m[0][2] * S05);
    I[2][0] = +(m[0][1] * S06 - m[0][2] * S07 + m[0][3] * S08);
    I[2][1] = -(m[0][0] * S06 - m[0][2] * S09 + m[0][3] * S10);
    I[2][2] = +(m[0][0] * S11 - m[0][1] * S09 + m[0][3] * S12);
    I[2][3] = -(m[0][0] * S08 - m[0][1] * S10 + m[0][2] * S12);
    I[3][0] = -(m[0][1] * S13 - m[0][2] * S14 + m[0][3] * S15);
    I[3][1] = +(m[0][0] * S13 - m[0][2] * S16 + m[0][3] * S17);
    I[3][2] = -(m[0][0] * S14 - m[0][1] * S16 + m[0][3] * S18);
    I[3][3] = +(m[0][0] * S15 - m[0][1] * S17 + m[0][2] * S18);
    float Determinant = +m[0][0] * I[0][0] + m[0][1] * I[0][1] + m[0][2] * I[0][2] + m[0][3] * I[0][3];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out->m[c][r] = I[c][r] / Determinant;
}

/* scene.cpp:158-182 (non-OBJ objects) */
void or_make_geom(int32_t type, int32_t materialid, pt_vec3 t, pt_vec3 r, pt_vec3 s, pt_geom* g) {
    memset(g, 0, sizeof(*g));
    g->type = type;
    g->materialid = materialid;
    g->translation = t; g->rotation = r; g->scale = s;
    or_build_transform(t, r, s, &g->transform);
    or_mat4_inverse(&g->transform, &g->inverseTransform);
    or_mat4_inverse_transpose(&g->transform, &g->invTranspose);
}

/* scene.cpp:184-213, then main.cpp:359-380 and runCuda's camchanged block main.cpp:423-444
 * (camchanged starts true, main.cpp:36, so the first frame always recomputes the basis).
 * Unqualified sin/cos/tan/atan on floats take the float overloads (CUDA/MSVC headers). */
void or_camera_setup(int32_t resx, int32_t resy, float fovy, pt_vec3 eye, pt_vec3 lookat, pt_vec3 up,
                     float aperture, pt_camera* cam) {
    memset(cam, 0, sizeof(*cam));
    cam->resolution.x = resx;
    cam->resolution.y = resy;
    cam->position = eye;
    cam->lookAt = lookat;
    cam->up = up;
    cam->focalDist = length3(sub3(cam->lookAt, cam->position));
    cam->aperture = aperture;
    float yscaled = tanf(fovy * (PI / 180));
    float xscaled = (yscaled * cam->resolution.x) / cam->resolution.y;
    float fovx = (atanf(xscaled) * 180) / PI;
    cam->fov = V2(fovx, fovy);
    cam->right = normalize3(cross3(cam->view, cam->up));     /* view is still zero here: NaN */
    cam->pixelLength = V2(2 * xscaled / (float)cam->resolution.x, 2 * yscaled / (float)cam->resolution.y);
    cam->view = normalize3(sub3(cam->lookAt, cam->position));
    /* main.cpp:359-380 */
    v3 view = cam->view;
    v3 viewXZ = V3(view.x, 0.0f, view.z);
    v3 viewZY = V3(0.0f, view.y, view.z);
    float phi = acosf(dot3(normalize3(viewXZ), V3(0, 0, -1)));
    float theta = acosf(dot3(normalize3(viewZY), V3(0, 1, 0)));
    v3 ogLookAt = cam->lookAt;
    float zoom = length3(sub3(cam->position, ogLookAt));
    /* main.cpp:423-444 */
    v3 cameraPosition;
    cameraPosition.x = zoom * sinf(phi) * sinf(theta);
    cameraPosition.y = zoom * cosf(theta);
    cameraPosition.z = zoom * cosf(phi) * sinf(theta);
    cam->view = neg3(normalize3(cameraPosition));
    v3 v = cam->view;
    v3 u = V3(0, 1, 0);
    v3 rr = cross3(v, u);
    cam->up = cross3(rr, v);
    cam->right = rr;
    cam->position = cameraPosition;
    cameraPosition = add3(cameraPosition, cam->lookAt);
    cam->position = cameraPosition;
    cam->focalDist = length3(sub3(cam->lookAt, cam->position));
}

/* scene.cpp:395-426 */
void or_triangle_tangents(pt_triangle* tri) {
    v3 p1 = tri->v1.position, p2 = tri->v2.position, p3 = tri->v3.position;
    v2 uv1 = tri->v1.uv, uv2 = tri->v2.uv, uv3 = tri->v3.uv;
    v3 dp1 = sub3(p2, p1), dp2 = sub3(p3, p1);
    v2 duv1 = sub2(uv2, uv1), duv2 = sub2(uv3, uv1);
    float det = duv1.x * duv2.y - duv1.y * duv2.x;
    if (fabsf(det) < 1e-8f) {
        v3 n = normalize3(cross3(dp1, dp2));
        v3 tangent = normalize3(dp1);
        v3 bitangent = normalize3(cross3(n, tangent));
        tri->dpdu = tangent;
        tri->dpdv = bitangent;
        return;
    }
    float invDet = 1.0f / det;
    tri->dpdu = muls3(sub3(muls3(dp1, duv2.y), muls3(dp2, duv1.y)), invDet);
    tri->dpdv = muls3(add3(muls3(neg3(dp1), duv2.x), muls3(dp2, duv1.x)), invDet);
}

/* scene.cpp:428-525 */
typedef struct { const pt_triangle* tris; pt_bvh_node* nodes; int32_t count; int32_t* idx; } bvh_builder;

static void bvh_bounds(bvh_builder* b, int start, int end, pt_bvh_node* node) {
    pt_aabb box;
    box.min = V3(FLT_MAX, FLT_MAX, FLT_MAX);
    box.max = V3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (int i = start; i < end; i++) {
        const pt_triangle* t = &b->tris[b->idx[i]];
        box.min = vmin3(box.min, t->v1.position);
        box.min = vmin3(box.min, t->v2.position);
        box.min = vmin3(box.min, t->v3.position);
        box.max = vmax3(box.max, t->v1.position);
        box.max = vmax3(box.max, t->v2.position);
        box.max = vmax3(box.max, t->v3.position);
    }
    node->aabb = box;
}

static int bvh_rec(bvh_builder* b, int start, int end) {
    int nodeIndex = b->count++;
    pt_bvh_node* nn = &b->nodes[nodeIndex];
    memset(nn, 0, sizeof(*nn));
    nn->aabb.min = V3(FLT_MAX, FLT_MAX, FLT_MAX);
    nn->aabb.max = V3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    bvh_bounds(b, start, end, nn);
    int numTris = end - start;
    const int leafThreshold = 4;
    if (numTris <= leafThreshold) {
        nn->start = start; nn->triCount = numTris; nn->left = -1; nn->right = -1;
        return nodeIndex;
    }
    pt_aabb cb;
    cb.min = V3(FLT_MAX, FLT_MAX, FLT_MAX);
    cb.max = V3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (int i = start; i < end; i++) {
        const pt_triangle* t = &b->tris[b->idx[i]];
        cb.min = vmin3(cb.min, t->centroid);
        cb.max = vmax3(cb.max, t->centroid);
    }
    v3 extent = sub3(cb.max, cb.min);
    int axis = 0;
    if (extent.y > extent.x && extent.y > extent.z) axis = 1;
    if (extent.z > extent.x) axis = 2;
    float splitPos = 0.5f * (comp3(cb.min, axis) + comp3(cb.max, axis));
    int mid = start;
    for (int i = start; i < end; i++) {
        int triIndex = b->idx[i];
        if (comp3(b->tris[triIndex].centroid, axis) < splitPos) {
            int tmp = b->idx[i]; b->idx[i] = b->idx[mid]; b->idx[mid] = tmp;
            mid++;
        }
    }
    if (mid == start || mid == end) mid = (start + end) / 2;
    int l = bvh_rec(b, start, mid);
    int r = bvh_rec(b, mid, end);
    nn = &b->nodes[nodeIndex];
    nn->left = l; nn->right = r; nn->start = -1; nn->triCount = 0;
    return nodeIndex;
}

int32_t or_build_bvh(const pt_triangle* tris, int32_t n, pt_bvh_node* nodes, int32_t* tri_indices) {
    for (int i = 0; i < n; i++) tri_indices[i] = i;
    if (n <= 0) return 0;
    bvh_builder b;
    b.tris = tris; b.nodes = nodes; b.count = 0; b.idx = tri_indices;
    bvh_rec(&b, 0, n);
    return b.count;
}

/* scene.cpp:226-363, one OBJ shape after tinyobj triangulation: faces are (v, vt, vn) index
 * triples (0-based, -1 = absent), 3 per face.  Returns triangles written. */
int32_t or_obj_to_triangles(const float* pos, const float* nrm, const float* tex, const int32_t* idx,
                            int32_t nfaces, int32_t materialID, const pt_mat4* transformMatrix,
                            const pt_mat4* invTransposeMatrix, pt_triangle* out) {
    int32_t ntri = 0;
    for (int f = 0; f < nfaces; ++f) {
        pt_vertex fv[3];
        for (int k = 0; k < 3; ++k) {
            const int32_t* ix = idx + (size_t)(f * 3 + k) * 3;
            pt_vertex nv;
            memset(&nv, 0, sizeof(nv));
            int vi = ix[0], ti = ix[1], ni = ix[2];
            v4 p = mat4_mul_v4(transformMatrix, V4(pos[3 * vi + 0], pos[3 * vi + 1], pos[3 * vi + 2], 1.0f));
            nv.position = V3(p.x, p.y, p.z);
            if (ni >= 0) {
                v4 n = mat4_mul_v4(invTransposeMatrix, V4(nrm[3 * ni + 0], nrm[3 * ni + 1], nrm[3 * ni + 2], 0.0f));
                nv.normal = normalize3(V3(n.x, n.y, n.z));
            }
            if (ti >= 0) nv.uv = V2(tex[2 * ti + 0], tex[2 * ti + 1]);
            else nv.uv = V2(0.0f, 0.0f);
            nv.materialID = materialID;
            fv[k] = nv;
        }
        int missing = 1;
        for (int k = 0; k < 3; ++k) if (length3(fv[k].normal) > 1e-6f) { missing = 0; break; }
        if (missing) {
            v3 e1 = sub3(fv[1].position, fv[0].position);
            v3 e2 = sub3(fv[2].position, fv[0].position);
            v3 fn = normalize3(cross3(e1, e2));
            for (int k = 0; k < 3; ++k) fv[k].normal = fn;
        }
        pt_triangle tri;
        memset(&tri, 0, sizeof(tri));
        tri.v1 = fv[0]; tri.v2 = fv[1]; tri.v3 = fv[2];
        tri.centroid = divs3(add3(add3(tri.v1.position, tri.v2.position), tri.v3.position), 3.0f);
        tri.materialID = materialID;
        or_triangle_tangents(&tri);
        out[ntri++] = tri;
    }
    return ntri;
}

void or_mat4_mul_v4(const pt_mat4* m, const pt_vec4* v, pt_vec4* out) { *out = mat4_mul_v4(m, *v); }

/* ------------------------------------------------------------------------------------------ */
/* batch probes for the reference pins (tests/test_ref_pins.py, oracle/ref_pins/ref_harness.cpp) */
/* ------------------------------------------------------------------------------------------ */
/* computeIntersections over n paths into zeroed records (pathtrace.cu:298-448, :699) */
void or_compute_intersections(const or_scene* s, const or_options* o, const pt_path_segment* paths, int32_t n,
                              pt_shadeable_isect* out) {
    memset(out, 0, sizeof(*out) * (size_t)n);
    for (int32_t i = 0; i < n; ++i) or_compute_intersection(s, o, &paths[i], &out[i]);
}
/* per (path, geom): box / sphere test (intersections.cu:3-109) -> {t, point, normal, outside};
 * point / normal / outside are reset on a miss (t == -1), where the reference leaves them unset */
void or_prim_probe(const pt_geom* geoms, int32_t ng, const pt_path_segment* paths, int32_t n, float* out) {
    for (int32_t i = 0; i < n; ++i) {
        for (int32_t g = 0; g < ng; ++g) {
            pt_vec3 p = {0, 0, 0}, nn = {0, 0, 0};
            int32_t outside = 1;
            float t = geoms[g].type == PT_CUBE ? or_box_test(&geoms[g], &paths[i].ray, &p, &nn, &outside)
                                               : or_sphere_test(&geoms[g], &paths[i].ray, &p, &nn, &outside);
            if (t == -1.f) { p = (pt_vec3){0, 0, 0}; nn = (pt_vec3){0, 0, 0}; outside = 1; }
            float* r = out + ((size_t)i * ng + g) * 8;
            r[0] = t; r[1] = p.x; r[2] = p.y; r[3] = p.z; r[4] = nn.x; r[5] = nn.y; r[6] = nn.z;
            memcpy(&r[7], &outside, 4);
        }
    }
}
/* per path: intersectTriangle on triangles [0, nt) -> {hit, t, u, v} (zeros on a miss), then
 * aabbIntersectionTest on nodes [0, nn) -> int (intersections.cu:112-145, 237-275) */
void or_tri_probe(const pt_triangle* tris, int32_t nt, const pt_bvh_node* nodes, int32_t nn,
                  const pt_path_segment* paths, int32_t n, int32_t* out) {
    for (int32_t i = 0; i < n; ++i) {
        int32_t* r = out + (size_t)i * (4 * nt + nn);
        for (int32_t k = 0; k < nt; ++k) {
            float t = 0, u = 0, v = 0;
            int32_t hit = or_triangle_test(&paths[i].ray, &tris[k].v1.position, &tris[k].v2.position,
                                           &tris[k].v3.position, &t, &u, &v);
            if (!hit) t = u = v = 0;
            r[4 * k] = hit;
            memcpy(&r[4 * k + 1], &t, 4);
            memcpy(&r[4 * k + 2], &u, 4);
            memcpy(&r[4 * k + 3], &v, 4);
        }
        for (int32_t k = 0; k < nn; ++k) r[4 * nt + k] = or_aabb_test(&nodes[k].aabb, &paths[i].ray);
    }
}
