/*
 * scene_structs.h — byte-layout-compatible restatement of the reference's scene PODs.
 *
 * Every struct here has exactly the size and field offsets of its counterpart in
 * /root/reference/src/sceneStructs.h (glm 0.9.6 types: vec3 = 3 floats, align 4;
 * mat4 = 4 column vec4s, column-major).  The C-ABI (pathtrace_abi.h) takes arrays of
 * these so a caller holding the reference's std::vector<Geom>/<Material>/... can hand
 * them over with a reinterpret_cast and no copy.
 *
 *   pt_ray                  <- Ray                   sceneStructs.h:18-22    (24 B)
 *   pt_geom                 <- Geom                  sceneStructs.h:24-34    (236 B)
 *   pt_material             <- Material              sceneStructs.h:36-57    (72 B)
 *   pt_vertex               <- Vertex                sceneStructs.h:69-75    (36 B)
 *   pt_triangle             <- Triangle              sceneStructs.h:78-88    (148 B)
 *   pt_aabb                 <- AABB                  sceneStructs.h:90-93    (24 B)
 *   pt_bvh_node             <- BVHNode               sceneStructs.h:95-101   (40 B)
 *   pt_camera               <- Camera                sceneStructs.h:103-117  (92 B)
 *   pt_path_segment         <- PathSegment           sceneStructs.h:128-134  (44 B)
 *   pt_shadeable_isect      <- ShadeableIntersection sceneStructs.h:147-157  (52 B)
 *
 * Plain C (C99) so the oracle, the C++ host code and the HIP kernels all include it.
 */
#ifndef PT_SCENE_STRUCTS_H
#define PT_SCENE_STRUCTS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float x, y; } pt_vec2;
typedef struct { float x, y, z; } pt_vec3;
typedef struct { float x, y, z, w; } pt_vec4;
typedef struct { int32_t x, y; } pt_ivec2;
/* column-major like glm: m[col][row] */
typedef struct { float m[4][4]; } pt_mat4;

/* GeomType, sceneStructs.h:12-16 */
enum { PT_SPHERE = 0, PT_CUBE = 1 };

typedef struct { pt_vec3 origin; pt_vec3 direction; } pt_ray;

typedef struct {
    int32_t type;              /* PT_SPHERE / PT_CUBE */
    int32_t materialid;
    pt_vec3 translation;
    pt_vec3 rotation;
    pt_vec3 scale;
    pt_mat4 transform;
    pt_mat4 inverseTransform;
    pt_mat4 invTranspose;
} pt_geom;

typedef struct {
    pt_vec3 color;
    struct { float exponent; pt_vec3 color; } specular;
    float hasReflective;
    float hasRefractive;
    float roughness;           /* reference default -1 (sceneStructs.h:48) */
    float metallic;            /* reference default -1 (sceneStructs.h:49) */
    float indexOfRefraction;
    float emittance;
    uint8_t hasTexture;        /* C++ bool */
    uint8_t _pad0[3];
    int32_t textureID;         /* default -1 */
    uint8_t hasBumpMap;        /* C++ bool */
    uint8_t _pad1[3];
    int32_t bumpID;            /* default -1 */
    float bumpScale;           /* default 0.5 */
} pt_material;

typedef struct {
    int32_t width, height, channels;
    int32_t _pad;
    const uint8_t* data;       /* host RGBA8 pixels (stbi_load(..., STBI_rgb_alpha)) */
} pt_texture;

typedef struct {
    int32_t materialID;
    pt_vec3 position;
    pt_vec3 normal;
    pt_vec2 uv;
} pt_vertex;

typedef struct {
    pt_vertex v1, v2, v3;
    pt_vec3 centroid;
    int32_t materialID;
    pt_vec3 dpdu;
    pt_vec3 dpdv;
} pt_triangle;

typedef struct { pt_vec3 min; pt_vec3 max; } pt_aabb;

typedef struct {
    pt_aabb aabb;
    int32_t left;
    int32_t right;
    int32_t start;
    int32_t triCount;
} pt_bvh_node;

typedef struct {
    pt_ivec2 resolution;
    pt_vec3 position;
    pt_vec3 lookAt;
    pt_vec3 view;
    pt_vec3 up;
    pt_vec3 right;
    pt_vec2 fov;
    pt_vec2 pixelLength;
    float aperture;
    float focalDist;
} pt_camera;

typedef struct {
    pt_ray ray;
    pt_vec3 color;             /* throughput */
    int32_t pixelIndex;
    int32_t remainingBounces;
} pt_path_segment;

typedef struct {
    float t;
    pt_vec3 surfaceNormal;
    int32_t materialId;
    pt_vec2 uv;
    pt_vec3 dpdu;
    pt_vec3 dpdv;
} pt_shadeable_isect;

/* uchar4 written by sendImageToPBO (pathtrace.cu:59-80) */
typedef struct { uint8_t x, y, z, w; } pt_uchar4;

#ifdef __cplusplus
}  /* extern "C" */
#define PT_STATIC_ASSERT static_assert
#else
#define PT_STATIC_ASSERT _Static_assert
#endif

/* Layout contract with sceneStructs.h (sizes measured from the reference with sizeof). */
PT_STATIC_ASSERT(sizeof(pt_ray) == 24, "Ray");
PT_STATIC_ASSERT(sizeof(pt_geom) == 236, "Geom");
PT_STATIC_ASSERT(sizeof(pt_material) == 72, "Material");
PT_STATIC_ASSERT(sizeof(pt_vertex) == 36, "Vertex");
PT_STATIC_ASSERT(sizeof(pt_triangle) == 148, "Triangle");
PT_STATIC_ASSERT(sizeof(pt_aabb) == 24, "AABB");
PT_STATIC_ASSERT(sizeof(pt_bvh_node) == 40, "BVHNode");
PT_STATIC_ASSERT(sizeof(pt_camera) == 92, "Camera");
PT_STATIC_ASSERT(sizeof(pt_path_segment) == 44, "PathSegment");
PT_STATIC_ASSERT(sizeof(pt_shadeable_isect) == 52, "ShadeableIntersection");

#endif /* PT_SCENE_STRUCTS_H */
