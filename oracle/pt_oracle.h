/*
 * pt_oracle.h — CPU restatement of the reference's wavefront path-tracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library, and only as the checker / CPU baseline — never as the product.
 *
 * Parity status (details in DESIGN.md "Oracle"):
 *   - RNG (utilhash + thrust::default_random_engine + uniform_real_distribution<float>):
 *     pinned bit-exactly against rocThrust (THRUST_VERSION 200805, the implementation in this
 *     image of the reference's third-party Thrust dependency) by oracle/ref_pins/rng_pin.cpp ->
 *     tests/golden/rng_pin.json.
 *   - glm 0.9.6 semantics (TRS matrices, inverse, inverseTranspose, normalize/reflect/refract),
 *     the camera set-up float order and the alphabetical material ids: pinned bit-exactly
 *     against the reference's own src/utilities.cpp, its vendored glm 0.9.6 and nlohmann json
 *     3.11.3, compiled from /root/reference by oracle/ref_pins/ingest_pin.cpp ->
 *     tests/golden/ingest_pin.json.
 *   - src/intersections.cu (box / sphere / triangle / aabb / BVH tests), src/scene.cpp (OBJ
 *     ingest, tangents, buildBVHRecursive), src/image.cpp (PNG bytes) and the sceneStructs.h
 *     layouts: pinned bit-exactly against the reference's own sources, compiled in place with
 *     g++ and the CUDA runtime headers this image ships (oracle/ref_pins/ref_harness.cpp ->
 *     tests/golden/ref_pin.json, tests/test_ref_pins.py).
 *   - src/interactions.cu (scatterRay and the BSDFs) needs thrust/random.h, which only rocThrust
 *     provides here and which clashes with the CUDA vector types: UNBUILDABLE.  Pinned
 *     statistically instead: the GPU (bit-exact with this oracle in trig_mode 1) renders ten of
 *     the reference authors' own committed 800x800 renders to within 0.16-0.22/255 mean tile
 *     difference (tests/test_ref_renders.py; the sweep of every image against every scene variant
 *     is tests/golden/ref_render_sweep.json): the diffuse branch (interactions.cu:92-108), the
 *     mirror branch (:111-118, :465-470: cornell_multiple_glass's reflective cube), transmissive
 *     (:146-168), glass + Fresnel (:173-235) and the aperture sample (pathtrace.cu:231-237); and the
 *     known answers SURVEY.md §8a records from a run of the reference (cornell per-bounce
 *     live-path counts, glass-scene segment total, first NaN pixel) match exactly
 *     (tests/test_oracle_pins.py).  The Cook-Torrance / microfacet branch (interactions.cu:238-435,
 *     :481-525) matches NO reference-held image (best mean tile difference 17-25/255 with the
 *     camera refitted): PARITY UNPINNED for it beyond this restatement.  Bit-level BSDF parity:
 *     unpinned.
 *
 * Layouts are the reference's own (include/pt/scene_structs.h): AoS PathSegment /
 * ShadeableIntersection, exactly as pathtrace.cu holds them.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include <stdint.h>
#include "pt/scene_structs.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    const pt_geom* geoms;          int32_t num_geoms;
    const pt_material* materials;  int32_t num_materials;
    const pt_triangle* triangles;  int32_t num_triangles;
    const int32_t* tri_indices;    int32_t num_tri_indices;
    const pt_bvh_node* bvh_nodes;  int32_t num_bvh_nodes;
    pt_camera camera;
    int32_t trace_depth;
    int32_t num_textures;
    const pt_texture* textures;    /* RGBA8 (stbi STBI_rgb_alpha) images, scene.cpp:366-392 */
} or_scene;

typedef struct {
    int32_t stream_compaction;   /* STREAM_COMPACTION (pathtrace.cu:21), default 1 */
    int32_t material_sort;       /* MATERIAL_SORTING  (pathtrace.cu:22), default 0 */
    int32_t bvh;                 /* BVH_ACCELERATION  (pathtrace.cu:24), default 1 */
    int32_t trig_mode;           /* 0 = glibc sinf/cosf/powf, 1 = pt_libm (bit-exact with GPU) */
    int32_t arg_order;           /* 0 = glm::vec2(u01(rng), u01(rng)) evaluated right-to-left
                                    (g++, the compiler of the reference build SURVEY measured),
                                    1 = left-to-right */
    int32_t num_threads;         /* OpenMP threads for the per-path loops (0 = default) */
} or_options;

/* ---- RNG (pathtrace.cu:51-56, intersections.h:13-22, thrust minstd_rand + u01) ---- */
uint32_t or_utilhash(uint32_t a);
void or_rng_draws(int32_t iter, int32_t index, int32_t depth, int32_t n, float* out);

/* ---- geometry (intersections.cu) ---- */
float or_box_test(const pt_geom* g, const pt_ray* r, pt_vec3* point, pt_vec3* normal, int32_t* outside);
float or_sphere_test(const pt_geom* g, const pt_ray* r, pt_vec3* point, pt_vec3* normal, int32_t* outside);
int32_t or_triangle_test(const pt_ray* r, const pt_vec3* v0, const pt_vec3* v1, const pt_vec3* v2,
                         float* t, float* u, float* v);
int32_t or_aabb_test(const pt_aabb* b, const pt_ray* r);
void or_compute_intersection(const or_scene* s, const or_options* o, const pt_path_segment* p,
                             pt_shadeable_isect* out);
/* batch probes for the reference pins (tests/test_ref_pins.py) */
void or_compute_intersections(const or_scene* s, const or_options* o, const pt_path_segment* paths, int32_t n,
                              pt_shadeable_isect* out);
void or_prim_probe(const pt_geom* geoms, int32_t ng, const pt_path_segment* paths, int32_t n, float* out);
void or_tri_probe(const pt_triangle* tris, int32_t nt, const pt_bvh_node* nodes, int32_t nn,
                  const pt_path_segment* paths, int32_t n, int32_t* out);

/* ---- shading (pathtrace.cu:521-621 + interactions.cu:438-542) ---- */
void or_shade(const or_scene* s, const or_options* o, int32_t iter, const pt_shadeable_isect* isect,
              pt_path_segment* path);
/* scatterRay on one path, for per-branch known-answer tests */
void or_scatter(const or_options* o, pt_path_segment* path, pt_vec3 intersect, pt_vec3 normal,
                const pt_material* m, int32_t iter);

/* ---- camera rays (pathtrace.cu:231-292) ---- */
void or_generate_ray(const pt_camera* cam, int32_t iter, int32_t trace_depth, int32_t x, int32_t y,
                     const or_options* o, pt_path_segment* out);

/* ---- one pathtrace() call (pathtrace.cu:639-787): accumulates into image[N*3];
 *      live_counts[b] = paths alive entering bounce b (b < trace_depth), -1 past the end;
 *      returns the number of bounces traced. ---- */
int32_t or_pathtrace(const or_scene* s, const or_options* o, int32_t iter, float* image,
                     int32_t* live_counts);
/* frame with the paths array exposed after each bounce (for per-bounce dumps) */
int32_t or_pathtrace_dump(const or_scene* s, const or_options* o, int32_t iter, float* image,
                          int32_t* live_counts, pt_path_segment* paths_after_bounce /* depth*N */);

/* sendImageToPBO (pathtrace.cu:59-80) */
void or_image_to_pbo(const float* image, int32_t n, int32_t iter, pt_uchar4* pbo);

/* ---- stream_compaction/cpu.cu (CPU baseline, config 1) ---- */
void or_cpu_scan(int32_t n, int32_t* odata, const int32_t* idata);
int32_t or_cpu_compact_without_scan(int32_t n, int32_t* odata, const int32_t* idata);
int32_t or_cpu_compact_with_scan(int32_t n, int32_t* odata, const int32_t* idata);

/* ---- scene ingest helpers (scene.cpp, utilities.cpp, main.cpp) ---- */
void or_build_transform(pt_vec3 t, pt_vec3 r, pt_vec3 s, pt_mat4* out);      /* utilities.cpp:85-93 */
void or_mat4_inverse(const pt_mat4* m, pt_mat4* out);                        /* glm compute_inverse */
void or_mat4_inverse_transpose(const pt_mat4* m, pt_mat4* out);              /* glm inverseTranspose */
void or_make_geom(int32_t type, int32_t materialid, pt_vec3 t, pt_vec3 r, pt_vec3 s, pt_geom* g);
/* scene.cpp:184-213 followed by main.cpp:359-380 and the first runCuda() recompute main.cpp:423-444 */
void or_camera_setup(int32_t resx, int32_t resy, float fovy, pt_vec3 eye, pt_vec3 lookat, pt_vec3 up,
                     float aperture, pt_camera* cam);
void or_triangle_tangents(pt_triangle* tri);                                 /* scene.cpp:395-426 */
/* scene.cpp:445-525; nodes must hold 2*n entries; returns node count */
int32_t or_build_bvh(const pt_triangle* tris, int32_t n, pt_bvh_node* nodes, int32_t* tri_indices);

int32_t or_obj_to_triangles(const float* pos, const float* nrm, const float* tex, const int32_t* idx,
                            int32_t nfaces, int32_t materialID, const pt_mat4* transformMatrix,
                            const pt_mat4* invTransposeMatrix, pt_triangle* out);
void or_mat4_mul_v4(const pt_mat4* m, const pt_vec4* v, pt_vec4* out);

/* glm helpers exposed for the glm pin test */
void or_glm_normalize(const pt_vec3* v, pt_vec3* out);
void or_glm_reflect(const pt_vec3* i, const pt_vec3* n, pt_vec3* out);
void or_glm_refract(const pt_vec3* i, const pt_vec3* n, float eta, pt_vec3* out);

#ifdef __cplusplus
}
#endif
#endif /* PT_ORACLE_H */
