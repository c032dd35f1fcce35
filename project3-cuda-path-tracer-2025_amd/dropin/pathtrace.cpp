// dropin/pathtrace.cpp — the drop-in replacement for the reference's src/pathtrace.cu.
//
// Compiled INSIDE the application's build, against the application's own headers: it includes
// the reference's "pathtrace.h" (-> scene.h -> sceneStructs.h with glm, utilities.h), so the four
// entry points below have exactly the signatures main.cpp calls (src/pathtrace.h:6-9) —
// including whatever `uchar4` the application's toolchain defines — and link against
// libptamd.so (C-ABI, include/pt/pathtrace_abi.h).  A maintainer replaces src/pathtrace.cu with
// this file in the source list and adds -I<framework>/include -lptamd.
//
//   InitDataContainer(GuiDataContainer*)   pathtrace.cu:103-106   -> pt_init_data_container
//   pathtraceInit(Scene*)                  pathtrace.cu:134-207   -> pt_init
//   pathtraceFree()                        pathtrace.cu:209-229   -> pt_free
//   pathtrace(uchar4*, int, int)           pathtrace.cu:639-787   -> pt_set_camera + pt_trace
//
// The reference's Scene vectors are handed over without a copy: their element types have the
// byte layout of the pt_* records (checked below, and field by field against sceneStructs.h in
// tests/test_ref_pins.py::test_struct_layout_matches_reference).  Behaviour follows pathtrace.cu:
// a non-owning Scene*, the trace depth and the camera re-read on every frame, scene->state.image overwritten with the
// accumulated image on every frame, and on any error a message then exit(EXIT_FAILURE)
// (checkCUDAErrorFn, pathtrace.cu:27-49).
#include "pathtrace.h"

#include <cstdio>
#include <cstdlib>

#include "pt/pathtrace_abi.h"

static_assert(sizeof(Geom) == sizeof(pt_geom), "Geom layout");
static_assert(sizeof(Material) == sizeof(pt_material), "Material layout");
static_assert(sizeof(Texture) == sizeof(pt_texture), "Texture layout");
static_assert(sizeof(Triangle) == sizeof(pt_triangle), "Triangle layout");
static_assert(sizeof(BVHNode) == sizeof(pt_bvh_node), "BVHNode layout");
static_assert(sizeof(Camera) == sizeof(pt_camera), "Camera layout");
static_assert(sizeof(glm::vec3) == 3 * sizeof(float), "image pixel layout");
static_assert(sizeof(uchar4) == sizeof(pt_uchar4), "PBO pixel layout");

namespace {
Scene* hst_scene = nullptr;     // non-owning (pathtrace.cu:82, 136)

void check(int rc, const char* msg, int line) {
    if (rc == PT_OK) return;
    std::fprintf(stderr, "HIP error (%s:%d): %s: %s\n", __FILE__, line, msg, pt_last_error());
    std::exit(EXIT_FAILURE);
}
#define PT_CHECK(rc, msg) check((rc), (msg), __LINE__)

template <class T, class U>
const U* as(const std::vector<T>& v) {
    return v.empty() ? nullptr : reinterpret_cast<const U*>(v.data());
}
}  // namespace

void InitDataContainer(GuiDataContainer* guiData) {
    PT_CHECK(pt_init_data_container(guiData ? &guiData->TracedDepth : nullptr), "InitDataContainer");
}

void pathtraceInit(Scene* scene) {
    hst_scene = scene;
    pt_scene_view v{};
    v.geoms = as<Geom, pt_geom>(scene->geoms);
    v.num_geoms = (int32_t)scene->geoms.size();
    v.materials = as<Material, pt_material>(scene->materials);
    v.num_materials = (int32_t)scene->materials.size();
    v.textures = as<Texture, pt_texture>(scene->textures);
    v.num_textures = (int32_t)scene->textures.size();
    v.triangles = as<Triangle, pt_triangle>(scene->triangles);
    v.num_triangles = (int32_t)scene->triangles.size();
    v.tri_indices = scene->triIndices.empty() ? nullptr : scene->triIndices.data();
    v.num_tri_indices = (int32_t)scene->triIndices.size();
    v.bvh_nodes = as<BVHNode, pt_bvh_node>(scene->bvhNodes);
    v.num_bvh_nodes = (int32_t)scene->bvhNodes.size();
    v.camera = *reinterpret_cast<const pt_camera*>(&scene->state.camera);
    v.trace_depth = scene->state.traceDepth;
    pt_options o;
    pt_default_options(&o);
    PT_CHECK(pt_init(&v, &o), "pathtraceInit");
}

void pathtraceFree() { PT_CHECK(pt_free(), "pathtraceFree"); }

void pathtrace(uchar4* pbo, int frame, int iteration) {
    if (!hst_scene) PT_CHECK(PT_E_STATE, "pathtrace before pathtraceInit");
    // the trace depth and the camera are re-read from the Scene every frame (pathtrace.cu:641-642)
    PT_CHECK(pt_set_trace_depth(hst_scene->state.traceDepth), "pathtrace traceDepth");
    PT_CHECK(pt_set_camera(reinterpret_cast<const pt_camera*>(&hst_scene->state.camera)), "pathtrace camera");
    float* img = hst_scene->state.image.empty() ? nullptr : &hst_scene->state.image[0].x;
    PT_CHECK(pt_trace(reinterpret_cast<pt_uchar4*>(pbo), frame, iteration, img), "pathtrace");
}
