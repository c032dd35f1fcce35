// pathtrace_cpp.cpp — the reference's C++ boundary (src/pathtrace.h:6-9) on top of the C-ABI.
#include <cstdio>
#include <cstdlib>

#include "pathtrace.h"

namespace {
Scene* hst_scene = nullptr;            // non-owning, like pathtrace.cu:82
GuiDataContainer* guiData = nullptr;   // pathtrace.cu:83
pt_options g_opts;
bool g_opts_set = false;

void check(int rc, const char* what) {
    if (rc == PT_OK) return;
    std::fprintf(stderr, "HIP error (%s): %s\n", what, pt_last_error());   // checkCUDAError, pathtrace.cu:38-47
    std::exit(EXIT_FAILURE);
}
}  // namespace

void pathtraceSetOptions(const pt_options& opts) {
    g_opts = opts;
    g_opts_set = true;
}

void InitDataContainer(GuiDataContainer* imGuiData) {
    guiData = imGuiData;
    pt_init_data_container(imGuiData ? &imGuiData->TracedDepth : nullptr);
}

void pathtraceInit(Scene* scene) {
    hst_scene = scene;
    if (!g_opts_set) pt_default_options(&g_opts);
    pt_scene_view v = scene->view();
    check(pt_init(&v, &g_opts), "pathtraceInit");
}

void pathtraceFree() { check(pt_free(), "pathtraceFree"); }

void pathtrace(uchar4* pbo, int frame, int iteration) {
    if (!hst_scene) check(PT_E_STATE, "pathtrace before pathtraceInit");
    // the reference re-reads the trace depth and the camera from the Scene every frame (pathtrace.cu:641-642)
    check(pt_set_trace_depth(hst_scene->state.traceDepth), "pathtrace traceDepth");
    check(pt_set_camera(&hst_scene->state.camera), "pathtrace camera");
    float* img = hst_scene->state.image.empty() ? nullptr : &hst_scene->state.image[0].x;
    check(pt_trace(pbo, frame, iteration, img), "pathtrace");
}
