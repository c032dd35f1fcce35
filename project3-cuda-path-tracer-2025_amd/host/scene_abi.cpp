// scene_abi.cpp — C-ABI access to the C++ scene loader (for the Python harness and any
// non-C++ caller): load a reference JSON scene, get the flat pt_scene_view pt_init takes.
#include <cstring>
#include <exception>
#include <string>

#include "scene.h"
#include "scene_file.h"
#include "png_decode.h"
#include "image_io.h"

namespace {
thread_local std::string g_scene_err;
}

extern "C" {

const char* pt_scene_last_error(void) { return g_scene_err.c_str(); }

int32_t pt_texture_load(const char* path, int32_t* width, int32_t* height, uint8_t* rgba, int64_t cap) {
    if (!path || !width || !height) return PT_E_INVALID;
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    std::string err;
    if (!ptio::png_load_rgba(path, w, h, px, err)) {
        g_scene_err = err;
        return PT_E_INVALID;
    }
    *width = w;
    *height = h;
    if (rgba && cap >= (int64_t)px.size()) std::memcpy(rgba, px.data(), px.size());
    return PT_OK;
}

// res <= 0 / depth < 0 keep the file's values; viewer_camera != 0 applies main.cpp's camera
// recompute (what every reference frame actually renders with)
int32_t pt_scene_load(const char* path, int32_t resx, int32_t resy, int32_t depth, int32_t viewer_camera,
                      pt_scene_file** out) {
    return pt_scene_load_ex(path, resx, resy, depth, viewer_camera ? PT_SCENE_VIEWER_CAMERA : 0, out);
}

int32_t pt_scene_load_ex(const char* path, int32_t resx, int32_t resy, int32_t depth, int32_t flags,
                         pt_scene_file** out) {
    if (!path || !out) return PT_E_INVALID;
    try {
        Scene* s = new Scene(path, resx, resy, depth, (flags & PT_SCENE_GPU_BVH) != 0);
        if (flags & PT_SCENE_VIEWER_CAMERA) applyViewerCamera(s->state.camera);
        *out = new pt_scene_file{s};
        return PT_OK;
    } catch (const std::exception& e) {
        g_scene_err = e.what();
        return PT_E_INVALID;
    }
}

int32_t pt_scene_get_view(const pt_scene_file* f, pt_scene_view* v) {
    if (!f || !v) return PT_E_INVALID;
    *v = f->scene->view();
    return PT_OK;
}

int32_t pt_scene_get_info(const pt_scene_file* f, int32_t* iterations, int32_t* trace_depth, char* image_name,
                          int32_t cap) {
    if (!f) return PT_E_INVALID;
    if (iterations) *iterations = (int32_t)f->scene->state.iterations;
    if (trace_depth) *trace_depth = f->scene->state.traceDepth;
    if (image_name && cap > 0) {
        std::strncpy(image_name, f->scene->state.imageName.c_str(), (size_t)cap - 1);
        image_name[cap - 1] = 0;
    }
    return PT_OK;
}

int32_t pt_scene_material_name(const pt_scene_file* f, int32_t id, char* buf, int32_t cap) {
    if (!f || id < 0 || id >= (int32_t)f->scene->materialNames.size() || !buf || cap <= 0) return PT_E_INVALID;
    std::strncpy(buf, f->scene->materialNames[id].c_str(), (size_t)cap - 1);
    buf[cap - 1] = 0;
    return PT_OK;
}

// main.cpp:395-419 saveImage + image.cpp:23-43 Image::savePNG: x-flip, divide by the sample
// count, clamp, x255 truncation, PNG bytes as stb_image_write writes them -> "<base_path>.png"
int32_t pt_save_png(const float* image, int32_t width, int32_t height, int32_t iteration, const char* base_path) {
    if (!image || width <= 0 || height <= 0 || !base_path) return PT_E_INVALID;
    std::vector<pt_vec3> img((size_t)width * height);
    std::memcpy(img.data(), image, img.size() * sizeof(pt_vec3));
    const std::vector<unsigned char> rgb = ptio::to_rgb8(img, width, height, (float)iteration);
    if (!ptio::write_png(std::string(base_path) + ".png", rgb, width, height)) {
        g_scene_err = std::string("cannot write ") + base_path + ".png";
        return PT_E_INVALID;
    }
    return PT_OK;
}

void pt_scene_free(pt_scene_file* f) {
    if (!f) return;
    delete f->scene;
    delete f;
}

}  // extern "C"
