// viewer.cpp — the reference's interactive viewer (src/main.cpp) without GLFW / OpenGL / ImGui:
// its camera-control state machine, runCuda(), saveImage and the pixels mainLoop draws, driven
// through include/pt/pt_viewer.h.  Float operations follow main.cpp statement by statement
// (glm 0.9.6 order, hmath.h); -ffp-contract=off keeps every rounding where the reference has it.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <sstream>
#include <string>
#include <vector>

#include "hmath.h"
#include "image_io.h"
#include "pt/pt_viewer.h"
#include "scene_file.h"

using namespace pth;

namespace {
thread_local std::string g_viewer_err;
constexpr float kPI = 3.1415926535897932384626422832795028841971f;   // utilities.h:7

int fail(int rc, const std::string& msg) {
    g_viewer_err = msg;
    return rc;
}

// main.cpp:69-76
std::string current_time_string() {
    time_t now;
    time(&now);
    char buf[sizeof "0000-00-00_00-00-00z"];
    strftime(buf, sizeof buf, "%Y-%m-%d_%H-%M-%Sz", gmtime(&now));
    return std::string(buf);
}
}  // namespace

struct pt_viewer {
    Scene* scene = nullptr;          // borrowed (main.cpp:44 Scene* scene)
    pt_options opts{};
    std::string image_dir, start_time;
    // main.cpp:29-47
    bool left = false, right = false, middle = false;
    double lastX = 0.0, lastY = 0.0;
    bool camchanged = true;
    float zoom = 0.f, theta = 0.f, phi = 0.f;
    v3 cameraPosition{}, ogLookAt{};
    int iteration = 0;
    int width = 0, height = 0;
    bool should_close = false, exited = false, initialised = false;
    int traced_depth = 0, saved = 0;
    void* pbo = nullptr;             // device uchar4[width*height] (the GL PBO's role)
    std::vector<pt_uchar4> shown;    // last PBO contents read back for pt_viewer_display
    bool have_frame = false;
};

extern "C" {

const char* pt_viewer_last_error(void) { return g_viewer_err.c_str(); }

int32_t pt_viewer_create(pt_scene_file* sf, const pt_options* opts, const char* image_dir, const char* time_tag,
                         pt_viewer** out) {
    if (!sf || !sf->scene || !out) return fail(PT_E_INVALID, "pt_viewer_create: null argument");
    pt_viewer* v = new pt_viewer;
    v->scene = sf->scene;
    if (opts) v->opts = *opts; else pt_default_options(&v->opts);
    v->image_dir = image_dir ? image_dir : "../img";
    v->start_time = time_tag ? time_tag : current_time_string();   // main.cpp:342
    // main.cpp:359-380
    Camera& cam = v->scene->state.camera;
    v->width = cam.resolution.x;
    v->height = cam.resolution.y;
    v3 view = cam.view;
    v3 up = cam.up;
    v3 right = cross(view, up);
    up = cross(right, view);
    (void)up;
    v->cameraPosition = cam.position;
    v3 viewXZ = V3(view.x, 0.0f, view.z);
    v3 viewZY = V3(0.0f, view.y, view.z);
    v->phi = std::acos(dot(normalize(viewXZ), V3(0, 0, -1)));
    v->theta = std::acos(dot(normalize(viewZY), V3(0, 1, 0)));
    v->ogLookAt = cam.lookAt;
    v->zoom = length(cam.position - v->ogLookAt);
    v->scene->state.image.assign((size_t)v->width * v->height, pt_vec3{0.f, 0.f, 0.f});
    pt_init_data_container(&v->traced_depth);   // main.cpp:386-387 InitDataContainer(guiData)
    *out = v;
    return PT_OK;
}

void pt_viewer_destroy(pt_viewer* v) {
    if (!v) return;
    if (v->initialised) pt_free();
    if (v->pbo) pt_device_free(v->pbo);
    pt_init_data_container(nullptr);
    delete v;
}

// main.cpp:504-514 (no ImGui window to capture the mouse)
int32_t pt_viewer_mouse_button(pt_viewer* v, int32_t button, int32_t action, int32_t mods) {
    (void)mods;
    if (!v) return fail(PT_E_INVALID, "null viewer");
    v->left = (button == PT_GLFW_MOUSE_BUTTON_LEFT && action == PT_GLFW_PRESS);
    v->right = (button == PT_GLFW_MOUSE_BUTTON_RIGHT && action == PT_GLFW_PRESS);
    v->middle = (button == PT_GLFW_MOUSE_BUTTON_MIDDLE && action == PT_GLFW_PRESS);
    return PT_OK;
}

// main.cpp:516-555
int32_t pt_viewer_cursor_pos(pt_viewer* v, double xpos, double ypos) {
    if (!v) return fail(PT_E_INVALID, "null viewer");
    if (xpos == v->lastX || ypos == v->lastY) return PT_OK;   // clicking back into the window
    if (v->left) {
        v->phi -= (xpos - v->lastX) / v->width;                  // float -= double (rounded once)
        v->theta -= (ypos - v->lastY) / v->height;
        v->theta = std::fmax(0.001f, std::fmin(v->theta, kPI));
        v->camchanged = true;
    } else if (v->right) {
        v->zoom += (ypos - v->lastY) / v->height;
        v->zoom = std::fmax(0.1f, v->zoom);
        v->camchanged = true;
    } else if (v->middle) {
        Camera& cam = v->scene->state.camera;
        v3 forward = cam.view;
        forward.y = 0.0f;
        forward = normalize(forward);
        v3 right = cam.right;
        right.y = 0.0f;
        right = normalize(right);
        // (float * vec3) * float, then -= / += componentwise
        cam.lookAt = cam.lookAt - (right * (float)(xpos - v->lastX)) * 0.01f;
        cam.lookAt = cam.lookAt + (forward * (float)(ypos - v->lastY)) * 0.01f;
        v->camchanged = true;
    }
    v->lastX = xpos;
    v->lastY = ypos;
    return PT_OK;
}

// main.cpp:481-502
int32_t pt_viewer_key(pt_viewer* v, int32_t key, int32_t scancode, int32_t action, int32_t mods) {
    (void)scancode;
    (void)mods;
    if (!v) return fail(PT_E_INVALID, "null viewer");
    if (action != PT_GLFW_PRESS) return PT_OK;
    switch (key) {
        case PT_GLFW_KEY_ESCAPE: {
            const int rc = pt_viewer_save_image(v, nullptr, 0);
            v->should_close = true;
            return rc;
        }
        case PT_GLFW_KEY_S:
            return pt_viewer_save_image(v, nullptr, 0);
        case PT_GLFW_KEY_SPACE:
            v->camchanged = true;
            v->scene->state.camera.lookAt = v->ogLookAt;
            return PT_OK;
        default:
            return PT_OK;
    }
}

// main.cpp:423-444
int32_t pt_viewer_update_camera(pt_viewer* v, int32_t* reset) {
    if (!v) return fail(PT_E_INVALID, "null viewer");
    if (reset) *reset = 0;
    if (!v->camchanged) return PT_OK;
    v->iteration = 0;
    Camera& cam = v->scene->state.camera;
    // float overloads of sin / cos (CUDA's and MSVC's headers), as applyViewerCamera
    v->cameraPosition.x = v->zoom * std::sin(v->phi) * std::sin(v->theta);
    v->cameraPosition.y = v->zoom * std::cos(v->theta);
    v->cameraPosition.z = v->zoom * std::cos(v->phi) * std::sin(v->theta);
    cam.view = -normalize(v->cameraPosition);
    v3 vv = cam.view;
    v3 u = V3(0, 1, 0);
    v3 r = cross(vv, u);
    cam.up = cross(r, vv);
    cam.right = r;
    cam.position = v->cameraPosition;
    v->cameraPosition = v->cameraPosition + cam.lookAt;
    cam.position = v->cameraPosition;
    v->camchanged = false;
    cam.focalDist = length(cam.lookAt - cam.position);
    if (reset) *reset = 1;
    return PT_OK;
}

// main.cpp:421-475
int32_t pt_viewer_run_frame(pt_viewer* v, int32_t* exited) {
    if (!v) return fail(PT_E_INVALID, "null viewer");
    if (exited) *exited = v->exited ? 1 : 0;
    if (v->exited) return fail(PT_E_STATE, "the viewer reached ITERATIONS and exited");
    int rc = pt_viewer_update_camera(v, nullptr);
    if (rc != PT_OK) return rc;
    if (v->iteration == 0) {   // pathtraceFree(); pathtraceInit(scene)
        if (v->initialised) {
            pt_free();
            v->initialised = false;
        }
        pt_scene_view view = v->scene->view();
        rc = pt_init(&view, &v->opts);
        if (rc != PT_OK) return fail(rc, std::string("pathtraceInit: ") + pt_last_error());
        v->initialised = true;
        if (!v->pbo) {
            const size_t bytes = sizeof(pt_uchar4) * (size_t)v->width * v->height;
            rc = pt_device_alloc((int64_t)bytes, &v->pbo);
            if (rc != PT_OK) return fail(rc, std::string("display PBO: ") + pt_last_error());
        }
    }
    if (v->iteration < (int)v->scene->state.iterations) {
        v->iteration++;
        rc = pt_set_camera(&v->scene->state.camera);   // pathtrace re-reads the Scene's camera
        if (rc == PT_OK)
            rc = pt_trace(static_cast<pt_uchar4*>(v->pbo), 0, v->iteration, &v->scene->state.image[0].x);
        if (rc != PT_OK) return fail(rc, std::string("pathtrace: ") + pt_last_error());
        // mainLoop uploads the PBO into the window's texture (main.cpp:312-314)
        v->shown.resize((size_t)v->width * v->height);
        rc = pt_device_read(v->shown.data(), v->pbo, (int64_t)(sizeof(pt_uchar4) * v->shown.size()));
        if (rc != PT_OK) return fail(rc, std::string("PBO readback: ") + pt_last_error());
        v->have_frame = true;
    } else {
        rc = pt_viewer_save_image(v, nullptr, 0);
        pt_free();
        v->initialised = false;
        v->exited = true;
        if (exited) *exited = 1;
        return rc;
    }
    return PT_OK;
}

int32_t pt_viewer_display(const pt_viewer* v, uint8_t* rgb, int64_t cap) {
    if (!v || !rgb) return fail(PT_E_INVALID, "null argument");
    const int64_t need = (int64_t)v->width * v->height * 3;
    if (cap < need) return fail(PT_E_INVALID, "display buffer too small");
    if (!v->have_frame) return fail(PT_E_STATE, "no frame traced yet");
    // quad texcoords (main.cpp:99-104): the window's top row is PBO row 0, its left column the
    // PBO's last column
    for (int y = 0; y < v->height; ++y)
        for (int X = 0; X < v->width; ++X) {
            const pt_uchar4& p = v->shown[(size_t)y * v->width + (v->width - 1 - X)];
            uint8_t* o = rgb + 3 * ((size_t)y * v->width + X);
            o[0] = p.x;
            o[1] = p.y;
            o[2] = p.z;
        }
    return PT_OK;
}

int32_t pt_viewer_title(const pt_viewer* v, char* buf, int32_t cap) {
    if (!v || !buf || cap <= 0) return fail(PT_E_INVALID, "null argument");
    const std::string t = "CIS565 Path Tracer | " + std::to_string(v->iteration) + " Iterations";
    std::strncpy(buf, t.c_str(), (size_t)cap - 1);
    buf[cap - 1] = 0;
    return PT_OK;
}

int32_t pt_viewer_get_state(const pt_viewer* v, pt_viewer_state* o) {
    if (!v || !o) return fail(PT_E_INVALID, "null argument");
    std::memset(o, 0, sizeof *o);
    o->zoom = v->zoom;
    o->theta = v->theta;
    o->phi = v->phi;
    o->iteration = v->iteration;
    o->camchanged = v->camchanged;
    o->left = v->left;
    o->right = v->right;
    o->middle = v->middle;
    o->last_x = v->lastX;
    o->last_y = v->lastY;
    o->should_close = v->should_close;
    o->exited = v->exited;
    o->traced_depth = v->traced_depth;
    o->saved_images = v->saved;
    o->og_look_at = v->ogLookAt;
    o->camera = v->scene->state.camera;
    return PT_OK;
}

// main.cpp:395-419
int32_t pt_viewer_save_image(pt_viewer* v, char* path_out, int32_t cap) {
    if (!v) return fail(PT_E_INVALID, "null viewer");
    float samples = v->iteration;
    std::ostringstream ss;
    ss << v->scene->state.imageName << "." << v->start_time << "." << samples << "samp";
    const std::string filename = v->image_dir + "/" + ss.str();
    const std::vector<unsigned char> rgb = ptio::to_rgb8(v->scene->state.image, v->width, v->height, samples);
    if (!ptio::write_png(filename + ".png", rgb, v->width, v->height))
        return fail(PT_E_INVALID, "cannot write " + filename + ".png");
    std::printf("Saved %s.png.\n", filename.c_str());   // image.cpp:42
    v->saved++;
    if (path_out && cap > 0) {
        std::strncpy(path_out, filename.c_str(), (size_t)cap - 1);
        path_out[cap - 1] = 0;
    }
    return PT_OK;
}

}  // extern "C"
