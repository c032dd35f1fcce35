/*
 * pt_viewer.h — the reference's interactive viewer (src/main.cpp:203-555) without a window:
 * the camera-control state machine of its GLFW callbacks, runCuda()'s camera recompute and
 * pathtraceFree/pathtraceInit restart, the per-frame pathtrace call, saveImage, the window
 * title and the displayed pixels, driven by the caller instead of glfwPollEvents.
 *
 *   main.cpp:359-380  pt_viewer_create    phi / theta / zoom / ogLookAt from the loaded camera
 *   main.cpp:481-502  pt_viewer_key       ESC (save + close), S (save), SPACE (re-centre lookAt)
 *   main.cpp:504-514  pt_viewer_mouse_button
 *   main.cpp:516-555  pt_viewer_cursor_pos  left: orbit, right: zoom, middle: pan lookAt
 *   main.cpp:421-444  pt_viewer_update_camera  the camchanged block of runCuda (host math only)
 *   main.cpp:421-475  pt_viewer_run_frame      runCuda(): restart on iteration 0, one pathtrace
 *                                              call per display frame, save + exit at ITERATIONS
 *   main.cpp:302-326  pt_viewer_display / pt_viewer_title: what mainLoop draws from the PBO
 *   main.cpp:395-419  pt_viewer_save_image   saveImage's file name and PNG
 *
 * Button / key / action codes are GLFW's.  ImGui's mouse capture (main.cpp:506) never applies:
 * there is no ImGui panel.  A viewer drives the library's process-global path tracer (one
 * viewer at a time, like the reference's one window).  Everything but pt_viewer_run_frame and
 * pt_viewer_display is host code and runs without a GPU.
 */
#ifndef PT_VIEWER_H
#define PT_VIEWER_H

#include <stdint.h>

#include "pt/pathtrace_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { PT_GLFW_RELEASE = 0, PT_GLFW_PRESS = 1 };
enum { PT_GLFW_MOUSE_BUTTON_LEFT = 0, PT_GLFW_MOUSE_BUTTON_RIGHT = 1, PT_GLFW_MOUSE_BUTTON_MIDDLE = 2 };
enum { PT_GLFW_KEY_SPACE = 32, PT_GLFW_KEY_S = 83, PT_GLFW_KEY_ESCAPE = 256 };

typedef struct pt_viewer pt_viewer;

typedef struct pt_viewer_state {
    float zoom, theta, phi;          /* main.cpp:40 */
    int32_t iteration;               /* main.cpp:47 (frames accumulated since the last restart) */
    int32_t camchanged;              /* main.cpp:36 */
    int32_t left, right, middle;     /* main.cpp:30-32 */
    double last_x, last_y;           /* main.cpp:33-34 */
    int32_t should_close;            /* glfwSetWindowShouldClose (ESC) */
    int32_t exited;                  /* runCuda reached ITERATIONS: saved, freed, exit(EXIT_SUCCESS) */
    int32_t traced_depth;            /* GuiDataContainer::TracedDepth (ImGui "Traced Depth") */
    int32_t saved_images;            /* saveImage calls so far */
    pt_vec3 og_look_at;              /* main.cpp:42 */
    pt_camera camera;                /* renderState->camera */
} pt_viewer_state;

/* main.cpp:343-387 after Scene loading: takes the scene as LOADED (pt_scene_load with
 * viewer_camera = 0; the viewer applies the camera recompute itself at its first frame, as
 * camchanged starts true).  The viewer borrows `scene` (it edits its camera, like the
 * reference's renderState) until pt_viewer_destroy.  `image_dir` replaces saveImage's "../img";
 * `time_tag` replaces startTimeString (NULL: currentTimeString(), "%Y-%m-%d_%H-%M-%Sz" UTC now).
 * `opts` NULL: pt_default_options. */
int32_t pt_viewer_create(pt_scene_file* scene, const pt_options* opts, const char* image_dir, const char* time_tag,
                         pt_viewer** out);
/* frees the viewer and, if it initialised the path tracer, pt_free */
void pt_viewer_destroy(pt_viewer* v);

int32_t pt_viewer_mouse_button(pt_viewer* v, int32_t button, int32_t action, int32_t mods);
int32_t pt_viewer_cursor_pos(pt_viewer* v, double xpos, double ypos);
int32_t pt_viewer_key(pt_viewer* v, int32_t key, int32_t scancode, int32_t action, int32_t mods);

/* runCuda's camchanged block alone (main.cpp:423-444): *reset = 1 when it ran (iteration -> 0) */
int32_t pt_viewer_update_camera(pt_viewer* v, int32_t* reset);
/* one runCuda() (main.cpp:421-475): *exited = 1 when ITERATIONS were reached (the image was saved
 * and the tracer freed; the reference exits the process there) */
int32_t pt_viewer_run_frame(pt_viewer* v, int32_t* exited);

/* the window's pixels as mainLoop draws the PBO (main.cpp:93-104, 302-326): width*height RGB8,
 * top row first, x mirrored (the quad's texcoords), sendImageToPBO's clamp(int(pix/iter*255))
 * values; cap >= width*height*3 */
int32_t pt_viewer_display(const pt_viewer* v, uint8_t* rgb, int64_t cap);
/* "CIS565 Path Tracer | <iteration> Iterations" (main.cpp:310) */
int32_t pt_viewer_title(const pt_viewer* v, char* buf, int32_t cap);
int32_t pt_viewer_get_state(const pt_viewer* v, pt_viewer_state* out);
/* saveImage (main.cpp:395-419): "<image_dir>/<imageName>.<time_tag>.<samples>samp.png"; the
 * accumulated host image (state.image) divided by the iteration count.  The written path (without
 * ".png") is copied into path_out when given. */
int32_t pt_viewer_save_image(pt_viewer* v, char* path_out, int32_t cap);
const char* pt_viewer_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PT_VIEWER_H */
