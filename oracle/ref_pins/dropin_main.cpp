// dropin_main.cpp — TEST INFRASTRUCTURE: a main.cpp-shaped, headless caller of the drop-in.
//
// Built by oracle/ref_pins/make_fixtures.sh into oracle/_ref/dropin_main from the reference's own
// headers and host sources (src/scene.cpp, utilities.cpp, stb.cpp: the Scene the application
// hands over) plus project3-cuda-path-tracer-2025_amd/dropin/pathtrace.cpp, linked against
// libptamd.so.  It makes exactly the calls of src/main.cpp — the camera set-up of :359-380, then
// runCuda (:421-475): camera recompute, pathtraceFree + pathtraceInit at iteration 0, one
// pathtrace(pbo, 0, iteration) per frame, pathtraceFree at the end — minus GLFW / ImGui / the GL
// PBO (pbo = NULL, the headless case the drop-in accepts).
//
//   dropin_main <scene.json> <frames> <out.f32> [F:D]  -> writes scene->state.image after the last
//                                                    frame and prints "traced_depth <n>"; with F:D
//                                                    the caller sets state.traceDepth = D before
//                                                    frame F (the reference re-reads it per frame,
//                                                    pathtrace.cu:641)
#include "pathtrace.h"

#include <cstdio>
#include <cstdlib>

int main(int argc, char** argv) {
    if (argc != 4 && argc != 5) {
        std::printf("Usage: %s SCENEFILE.json FRAMES OUT.f32 [FRAME:DEPTH]\n", argv[0]);
        return 1;
    }
    int depth_frame = -1, depth_value = 0;
    if (argc == 5 && std::sscanf(argv[4], "%d:%d", &depth_frame, &depth_value) != 2) return 1;
    Scene* scene = new Scene(argv[1]);
    GuiDataContainer* guiData = new GuiDataContainer();
    RenderState* renderState = &scene->state;
    Camera& cam = renderState->camera;

    // main.cpp:359-380
    glm::vec3 view = cam.view;
    glm::vec3 up = cam.up;
    glm::vec3 right = glm::cross(view, up);
    up = glm::cross(right, view);
    glm::vec3 cameraPosition = cam.position;
    glm::vec3 viewXZ = glm::vec3(view.x, 0.0f, view.z);
    glm::vec3 viewZY = glm::vec3(0.0f, view.y, view.z);
    float phi = glm::acos(glm::dot(glm::normalize(viewXZ), glm::vec3(0, 0, -1)));
    float theta = glm::acos(glm::dot(glm::normalize(viewZY), glm::vec3(0, 1, 0)));
    glm::vec3 ogLookAt = cam.lookAt;
    float zoom = glm::length(cam.position - ogLookAt);
    (void)right;
    (void)up;

    InitDataContainer(guiData);   // main.cpp:387

    const int frames = std::atoi(argv[2]);
    int iteration = 0;
    bool camchanged = true;
    while (true) {   // runCuda, main.cpp:421-475
        if (camchanged) {
            iteration = 0;
            // float overloads, as MSVC's <cmath> gives main.cpp's unqualified calls (the reference
            // was built on Windows 10, README.md:19); g++ alone would pick ::sin(double)
            cameraPosition.x = zoom * std::sin(phi) * std::sin(theta);
            cameraPosition.y = zoom * std::cos(theta);
            cameraPosition.z = zoom * std::cos(phi) * std::sin(theta);
            cam.view = -glm::normalize(cameraPosition);
            glm::vec3 v = cam.view;
            glm::vec3 u = glm::vec3(0, 1, 0);
            glm::vec3 r = glm::cross(v, u);
            cam.up = glm::cross(r, v);
            cam.right = r;
            cam.position = cameraPosition;
            cameraPosition += cam.lookAt;
            cam.position = cameraPosition;
            camchanged = false;
            cam.focalDist = glm::length(cam.lookAt - cam.position);
        }
        if (iteration == 0) {
            pathtraceFree();
            pathtraceInit(scene);
        }
        if (iteration < frames) {
            uchar4* pbo_dptr = NULL;
            iteration++;
            if (iteration == depth_frame) renderState->traceDepth = depth_value;
            pathtrace(pbo_dptr, 0, iteration);
        } else {
            break;
        }
    }
    std::FILE* f = std::fopen(argv[3], "wb");
    if (!f) return 2;
    std::fwrite(renderState->image.data(), sizeof(glm::vec3), renderState->image.size(), f);
    std::fclose(f);
    std::printf("traced_depth %d\n", guiData->TracedDepth);
    pathtraceFree();
    delete guiData;
    delete scene;
    return 0;
}
