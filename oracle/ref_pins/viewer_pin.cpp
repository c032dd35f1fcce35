// viewer_pin.cpp — TEST INFRASTRUCTURE: pins the headless viewer (include/pt/pt_viewer.h,
// project3-cuda-path-tracer-2025_amd/host/viewer.cpp) to the reference's interactive camera.
//
// Built by oracle/ref_pins/make_fixtures.sh into oracle/_ref/viewer_pin against the reference's
// own headers and host sources: the Scene comes from src/scene.cpp (+ utilities.cpp, stb.cpp) and
// glm is the reference's vendored 0.9.6.  main.cpp's unqualified sin / cos on floats are the
// FLOAT overloads where the reference was built (Windows 10, README.md:19: MSVC's <cmath>
// declares them in the global namespace); g++ would resolve them to ::sin(double), so they are
// spelled std::sin / std::cos here (a 1-ulp difference in view.y otherwise).  main.cpp itself needs
// GLFW / GLEW / ImGui / OpenGL and cannot be built here, so the bodies of its camera code --
// main.cpp:359-380 (set-up), 481-502 (keyCallback), 504-514 (mouseButtonCallback), 516-555
// (mousePositionCallback) and 423-444 (runCuda's camchanged block) -- are restated below
// statement for statement on those types.
//
//   viewer_pin <scene.json> <events.txt>  -> JSON on stdout: after every `frame` event, whether the
//                                            camera was recomputed and the camera / phi / theta / zoom bits
// Event lines: "button B A", "cursor X Y", "key K", "frame [N]" ('#' comments), as pt_render --events.
#include "scene.h"
#include "sceneStructs.h"
#include "utilities.h"

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

static uint32_t bits(float f) { uint32_t b; std::memcpy(&b, &f, 4); return b; }
static void pv3(const char* k, const glm::vec3& v) {
    std::printf("\"%s\": [%u, %u, %u], ", k, bits(v.x), bits(v.y), bits(v.z));
}

// main.cpp:28-47
static bool leftMousePressed = false, rightMousePressed = false, middleMousePressed = false;
static double lastX, lastY;
static bool camchanged = true;
static float zoom, theta, phi;
static glm::vec3 cameraPosition, ogLookAt;
static Scene* scene;
static RenderState* renderState;
static int width, height;

int main(int argc, char** argv) {
    if (argc != 3) {
        std::printf("Usage: %s SCENEFILE.json EVENTS.txt\n", argv[0]);
        return 1;
    }
    scene = new Scene(argv[1]);
    // main.cpp:359-380
    renderState = &scene->state;
    Camera& cam = renderState->camera;
    width = cam.resolution.x;
    height = cam.resolution.y;
    glm::vec3 view = cam.view;
    glm::vec3 up = cam.up;
    glm::vec3 right = glm::cross(view, up);
    up = glm::cross(right, view);
    cameraPosition = cam.position;
    glm::vec3 viewXZ = glm::vec3(view.x, 0.0f, view.z);
    glm::vec3 viewZY = glm::vec3(0.0f, view.y, view.z);
    phi = glm::acos(glm::dot(glm::normalize(viewXZ), glm::vec3(0, 0, -1)));
    theta = glm::acos(glm::dot(glm::normalize(viewZY), glm::vec3(0, 1, 0)));
    ogLookAt = cam.lookAt;
    zoom = glm::length(cam.position - ogLookAt);
    (void)up;

    std::ifstream in(argv[2]);
    std::string line;
    bool first = true;
    std::printf("{\"frames\": [\n");
    while (std::getline(in, line)) {
        const auto hash = line.find('#');
        if (hash != std::string::npos) line.resize(hash);
        std::istringstream ls(line);
        std::string cmd;
        if (!(ls >> cmd)) continue;
        if (cmd == "button") {   // main.cpp:504-514
            int button = 0, action = 0;
            ls >> button >> action;
            leftMousePressed = (button == 0 && action == 1);
            rightMousePressed = (button == 1 && action == 1);
            middleMousePressed = (button == 2 && action == 1);
        } else if (cmd == "cursor") {   // main.cpp:516-555
            double xpos = 0, ypos = 0;
            ls >> xpos >> ypos;
            if (xpos == lastX || ypos == lastY) continue;
            if (leftMousePressed) {
                phi -= (xpos - lastX) / width;
                theta -= (ypos - lastY) / height;
                theta = std::fmax(0.001f, std::fmin(theta, PI));
                camchanged = true;
            } else if (rightMousePressed) {
                zoom += (ypos - lastY) / height;
                zoom = std::fmax(0.1f, zoom);
                camchanged = true;
            } else if (middleMousePressed) {
                renderState = &scene->state;
                Camera& c = renderState->camera;
                glm::vec3 forward = c.view;
                forward.y = 0.0f;
                forward = glm::normalize(forward);
                glm::vec3 r = c.right;
                r.y = 0.0f;
                r = glm::normalize(r);
                c.lookAt -= (float)(xpos - lastX) * r * 0.01f;
                c.lookAt += (float)(ypos - lastY) * forward * 0.01f;
                camchanged = true;
            }
            lastX = xpos;
            lastY = ypos;
        } else if (cmd == "key") {   // main.cpp:481-502 (S / ESC save only; no camera effect)
            int key = 0;
            ls >> key;
            if (key == 32) {
                camchanged = true;
                renderState = &scene->state;
                renderState->camera.lookAt = ogLookAt;
            }
        } else if (cmd == "frame") {   // runCuda, main.cpp:423-444
            const bool reset = camchanged;
            if (camchanged) {
                Camera& c = renderState->camera;
                cameraPosition.x = zoom * std::sin(phi) * std::sin(theta);
                cameraPosition.y = zoom * std::cos(theta);
                cameraPosition.z = zoom * std::cos(phi) * std::sin(theta);
                c.view = -glm::normalize(cameraPosition);
                glm::vec3 v = c.view;
                glm::vec3 u = glm::vec3(0, 1, 0);
                glm::vec3 r = glm::cross(v, u);
                c.up = glm::cross(r, v);
                c.right = r;
                c.position = cameraPosition;
                cameraPosition += c.lookAt;
                c.position = cameraPosition;
                camchanged = false;
                c.focalDist = glm::length(c.lookAt - c.position);
            }
            const Camera& c = renderState->camera;
            std::printf("%s{\"reset\": %d, \"phi\": %u, \"theta\": %u, \"zoom\": %u, ", first ? "" : ",\n", reset ? 1 : 0,
                        bits(phi), bits(theta), bits(zoom));
            first = false;
            pv3("position", c.position);
            pv3("lookAt", c.lookAt);
            pv3("view", c.view);
            pv3("up", c.up);
            pv3("right", c.right);
            std::printf("\"focalDist\": %u}", bits(c.focalDist));
        }
    }
    std::printf("\n]}\n");
    return 0;
}
