// ingest_pin.cpp — pins the oracle's scene-ingest float math against the reference's OWN
// code where it builds here without stand-ins:
//   * src/utilities.cpp (utilityCore::buildTransformationMatrix) compiled from the reference
//     sources in place, with the reference's vendored glm 0.9.6 and nlohmann json 3.11.3;
//   * glm::inverse / glm::inverseTranspose / normalize / reflect / refract from that glm.
// scene.cpp / main.cpp cannot be compiled (sceneStructs.h includes cuda_runtime.h), so the
// ~20 lines of camera set-up they perform (scene.cpp:184-213, main.cpp:359-380, 423-444)
// are restated below ON TOP OF the reference's glm, to pin the oracle's float ordering.
// Output: JSON on stdout.  Build/run recipe: oracle/ref_pins/make_fixtures.sh.
#include "utilities.h"
#include "json.hpp"
#include <glm/glm.hpp>
#include <glm/gtc/matrix_inverse.hpp>
#include <cstdio>
#include <cstring>
#include <cstdint>
#include <fstream>
#include <string>

using json = nlohmann::json;

static uint32_t bits(float f) { uint32_t b; std::memcpy(&b, &f, 4); return b; }
static void pv3(const glm::vec3& v) { std::printf("[%u, %u, %u]", bits(v.x), bits(v.y), bits(v.z)); }
static void pm4(const glm::mat4& m) {
    std::printf("[");
    for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) std::printf("%s%u", (c || r) ? ", " : "", bits(m[c][r]));
    std::printf("]");
}

int main(int argc, char** argv) {
    std::printf("{\"scenes\": {\n");
    for (int a = 1; a < argc; ++a) {
        std::ifstream f(argv[a]);
        json data = json::parse(f);
        std::printf("%s\"%s\": {\"materials\": [", a > 1 ? ",\n" : "", argv[a]);
        bool first = true;
        for (const auto& item : data["Materials"].items()) {
            std::printf("%s\"%s\"", first ? "" : ", ", item.key().c_str());
            first = false;
        }
        std::printf("], \"objects\": [");
        first = true;
        for (const auto& p : data["Objects"]) {
            glm::vec3 t(p["TRANS"][0], p["TRANS"][1], p["TRANS"][2]);
            glm::vec3 r(p["ROTAT"][0], p["ROTAT"][1], p["ROTAT"][2]);
            glm::vec3 s(p["SCALE"][0], p["SCALE"][1], p["SCALE"][2]);
            glm::mat4 T = utilityCore::buildTransformationMatrix(t, r, s);
            std::printf("%s{\"transform\": ", first ? "" : ",\n  ");
            first = false;
            pm4(T);
            std::printf(", \"inverse\": ");
            pm4(glm::inverse(T));
            std::printf(", \"invTranspose\": ");
            pm4(glm::inverseTranspose(T));
            std::printf("}");
        }
        // camera: scene.cpp:184-213 then main.cpp:359-380 and runCuda's first recompute
        const auto& cd = data["Camera"];
        glm::ivec2 res(cd["RES"][0], cd["RES"][1]);
        float fovy = cd["FOVY"];
        glm::vec3 position(cd["EYE"][0], cd["EYE"][1], cd["EYE"][2]);
        glm::vec3 lookAt(cd["LOOKAT"][0], cd["LOOKAT"][1], cd["LOOKAT"][2]);
        float yscaled = std::tan(fovy * (PI / 180));
        float xscaled = (yscaled * res.x) / res.y;
        glm::vec2 pixelLength(2 * xscaled / (float)res.x, 2 * yscaled / (float)res.y);
        glm::vec3 view = glm::normalize(lookAt - position);
        float phi = glm::acos(glm::dot(glm::normalize(glm::vec3(view.x, 0.0f, view.z)), glm::vec3(0, 0, -1)));
        float theta = glm::acos(glm::dot(glm::normalize(glm::vec3(0.0f, view.y, view.z)), glm::vec3(0, 1, 0)));
        float zoom = glm::length(position - lookAt);
        glm::vec3 cp;
        cp.x = zoom * std::sin(phi) * std::sin(theta);
        cp.y = zoom * std::cos(theta);
        cp.z = zoom * std::cos(phi) * std::sin(theta);
        glm::vec3 v = -glm::normalize(cp);
        glm::vec3 rr = glm::cross(v, glm::vec3(0, 1, 0));
        glm::vec3 up = glm::cross(rr, v);
        cp += lookAt;
        std::printf("], \"camera\": {\"view\": "); pv3(v);
        std::printf(", \"up\": "); pv3(up);
        std::printf(", \"right\": "); pv3(rr);
        std::printf(", \"position\": "); pv3(cp);
        std::printf(", \"focalDist\": %u", bits(glm::length(lookAt - cp)));
        std::printf(", \"pixelLength\": [%u, %u]}}", bits(pixelLength.x), bits(pixelLength.y));
    }
    // glm vector semantics on a deterministic sample
    std::printf("\n}, \"glm\": [\n");
    uint32_t s = 2463534242u;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return (float)(s % 2000001u) / 1000000.0f - 1.0f; };
    for (int k = 0; k < 256; ++k) {
        glm::vec3 I(rnd(), rnd(), rnd()), N(rnd(), rnd(), rnd());
        float eta = 0.5f + (rnd() + 1.0f);
        glm::vec3 n = glm::normalize(N);
        std::printf("%s{\"I\": ", k ? ",\n" : ""); pv3(I);
        std::printf(", \"N\": "); pv3(N);
        std::printf(", \"eta\": %u, \"normalize\": ", bits(eta)); pv3(n);
        std::printf(", \"reflect\": "); pv3(glm::reflect(I, n));
        std::printf(", \"refract\": "); pv3(glm::refract(glm::normalize(I), n, eta));
        std::printf("}");
    }
    std::printf("\n]}\n");
    return 0;
}
