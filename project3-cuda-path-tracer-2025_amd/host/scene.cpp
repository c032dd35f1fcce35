// scene.cpp — scene ingest for the MI355X path tracer: a C++ restatement of the reference's
// host-side loader (src/scene.cpp, src/utilities.cpp:85-93, and the viewer camera of
// src/main.cpp:359-380 / 423-444).  Everything it produces is consumed bit-for-bit by the
// kernels (material ids, matrices, camera, BVH layout), so the float math follows glm 0.9.6's
// operation order exactly (hmath.h) and is checked against the reference's own glm /
// utilities.cpp by tests/test_scene_ingest.py.
#include <cfloat>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "hmath.h"
#include "json_lite.h"
#include "scene.h"
#include "png_decode.h"

using namespace pth;

namespace {
// utilities.h:13
constexpr float PI = 3.1415926535897932384626422832795028841971f;

// gtc/matrix_transform.inl translate / rotate / scale
pt_mat4 translate(const pt_mat4& m, v3 v) {
    pt_mat4 r = m;
    setcol(r, 3, col(m, 0) * v.x + col(m, 1) * v.y + col(m, 2) * v.z + col(m, 3));
    return r;
}
pt_mat4 rotate(const pt_mat4& m, float angle, v3 v) {
    const float c = std::cos(angle);
    const float s = std::sin(angle);
    v3 axis = normalize(v);
    v3 temp = axis * (1.0f - c);
    float R[3][3];
    R[0][0] = c + temp.x * axis.x;
    R[0][1] = 0 + temp.x * axis.y + s * axis.z;
    R[0][2] = 0 + temp.x * axis.z - s * axis.y;
    R[1][0] = 0 + temp.y * axis.x - s * axis.z;
    R[1][1] = c + temp.y * axis.y;
    R[1][2] = 0 + temp.y * axis.z + s * axis.x;
    R[2][0] = 0 + temp.z * axis.x + s * axis.y;
    R[2][1] = 0 + temp.z * axis.y - s * axis.x;
    R[2][2] = c + temp.z * axis.z;
    pt_mat4 r;
    for (int j = 0; j < 3; ++j) setcol(r, j, col(m, 0) * R[j][0] + col(m, 1) * R[j][1] + col(m, 2) * R[j][2]);
    setcol(r, 3, col(m, 3));
    return r;
}
pt_mat4 scale(const pt_mat4& m, v3 v) {
    pt_mat4 r;
    setcol(r, 0, col(m, 0) * v.x);
    setcol(r, 1, col(m, 1) * v.y);
    setcol(r, 2, col(m, 2) * v.z);
    setcol(r, 3, col(m, 3));
    return r;
}

v3 vec3_of(const ptj::Value& a) { return V3(a[0].as_float(), a[1].as_float(), a[2].as_float()); }

std::string read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

// scene.cpp:395-426
void computeTriangleTangents(Triangle& tri) {
    v3 p1 = tri.v1.position, p2 = tri.v2.position, p3 = tri.v3.position;
    v2 uv1 = tri.v1.uv, uv2 = tri.v2.uv, uv3 = tri.v3.uv;
    v3 dp1 = p2 - p1, dp2 = p3 - p1;
    v2 duv1 = uv2 - uv1, duv2 = uv3 - uv1;
    float det = duv1.x * duv2.y - duv1.y * duv2.x;
    if (std::fabs(det) < 1e-8f) {
        v3 n = normalize(cross(dp1, dp2));
        v3 tangent = normalize(dp1);
        v3 bitangent = normalize(cross(n, tangent));
        tri.dpdu = tangent;
        tri.dpdv = bitangent;
        return;
    }
    float invDet = 1.0f / det;
    tri.dpdu = (dp1 * duv2.y - dp2 * duv1.y) * invDet;
    tri.dpdv = ((-dp1) * duv2.x + dp2 * duv1.x) * invDet;
}

// scene.cpp:428-525 (node bounds, longest-axis midpoint split with the reference's axis
// selection, in-place swap partition, median fallback, leaves of <= 4)
struct BVHBuilder {
    const std::vector<Triangle>& tris;
    std::vector<BVHNode>& nodes;
    std::vector<int>& idx;

    void bounds(int start, int end, BVHNode& node) {
        AABB b;
        b.min = V3(FLT_MAX, FLT_MAX, FLT_MAX);
        b.max = V3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
        for (int i = start; i < end; i++) {
            const Triangle& t = tris[idx[i]];
            b.min = vmin(b.min, t.v1.position);
            b.min = vmin(b.min, t.v2.position);
            b.min = vmin(b.min, t.v3.position);
            b.max = vmax(b.max, t.v1.position);
            b.max = vmax(b.max, t.v2.position);
            b.max = vmax(b.max, t.v3.position);
        }
        node.aabb = b;
    }
    int build(int start, int end) {
        int nodeIndex = (int)nodes.size();
        BVHNode fresh{};
        fresh.aabb.min = V3(FLT_MAX, FLT_MAX, FLT_MAX);
        fresh.aabb.max = V3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
        nodes.push_back(fresh);
        bounds(start, end, nodes[nodeIndex]);
        int numTris = end - start;
        if (numTris <= 4) {
            nodes[nodeIndex].start = start;
            nodes[nodeIndex].triCount = numTris;
            nodes[nodeIndex].left = -1;
            nodes[nodeIndex].right = -1;
            return nodeIndex;
        }
        AABB cb;
        cb.min = V3(FLT_MAX, FLT_MAX, FLT_MAX);
        cb.max = V3(-FLT_MAX, -FLT_MAX, -FLT_MAX);
        for (int i = start; i < end; i++) {
            cb.min = vmin(cb.min, tris[idx[i]].centroid);
            cb.max = vmax(cb.max, tris[idx[i]].centroid);
        }
        v3 extent = cb.max - cb.min;
        int axis = 0;
        if (extent.y > extent.x && extent.y > extent.z) axis = 1;
        if (extent.z > extent.x) axis = 2;
        float splitPos = 0.5f * (comp(cb.min, axis) + comp(cb.max, axis));
        int mid = start;
        for (int i = start; i < end; i++) {
            if (comp(tris[idx[i]].centroid, axis) < splitPos) {
                std::swap(idx[i], idx[mid]);
                mid++;
            }
        }
        if (mid == start || mid == end) mid = (start + end) / 2;
        int l = build(start, mid);
        int r = build(mid, end);
        nodes[nodeIndex].left = l;
        nodes[nodeIndex].right = r;
        nodes[nodeIndex].start = -1;
        nodes[nodeIndex].triCount = 0;
        return nodeIndex;
    }
};

struct ObjIndex {
    int v, t, n;
};

// tinyobj::LoadObj(triangulate=true) for the v / vt / vn / f records the scenes use:
// triangles as-is, quads split on the shorter diagonal (tiny_obj_loader.h:1520-1628),
// larger polygons fanned.
void parse_obj(const std::string& path, std::vector<float>& pos, std::vector<float>& nrm, std::vector<float>& tex,
               std::vector<ObjIndex>& faces) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("Failed to load " + path);   // scene.cpp:245-247
    std::string line;
    auto resolve = [](const std::string& tok, size_t n) -> int {
        if (tok.empty()) return -1;
        long i = std::strtol(tok.c_str(), nullptr, 10);
        return i > 0 ? (int)(i - 1) : (int)((long)n + i);
    };
    while (std::getline(f, line)) {
        std::istringstream ls(line);
        std::string tag;
        if (!(ls >> tag)) continue;
        if (tag == "v") {
            std::string a, b, c;
            ls >> a >> b >> c;
            pos.push_back((float)std::strtod(a.c_str(), nullptr));
            pos.push_back((float)std::strtod(b.c_str(), nullptr));
            pos.push_back((float)std::strtod(c.c_str(), nullptr));
        } else if (tag == "vn") {
            std::string a, b, c;
            ls >> a >> b >> c;
            nrm.push_back((float)std::strtod(a.c_str(), nullptr));
            nrm.push_back((float)std::strtod(b.c_str(), nullptr));
            nrm.push_back((float)std::strtod(c.c_str(), nullptr));
        } else if (tag == "vt") {
            std::string a, b;
            ls >> a;
            if (!(ls >> b)) b = "0";
            tex.push_back((float)std::strtod(a.c_str(), nullptr));
            tex.push_back((float)std::strtod(b.c_str(), nullptr));
        } else if (tag == "f") {
            std::vector<ObjIndex> poly;
            std::string tok;
            while (ls >> tok) {
                std::string parts[3];
                int k = 0;
                for (char ch : tok) {
                    if (ch == '/') { if (++k > 2) break; }
                    else parts[k] += ch;
                }
                poly.push_back(ObjIndex{resolve(parts[0], pos.size() / 3), resolve(parts[1], tex.size() / 2),
                                        resolve(parts[2], nrm.size() / 3)});
            }
            if (poly.size() < 3) continue;
            for (const ObjIndex& ix : poly)   // before the quad split reads positions
                if (ix.v < 0 || 3 * (size_t)ix.v + 2 >= pos.size()) throw std::runtime_error("bad vertex index in " + path);
            if (poly.size() == 3) {
                faces.insert(faces.end(), poly.begin(), poly.end());
            } else if (poly.size() == 4) {
                auto P = [&](int q, int c) { return pos[3 * (size_t)poly[q].v + c]; };
                float e02x = P(2, 0) - P(0, 0), e02y = P(2, 1) - P(0, 1), e02z = P(2, 2) - P(0, 2);
                float e13x = P(3, 0) - P(1, 0), e13y = P(3, 1) - P(1, 1), e13z = P(3, 2) - P(1, 2);
                float sqr02 = e02x * e02x + e02y * e02y + e02z * e02z;
                float sqr13 = e13x * e13x + e13y * e13y + e13z * e13z;
                const int* order;
                static const int a02[6] = {0, 1, 2, 0, 2, 3}, a13[6] = {0, 1, 3, 1, 2, 3};
                order = sqr02 < sqr13 ? a02 : a13;
                for (int q = 0; q < 6; ++q) faces.push_back(poly[order[q]]);
            } else {
                for (size_t i = 1; i + 1 < poly.size(); ++i) {
                    faces.push_back(poly[0]);
                    faces.push_back(poly[i]);
                    faces.push_back(poly[i + 1]);
                }
            }
        }
    }
}

}  // namespace

// utilities.cpp:85-93
pt_mat4 buildTransformationMatrix(pt_vec3 translation, pt_vec3 rotation, pt_vec3 s) {
    pt_mat4 I = identity();
    pt_mat4 translationMat = translate(I, translation);
    pt_mat4 rotationMat = rotate(I, rotation.x * (float)PI / 180, V3(1, 0, 0));
    rotationMat = mul(rotationMat, rotate(I, rotation.y * (float)PI / 180, V3(0, 1, 0)));
    rotationMat = mul(rotationMat, rotate(I, rotation.z * (float)PI / 180, V3(0, 0, 1)));
    pt_mat4 scaleMat = scale(I, s);
    return mul(mul(translationMat, rotationMat), scaleMat);
}

// glm 0.9.6 detail::compute_inverse(tmat4x4) (type_mat4x4.inl:37-92)
pt_mat4 glmInverse(const pt_mat4& mm) {
    const float(*m)[4] = mm.m;
    float C00 = m[2][2] * m[3][3] - m[3][2] * m[2][3], C02 = m[1][2] * m[3][3] - m[3][2] * m[1][3],
          C03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float C04 = m[2][1] * m[3][3] - m[3][1] * m[2][3], C06 = m[1][1] * m[3][3] - m[3][1] * m[1][3],
          C07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float C08 = m[2][1] * m[3][2] - m[3][1] * m[2][2], C10 = m[1][1] * m[3][2] - m[3][1] * m[1][2],
          C11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float C12 = m[2][0] * m[3][3] - m[3][0] * m[2][3], C14 = m[1][0] * m[3][3] - m[3][0] * m[1][3],
          C15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float C16 = m[2][0] * m[3][2] - m[3][0] * m[2][2], C18 = m[1][0] * m[3][2] - m[3][0] * m[1][2],
          C19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float C20 = m[2][0] * m[3][1] - m[3][0] * m[2][1], C22 = m[1][0] * m[3][1] - m[3][0] * m[1][1],
          C23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    v4 F0 = V4(C00, C00, C02, C03), F1 = V4(C04, C04, C06, C07), F2 = V4(C08, C08, C10, C11);
    v4 F3 = V4(C12, C12, C14, C15), F4 = V4(C16, C16, C18, C19), F5 = V4(C20, C20, C22, C23);
    v4 Vec0 = V4(m[1][0], m[0][0], m[0][0], m[0][0]);
    v4 Vec1 = V4(m[1][1], m[0][1], m[0][1], m[0][1]);
    v4 Vec2 = V4(m[1][2], m[0][2], m[0][2], m[0][2]);
    v4 Vec3 = V4(m[1][3], m[0][3], m[0][3], m[0][3]);
    v4 Inv0 = Vec1 * F0 - Vec2 * F1 + Vec3 * F2;
    v4 Inv1 = Vec0 * F0 - Vec2 * F3 + Vec3 * F4;
    v4 Inv2 = Vec0 * F1 - Vec1 * F3 + Vec3 * F5;
    v4 Inv3 = Vec0 * F2 - Vec1 * F4 + Vec2 * F5;
    v4 SignA = V4(+1, -1, +1, -1), SignB = V4(-1, +1, -1, +1);
    pt_mat4 inv;
    setcol(inv, 0, Inv0 * SignA);
    setcol(inv, 1, Inv1 * SignB);
    setcol(inv, 2, Inv2 * SignA);
    setcol(inv, 3, Inv3 * SignB);
    v4 Row0 = V4(inv.m[0][0], inv.m[1][0], inv.m[2][0], inv.m[3][0]);
    v4 Dot0 = col(mm, 0) * Row0;
    float Dot1 = (Dot0.x + Dot0.y) + (Dot0.z + Dot0.w);
    float OneOverDeterminant = 1.0f / Dot1;
    pt_mat4 r;
    for (int c = 0; c < 4; ++c) setcol(r, c, col(inv, c) * OneOverDeterminant);
    return r;
}

// glm 0.9.6 gtc/matrix_inverse.inl:95-147 inverseTranspose(tmat4x4)
pt_mat4 glmInverseTranspose(const pt_mat4& mm) {
    const float(*m)[4] = mm.m;
    float S00 = m[2][2] * m[3][3] - m[3][2] * m[2][3], S01 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float S02 = m[2][1] * m[3][2] - m[3][1] * m[2][2], S03 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float S04 = m[2][0] * m[3][2] - m[3][0] * m[2][2], S05 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float S06 = m[1][2] * m[3][3] - m[3][2] * m[1][3], S07 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float S08 = m[1][1] * m[3][2] - m[3][1] * m[1][2], S09 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float S10 = m[1][0] * m[3][2] - m[3][0] * m[1][2], S11 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float S12 = m[1][0] * m[3][1] - m[3][0] * m[1][1], S13 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float S14 = m[1][1] * m[2][3] - m[2][1] * m[1][3], S15 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float S16 = m[1][0] * m[2][3] - m[2][0] * m[1][3], S17 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float S18 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    float I[4][4];
    I[0][0] = +(m[1][1] * S00 - m[1][2] * S01 + m[1][3] * S02);
    I[0][1] = -(m[1][0] * S00 - m[1][2] * S03 + m[1][3] * S04);
    I[0][2] = +(m[1][0] * S01 - m[1][1] * S03 + m[1][3] * S05);
    I[0][3] = -(m[1][0] * S02 - m[1][1] * S04 + m[1][2] * S05);
    I[1][0] = -(m[0][1] * S00 - m[0][2] * S01 + m[0][3] * S02);
    I[1][1] = +(m[0][0] * S00 - m[0][2] * S03 + m[0][3] * S04);
    I[1][2] = -(m[0][0] * S01 - m[0][1] * S03 + m[0][3] * S05);
    I[1][3] = +(m[0][0] * S02 - m[0][1] * S04 + m[0][2] * S05);
    I[2][0] = +(m[0][1] * S06 - m[0][2] * S07 + m[0][3] * S08);
    I[2][1] = -(m[0][0] * S06 - m[0][2] * S09 + m[0][3] * S10);
    I[2][2] = +(m[0][0] * S11 - m[0][1] * S09 + m[0][3] * S12);
    I[2][3] = -(m[0][0] * S08 - m[0][1] * S10 + m[0][2] * S12);
    I[3][0] = -(m[0][1] * S13 - m[0][2] * S14 + m[0][3] * S15);
    I[3][1] = +(m[0][0] * S13 - m[0][2] * S16 + m[0][3] * S17);
    I[3][2] = -(m[0][0] * S14 - m[0][1] * S16 + m[0][3] * S18);
    I[3][3] = +(m[0][0] * S15 - m[0][1] * S17 + m[0][2] * S18);
    float det = +m[0][0] * I[0][0] + m[0][1] * I[0][1] + m[0][2] * I[0][2] + m[0][3] * I[0][3];
    pt_mat4 r;
    for (int c = 0; c < 4; ++c)
        for (int k = 0; k < 4; ++k) r.m[c][k] = I[c][k] / det;
    return r;
}

void applyViewerCamera(Camera& cam) {
    // main.cpp:359-380
    v3 view = cam.view;
    v3 viewXZ = V3(view.x, 0.0f, view.z);
    v3 viewZY = V3(0.0f, view.y, view.z);
    float phi = std::acos(dot(normalize(viewXZ), V3(0, 0, -1)));
    float theta = std::acos(dot(normalize(viewZY), V3(0, 1, 0)));
    v3 ogLookAt = cam.lookAt;
    float zoom = length(cam.position - ogLookAt);
    // main.cpp:423-444 (float overloads of sin/cos, as CUDA's and MSVC's headers provide)
    v3 cameraPosition;
    cameraPosition.x = zoom * std::sin(phi) * std::sin(theta);
    cameraPosition.y = zoom * std::cos(theta);
    cameraPosition.z = zoom * std::cos(phi) * std::sin(theta);
    cam.view = -normalize(cameraPosition);
    v3 v = cam.view;
    v3 u = V3(0, 1, 0);
    v3 r = cross(v, u);
    cam.up = cross(r, v);
    cam.right = r;
    cameraPosition = cameraPosition + cam.lookAt;
    cam.position = cameraPosition;
    cam.focalDist = length(cam.lookAt - cam.position);
}

Scene::Scene(std::string filename) : Scene(std::move(filename), 0, 0, -1) {}

Scene::Scene(std::string filename, int resx, int resy, int depth, bool gpu_bvh) : gpuBVH(gpu_bvh) {
    auto dot_pos = filename.find_last_of('.');
    std::string ext = dot_pos == std::string::npos ? "" : filename.substr(dot_pos);
    if (ext != ".json") throw std::runtime_error("Couldn't read from " + filename);   // scene.cpp:30-35
    loadFromJSON(filename, resx, resy, depth);
}

Scene::~Scene() = default;

// loadTexture (scene.cpp:366-392): RGBA8 via the framework's PNG decoder (stbi_load with
// STBI_rgb_alpha in the reference; every texture the reference's scenes name is a PNG).
int Scene::loadTexture(const std::string& texturePath) {
    int w = 0, h = 0;
    std::vector<uint8_t> rgba;
    std::string err;
    if (!ptio::png_load_rgba(texturePath, w, h, rgba, err)) {
        std::fprintf(stderr, "Failed to load texture image: %s (%s)\n", texturePath.c_str(), err.c_str());
        return -1;
    }
    texturePixels.push_back(std::move(rgba));
    Texture t{};
    t.width = w;
    t.height = h;
    t.channels = 4;
    t.data = texturePixels.back().data();
    int id = (int)textures.size();
    textures.push_back(t);
    return id;
}

void Scene::loadFromJSON(const std::string& jsonName, int resx, int resy, int depth) {
    ptj::Value data = ptj::parse(read_file(jsonName));
    const ptj::Value& materialsData = data["Materials"];
    std::map<std::string, int> MatNameToID;
    for (const auto& item : materialsData.as_object()) {   // std::map order == nlohmann object order
        const std::string& name = item.first;
        const ptj::Value& p = item.second;
        Material m{};
        m.roughness = -1.f;
        m.metallic = -1.f;
        m.textureID = -1;
        m.bumpID = -1;
        m.bumpScale = 0.5f;
        std::string type = p.contains("TYPE") && p["TYPE"].kind == ptj::Value::String ? p["TYPE"].s : "";
        if (type == "Diffuse") {
            m.color = vec3_of(p["RGB"]);
        } else if (type == "Emitting") {
            m.color = vec3_of(p["RGB"]);
            m.emittance = p["EMITTANCE"].as_float();
        } else if (type == "Glass") {
            m.hasReflective = 1;
            m.hasRefractive = 1;
            m.indexOfRefraction = p["IOR"].as_float();
            m.color = vec3_of(p["RGB"]);
        } else if (type == "Reflective") {
            m.hasReflective = 1;
            m.hasRefractive = 0;
            m.color = vec3_of(p["RGB"]);
        } else if (type == "Transmissive") {
            m.hasReflective = 0;
            m.hasRefractive = 1;
            m.indexOfRefraction = p["IOR"].as_float();
            m.color = vec3_of(p["RGB"]);
        } else if (type == "Microfacet") {
            m.roughness = p["ROUGHNESS"].as_float();
            m.metallic = p["METALLIC"].as_float();
            m.indexOfRefraction = p["IOR"].as_float();
            m.color = vec3_of(p["RGB"]);
        }
        // TEXTURE / BUMP_MAP (scene.cpp:102-133): path relative to the JSON's directory; a
        // texture that fails to load gets id -1 while hasTexture / hasBumpMap stay set.
        auto tex_base = [&]() {
            size_t lastSlashPos = jsonName.find_last_of("/\\");
            std::string basePath = lastSlashPos == std::string::npos ? jsonName : jsonName.substr(0, lastSlashPos);
            if (!basePath.empty() && basePath.back() != '/' && basePath.back() != '\\') basePath += "/";
            return basePath;
        };
        if (p.contains("TEXTURE")) {
            m.textureID = loadTexture(tex_base() + p["TEXTURE"].as_string());
            m.hasTexture = 1;
        }
        if (p.contains("BUMP_MAP")) {
            m.bumpID = loadTexture(tex_base() + p["BUMP_MAP"].as_string());
            m.hasBumpMap = 1;
            m.bumpScale = p["BUMP_SCALE"].as_float();
        }
        MatNameToID[name] = (int)materials.size();
        materials.push_back(m);
        materialNames.push_back(name);
    }
    auto mat_of = [&](const ptj::Value& p) -> int {
        // unordered_map::operator[] default-inserts 0 for unknown names (scene.cpp:148, 173)
        auto it = MatNameToID.find(p["MATERIAL"].as_string());
        return it == MatNameToID.end() ? 0 : it->second;
    };
    for (const ptj::Value& p : data["Objects"].as_array()) {
        const std::string& type = p["TYPE"].as_string();
        if (type == "obj") {
            size_t lastSlashPos = jsonName.find_last_of("/\\");
            std::string basePath = lastSlashPos == std::string::npos ? jsonName : jsonName.substr(0, lastSlashPos);
            std::string objPath = basePath + p["PATH"].as_string();
            pt_mat4 T = buildTransformationMatrix(vec3_of(p["TRANS"]), vec3_of(p["ROTAT"]), vec3_of(p["SCALE"]));
            pt_mat4 IT = glmInverseTranspose(T);
            loadFromOBJ(objPath, mat_of(p), T, IT);
        } else {
            Geom g{};
            g.type = type == "cube" ? PT_CUBE : PT_SPHERE;
            g.materialid = mat_of(p);
            g.translation = vec3_of(p["TRANS"]);
            g.rotation = vec3_of(p["ROTAT"]);
            g.scale = vec3_of(p["SCALE"]);
            g.transform = buildTransformationMatrix(g.translation, g.rotation, g.scale);
            g.inverseTransform = glmInverse(g.transform);
            g.invTranspose = glmInverseTranspose(g.transform);
            geoms.push_back(g);
        }
    }
    // camera, scene.cpp:184-213
    const ptj::Value& cd = data["Camera"];
    Camera& camera = state.camera;
    camera = Camera{};
    camera.resolution.x = resx > 0 ? resx : cd["RES"][0].as_int();
    camera.resolution.y = resy > 0 ? resy : cd["RES"][1].as_int();
    // the wavefront indexes pixels with 32-bit ints (the reference's too): a frame of at most 2^28
    if (camera.resolution.x <= 0 || camera.resolution.y <= 0 || camera.resolution.x > 65536 ||
        camera.resolution.y > 65536 || (int64_t)camera.resolution.x * camera.resolution.y > (int64_t(1) << 28))
        throw std::runtime_error("bad RES " + std::to_string(camera.resolution.x) + "x" +
                                 std::to_string(camera.resolution.y));
    float fovy = cd["FOVY"].as_float();
    state.iterations = (unsigned)cd["ITERATIONS"].as_int();
    state.traceDepth = depth >= 0 ? depth : cd["DEPTH"].as_int();
    state.imageName = cd["FILE"].as_string();
    camera.position = vec3_of(cd["EYE"]);
    camera.lookAt = vec3_of(cd["LOOKAT"]);
    camera.up = vec3_of(cd["UP"]);
    camera.focalDist = length(camera.lookAt - camera.position);
    // required like every other camera key: the reference's const json operator[] asserts on a
    // missing key (scene.cpp:198; scenes/sphere.json has no APERTURE and aborts the reference)
    camera.aperture = cd["APERTURE"].as_float();
    float yscaled = std::tan(fovy * (PI / 180));
    float xscaled = (yscaled * camera.resolution.x) / camera.resolution.y;
    float fovx = (std::atan(xscaled) * 180) / PI;
    camera.fov = pt_vec2{fovx, fovy};
    camera.right = normalize(cross(camera.view, camera.up));   // view not yet set (NaN), as in the reference
    camera.pixelLength = pt_vec2{2 * xscaled / (float)camera.resolution.x, 2 * yscaled / (float)camera.resolution.y};
    camera.view = normalize(camera.lookAt - camera.position);
    state.image.assign((size_t)camera.resolution.x * camera.resolution.y, pt_vec3{0, 0, 0});
    if (!triangles.empty()) buildBVH();
}

// scene.cpp:226-363
void Scene::loadFromOBJ(const std::string& objName, int materialID, const pt_mat4& T, const pt_mat4& IT) {
    std::vector<float> pos, nrm, tex;
    std::vector<ObjIndex> faces;
    parse_obj(objName, pos, nrm, tex, faces);
    for (size_t f = 0; f + 2 < faces.size(); f += 3) {
        Vertex fv[3];
        for (int k = 0; k < 3; ++k) {
            const ObjIndex& ix = faces[f + k];
            Vertex nv{};
            if (ix.v < 0 || 3 * (size_t)ix.v + 2 >= pos.size()) throw std::runtime_error("bad vertex index in " + objName);
            v4 p = mul(T, V4(pos[3 * ix.v], pos[3 * ix.v + 1], pos[3 * ix.v + 2], 1.0f));
            nv.position = V3(p.x, p.y, p.z);
            if (ix.n >= 0 && 3 * (size_t)ix.n + 2 < nrm.size()) {
                v4 n = mul(IT, V4(nrm[3 * ix.n], nrm[3 * ix.n + 1], nrm[3 * ix.n + 2], 0.0f));
                nv.normal = normalize(V3(n.x, n.y, n.z));
            }
            if (ix.t >= 0 && 2 * (size_t)ix.t + 1 < tex.size()) nv.uv = pt_vec2{tex[2 * ix.t], tex[2 * ix.t + 1]};
            else nv.uv = pt_vec2{0.0f, 0.0f};
            nv.materialID = materialID;
            fv[k] = nv;
        }
        bool missingNormals = true;
        for (const Vertex& vtx : fv)
            if (length(vtx.normal) > 1e-6f) { missingNormals = false; break; }
        if (missingNormals) {
            v3 faceNormal = normalize(cross(fv[1].position - fv[0].position, fv[2].position - fv[0].position));
            for (Vertex& vtx : fv) vtx.normal = faceNormal;
        }
        Triangle tri{};
        tri.v1 = fv[0];
        tri.v2 = fv[1];
        tri.v3 = fv[2];
        tri.centroid = (tri.v1.position + tri.v2.position + tri.v3.position) / 3.0f;
        tri.materialID = materialID;
        computeTriangleTangents(tri);
        triangles.push_back(tri);
        for (const Vertex& vtx : fv) vertices.push_back(vtx);
    }
}

// scene.cpp:445-457
void Scene::buildBVH() {
    bvhNodes.clear();
    triIndices.resize(triangles.size());
    for (int i = 0; i < (int)triangles.size(); i++) triIndices[i] = i;
    if (triangles.empty()) return;
    if (gpuBVH) {   // the same recursion on the GPU (csrc/pt_bvh_build.hip), same bits
#ifdef PT_HOST_ONLY   // the sanitizer build of the ingest (Makefile `asan`): no device code linked
        throw std::runtime_error("GPU BVH build: not in this host-only build");
#else
        const int n = (int)triangles.size();
        bvhNodes.resize(2 * (size_t)n - 1);
        int32_t count = 0;
        const int32_t rc = pt_bvh_build(triangles.data(), n, bvhNodes.data(), (int32_t)bvhNodes.size(), &count,
                                        triIndices.data());
        if (rc != PT_OK) throw std::runtime_error(std::string("GPU BVH build: ") + pt_bvh_build_last_error());
        bvhNodes.resize((size_t)count);
        return;
#endif
    }
    bvhNodes.reserve(2 * triangles.size());
    BVHBuilder b{triangles, bvhNodes, triIndices};
    b.build(0, (int)triangles.size());
}

pt_scene_view Scene::view() const {
    pt_scene_view v{};
    v.geoms = geoms.data();
    v.num_geoms = (int32_t)geoms.size();
    v.materials = materials.data();
    v.num_materials = (int32_t)materials.size();
    v.textures = textures.data();
    v.num_textures = (int32_t)textures.size();
    v.triangles = triangles.data();
    v.num_triangles = (int32_t)triangles.size();
    v.tri_indices = triIndices.data();
    v.num_tri_indices = (int32_t)triIndices.size();
    v.bvh_nodes = bvhNodes.data();
    v.num_bvh_nodes = (int32_t)bvhNodes.size();
    v.camera = state.camera;
    v.trace_depth = state.traceDepth;
    return v;
}
