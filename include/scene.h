// scene.h — C++ mirror of the reference's scene ingest interface (src/scene.h:6-28,
// src/sceneStructs.h), so code written against the reference's Scene compiles against this
// framework.  The reference's glm-typed structs are replaced by the layout-identical
// pt_* PODs of pt/scene_structs.h, aliased to the reference's names.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "pt/pathtrace_abi.h"
#include "pt/scene_structs.h"

using Geom = pt_geom;
using Material = pt_material;
using Texture = pt_texture;
using Vertex = pt_vertex;
using Triangle = pt_triangle;
using AABB = pt_aabb;
using BVHNode = pt_bvh_node;
using Camera = pt_camera;
using PathSegment = pt_path_segment;
using ShadeableIntersection = pt_shadeable_isect;
using uchar4 = pt_uchar4;

// sceneStructs.h:119-126
struct RenderState {
    Camera camera;
    unsigned int iterations = 0;
    int traceDepth = 0;
    std::vector<pt_vec3> image;
    std::string imageName;
};

// utilities.h:22-27
class GuiDataContainer {
public:
    GuiDataContainer() : TracedDepth(0) {}
    int TracedDepth;
};

class Scene {
public:
    // scene.cpp:22-37; throws std::runtime_error where the reference exit()s / throws
    explicit Scene(std::string filename);
    // same, with RES (<= 0: keep) / DEPTH (< 0: keep) overridden before the camera is derived;
    // gpuBVH: build the BVH with pt_bvh_build on the current HIP device (same tree, bit for bit)
    Scene(std::string filename, int resx, int resy, int depth, bool gpuBVH = false);
    ~Scene();

    std::vector<Geom> geoms;
    std::vector<Material> materials;
    std::vector<Texture> textures;
    std::vector<Vertex> vertices;
    std::vector<Triangle> triangles;
    std::vector<int> triIndices;
    std::vector<BVHNode> bvhNodes;
    RenderState state;

    // framework additions
    std::vector<std::string> materialNames;   // index = material id (alphabetical)
    std::vector<std::vector<uint8_t>> texturePixels;   // RGBA8 storage behind textures[i].data
    pt_scene_view view() const;               // borrowed flat view for pt_init

private:
    void loadFromJSON(const std::string& jsonName, int resx, int resy, int depth);
    void loadFromOBJ(const std::string& objName, int materialID, const pt_mat4& transformMatrix,
                     const pt_mat4& invTransposeMatrix);
    void buildBVH();
    bool gpuBVH = false;
    int loadTexture(const std::string& texturePath);
};

// The interactive viewer's camera recompute that every reference frame sees: main.cpp:359-380
// (phi/theta/zoom from the loaded view) followed by runCuda()'s camchanged block
// main.cpp:423-444 (camchanged starts true, main.cpp:36).
void applyViewerCamera(Camera& cam);

// utilities.cpp:85-93 and the glm 0.9.6 matrix helpers scene.cpp uses
pt_mat4 buildTransformationMatrix(pt_vec3 translation, pt_vec3 rotation, pt_vec3 scale);
pt_mat4 glmInverse(const pt_mat4& m);
pt_mat4 glmInverseTranspose(const pt_mat4& m);
