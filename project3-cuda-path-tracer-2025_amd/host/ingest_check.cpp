// ingest_check.cpp — the host ingest behind the C-ABI, driven standalone for the sanitizer build
// (Makefile target `asan`: host/*.cpp with -fsanitize=address,undefined, no device code).
//
// The files a caller hands the library are untrusted: scene JSON (host/json_lite.h), OBJ meshes
// (host/scene.cpp's reader) and PNG textures (host/png_decode.cpp, a from-scratch inflate).  The
// reference's failure semantics are an exception for a scene it cannot read (scene.cpp:245-247,
// "Failed to load") and -1 for a texture it cannot decode (scene.cpp:372-375, shown as magenta);
// here: PT_E_INVALID with a message, and textureID -1.  Every input must end in one of those or
// in a loaded scene -- never in a sanitizer report.
//
//   ingest_check scene FILE.json...   pt_scene_load_ex (host BVH) + the SAH traversal tree over its
//                                     leaves + pt_scene_get_view; prints "scene rc=<rc> ..."
//   ingest_check png FILE...          pt_texture_load (size query, then decode); "png rc=<rc> w h"
//   ingest_check savepng OUT W H      pt_save_png of a W x H test image with NaN / inf / negatives
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "pt/pathtrace_abi.h"
#include "trav_tree.h"

static int check_scene(const char* path) {
    pt_scene_file* f = nullptr;
    const int rc = pt_scene_load_ex(path, -1, -1, -1, PT_SCENE_VIEWER_CAMERA, &f);
    if (rc != PT_OK) {
        std::printf("scene rc=%d err=%s\n", rc, pt_scene_last_error());
        return rc;
    }
    pt_scene_view v{};
    pt_scene_get_view(f, &v);
    int32_t iters = 0, depth = 0;
    char name[256];
    pt_scene_get_info(f, &iters, &depth, name, (int32_t)sizeof name);
    int bad_tex = 0;
    for (int i = 0; i < v.num_materials; ++i) {
        char mname[128];
        pt_scene_material_name(f, i, mname, (int32_t)sizeof mname);
        if ((v.materials[i].hasTexture && v.materials[i].textureID < 0) ||
            (v.materials[i].hasBumpMap && v.materials[i].bumpID < 0))
            ++bad_tex;
    }
    // the SAH traversal hierarchy pt_init builds over the BVH's leaves (host part of the path)
    std::vector<float> lo, hi, s;
    for (int i = 0; i < v.num_bvh_nodes; ++i) {
        const pt_bvh_node& nd = v.bvh_nodes[i];
        if (!(nd.triCount > 0 && nd.start >= 0)) continue;
        const float l[3] = {nd.aabb.min.x, nd.aabb.min.y, nd.aabb.min.z};
        const float h[3] = {nd.aabb.max.x, nd.aabb.max.y, nd.aabb.max.z};
        for (int a = 0; a < 3; ++a) {
            lo.push_back(l[a]);
            hi.push_back(h[a]);
        }
        s.push_back(1.0f);
    }
    std::vector<pth::TravInner> tree;
    int height = 0;
    const bool sah = pth::build_sah_tree(lo, hi, s, tree, height);
    // the same tree under every numbering (breadth-first top levels, preorder below): walk both
    // from the root and compare every child's box, cull size and leaf id
    int orders_equal = sah ? 1 : -1;
    for (int levels : {0, 1, 4, 8}) {
        if (!sah || s.size() > 20000) break;   // (the 262k / 1.0M stand-ins: too slow under ASan)
        std::vector<pth::TravInner> t2;
        int h2 = 0;
        if (!pth::build_sah_tree(lo, hi, s, t2, h2, levels) || h2 != height || t2.size() != tree.size()) {
            orders_equal = 0;
            break;
        }
        std::vector<std::pair<int, int>> st{{0, 0}};
        size_t seen = 0;
        while (!st.empty() && orders_equal) {
            const auto [a, b] = st.back();
            st.pop_back();
            ++seen;
            for (int c = 0; c < 2; ++c) {
                const pth::TravChild &x = tree[a].c[c], &y = t2[b].c[c];
                bool same = x.leaf == y.leaf && x.s == y.s && (!x.leaf || x.ref == y.ref);
                for (int k = 0; k < 3; ++k) same = same && x.lo[k] == y.lo[k] && x.hi[k] == y.hi[k];
                if (!same) orders_equal = 0;
                else if (!x.leaf) st.push_back({x.ref, y.ref});
            }
        }
        if (seen != tree.size()) orders_equal = 0;
    }
    if (sah && s.size() > 20000) orders_equal = -2;   // not checked
    // the tightest height bound (1 + ceil(log2 leaves)): every leaf still in the tree exactly once
    int tight = -1, tight_leaves = 0;
    if (sah) {
        std::vector<pth::TravInner> t3;
        int h3 = 0;
        if (pth::build_sah_tree(lo, hi, s, t3, h3, 1 << 30, 1)) {
            tight = h3;
            std::vector<int> seen(s.size(), 0);
            for (const pth::TravInner& t : t3)
                for (const pth::TravChild& c : t.c)
                    if (c.leaf && c.ref >= 0 && c.ref < (int)s.size()) seen[c.ref]++;
            for (int x : seen) tight_leaves += x == 1;
        }
    }
    // the 4-wide records: every leaf in exactly one record, every record but the root referenced
    // exactly once and after its parent... 2..4 children, each child's box the tree's own
    int quads = -1, quad_ok = -1, quad_need = -1;
    if (sah) {
        std::vector<pth::QuadRecord> qr;
        pth::build_quad_records(tree, 6, qr, quad_need);
        quads = (int)qr.size();
        quad_ok = 1;
        std::vector<int> leaf_seen(s.size(), 0), rec_seen(qr.size(), 0);
        for (const pth::QuadRecord& r : qr) {
            if (r.n < 2 || r.n > 4) quad_ok = 0;
            for (int i = 0; i < r.n; ++i) {
                const pth::TravChild& c = r.c[i];
                if (c.leaf) {
                    if (c.ref < 0 || c.ref >= (int)s.size()) quad_ok = 0;
                    else leaf_seen[c.ref]++;
                } else if (c.ref <= 0 || c.ref >= (int)qr.size()) {
                    quad_ok = 0;
                } else {
                    rec_seen[c.ref]++;
                }
                for (int a = 0; a < 3; ++a)
                    if (!(c.lo[a] <= c.hi[a])) quad_ok = 0;
            }
        }
        for (int x : leaf_seen) quad_ok &= x == 1;
        for (size_t q = 1; q < rec_seen.size(); ++q) quad_ok &= rec_seen[q] == 1;
        if (!rec_seen.empty()) quad_ok &= rec_seen[0] == 0;
    }
    std::printf("scene rc=0 geoms=%d materials=%d triangles=%d nodes=%d depth=%d textures=%d bad_tex=%d sah=%d "
                "sah_orders_equal=%d sah_tight=%d leaves=%zu tight_leaves=%d quads=%d quad_ok=%d quad_stack=%d\n",
                v.num_geoms, v.num_materials, v.num_triangles, v.num_bvh_nodes, depth, v.num_textures, bad_tex,
                sah ? height : -1, orders_equal, tight, s.size(), tight_leaves, quads, quad_ok, quad_need);
    pt_scene_free(f);
    return 0;
}

static int check_png(const char* path) {
    int32_t w = 0, h = 0;
    int rc = pt_texture_load(path, &w, &h, nullptr, 0);
    if (rc == PT_OK) {
        std::vector<uint8_t> px((size_t)w * h * 4);
        rc = pt_texture_load(path, &w, &h, px.data(), (int64_t)px.size());
    }
    if (rc != PT_OK) std::printf("png rc=%d err=%s\n", rc, pt_scene_last_error());
    else std::printf("png rc=0 %d %d\n", w, h);
    return rc;
}

static int save_png(const char* out, int w, int h) {
    std::vector<float> img((size_t)w * h * 3);
    for (size_t i = 0; i < img.size(); ++i) img[i] = (float)((i * 37) % 300) / 7.0f - 3.0f;
    if (!img.empty()) img[0] = std::numeric_limits<float>::quiet_NaN();
    if (img.size() > 1) img[1] = std::numeric_limits<float>::infinity();
    if (img.size() > 2) img[2] = -std::numeric_limits<float>::infinity();
    const int rc = pt_save_png(img.data(), w, h, 3, out);
    std::printf("savepng rc=%d\n", rc);
    return rc;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s scene|png FILE... | savepng OUT W H\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    if (mode == "savepng" && argc == 5) return save_png(argv[2], std::atoi(argv[3]), std::atoi(argv[4])) == 0 ? 0 : 1;
    for (int i = 2; i < argc; ++i) {
        std::printf("%s: ", argv[i]);
        if (mode == "scene") check_scene(argv[i]);
        else if (mode == "png") check_png(argv[i]);
        else return 2;
        std::fflush(stdout);
    }
    return 0;
}
