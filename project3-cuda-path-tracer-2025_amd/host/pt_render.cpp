// pt_render.cpp — headless driver that replaces the reference's GL viewer (src/main.cpp):
// load a scene, apply the viewer's camera recompute, run iterations 1..spp through the
// reference's C++ boundary (pathtraceInit / pathtrace / pathtraceFree), and save the result
// like saveImage (main.cpp:395-419): x-flipped, averaged, clamped 8-bit PNG, plus the raw
// accumulated float image as PFM.
//
//   pt_render SCENE.json [--spp N] [--res WxH] [--depth D] [--out PREFIX]
//             [--pipeline fused|staged] [--sort] [--no-compaction] [--no-bvh] [--device K] [--gpu-bvh]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "image_io.h"
#include "pathtrace.h"

int main(int argc, char** argv) {
    if (argc < 2) {
        std::printf("Usage: %s SCENEFILE.json [--spp N] [--res WxH] [--depth D] [--out PREFIX] "
                    "[--pipeline fused|staged] [--sort] [--no-compaction] [--no-bvh] [--device K] [--gpu-bvh]\n", argv[0]);
        return 1;
    }
    std::string scene_file = argv[1], out;
    bool gpu_bvh = false;
    int spp = -1, resx = 0, resy = 0, depth = -1;
    pt_options opts;
    pt_default_options(&opts);
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (a == "--spp") spp = std::atoi(next());
        else if (a == "--res") { if (std::sscanf(next(), "%dx%d", &resx, &resy) != 2) return 2; }
        else if (a == "--depth") depth = std::atoi(next());
        else if (a == "--out") out = next();
        else if (a == "--pipeline") opts.pipeline = std::strcmp(next(), "staged") == 0 ? PT_PIPELINE_STAGED : PT_PIPELINE_FUSED;
        else if (a == "--sort") opts.material_sort = 1;
        else if (a == "--no-compaction") opts.stream_compaction = 0;
        else if (a == "--no-bvh") opts.bvh = 0;
        else if (a == "--device") opts.device = std::atoi(next());
        else if (a == "--gpu-bvh") gpu_bvh = true;
        else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
    }
    Scene* scene = nullptr;
    try {
        scene = new Scene(scene_file, resx, resy, depth, gpu_bvh);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    applyViewerCamera(scene->state.camera);   // main.cpp:359-380 + runCuda's first recompute
    GuiDataContainer gui;
    InitDataContainer(&gui);
    pathtraceSetOptions(opts);
    pathtraceInit(scene);
    const int iterations = spp > 0 ? spp : (int)scene->state.iterations;
    const int width = scene->state.camera.resolution.x, height = scene->state.camera.resolution.y;
    auto t0 = std::chrono::steady_clock::now();
    for (int iteration = 1; iteration <= iterations; ++iteration) pathtrace(nullptr, 0, iteration);
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    pt_frame_stats st;
    pt_get_frame_stats(&st);
    std::printf("%s: %dx%d depth %d, %d spp in %.3f s (%.3f ms/frame incl. %zu-byte image copy), last frame %lld segments\n",
                scene_file.c_str(), width, height, scene->state.traceDepth, iterations, secs, 1e3 * secs / iterations,
                sizeof(float) * 3 * (size_t)width * height, (long long)st.segments);
    if (out.empty()) out = scene->state.imageName + "." + std::to_string(iterations) + "samp";
    std::vector<unsigned char> rgb = ptio::to_rgb8(scene->state.image, width, height, (float)iterations);
    bool ok = ptio::write_png(out + ".png", rgb, width, height) && ptio::write_pfm(out + ".pfm", scene->state.image, width, height);
    std::printf("Saved %s.png / %s.pfm\n", out.c_str(), out.c_str());
    pathtraceFree();
    delete scene;
    return ok ? 0 : 1;
}
