// pt_render.cpp — headless driver that replaces the reference's GL viewer (src/main.cpp):
// load a scene, apply the viewer's camera recompute, run iterations 1..spp through the
// reference's C++ boundary (pathtraceInit / pathtrace / pathtraceFree), and save the result
// like saveImage (main.cpp:395-419): x-flipped, averaged, clamped 8-bit PNG, plus the raw
// accumulated float image as PFM.
//
//   pt_render SCENE.json [--spp N] [--res WxH] [--depth D] [--out PREFIX]
//             [--pipeline fused|staged] [--sort] [--no-compaction] [--no-bvh] [--device K] [--gpu-bvh]
//             [--devices N | --devices K0,K1,...] [--combine peer|rccl]
//             [--events FILE [--img-dir DIR] [--time-tag TAG]]
//
// --events replays a recorded window session through the viewer state machine of
// include/pt/pt_viewer.h (main.cpp's GLFW callbacks + runCuda) instead of rendering --spp frames.
// One event per line ('#' starts a comment):
//   button B A        mouseButtonCallback(button B, action A)   (GLFW codes: 0 left, 1 right, 2 middle; 1 press)
//   cursor X Y        mousePositionCallback(X, Y)
//   key K             keyCallback(key K, GLFW_PRESS)           (32 space, 83 S, 256 escape)
//   frame [N]         N mainLoop iterations (runCuda; default 1)
//   display FILE.png  write the window's pixels (the PBO as mainLoop draws it)
// The session ends at the end of the file, on ESC (window closed) or when runCuda reaches
// ITERATIONS (image saved, process exits), like the reference's main loop.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#include "image_io.h"
#include "pathtrace.h"
#include "pt/pt_viewer.h"

static int run_events(const std::string& scene_file, const pt_options& opts, int resx, int resy, int depth,
                      const std::string& events, const std::string& img_dir, const std::string& time_tag) {
    pt_scene_file* sf = nullptr;
    if (pt_scene_load(scene_file.c_str(), resx, resy, depth, 0, &sf) != PT_OK) {
        std::fprintf(stderr, "%s\n", pt_scene_last_error());
        return 1;
    }
    pt_viewer* v = nullptr;
    if (pt_viewer_create(sf, &opts, img_dir.c_str(), time_tag.empty() ? nullptr : time_tag.c_str(), &v) != PT_OK) {
        std::fprintf(stderr, "%s\n", pt_viewer_last_error());
        pt_scene_free(sf);
        return 1;
    }
    std::ifstream in(events);
    if (!in) {
        std::fprintf(stderr, "cannot read %s\n", events.c_str());
        return 2;
    }
    std::string line;
    int rc = PT_OK, exited = 0, lineno = 0, frames = 0;
    auto t0 = std::chrono::steady_clock::now();
    while (rc == PT_OK && !exited && std::getline(in, line)) {
        ++lineno;
        const auto hash = line.find('#');
        if (hash != std::string::npos) line.resize(hash);
        std::istringstream ls(line);
        std::string cmd;
        if (!(ls >> cmd)) continue;
        if (cmd == "button") {
            int b = 0, a = 0;
            ls >> b >> a;
            rc = pt_viewer_mouse_button(v, b, a, 0);
        } else if (cmd == "cursor") {
            double x = 0, y = 0;
            ls >> x >> y;
            rc = pt_viewer_cursor_pos(v, x, y);
        } else if (cmd == "key") {
            int k = 0;
            ls >> k;
            rc = pt_viewer_key(v, k, 0, PT_GLFW_PRESS, 0);
            pt_viewer_state st;
            pt_viewer_get_state(v, &st);
            if (st.should_close) break;
        } else if (cmd == "frame") {
            int n = 1;
            ls >> n;
            for (int i = 0; i < n && rc == PT_OK && !exited; ++i, ++frames) rc = pt_viewer_run_frame(v, &exited);
        } else if (cmd == "display") {
            std::string f;
            ls >> f;
            pt_viewer_state st;
            pt_viewer_get_state(v, &st);
            const int w = st.camera.resolution.x, h = st.camera.resolution.y;
            std::vector<unsigned char> rgb((size_t)w * h * 3);
            rc = pt_viewer_display(v, rgb.data(), (int64_t)rgb.size());
            if (rc == PT_OK && !ptio::write_png(f, rgb, w, h)) rc = PT_E_INVALID;
        } else {
            std::fprintf(stderr, "%s:%d: unknown event '%s'\n", events.c_str(), lineno, cmd.c_str());
            rc = PT_E_INVALID;
        }
    }
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    char title[128];
    pt_viewer_title(v, title, sizeof title);
    pt_viewer_state st;
    pt_viewer_get_state(v, &st);
    if (rc != PT_OK) std::fprintf(stderr, "viewer: %s\n", pt_viewer_last_error());
    std::printf("%s: %d display frames in %.3f s; %s; traced depth %d; %d image(s) saved%s\n", scene_file.c_str(),
                frames, secs, title, st.traced_depth, st.saved_images, exited ? "; reached ITERATIONS" : "");
    pt_viewer_destroy(v);
    pt_scene_free(sf);
    return rc == PT_OK ? 0 : 1;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::printf("Usage: %s SCENEFILE.json [--spp N] [--res WxH] [--depth D] [--out PREFIX] "
                    "[--pipeline fused|staged] [--sort] [--no-compaction] [--no-bvh] [--device K] [--gpu-bvh] "
                    "[--devices N|K0,K1,... [--combine peer|rccl]] "
                    "[--events FILE [--img-dir DIR] [--time-tag TAG]]\n", argv[0]);
        return 1;
    }
    std::string scene_file = argv[1], out, events, img_dir = "../img", time_tag;
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
        else if (a == "--devices") {   // every frame split into pixel shards over these GPUs
            const std::string d = next();
            opts.num_devices = 0;
            if (d.find(',') == std::string::npos) {
                opts.num_devices = std::max(0, std::min(PT_MAX_DEVICES, std::atoi(d.c_str())));
                for (int k = 0; k < PT_MAX_DEVICES; ++k) opts.device_ids[k] = k;
            } else {
                for (size_t s = 0; s <= d.size() && opts.num_devices < PT_MAX_DEVICES;) {
                    const size_t e = std::min(d.find(',', s), d.size());
                    const std::string tok = d.substr(s, e - s);
                    char* end = nullptr;
                    const long v = std::strtol(tok.c_str(), &end, 10);
                    if (tok.empty() || *end != '\0' || v < 0) {   // "0,,1", "0,1,", "0,x"
                        std::fprintf(stderr, "--devices: bad device id '%s' in '%s'\n", tok.c_str(), d.c_str());
                        return 2;
                    }
                    opts.device_ids[opts.num_devices++] = (int32_t)v;
                    s = e + 1;
                }
            }
        } else if (a == "--combine") opts.combine = std::strcmp(next(), "rccl") == 0 ? PT_COMBINE_RCCL : PT_COMBINE_PEER;
        else if (a == "--events") events = next();
        else if (a == "--img-dir") img_dir = next();
        else if (a == "--time-tag") time_tag = next();
        else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
    }
    if (!events.empty()) return run_events(scene_file, opts, resx, resy, depth, events, img_dir, time_tag);
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
