/*
 * pathtrace_abi.h — the drop-in C-ABI of the MI355X wavefront path tracer (libptamd.so).
 *
 * It replaces the reference's hot-path boundary, src/pathtrace.h:6-9:
 *
 *     void InitDataContainer(GuiDataContainer* guiData);   -> pt_init_data_container
 *     void pathtraceInit(Scene* scene);                    -> pt_init   (+ C++ mirror in include/pathtrace.h)
 *     void pathtraceFree();                                -> pt_free
 *     void pathtrace(uchar4* pbo, int frame, int iteration)-> pt_trace
 *
 * with plain pointers + counts instead of the reference's Scene* (src/scene.h:6-28), and
 * error codes instead of exit(EXIT_FAILURE) (pathtrace.cu:27-49).  The C++ mirror in
 * include/pathtrace.h keeps the reference's exact void signatures on top of this ABI.
 *
 * State is process-global like the reference's file-static device buffers
 * (pathtrace.cu:82-101); the library is not re-entrant.  One process may drive several GPUs:
 * pt_options.num_devices > 1 splits every frame into pixel shards, one per device, traced
 * concurrently and combined into the first device's image after every pt_trace / pt_trace_frames
 * call (over xGMI peer access or RCCL) -- the same pathtrace() call, the same image, bit for bit.  All arrays are in the reference's
 * own layouts (include/pt/scene_structs.h); the library converts them once, at pt_init, to
 * its device layout.  Every function returns PT_OK (0) or a negative PT_E* code;
 * pt_last_error() gives the message.
 */
#ifndef PT_PATHTRACE_ABI_H
#define PT_PATHTRACE_ABI_H

#include <stddef.h>
#include <stdint.h>

#include "pt/scene_structs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* 2: pt_options gained num_devices / device_ids / combine, pt_frame_stats queued_total,
 *    pt_kernel_times tail_ms / tail_from; pt_set_trace_depth
 * 3: pt_frame_stats handed_total / handed_stack_total; pt_set_speculation */
#define PT_ABI_VERSION 3
#define PT_MAX_DEVICES 16

enum {
    PT_OK = 0,
    PT_E_INVALID = -1,      /* bad argument / scene */
    PT_E_STATE = -2,        /* call order (e.g. pt_trace before pt_init) */
    PT_E_HIP = -3,          /* HIP runtime error */
    PT_E_NODEVICE = -4,     /* no gfx950 device visible */
    PT_E_UNSUPPORTED = -5
};

/* Flat view of the reference's Scene (src/scene.h:20-27).  Borrowed for the duration of
 * pt_init only (the library copies what it needs to the device; the reference kept a
 * non-owning Scene* and re-read traceDepth/camera each frame — pt_set_camera covers that). */
typedef struct pt_scene_view {
    const pt_geom* geoms;          int32_t num_geoms;
    const pt_material* materials;  int32_t num_materials;
    const pt_texture* textures;    int32_t num_textures;
    const pt_triangle* triangles;  int32_t num_triangles;
    const int32_t* tri_indices;    int32_t num_tri_indices;
    const pt_bvh_node* bvh_nodes;  int32_t num_bvh_nodes;
    pt_camera camera;
    int32_t trace_depth;           /* RenderState::traceDepth */
} pt_scene_view;

enum { PT_PIPELINE_FUSED = 0, PT_PIPELINE_STAGED = 1 };
enum { PT_SHARD_NONE = 0, PT_SHARD_PIXELS = 1, PT_SHARD_SAMPLES = 2 };
enum { PT_COMBINE_PEER = 0, PT_COMBINE_RCCL = 1 };

typedef struct pt_options {
    int32_t stream_compaction;   /* STREAM_COMPACTION (pathtrace.cu:21), default 1 */
    int32_t material_sort;       /* MATERIAL_SORTING  (pathtrace.cu:22), default 0.  Staged
                                    pipeline: a stable counting sort of the wavefront by
                                    materialId before shading (k_sort_*).  Fused pipeline: the
                                    block's paths are regrouped by material in LDS between
                                    intersection and shading (scenes of <= 63 materials; mesh
                                    hits shaded by the BVH queue kernel are not regrouped).
                                    Results do not depend on path order either way */
    int32_t bvh;                 /* BVH_ACCELERATION  (pathtrace.cu:24), default 1 */
    int32_t arg_order;           /* 0: glm::vec2(u01(rng), u01(rng)) right-to-left (g++), 1: left-to-right */
    int32_t pipeline;            /* PT_PIPELINE_FUSED (default) or PT_PIPELINE_STAGED (one kernel per stage) */
    int32_t use_graph;           /* capture a frame in a hipGraph and replay it (default 1) */
    int32_t device;              /* HIP device ordinal (default 0) */
    int32_t shard_mode;          /* PT_SHARD_*: multi-GPU partition of one frame (default NONE) */
    int32_t shard_rank;
    int32_t shard_count;
    int32_t shard_rows;          /* PIXELS mode: height of the interleaved row bands (default 8) */
    int32_t block_size;          /* threads per block of the per-path kernels (default 256) */
    int32_t variant;             /* fused-kernel variant bits (1: per-wave compaction atomics,
                                    2: per-lane candidate queue for the geom tests, 4: section
                                    timing (tools), 8: exact geom tests redistributed over the
                                    wave's lanes, 16: BVH traversal with exact-decision fast box
                                    tests, near-first order and certified t-culling, 32: rays
                                    that enter the mesh's root box are queued and traversed in
                                    full waves by a second kernel per bounce, 64: keep 16 on the
                                    reference node array instead of the paired-children layout,
                                    128: with 8, the exact-test exchange spans the whole block,
                                    256: 4-wide BVH nodes, 512: material grouping, set by
                                    material_sort; 1024 is set by pt_init itself when no material
                                    has a texture or bump map: the kernels built without texel
                                    fetches); results are bit-identical for every value.  Default
                                    2|8|16|32|128 */
    int32_t frames_per_pass;     /* pt_trace_frames traces F frames per wavefront pass (1..256;
                                    0 = auto: ~84M paths in flight, e.g. 128 at 800x800, 256 for
                                    a 1/8 pixel shard of it).  The image is bit-identical
                                    to frame-by-frame tracing: terminated paths of a pass land in
                                    per-frame planes that are added in frame order. */
    /* ---- ABI 2: several GPUs behind one pathtrace() ---- */
    int32_t num_devices;         /* 0 or 1: one device (`device`).  N > 1: N shard contexts; shard k traces the
                                    interleaved row bands (y / shard_rows) % N == k on device device_ids[k]
                                    (entries may repeat: shards on one GPU run on their own streams).
                                    Requires shard_mode == PT_SHARD_NONE (this is the in-process form of
                                    PT_SHARD_PIXELS).  pt_default_options reads PT_DEVICES from the
                                    environment: "N" (devices 0..N-1) or a list "0,1,1" */
    int32_t device_ids[PT_MAX_DEVICES];   /* default k -> k */
    int32_t combine;             /* how shard images reach the first device's image: PT_COMBINE_PEER (default:
                                    a kernel on the first device reads each shard's pixels over xGMI peer
                                    access) or PT_COMBINE_RCCL (each shard packs its pixels, one RCCL group of
                                    send / recv over a communicator of the distinct devices, librccl.so loaded
                                    at pt_init).  Environment default: PT_COMBINE=rccl|peer */
} pt_options;

typedef struct pt_frame_stats {
    int32_t iteration;           /* iteration of the last traced frame */
    int32_t bounces;             /* trace depth */
    int64_t live[64];            /* paths entering bounce b (b < bounces) */
    int64_t segments;            /* sum of live[] = the metric's path segments */
    int64_t pixels;              /* pixels traced by this process */
    int64_t frames_total;        /* frames traced since pt_init / pt_reset_stats */
    int64_t live_total[65];      /* per-bounce live counts summed over those frames */
    int64_t segments_total;      /* path segments traced over those frames */
    int32_t frames_per_pass;     /* resolved F; live[] / segments above cover the last pass */
    int32_t last_pass_frames;
    int64_t queued_total[65];    /* mesh scenes, fused pipeline: per-bounce paths queued for the BVH
                                    traversal kernel, summed over frames_total frames (0 otherwise) */
    int64_t handed_total[65];    /* ... of those, traversals handed over to the refilling waves */
    int64_t handed_stack_total[65];  /* ... and the stack entries they carried */
} pt_frame_stats;

int32_t pt_abi_version(void);
const char* pt_last_error(void);
void pt_default_options(pt_options* opts);

/* InitDataContainer (pathtrace.cu:103-106): `traced_depth` (GuiDataContainer::TracedDepth)
 * receives the number of bounces traced after each pt_trace; NULL disables. */
int32_t pt_init_data_container(int32_t* traced_depth);

/* pathtraceInit (pathtrace.cu:134-207): upload the scene, size the wavefront for
 * camera.resolution, zero the accumulated image.  Calling it again re-initialises. */
int32_t pt_init(const pt_scene_view* scene, const pt_options* opts);

/* pathtraceFree (pathtrace.cu:209-229). Safe to call when not initialised. */
int32_t pt_free(void);

/* pathtrace(pbo, frame, iteration) (pathtrace.cu:639-787): trace one sample per pixel with
 * 1-based `iteration`, add it into the accumulated image, write the 8-bit preview into
 * `pbo_device` (a DEVICE pointer of width*height pt_uchar4, or NULL), and copy the
 * accumulated (not averaged) image into `host_image` (width*height*3 floats, or NULL) —
 * the reference copies into scene->state.image every call (pathtrace.cu:783-784).  The copy goes
 * straight into the caller's (pageable) memory; nothing about `host_image` is kept between calls. */
int32_t pt_trace(pt_uchar4* pbo_device, int32_t frame, int32_t iteration, float* host_image);

/* Trace `count` frames with iterations first_iteration .. first_iteration+count-1, image stays
 * in HBM (no host copy, no PBO).  The throughput path used by bench.py. */
int32_t pt_trace_frames(int32_t first_iteration, int32_t count);
/* Capture (hipGraph) every pass size a later pt_trace_frames(., count) replays, so that call
 * launches only.  Optional: pt_trace_frames captures on first use. */
int32_t pt_prepare_frames(int32_t count);

/* Block until all queued work finished. */
int32_t pt_synchronize(void);

/* Accumulated image: host copy (n_floats >= width*height*3) / raw device pointer.  The caller may
 * read or write through the device pointer between pt_trace calls: pt_get_image_device drops a
 * speculated next frame (pt_trace with a host copy traces frame N + 1 ahead from the image as it
 * was), so the next pt_trace traces from whatever the caller left in the buffer. */
int32_t pt_get_image(float* host_out, int64_t n_floats);
int32_t pt_get_image_device(void** device_ptr, int64_t* n_floats);
/* Overwrite the accumulated image (host data), e.g. after a multi-GPU reduce. */
int32_t pt_set_image(const float* host_in, int64_t n_floats);

/* Device memory for callers without the HIP headers (a PBO for pt_trace's pbo_device, as the
 * headless viewer of pt/pt_viewer.h uses): hipMalloc / hipFree / synchronous hipMemcpy D->H
 * (after the library's stream drained).  pt_device_alloc fails with PT_E_NODEVICE without a GPU. */
int32_t pt_device_alloc(int64_t bytes, void** out);
int32_t pt_device_free(void* p);
int32_t pt_device_read(void* host_dst, const void* device_src, int64_t bytes);

int32_t pt_get_frame_stats(pt_frame_stats* out);
/* Zero the running totals of pt_frame_stats (frames_total, live_total, segments_total). */
int32_t pt_reset_stats(void);

/* Camera update without re-upload (main.cpp:423-444 path); resets nothing else. */
int32_t pt_set_camera(const pt_camera* camera);
/* RenderState::traceDepth, re-read by the reference at every pathtrace() call (pathtrace.cu:641):
 * the depth of the next frames (0 .. 64); resets nothing else. */
int32_t pt_set_trace_depth(int32_t depth);
/* Next-frame speculation of single-frame calls that copy the image out (pt_trace with host_image:
 * frame N + 1 is traced while frame N's image crosses PCIe; results bit-identical either way).
 * On by default (PT_SPECULATE=0 in the environment at pt_init: off); off drops a speculated frame. */
int32_t pt_set_speculation(int32_t enabled);

/* ---- scene ingest (C++ restatement of scene.cpp, host/scene.cpp) for non-C++ callers ---- */
typedef struct pt_scene_file pt_scene_file;
/* Load a reference JSON scene.  res_x/res_y <= 0 / depth < 0 keep the file's RES/DEPTH (overriding
 * them recomputes pixelLength exactly as editing the file would).  viewer_camera != 0 applies
 * main.cpp:359-380 + 423-444, the camera the reference's frames are rendered with. */
int32_t pt_scene_load(const char* json_path, int32_t res_x, int32_t res_y, int32_t depth, int32_t viewer_camera,
                      pt_scene_file** out);
/* Same, with flags: PT_SCENE_VIEWER_CAMERA (= viewer_camera above), PT_SCENE_GPU_BVH (build the BVH
 * on the current HIP device with pt_bvh_build instead of on the host; the same nodes and triIndices). */
enum { PT_SCENE_VIEWER_CAMERA = 1, PT_SCENE_GPU_BVH = 2 };
int32_t pt_scene_load_ex(const char* json_path, int32_t res_x, int32_t res_y, int32_t depth, int32_t flags,
                         pt_scene_file** out);
/* View borrowed from the scene file (valid until pt_scene_free). */
int32_t pt_scene_get_view(const pt_scene_file* scene, pt_scene_view* view);
int32_t pt_scene_get_info(const pt_scene_file* scene, int32_t* iterations, int32_t* trace_depth, char* image_name,
                          int32_t cap);
int32_t pt_scene_material_name(const pt_scene_file* scene, int32_t id, char* buf, int32_t cap);
void pt_scene_free(pt_scene_file* scene);
const char* pt_scene_last_error(void);
/* Scene::loadTexture's decode (scene.cpp:366-392, stbi_load(..., STBI_rgb_alpha)): PNG -> RGBA8.
 * Writes width/height; copies w*h*4 bytes into rgba when cap is large enough (rgba may be
 * NULL to query the size).  PT_E_INVALID + pt_scene_last_error() on a decode failure. */
int32_t pt_texture_load(const char* path, int32_t* width, int32_t* height, uint8_t* rgba, int64_t cap);

/* Scene::buildBVH + buildBVHRecursive (scene.cpp:445-525) on the current HIP device: bounds,
 * longest-axis midpoint split, the in-place swap partition and the median fallback, level by level
 * on the GPU, with the reference's preorder node numbering -- the same bvhNodes and triIndices as the
 * host build, bit for bit (csrc/pt_bvh_build.hip).  `nodes` holds cap >= 2n - 1 entries;
 * *num_nodes receives the count; tri_indices receives n entries.  PT_E_NODEVICE without a GPU. */
int32_t pt_bvh_build(const pt_triangle* triangles, int32_t n, pt_bvh_node* nodes, int32_t cap, int32_t* num_nodes,
                     int32_t* tri_indices);
const char* pt_bvh_build_last_error(void);

/* saveImage (main.cpp:395-419) + Image::savePNG (image.cpp:23-43): writes "<base_path>.png" from an
 * accumulated host image (width*height*3 floats) traced `iteration` samples per pixel — x-flipped,
 * divided by the sample count, clamped, x255-truncated, encoded byte-identically to the reference's
 * stb_image_write 0.98.  PT_E_INVALID + pt_scene_last_error() on an I/O error. */
int32_t pt_save_png(const float* image, int32_t width, int32_t height, int32_t iteration, const char* base_path);

/* ---- test entry points: run one production kernel on caller data (reference layouts) ---- */
/* generateRayFromCamera for every pixel of this process's shard -> out[pixels] */
int32_t pt_test_camera(int32_t iteration, pt_path_segment* out, int64_t n);
/* computeIntersections on n paths -> isects (zeroed + t=-1 semantics of pathtrace.cu:699,423) */
int32_t pt_test_intersect(const pt_path_segment* paths, int64_t n, pt_shadeable_isect* isects);
/* kernShadeMaterialProper on n (isect, path) pairs, in place; terminated paths are NOT
 * gathered (image untouched) */
int32_t pt_test_shade(int32_t iteration, const pt_shadeable_isect* isects, pt_path_segment* paths, int64_t n);
/* stable partition of n paths on remainingBounces > 0 -> out (alive first, in order);
 * returns the alive count through *alive */
int32_t pt_test_compact(const pt_path_segment* paths, int64_t n, pt_path_segment* out, int64_t* alive);
/* stable sort of n (isect, path) pairs by materialId -> permutation perm[n] */
int32_t pt_test_sort(const pt_shadeable_isect* isects, int64_t n, int32_t* perm);
/* first n draws of makeSeededRandomEngine(iter, index, depth) for m seeds -> out[m*n] */
int32_t pt_test_rng(const int32_t* iter_index_depth, int64_t m, int32_t n, float* out);
/* sendImageToPBO on a caller image (host, n pixels) -> pbo (host) */
int32_t pt_test_pbo(const float* image, int64_t n, int32_t iteration, pt_uchar4* pbo);

/* ---- kernel timing (HIP events on the library's stream) for bench.py ---- */
typedef struct pt_kernel_times {
    int32_t frames;
    float frame_ms;              /* stream time of the whole run / frames */
    float bounce_ms[64];         /* per-launch kernel time of bounce b (see pt_profile_frames) */
    float compact_ms;            /* staged: total compaction-kernel time per frame */
    float intersect_ms, shade_ms, camera_ms, sort_ms;
    int64_t compact_bytes;       /* reserved */
    int64_t frame_bytes;         /* reserved */
    float compact_scan_ms;       /* staged: compaction count + scan kernels per frame (compact_ms = scatter) */
    int32_t passes;              /* wavefront passes the `frames` frames were traced in */
    float combine_ms;            /* k_combine (per-frame planes -> image) per frame */
    float bvh_ms[64];            /* split BVH traversal (variant 32): k_bvh_bounce's part of bounce_ms[b] */
    float tail_ms;               /* single-frame passes of primitive-only scenes: the one k_tail launch that
                                    runs bounces tail_from .. depth-1 (per pass; bounce_ms[b >= tail_from]
                                    stay 0 then) */
    int32_t tail_from;           /* first bounce k_tail ran (0: no k_tail launch) */
} pt_kernel_times;
/* Trace `count` frames with iterations first_iteration.. eagerly, every kernel launched with
 * hipExtLaunchKernel start/stop events (timestamps of that dispatch itself) and no host
 * synchronisation until all frames are queued; returns per-kernel average durations and the
 * stream-level frame time.  bounce_ms[b]: average duration of ONE launch of the fused bounce
 * kernel b, or (staged) of the compaction scatter kernel of bounce b; the other *_ms fields are
 * per frame.  Frames are grouped into passes exactly as pt_trace_frames groups them. */
int32_t pt_profile_frames(int32_t first_iteration, int32_t count, pt_kernel_times* out);

/* Tools: counters filled by the fused kernel when pt_options.variant has bit 4 (section timing):
 * [0..5] shader-clock cycles per section summed over waves (load, cull, exact tests, hit finish,
 * shade, gather+compact+store), [6] exact geom tests, [7] candidates, [8] candidate-loop
 * iterations (per wave), [9] waves, [10] live lanes, [11] BVH node + leaf visits, [12] leaf
 * triangles, [13] traversed rays, [14] box-decision mismatches (node-array traversal), [15] wave
 * traversal iterations, [16] leaf visits, [17] traversed rays whose mesh hit wins, [18] node
 * visits of the rays whose mesh hit does not win, [19] rays culled at the root, [20..35] wave
 * traversal iterations by active lanes in bins of 4 (1-4, 5-8, ..), [36..51] the same for the
 * handed-over traversals' kernel, [52..67] handed-over rays by stack depth (8 buckets: count,
 * nodes visited after), [68..71] by a hit found before (no: count, nodes; yes: count, nodes);
 * [72] candidate-table pre-test superset sizes over the live lanes, [73] the sum over waves of
 * each wave's largest superset, [74] of the size of the union of the wave's supersets; n <= 76.  `reset` zeroes them after the read. */
int32_t pt_debug_section_counters(uint64_t* out, int32_t n, int32_t reset);

/* Next-frame speculation (pt_set_speculation): frames speculated and frames taken over since
 * pt_init, summed over the context's shards (either pointer may be NULL).  Tests and tools. */
int32_t pt_debug_spec_counts(int64_t* launched, int64_t* adopted);

#ifdef __cplusplus
}
#endif
#endif /* PT_PATHTRACE_ABI_H */
