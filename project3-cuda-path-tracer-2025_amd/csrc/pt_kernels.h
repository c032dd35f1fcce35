// pt_kernels.h — per-path stage functions shared by the fused and the staged pipelines.
//
//   camera_ray      generateRayFromCamera         pathtrace.cu:231-292
//   intersect_scene computeIntersections          pathtrace.cu:298-448 (+ intersections.cu)
//   shade_path      kernShadeMaterialProper       pathtrace.cu:521-621 (+ interactions.cu)
//
// Each is a pure function of (scene, path, iteration), so the fused bounce kernel and the
// one-kernel-per-stage pipeline run literally the same code.
#pragma once

#include "pt_device.h"
#include "pt/pt_texture.h"

namespace ptd {

constexpr int NSEG = 8;        // output segments of the fused compaction (one per XCD group)
constexpr int LDS_GEOMS = 64;  // fused kernel: geom tables up to this size are staged in LDS
constexpr int MAXB = 64;       // max trace depth supported by the frame control block
constexpr int BLOCK = 256;     // threads per block of the per-path kernels
constexpr int MAXSTACK = 64;   // reference BVH stack (intersections.cu:167)
constexpr int CNT_PAD = 32;    // one 128-byte cache line per live counter (atomics on separate lines)

// kernel variants (pt_options.variant bits), selectable at run time for in-process A/B
enum : int {
    VAR_WAVE_ATOMIC = 1,   // compaction: one atomic per wave, no block barrier
    VAR_CAND_QUEUE = 2,    // intersection: per-lane queue of candidate geoms (see intersect_scene_q)
    VAR_SECTION_TIMING = 4,    // tools only: per-wave shader-clock section times into g_sections
    VAR_WAVE_REDIST = 8,   // intersection: the wave's (ray, candidate) pairs spread over all 64 lanes
    VAR_BVH_FAST = 16,     // BVH: exact-decision fast AABB test, near-first order, certified t-culling
    VAR_CTILE8 = 16,       // staged compaction: 8 items per thread (2048-item tiles)
    VAR_BVH_SPLIT = 32,    // fused + BVH_FAST + pair layout: rays that enter the mesh's root box are
                           // queued and traversed (then shaded) by k_bvh_bounce in full waves
    VAR_BVH_NODES = 64,    // host only: BVH_FAST on the node array instead of the DevPair layout (A/B)
    VAR_BLOCK_REDIST = 128,  // with VAR_WAVE_REDIST: the exchange spans the block (block_intersect)
    VAR_MAT_GROUP = 512,   // fused MATERIAL_SORTING: the block's paths regrouped by material between
                           // intersection and shading (group_by_material); set by pt_options.material_sort
    VAR_NO_TEX = 1024,     // host-set: no material samples a texture or bump map, so the fused kernels'
                           // shading is compiled without the texel fetches (whose registers otherwise set
                           // the kernels' VGPR count and occupancy)
};

struct CamDev {
    int resx, resy;
    f3 position, view, up, right;
    float plx, ply;
    float aperture, focalDist;
};

struct ShardDev {
    int mode;          // PT_SHARD_*
    int rank, count, rows;
    int local_pixels;
};

struct SceneDev {
    const DevGeom* geoms;
    const DevCull* cull;      // candidate pre-test records, one per geom
    const DevMaterial* mats;
    const DevNode* nodes;
    const DevTriHot* hot;
    const DevTriCold* cold;
    int num_geoms, num_mats, num_nodes, num_tris;
    int trace_depth, arg_order, use_bvh, stack_depth;
    int pair_stack_depth;     // bvh_intersect_pairs' push bound (<= stack_depth)
    CamDev cam;
    ShardDev shard;
    float* contrib;     // passes of F > 1 frames: [slot][pixel] float3 of each terminated path
    const float4* node_aux;   // per BVH node: MT error coefficient, max edge, reference DFS rank
    const uint32_t* texels;   // all textures' RGBA8 texels, concatenated
    const int4* texinfo;      // per texture: texel offset, width, height
    int num_textures;
    // VAR_BVH_FAST layout (pairs != null when the tree allows it, see DevPair)
    const DevPair* pairs;
    // 4-wide layout of the same hierarchy (trav_inner4, trees past the L2; null: pairs only):
    // num_quads records of 8 float4 = one 128-B line each, leaves referenced as num_quads + leaf
    const float4* quads;
    int num_quads;
    // traversal stack of the split kernels: entries [0, stack_lds) in the block's LDS, deeper
    // ones (rare) in `spill`, spill_stride entries per traversal-queue slot (TravState::qs)
    int stack_lds, spill_stride;
    int* spill;
    const DevTriHot* hot4;    // 4-slot triangle groups per leaf; slot 0's c.z = count (int bits)
    const float4* leaf9;      // per leaf, 9 float4: v0.x v0.y v0.z e1.x .. e2.z, each over the 4 slots
    int num_pairs, root_ref;
    int ref_shift;            // pair-layout stack entries: ref << ref_shift | T field (pack_ref)
    float4 root_lo, root_hi;  // root box (w: root s)
    float cull_c0;            // c = s^2 * cull_c0 (64 2^-24 / 1e-5, rounded up)
    float cull_E;             // scene extent (rounded up): cE = c * cull_E
    // candidate table of the pre-test (scenes of GRID_MIN_GEOMS..64 geoms; null: flat pre-test):
    // per (origin cell, direction bin) the geoms a ray from that cell in that cone can hit
    const unsigned long long* grid;
    unsigned long long grid_all;   // every geom (rays outside the table's domain)
    float grid_lo[3], grid_inv[3]; // cell = floor((o - grid_lo) * grid_inv), GRID_G per axis
};

// The candidate table's resolution: GRID_G^3 origin cells x 6 faces x GRID_B^2 direction bins.
// An entry is the AND of one mask per ratio bin (build_candidate_table), so the table is stored
// separably (PT_GRID_SEP): 2 GRID_B masks per (cell, face), 2.65 MB at 12 / 16 (L2-resident).
// 16 / 16 against 8 / 8: khaslana superset 5.68 -> 3.60 per ray, 13.8 -> 8.4 at the wave maximum,
// frame -3 %; 12 / 16 times the same as 16 / 16 with 10 % less k_bounce traffic
#ifndef PT_GRID_G
#define PT_GRID_G 12
#endif
#ifndef PT_GRID_B
#define PT_GRID_B 16
#endif
#ifndef PT_GRID_SEP
#define PT_GRID_SEP 1
#endif
constexpr int GRID_G = PT_GRID_G;
constexpr int GRID_B = PT_GRID_B;
constexpr int GRID_MIN_GEOMS = 16;

// frame control block (device memory); zeroed / advanced by k_frame_begin every frame
struct FrameCtl {
    int iter;           // iteration of the pass's first frame (slot s traces iter + s)
    int batch;          // frames in the current pass
    int plane;          // 1: a single-frame pass stores its contributions to plane 0 (speculative frame)
    int _pad;
    unsigned long long frames;              // frames started since the last stats reset
    unsigned long long tot[MAXB + 1];       // sum over finished frames of paths entering bounce b
    unsigned long long qtot[MAXB + 1];      // the same for qcnt (paths of bounce b queued for traversal)
    unsigned long long htot[MAXB + 1];      // ... traversals handed over to k_bvh_tail_trav (qcnt[b][s][3])
    unsigned long long hstk[MAXB + 1];      // ... their saved stack entries (qcnt[b][s][4])
    int cnt[MAXB + 1][NSEG][CNT_PAD];       // paths entering bounce b, per output segment ([..][0])
    // VAR_BVH_SPLIT: paths of bounce b queued for traversal, per queue segment (blockIdx % NSEG of
    // the queuing k_bounce block).  One counter per segment, not one for the whole queue: every
    // block's returning atomic on ONE word serialised at the memory side (~88 / us, the guide's
    // 'dequeue' row) -- 43k blocks per launch put a ~0.5 ms floor under k_bounce in mesh scenes
    int qcnt[MAXB + 1][NSEG][CNT_PAD];
};

// VAR_SECTION_TIMING (tools/section_times.py): wave-level s_memtime deltas per kernel section and
// per-lane work counters, summed by the first active lane of each wave
enum { SEC_LOAD, SEC_CULL, SEC_EXACT, SEC_FINISH, SEC_SHADE, SEC_STORE, SEC_N_EXACT, SEC_N_CAND, SEC_N_ITERS,
       SEC_N_WAVES, SEC_N_LANES, SEC_N_NODES, SEC_N_TRIS, SEC_N_BVH_RAYS, SEC_N_BVH_ITERS, SEC_N_BVH_WITERS,
       SEC_N_LEAVES, SEC_N_BVH_HITS, SEC_N_MISS_NODES, SEC_N_ROOT_CULLED,
       SEC_BVH_LANES_HIST,                    // 16 bins: wave traversal steps by active lanes (1-4, 5-8, ..)
       SEC_TAIL_LANES_HIST = SEC_BVH_LANES_HIST + 16,   // the same for k_bvh_tail_trav's steps
       SEC_TAIL_BY_SP = SEC_TAIL_LANES_HIST + 16,   // handed-over rays by stack depth at the hand-over
                                                    // (0, 1, 2, 3, 4-5, 6-7, 8-11, 12+): count, nodes after
       SEC_TAIL_BY_HIT = SEC_TAIL_BY_SP + 16,       // ... by "a hit found before": no (count, nodes), yes
       SEC_N_SUP = SEC_TAIL_BY_HIT + 4,             // candidate table: superset sizes over the live lanes
       SEC_N_SUP_WMAX,                              // ... and the sum over waves of the wave's largest
       SEC_N_SUP_WUNION,                            // ... and of the size of the union of the wave's supersets
       SEC_COUNT };
constexpr int SEC_SLOTS = 76;
__device__ unsigned long long g_sections[SEC_SLOTS];
PT_DEV uint64_t sec_clock() { return __builtin_amdgcn_s_memtime(); }
PT_DEV void sec_add(int k, uint64_t v) {
    // one atomic per wave: the first active lane adds the wave's value
    if (__builtin_amdgcn_read_exec() == 0) return;
    const int lane = threadIdx.x & 63;
    const int first = __builtin_ctzll(__builtin_amdgcn_read_exec());
    if (lane == first) atomicAdd(&g_sections[k], (unsigned long long)v);
}
PT_DEV void sec_add_lanes(int k, int v) {    // sum over the active lanes (may be called divergently)
    if (v) atomicAdd(&g_sections[k], (unsigned long long)v);
}

// a wavefront of paths: three float4 streams
struct PathBuf {
    float4* A;   // origin.xyz | pixelIndex
    float4* B;   // direction.xyz | remainingBounces
    float4* C;   // throughput.rgb | unused
};

PT_DEV PathReg load_path(const PathBuf& b, int i) {
    float4 a = b.A[i], d = b.B[i], c = b.C[i];
    PathReg p;
    p.o = mk(a.x, a.y, a.z);
    p.pix = __float_as_int(a.w);
    p.d = mk(d.x, d.y, d.z);
    p.rb = __float_as_int(d.w);
    p.c = mk(c.x, c.y, c.z);
    p.slot = __float_as_int(c.w);
    return p;
}
PT_DEV void store_path(const PathBuf& b, int i, const PathReg& p) {
    b.A[i] = make_float4(p.o.x, p.o.y, p.o.z, __int_as_float(p.pix));
    b.B[i] = make_float4(p.d.x, p.d.y, p.d.z, __int_as_float(p.rb));
    b.C[i] = make_float4(p.c.x, p.c.y, p.c.z, __int_as_float(p.slot));
}

// local path id of this process -> global pixel index (PIXELS shard: interleaved row bands)
PT_DEV int shard_pixel_of(const ShardDev& sh, int W, int l) {
    if (sh.mode != 1) return l;
    int lr = l / W, x = l - lr * W;
    int band = lr / sh.rows, within = lr - band * sh.rows;
    int y = (band * sh.count + sh.rank) * sh.rows + within;
    return x + y * W;
}
PT_DEV int shard_pixel(const SceneDev& sc, int l) { return shard_pixel_of(sc.shard, sc.cam.resx, l); }

// generateRayFromCamera + sampleAperture (pathtrace.cu:231-292) for pixel `index`
PT_DEV PathReg camera_ray(const CamDev& cam, int iter, int trace_depth, int index) {
    int y = index / cam.resx;
    int x = index - y * cam.resx;
    Rng rng = rng_make(iter, index, 0);
    float jitterX = u01(rng);
    float jitterY = u01(rng);
    float sx = (float)x + jitterX - (float)cam.resx * 0.5f;
    float sy = (float)y + jitterY - (float)cam.resy * 0.5f;
    f3 pixelPoint = cam.view - (cam.right * cam.plx) * sx - (cam.up * cam.ply) * sy;
    f3 rayDir = normalize(pixelPoint);
    f3 focalPoint = cam.position + rayDir * cam.focalDist;
    float r = cam.aperture * __builtin_sqrtf(u01(rng));
    float theta = 2.0f * PI * u01(rng);
    float s, c;
    pt_sincosf(theta, &s, &c);
    f3 apertureOffset = mk(r * c, r * s, 0.0f);
    PathReg p;
    p.o = cam.position + apertureOffset;
    p.c = mk(1.f, 1.f, 1.f);
    p.d = normalize(focalPoint - p.o);
    p.pix = index;
    p.rb = trace_depth;
    p.slot = 0;
    return p;
}

struct Hit {
    float t;        // -1 on miss
    f3 n;
    int mat;
    int tri;        // winning triangle (reference index) or -1
    float u, v;
};

// bvhMeshIntersectionTest (intersections.cu:148-234): same DFS order (push left, push right,
// pop right first), same strict `t < t_hit` acceptance, so exact-t ties resolve identically.
// `stack` is this thread's column of an LDS array (stride BLOCK).  Returns the winner's leaf
// slot (index into the leaf-ordered hot triangle array) in `btri`.
template <bool COUNT = false>
PT_DEV float bvh_intersect(const SceneDev& sc, f3 ro, f3 rd, int* stack, float& bu, float& bv, int& btri) {
    int n_nodes = 0, n_tris = 0;
    float t_hit = FLT_MAX_;
    bool hit = false;
    btri = -1;
    int sp = 0;
    stack[0] = 0;
    sp = 1;
    while (sp > 0) {
        if (COUNT) sec_add(SEC_N_BVH_WITERS, 1);
        int ni = stack[(--sp) * BLOCK];
        DevNode nd = sc.nodes[ni];
        if (COUNT) n_nodes++;
        if (!aabb_test(nd.lo, nd.hi, ro, rd)) continue;
        int a = __float_as_int(nd.lo.w), b = __float_as_int(nd.hi.w);
        if (b <= -2) {
            int cnt = -b - 2;
            if (COUNT) n_tris += cnt;
            for (int i = 0; i < cnt; ++i) {
                DevTriHot th = sc.hot[a + i];
                f3 v0 = mk(th.a.x, th.a.y, th.a.z);
                f3 v1 = mk(th.a.w, th.b.x, th.b.y);
                f3 v2 = mk(th.b.z, th.b.w, th.c.x);
                float t, u, v;
                if (tri_test(ro, rd, v0, v1, v2, t, u, v)) {
                    if (t < t_hit && t > 0.0f) {
                        hit = true;
                        t_hit = t;
                        bu = u;
                        bv = v;
                        btri = a + i;
                    }
                }
            }
        } else {
            if (a >= 0 && sp < sc.stack_depth) stack[(sp++) * BLOCK] = a;
            if (b >= 0 && sp < sc.stack_depth) stack[(sp++) * BLOCK] = b;
        }
    }
    if (COUNT) {
        sec_add_lanes(SEC_N_NODES, n_nodes);
        sec_add_lanes(SEC_N_TRIS, n_tris);
        sec_add_lanes(SEC_N_BVH_RAYS, 1);
    }
    return hit ? t_hit : -1.f;
}

// ---- faster traversal with the SAME result (VAR_BVH_FAST) ----------------------------------
// 1. aabb_decide(): the reference's aabbIntersectionTest decision, computed with rcp slabs.
//    Each slab distance differs from the reference's fl((b - o) / d) by < 2^-22 relative and
//    has the same sign, so `t_max > 0` is decided exactly and `t_max >= t_min` whenever the gap
//    exceeds 1e-6 (|t_min| + |t_max|); otherwise (or for a NaN ray) the reference arithmetic
//    decides.  The visited node set is therefore the reference's.
// 2. Children are visited nearest-entry first.  Ties in t are resolved by the reference's visit
//    order (DFS rank of the leaf, then the slot), so the winner is the reference's: the first
//    triangle of minimal t in ITS order.
// 3. A node is skipped when its entry distance exceeds the best t so far (t_limit = the geoms'
//    t_min included) by more than the Moller-Trumbore error bound of any triangle below it, so
//    no skipped triangle could have tied or won.  For edges up to s and |det| >= 1e-5 (which
//    intersectTriangle requires) with |d| = 1, the computed t of a hit differs from the
//    geometric one by at most t * c (2 + s / t) (cross/dot rounding, relative) + c E (rounding
//    of v1 - v0, v2 - v0, o - v0 for coordinates up to E, absolute), c = 64 * 2^-24 * s^2 / 1e-5
//    (about 10x the first-order bound).  aux = (c, s, DFS rank, c E).
PT_DEV bool aabb_decide(float4 lo, float4 hi, f3 ro, f3 rd, f3 rr, bool exact, float& entry) {
    float tmin = -FLT_MAX_, tmax = FLT_MAX_;
    const float bmin[3] = {lo.x, lo.y, lo.z};
    const float bmax[3] = {hi.x, hi.y, hi.z};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float dir = comp(rd, i), origin = comp(ro, i);
        if (__builtin_fabsf(dir) < 0.00001f) {
            if (origin < bmin[i] || origin > bmax[i]) return false;
        } else {
            const float r = comp(rr, i);
            const float t1 = (bmin[i] - origin) * r, t2 = (bmax[i] - origin) * r;
            tmin = __builtin_fmaxf(tmin, __builtin_fminf(t1, t2));
            tmax = __builtin_fminf(tmax, __builtin_fmaxf(t1, t2));
        }
    }
    entry = tmin;
    if (!exact) {
        if (!(tmax > 0.f)) return false;
        const float e = 1e-6f * (__builtin_fabsf(tmin) + __builtin_fabsf(tmax));
        if (tmax - tmin > e) return true;
        if (tmin - tmax > e) return false;
    }
    return aabb_test(lo, hi, ro, rd);
}
// aabb_decide for a ray that is finite with every |d| >= 1e-5 (no per-axis "parallel" branch,
// no exact-mode branch): the same slab values, max / min taken in another association (exact
// operations, no NaN can arise), the same certain-pass / certain-fail thresholds.  `amb` is set
// when neither is certain; the caller then asks aabb_test (the reference arithmetic).
PT_DEV bool aabb_fast(float4 lo, float4 hi, f3 ro, f3 rr, float& entry, bool& amb) {
    const float t1x = (lo.x - ro.x) * rr.x, t2x = (hi.x - ro.x) * rr.x;
    const float t1y = (lo.y - ro.y) * rr.y, t2y = (hi.y - ro.y) * rr.y;
    const float t1z = (lo.z - ro.z) * rr.z, t2z = (hi.z - ro.z) * rr.z;
    const float tmin = __builtin_fmaxf(__builtin_fmaxf(-FLT_MAX_, __builtin_fminf(t1x, t2x)),
                                       __builtin_fmaxf(__builtin_fminf(t1y, t2y), __builtin_fminf(t1z, t2z)));
    const float tmax = __builtin_fminf(__builtin_fminf(FLT_MAX_, __builtin_fmaxf(t1x, t2x)),
                                       __builtin_fminf(__builtin_fmaxf(t1y, t2y), __builtin_fmaxf(t1z, t2z)));
    entry = tmin;
    const float e = 1e-6f * (__builtin_fabsf(tmin) + __builtin_fabsf(tmax));
    const bool pos = tmax > 0.f;
    const bool yes = pos & (tmax - tmin > e);
    const bool no = !pos | (tmin - tmax > e);
    amb = !(yes | no);
    return yes;
}
PT_DEV bool node_culled(float entry, float4 aux, float t_best) {
    if (!(entry > 0.0f)) return false;
    const float rho = aux.x * (2.0f + aux.y * __builtin_amdgcn_rcpf(t_best) * 1.001f) + 1e-6f;
    return entry * (1.0f - 1e-6f) > t_best * (1.0f + rho) + aux.w;
}
// stack entry: node (16 bits) | entry distance truncated to bf16 (a lower bound for entry >= 0)
PT_DEV uint32_t pack_entry(int node, float entry) {
    const uint32_t eb = __float_as_uint(__builtin_fmaxf(entry, 0.0f)) >> 16;
    return ((uint32_t)node << 16) | eb;
}
template <bool COUNT = false>
PT_DEV float bvh_intersect_fast(const SceneDev& sc, f3 ro, f3 rd, int* stack, float t_limit, float& bu, float& bv,
                                int& btri) {
    int n_nodes = 0, n_tris = 0;
    const bool exact = !(ro.x - ro.x == 0.f && ro.y - ro.y == 0.f && ro.z - ro.z == 0.f &&
                         rd.x - rd.x == 0.f && rd.y - rd.y == 0.f && rd.z - rd.z == 0.f);   // NaN / inf ray
    const f3 rr = mk(__builtin_amdgcn_rcpf(rd.x), __builtin_amdgcn_rcpf(rd.y), __builtin_amdgcn_rcpf(rd.z));
    const bool packed = sc.num_nodes <= 65536;
    float t_hit = FLT_MAX_;
    bool hit = false;
    int hit_rank = 0x7fffffff, hit_i = 0;
    btri = -1;
    float e0;
    if (!aabb_decide(sc.nodes[0].lo, sc.nodes[0].hi, ro, rd, rr, exact, e0)) return -1.f;
    int sp = 0;
    stack[0] = packed ? (int)pack_entry(0, e0) : 0;
    sp = 1;
    while (sp > 0) {
        if (COUNT) sec_add(SEC_N_BVH_WITERS, 1);
        const uint32_t w = (uint32_t)stack[(--sp) * BLOCK];
        const int ni = packed ? (int)(w >> 16) : (int)w;
        const float t_best = __builtin_fminf(t_hit, t_limit);
        const float4 aux = sc.node_aux[ni];
        if (packed && node_culled(__uint_as_float(w << 16), aux, t_best)) continue;
        const DevNode nd = sc.nodes[ni];
        const int a = __float_as_int(nd.lo.w), b = __float_as_int(nd.hi.w);
        if (COUNT) n_nodes++;
        if (b <= -2) {
            const int cnt = -b - 2;
            if (COUNT) n_tris += cnt;
            const int rank = __float_as_int(aux.z);
            for (int i = 0; i < cnt; ++i) {
                const DevTriHot th = sc.hot[a + i];
                const f3 v0 = mk(th.a.x, th.a.y, th.a.z);
                const f3 v1 = mk(th.a.w, th.b.x, th.b.y);
                const f3 v2 = mk(th.b.z, th.b.w, th.c.x);
                float t, u, v;
                if (tri_test(ro, rd, v0, v1, v2, t, u, v) && t > 0.0f &&
                    (t < t_hit || (t == t_hit && (rank < hit_rank || (rank == hit_rank && i < hit_i))))) {
                    hit = true;
                    t_hit = t;
                    hit_rank = rank;
                    hit_i = i;
                    bu = u;
                    bv = v;
                    btri = a + i;
                }
            }
        } else {
            float ea = 0.f, eb = 0.f;
            bool pa = a >= 0 && aabb_decide(sc.nodes[a].lo, sc.nodes[a].hi, ro, rd, rr, exact, ea);
            bool pb = b >= 0 && aabb_decide(sc.nodes[b].lo, sc.nodes[b].hi, ro, rd, rr, exact, eb);
            if (COUNT) {   // debug: the fast decision must equal the reference test
                const bool ra = a >= 0 && aabb_test(sc.nodes[a].lo, sc.nodes[a].hi, ro, rd);
                const bool rb = b >= 0 && aabb_test(sc.nodes[b].lo, sc.nodes[b].hi, ro, rd);
                sec_add_lanes(SEC_N_BVH_ITERS, (ra != pa) + (rb != pb));
            }
            const float tb2 = __builtin_fminf(t_hit, t_limit);
            if (pa && node_culled(ea, sc.node_aux[a], tb2)) pa = false;
            if (pb && node_culled(eb, sc.node_aux[b], tb2)) pb = false;
            // push the farther child first so the nearer one is popped first
            int n1 = a, n2 = b;
            float e1 = ea, e2 = eb;
            bool p1 = pa, p2 = pb;
            if (pa && pb && ea < eb) {
                n1 = b; n2 = a; e1 = eb; e2 = ea;
            }
            if (p1 && sp < sc.stack_depth) stack[(sp++) * BLOCK] = packed ? (int)pack_entry(n1, e1) : n1;
            if (p2 && sp < sc.stack_depth) stack[(sp++) * BLOCK] = packed ? (int)pack_entry(n2, e2) : n2;
        }
    }
    if (COUNT) {
        sec_add_lanes(SEC_N_NODES, n_nodes);
        sec_add_lanes(SEC_N_TRIS, n_tris);
        sec_add_lanes(SEC_N_BVH_RAYS, 1);
    }
    return hit ? t_hit : -1.f;
}

// VAR_BVH_FAST on the pair layout: the same visited-node decisions, cull bound and tie rule as
// bvh_intersect_fast, restructured for fewer dependent fetches.
//  * the node being expanded is a 64-B DevPair of its children: one record fetch yields both
//    boxes (exact-decision aabb_decide), their refs and their cull sizes;
//  * the nearer accepted child is expanded next without touching the stack; the farther one is
//    pushed as [ref | T] (pack_ref), where T is the cull threshold of node_culled solved for t_best
//    (culled iff t_best < T, T rounded down), so a pop needs no fetch to decide the cull;
//  * leaf triangles live in 4-slot groups in reference visit order: ties on t go to the smaller
//    hot4 index, i.e. to the triangle the reference meets first.
// node_culled(entry, {c, s, ., cE}, t): entry(1-1e-6) > t(1 + c(2 + 1.001 s/t) + 1e-6) + cE
//   <=> t < (entry(1-1e-6) - 1.001 c s - cE) / (1 + 2c + 1e-6); evaluated with extra 1e-6 slack
//   on each side for the float rounding of this rearrangement.
PT_DEV float cull_threshold(const SceneDev& sc, float entry, float s) {
    const float c = (s * s) * sc.cull_c0;
    const float num = entry * (1.0f - 2e-6f) - (c * s * 1.002f + c * sc.cull_E * (1.0f + 1e-6f));
    const float T = num * __builtin_amdgcn_rcpf(1.0f + 2.0f * c + 2e-6f) * (1.0f - 1e-6f);
    return T > 0.0f ? T : 0.0f;      // NaN (inf - inf on degenerate data) -> 0: never culled
}
// Stack entry of the pair layout: [ref : 32 - S | T field : S], S = SceneDev::ref_shift (the
// fewest ref bits the tree's P + L refs need, so small trees keep more of T).  The field holds the
// top S bits of u = clamp(bits(T), T_BIAS, T_BIAS + 2^30 - 1) - T_BIAS, i.e. T's exponent from
// 2^-17 to 2^111 and as much mantissa as fits; truncation rounds T down, which only culls less.
// Below 2^-17 the field is 0 and decodes to 2^-17: a cull then needs t_best < 2^-17, and with
// t_best below 1e-5 no triangle can be accepted at all (tri_test_e rejects t <= 1e-5), so such a
// cull never changes a result.  Refs up to 2^24 - 1 (S >= 8).
constexpr uint32_t T_BIAS = 0x37000000u;   // bits of 2^-17
PT_DEV uint32_t pack_ref(int ref, float T, int S) {
    const uint32_t b = __float_as_uint(T);
    const uint32_t u = __builtin_elementwise_min(__builtin_elementwise_max(b, T_BIAS), T_BIAS + 0x3fffffffu) - T_BIAS;
    return ((uint32_t)ref << S) | (u >> (30 - S));
}
PT_DEV float unpack_T(uint32_t w, int S) {
    return __uint_as_float((__builtin_amdgcn_ubfe(w, 0, S) << (30 - S)) + T_BIAS);
}
// cull_threshold from the per-child constants the host packs into DevPair's hi.w (pack_cull in
// pt_runtime.hip): high half A >= 1.002 c s + c E (1 + 1e-6), low half d >= 1 - (1 - 1e-6) /
// (1 + 2c + 2e-6), both rounded UP to 16-bit floats.  T = (entry (1 - 2e-6) - A)(1 - d), two fmas
// (each one rounding, covered by the 1e-6 factor), never exceeds the certified threshold
// (entry (1 - 1e-6) - 1.001 c s - c E) / (1 + 2c + 1e-6).  NaN / negative -> 0: never culled.
PT_DEV float cull_threshold_packed(float entry, float w) {
    const uint32_t b = __float_as_uint(w);
    const float A = __uint_as_float(b & 0xffff0000u), d = __uint_as_float(b << 16);
    const float x = __builtin_fmaf(entry, 1.0f - 2e-6f, -A);
    return __builtin_fmaxf(__builtin_fmaf(-d, x, x), 0.0f);
}

// traversal state of one ray on the pair layout
struct TravState {
    f3 ro, rd, rr;
    float t_hit, bu, bv;   // t_hit starts at t_limit (the primitives' t): see trav_begin
    int btri, cur, sp;
    int qs;       // traversal-queue slot (the spill area's row; -1: LDS stack only)
    float curT;   // certified cull threshold of st.cur (0: none)
    bool exact;
    bool wfast;   // wave-uniform: every ray of the wave is finite with all |d| >= 1e-5 (aabb_fast)
};
// the ray's part of the state (wfast over the lanes that call it together)
PT_DEV void trav_ray(TravState& st, f3 ro, f3 rd) {
    st.ro = ro;
    st.rd = rd;
    st.exact = !(ro.x - ro.x == 0.f && ro.y - ro.y == 0.f && ro.z - ro.z == 0.f &&
                 rd.x - rd.x == 0.f && rd.y - rd.y == 0.f && rd.z - rd.z == 0.f);   // NaN / inf ray
    const bool par = __builtin_fabsf(rd.x) < 0.00001f || __builtin_fabsf(rd.y) < 0.00001f ||
                     __builtin_fabsf(rd.z) < 0.00001f;
    st.wfast = __all(!(st.exact || par));
    st.rr = mk(__builtin_amdgcn_rcpf(rd.x), __builtin_amdgcn_rcpf(rd.y), __builtin_amdgcn_rcpf(rd.z));
}
PT_DEV void trav_begin(const SceneDev& sc, TravState& st, f3 ro, f3 rd, float t_limit) {
    trav_ray(st, ro, rd);
    // t_hit starts at the primitives' t_limit instead of FLT_MAX: the culls used min(t_hit,
    // t_limit), which is then t_hit itself, and a triangle farther than t_limit can never win (the
    // primitive keeps ties, make_hit's strict `<`), so the result is the same and the traversal
    // carries one register fewer.  "No triangle" is btri still at its sentinel.
    st.t_hit = t_limit;
    st.bu = st.bv = 0.f;
    st.btri = 0x7fffffff;
    st.sp = 0;
    st.qs = -1;
    st.curT = 0.f;
    float e0;
    st.cur = (aabb_decide(sc.root_lo, sc.root_hi, ro, rd, st.rr, st.exact, e0) &&
              !(t_limit < cull_threshold(sc, e0, sc.root_hi.w)))
                 ? sc.root_ref
                 : -1;
}
// stack entry i of the ray: the block's LDS below sc.stack_lds, its spill row above (split kernels)
PT_DEV int* trav_slot(const SceneDev& sc, const TravState& st, int* stack, int i) {
    return (i < sc.stack_lds || st.qs < 0) ? stack + i * BLOCK
                                           : sc.spill + (size_t)st.qs * sc.spill_stride + (i - sc.stack_lds);
}
PT_DEV void trav_push(const SceneDev& sc, TravState& st, int* stack, uint32_t w) {
    if (st.sp < sc.pair_stack_depth) *trav_slot(sc, st, stack, st.sp++) = (int)w;
}
// pop the nearest stack entry whose certified cull does not reject it (st.cur = -1: empty)
PT_DEV void trav_pop(const SceneDev& sc, TravState& st, int* stack) {
    const float tb = st.t_hit;
    const int S = sc.ref_shift;
    st.cur = -1;
    while (st.sp > 0) {
        const uint32_t w = (uint32_t)*trav_slot(sc, st, stack, --st.sp);
        const float T = unpack_T(w, S);
        if (!(tb < T)) {
            st.cur = (int)(w >> S);
            st.curT = T;
            break;
        }
    }
}
// expand the internal node st.cur: both child boxes decided exactly (aabb_fast / aabb_decide),
// certified culls, the nearer passing child continues (true) and the farther one is pushed;
// false: no child passes (the caller pops)
template <bool COUNT = false>
PT_DEV bool trav_inner(const SceneDev& sc, TravState& st, int* stack, int& n_nodes) {
    const float t_best = st.t_hit;
    if (COUNT) n_nodes++;
    const DevPair pr = sc.pairs[st.cur];
    PT_HOOK(PROBE_INNER, sc, st.cur, pr);
    float el = 0.f, er = 0.f;
    bool pl, pb;
    if (st.wfast) {   // wave-uniform
        bool al, ar;
        pl = aabb_fast(pr.l_lo, pr.l_hi, st.ro, st.rr, el, al);
        pb = aabb_fast(pr.r_lo, pr.r_hi, st.ro, st.rr, er, ar);
        if (al | ar) {   // rare: a gap within the rcp slabs' error, the reference decides
            if (al) pl = aabb_test(pr.l_lo, pr.l_hi, st.ro, st.rd);
            if (ar) pb = aabb_test(pr.r_lo, pr.r_hi, st.ro, st.rd);
        }
    } else {
        pl = aabb_decide(pr.l_lo, pr.l_hi, st.ro, st.rd, st.rr, st.exact, el);
        pb = aabb_decide(pr.r_lo, pr.r_hi, st.ro, st.rd, st.rr, st.exact, er);
    }
    const float Tl = cull_threshold_packed(el, pr.l_hi.w);
    const float Tr = cull_threshold_packed(er, pr.r_hi.w);
    pl = pl && !(t_best < Tl);
    pb = pb && !(t_best < Tr);
    const int rl = __float_as_int(pr.l_lo.w), rrf = __float_as_int(pr.r_lo.w);
    if (pl && pb) {
        const bool lfirst = el <= er;
        st.cur = lfirst ? rl : rrf;
        st.curT = lfirst ? Tl : Tr;
        const int far = lfirst ? rrf : rl;
        const float Tf = lfirst ? Tr : Tl;
        trav_push(sc, st, stack, pack_ref(far, Tf, sc.ref_shift));
        return true;
    }
    if (pl | pb) {
        st.cur = pl ? rl : rrf;
        st.curT = pl ? Tl : Tr;
        return true;
    }
    return false;
}
// test the 4 slots of leaf `leaf` (ref - num_pairs): 9 float4, component k of slots 0..3, the
// edges v1 - v0, v2 - v0 precomputed (same float rounding).  Unused slots are all-zero (det = 0:
// rejected; a NaN ray gets t = NaN, which `t > 0` never accepts).  Ties on t go to the smaller
// slot (the reference's visit order), so the order leaves are tested in does not matter.
template <bool COUNT = false>
PT_DEV void trav_leaf(const SceneDev& sc, TravState& st, int leaf, int& n_nodes, int& n_tris) {
    const int base = 4 * leaf;
    if (COUNT) {
        n_nodes++;
        n_tris += __float_as_int(sc.hot4[base].c.z);
        sec_add_lanes(SEC_N_LEAVES, 1);
    }
    const v4f* L = reinterpret_cast<const v4f*>(sc.leaf9) + 9 * (size_t)leaf;
    v4f c[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) c[k] = L[k];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f3 v0 = mk(c[0][i], c[1][i], c[2][i]);
        const f3 e1 = mk(c[3][i], c[4][i], c[5][i]);
        const f3 e2 = mk(c[6][i], c[7][i], c[8][i]);
        float t, u, v;
        if (tri_test_e(st.ro, st.rd, v0, e1, e2, t, u, v) && t > 0.0f &&
            (t < st.t_hit || (t == st.t_hit && base + i < st.btri))) {
            st.t_hit = t;
            st.bu = u;
            st.bv = v;
            st.btri = base + i;
        }
    }
}
// 4-wide node (SceneDev::quads): up to four children of the same hierarchy -- a pair's children,
// or for an inner child its own two children (two levels in one record) -- in ONE 128-B line:
// float4 [0..2] lo.x / lo.y / lo.z of children 0..3, [3..5] hi.x / hi.y / hi.z, [6] refs (int
// bits, -1: no child), [7] cull constants (pack_cull).  Every passing, not culled child is kept:
// the nearest continues, the others are pushed farthest first (so they pop nearest first).  Box
// decisions and culls are trav_inner's, child by child, so the visited leaves are the same.
template <bool COUNT = false>
PT_DEV bool trav_inner4(const SceneDev& sc, TravState& st, int* stack, int& n_nodes) {
    const float t_best = st.t_hit;
    if (COUNT) n_nodes++;
    const v4f* Q = reinterpret_cast<const v4f*>(sc.quads) + 8 * (size_t)st.cur;
    v4f q[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) q[k] = Q[k];
    float key[4], T[4];
    int ref[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float4 lo = make_float4(q[0][i], q[1][i], q[2][i], 0.f);
        const float4 hi = make_float4(q[3][i], q[4][i], q[5][i], 0.f);
        ref[i] = __float_as_int(q[6][i]);
        float e = 0.f;
        bool p;
        if (st.wfast) {   // wave-uniform
            bool amb;
            p = aabb_fast(lo, hi, st.ro, st.rr, e, amb);
            if (amb && ref[i] >= 0) p = aabb_test(lo, hi, st.ro, st.rd);   // rare: the reference decides
        } else {
            p = aabb_decide(lo, hi, st.ro, st.rd, st.rr, st.exact, e);
        }
        T[i] = cull_threshold_packed(e, q[7][i]);
        p = p && ref[i] >= 0 && !(t_best < T[i]);
        key[i] = p ? e : __builtin_inff();
    }
    // order the four by entry (a network of five compare-exchanges; failed children last)
    auto cx = [&](int a, int b) {
        if (key[b] < key[a]) {
            float tk = key[a]; key[a] = key[b]; key[b] = tk;
            float tt = T[a]; T[a] = T[b]; T[b] = tt;
            int tr = ref[a]; ref[a] = ref[b]; ref[b] = tr;
        }
    };
    cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2);
    if (!(key[0] < __builtin_inff())) return false;    // no child passes: the caller pops
    const int S = sc.ref_shift;
#pragma unroll
    for (int i = 3; i >= 1; --i)
        if (key[i] < __builtin_inff()) trav_push(sc, st, stack, pack_ref(ref[i], T[i], S));
    st.cur = ref[0];
    st.curT = T[0];
    return true;
}

// one node expansion or one leaf; st.cur < 0 afterwards: the ray is finished
template <bool COUNT = false, bool QUAD = false>
PT_DEV void trav_step(const SceneDev& sc, TravState& st, int* stack, int& n_nodes, int& n_tris) {
    const int P = QUAD ? sc.num_quads : sc.num_pairs;
    bool next = false;
    if (st.cur < P) {
        next = QUAD ? trav_inner4<COUNT>(sc, st, stack, n_nodes) : trav_inner<COUNT>(sc, st, stack, n_nodes);
    } else {
        trav_leaf<COUNT>(sc, st, st.cur - P, n_nodes, n_tris);
    }
    if (!next) trav_pop(sc, st, stack);
}
// result of a finished traversal: t (-1: no triangle), u, v, hot4 slot (-1)
PT_DEV float trav_result(const TravState& st, float& bu, float& bv, int& btri) {
    if (st.btri == 0x7fffffff) {
        btri = -1;
        return -1.f;
    }
    bu = st.bu;
    bv = st.bv;
    btri = st.btri;
    return st.t_hit;
}

// A ray's traversal handed from one wave to another (k_bvh_bounce -> k_bvh_tail_trav): the best hit so
// far, the node to expand next and the stack.  The culls' thresholds ride in the stack entries and
// the ray's reciprocals, exactness and the wave's fast-box flag are recomputed; which box routine
// a wave uses never changes a decision, so the resumed traversal visits what the ray would have.
PT_DEV float4 trav_saved_hit(const TravState& st) {
    return make_float4(st.t_hit, st.bu, st.bv, __int_as_float(st.btri));
}
// node to expand next (refs < 2^24) | stack depth (<= MAXSTACK) << 24
PT_DEV int trav_saved_node(const TravState& st) { return st.cur | (st.sp << 24); }
PT_DEV void trav_resume(TravState& st, f3 ro, f3 rd, float4 hit, int node, int qs) {
    trav_ray(st, ro, rd);
    st.qs = qs;
    st.t_hit = hit.x;
    st.bu = hit.y;
    st.bv = hit.z;
    st.btri = __float_as_int(hit.w);
    st.cur = node & 0xffffff;
    st.sp = node >> 24;
    st.curT = 0.f;
}
// expand nodes until the ray is finished (st.cur < 0) or -- defer > 0 -- until no more than
// `defer` lanes of the wave are still traversing: those stop with st.cur >= 0 (wave steps with a
// handful of lanes cost a wave slot each for a few lanes of work; k_bvh_tail_trav resumes them in
// full waves).  Counters (COUNT) as bvh_intersect_pairs', the per-ray ones left to the caller.
template <bool COUNT = false, bool QUAD = false>
PT_DEV void trav_run(const SceneDev& sc, TravState& st, int* stack, int defer, int& n_nodes, int& n_tris,
                     int hist = SEC_BVH_LANES_HIST) {
    while (st.cur >= 0) {
        const int lanes = __popcll(__builtin_amdgcn_read_exec());   // wave-uniform
        if (lanes <= defer) break;
        if (COUNT) {
            sec_add(SEC_N_BVH_WITERS, 1);
            sec_add(hist + (lanes - 1) / 4, 1);
        }
        trav_step<COUNT, QUAD>(sc, st, stack, n_nodes, n_tris);
    }
}

template <bool COUNT = false>
PT_DEV float bvh_intersect_pairs(const SceneDev& sc, f3 ro, f3 rd, int* stack, float t_limit, float& bu, float& bv,
                                 int& btri) {
    int n_nodes = 0, n_tris = 0;
    TravState st;
    trav_begin(sc, st, ro, rd, t_limit);
    if (COUNT) sec_add_lanes(SEC_N_ROOT_CULLED, st.cur < 0 ? 1 : 0);
    while (st.cur >= 0) {
        if (COUNT) {
            sec_add(SEC_N_BVH_WITERS, 1);
            sec_add(SEC_BVH_LANES_HIST + (__popcll(__builtin_amdgcn_read_exec()) - 1) / 4, 1);
        }
        trav_step<COUNT>(sc, st, stack, n_nodes, n_tris);
    }
    if (COUNT) {
        sec_add_lanes(SEC_N_NODES, n_nodes);
        sec_add_lanes(SEC_N_TRIS, n_tris);
        sec_add_lanes(SEC_N_BVH_RAYS, 1);
        const bool hit = st.btri != 0x7fffffff && st.t_hit < t_limit;   // the mesh changes the winner
        sec_add_lanes(SEC_N_BVH_HITS, hit ? 1 : 0);
        sec_add_lanes(SEC_N_MISS_NODES, hit ? 0 : n_nodes);
    }
    return trav_result(st, bu, bv, btri);
}

// VAR_BVH_SPLIT: does bvh_intersect_pairs do anything for this ray beyond its root test?  The
// same root decision and root cull as bvh_intersect_pairs; false means the mesh cannot change the
// primitive winner (t_limit), true means the ray is queued for k_bvh_bounce.
PT_DEV bool bvh_root_needed(const SceneDev& sc, f3 ro, f3 rd, float t_limit) {
    const bool exact = !(ro.x - ro.x == 0.f && ro.y - ro.y == 0.f && ro.z - ro.z == 0.f &&
                         rd.x - rd.x == 0.f && rd.y - rd.y == 0.f && rd.z - rd.z == 0.f);
    const f3 rr = mk(__builtin_amdgcn_rcpf(rd.x), __builtin_amdgcn_rcpf(rd.y), __builtin_amdgcn_rcpf(rd.z));
    float e0;
    if (!aabb_decide(sc.root_lo, sc.root_hi, ro, rd, rr, exact, e0)) return false;
    return !(t_limit < cull_threshold(sc, e0, sc.root_hi.w));
}

// Conservative pre-test of one geom (approximate arithmetic, never decides a result): true
// when the exact test is CERTAIN not to update (t_min, winner) — the ray line misses the geom's
// margin-expanded world box, or enters it farther than t_min.  Slabs as fma(bound, 1/d, -o/d)
// with 1/d clamped to +-1e20 (finite inputs never make a NaN).  A NaN or infinite ray skips
// everything, which is what its exact tests return too: a NaN/inf distance never wins
// (`t > 0 && t_min > t`).
struct CullRay {
    f3 id;       // clamped approximate 1 / direction
    f3 rid;      // origin * id
    float rdlen;
};
PT_DEV float clamp_inv(float x) {
    return __builtin_fminf(__builtin_fmaxf(__builtin_amdgcn_rcpf(x), -1e20f), 1e20f);
}
PT_DEV CullRay cull_ray(f3 ro, f3 rd) {
    CullRay c;
    c.id = mk(clamp_inv(rd.x), clamp_inv(rd.y), clamp_inv(rd.z));
    c.rid = mk(ro.x * c.id.x, ro.y * c.id.y, ro.z * c.id.z);
    c.rdlen = __builtin_amdgcn_sqrtf(__builtin_fmaf(rd.x, rd.x, __builtin_fmaf(rd.y, rd.y, rd.z * rd.z)));
    return c;
}
template <bool FARTHER = true>
PT_DEV bool cull_geom(const DevGeom& g, const CullRay& c, float t_min) {
    const float a0 = __builtin_fmaf(g.box_lo[0], c.id.x, -c.rid.x), b0 = __builtin_fmaf(g.box_hi[0], c.id.x, -c.rid.x);
    const float a1 = __builtin_fmaf(g.box_lo[1], c.id.y, -c.rid.y), b1 = __builtin_fmaf(g.box_hi[1], c.id.y, -c.rid.y);
    const float a2 = __builtin_fmaf(g.box_lo[2], c.id.z, -c.rid.z), b2 = __builtin_fmaf(g.box_hi[2], c.id.z, -c.rid.z);
    const float t0 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(a0, b0), __builtin_fminf(a1, b1)),
                                     __builtin_fmaxf(__builtin_fminf(a2, b2), -1e-2f));
    const float t1 = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(a0, b0), __builtin_fmaxf(a1, b1)),
                                     __builtin_fmaxf(a2, b2));
    if (!(t1 >= t0)) return true;                                   // certain miss (or NaN ray)
    return FARTHER && t0 > 0.0f && t0 * c.rdlen * (1.0f - 1e-5f) - 1e-4f > t_min;  // certainly farther
}

// winner normal, BVH meshes (bvhMeshIntersectionTest, strict `<` so primitives win ties),
// miss / facing conventions of pathtrace.cu:397-446
// the winner's hit record from the primitive winner (t_min, win, seed) and the mesh result
// (tb, u, v, slot of the winning triangle in `hot`; tb <= 0: none), pathtrace.cu:397-446
PT_DEV Hit make_hit(const SceneDev& sc, f3 rd, float t_min, int win, f3 seed, float tb, float u,
                    float v, int tri, const DevTriHot* hot) {
    Hit h;
    h.tri = -1;
    h.u = 0.f;
    h.v = 0.f;
    f3 normal = mk(0.f, 0.f, 0.f);
    int hit_index = -1;   // reference hit_geom_index: prim -> its materialid, mesh -> -2
    int mat = 0;
    if (win >= 0) {
        const DevGeom& g = sc.geoms[win];   // itr: global (not in the LDS hot table)
        normal = normalize(xform(g.itr, seed, 0.0f));
        hit_index = g.materialid;
        mat = g.materialid;
    }
    if (tb > 0.0f && tb < t_min) {
        t_min = tb;
        hit_index = -2;
        DevTriHot th = hot[tri];
        int tri_index = __float_as_int(th.c.y);
        const DevTriCold& cd = sc.cold[tri_index];
        mat = cd.materialID;
        h.tri = tri_index;
        h.u = u;
        h.v = v;
        f3 n0 = mk(cd.n0[0], cd.n0[1], cd.n0[2]);
        f3 n1 = mk(cd.n1[0], cd.n1[1], cd.n1[2]);
        f3 n2 = mk(cd.n2[0], cd.n2[1], cd.n2[2]);
        if (length(n0) < 1e-6f || length(n1) < 1e-6f || length(n2) < 1e-6f) {
            f3 v0 = mk(th.a.x, th.a.y, th.a.z);
            f3 v1 = mk(th.a.w, th.b.x, th.b.y);
            f3 v2 = mk(th.b.z, th.b.w, th.c.x);
            normal = normalize(cross(v1 - v0, v2 - v0));
        } else {
            float w0 = 1.0f - u - v;
            normal = normalize((w0 * n0 + u * n1) + v * n2);
        }
    }
    if (hit_index == -1) {
        h.t = -1.0f;
        h.n = mk(0.f, 0.f, 0.f);
        h.mat = 0;
        return h;
    }
    if (dot(rd, normal) > 0.0f) normal = -normal;
    h.t = t_min;
    h.n = normal;
    h.mat = mat;
    return h;
}

// winner normal, BVH meshes (bvhMeshIntersectionTest, strict `<` so primitives win ties),
// miss / facing conventions of pathtrace.cu:397-446
template <bool HAS_BVH, bool BVH_FAST = false, bool COUNT = false>
PT_DEV Hit finish_hit(const SceneDev& sc, f3 ro, f3 rd, int* stack, float t_min, int win,
                      f3 seed, bool traverse = true) {
    float tb = -1.f, u = 0.f, v = 0.f;
    int tri = -1;
    const bool pairs = BVH_FAST && sc.pairs != nullptr;
    if (HAS_BVH && traverse && sc.use_bvh && sc.num_nodes > 0)
        tb = pairs ? bvh_intersect_pairs<COUNT>(sc, ro, rd, stack, t_min, u, v, tri)
           : BVH_FAST ? bvh_intersect_fast<COUNT>(sc, ro, rd, stack, t_min, u, v, tri)
                      : bvh_intersect<COUNT>(sc, ro, rd, stack, u, v, tri);
    return make_hit(sc, rd, t_min, win, seed, tb, u, v, tri, pairs ? sc.hot4 : sc.hot);
}

// computeIntersections for one ray (pathtrace.cu:298-448).  Per-geom work keeps only what
// decides the winner (t and the normal "seed"); the world normal is derived once for the
// winner — the same value the reference computes for every candidate and then keeps.
template <bool HAS_BVH, bool BVH_FAST = false>
PT_DEV Hit intersect_scene(const SceneDev& sc, f3 ro, f3 rd, int* stack) {
    float t_min = FLT_MAX_;
    int win = -1;
    f3 seed = mk(0.f, 0.f, 0.f);
    const CullRay cr = cull_ray(ro, rd);
    for (int i = 0; i < sc.num_geoms; ++i) {
        const DevGeom& g = sc.geoms[i];
        if (cull_geom(g, cr, t_min)) continue;
        f3 s;
        float t = geom_test(hot(g), ro, rd, s);
        if (t > 0.0f && t_min > t) {
            t_min = t;
            win = i;
            seed = s;
        }
    }
    return finish_hit<HAS_BVH, BVH_FAST>(sc, ro, rd, stack, t_min, win, seed);
}

// computeIntersections with the exact per-geom tests driven by a per-lane candidate queue:
// pass 1 runs the cheap cull for every geom (certain misses drop out), pass 2 lets every lane
// pop ITS next candidate (increasing geom index, so the first-minimum tie rule is unchanged)
// and re-checks the cull against its current t_min before the exact test.  The wave executes
// max-over-lanes(candidates) exact tests instead of one per geom any lane needs.
// `lgeoms`: the block's LDS copy of the geom table (the caller's job; sc.num_geoms <= 64).
// NEAR_FIRST (camera rays: neighbouring lanes share their nearest candidate, so the first test
// is wave-coherent): each lane tests its candidate of smallest conservative entry distance
// first; the rest, in index order, are then mostly re-culled as certainly farther.  Tested out
// of index order, the first-minimum rule becomes "smaller t, or equal t and smaller index".
PT_DEV float cull_entry(const DevGeom& g, const CullRay& c) {   // +inf: certain miss
    const float a0 = __builtin_fmaf(g.box_lo[0], c.id.x, -c.rid.x), b0 = __builtin_fmaf(g.box_hi[0], c.id.x, -c.rid.x);
    const float a1 = __builtin_fmaf(g.box_lo[1], c.id.y, -c.rid.y), b1 = __builtin_fmaf(g.box_hi[1], c.id.y, -c.rid.y);
    const float a2 = __builtin_fmaf(g.box_lo[2], c.id.z, -c.rid.z), b2 = __builtin_fmaf(g.box_hi[2], c.id.z, -c.rid.z);
    const float t0 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(a0, b0), __builtin_fminf(a1, b1)),
                                     __builtin_fmaxf(__builtin_fminf(a2, b2), -1e-2f));
    const float t1 = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(a0, b0), __builtin_fmaxf(a1, b1)),
                                     __builtin_fmaxf(a2, b2));
    return (t1 >= t0) ? t0 : __builtin_inff();
}
// The pre-test from the candidate table (sc.grid): the table gives each lane a superset of the
// geoms its ray can hit at all -- built on the host (pt_init, build_candidate_table) by interval
// arithmetic over every origin in the cell (grown by the cell computation's rounding) and every
// direction in the bin (grown by the bin computation's rounding), against the same conservative
// world boxes the pre-test uses, which contain every exact hit point.  Each lane then runs the
// flat pre-test's arithmetic (cull_candidates, bit for bit) on its own superset only, reading the
// records from the block's LDS copy (`lc`, 3 float4 per geom).  A geom outside the superset cannot
// be hit, so the exact tests of the candidates that remain find the same first minimum.  Rays
// whose origin lies outside the table or whose direction is not finite take every geom.
PT_DEV uint64_t grid_superset(const SceneDev& sc, f3 ro, f3 rd) {
    const float fx = (ro.x - sc.grid_lo[0]) * sc.grid_inv[0];
    const float fy = (ro.y - sc.grid_lo[1]) * sc.grid_inv[1];
    const float fz = (ro.z - sc.grid_lo[2]) * sc.grid_inv[2];
    constexpr float G = (float)GRID_G;
    const float ax = __builtin_fabsf(rd.x), ay = __builtin_fabsf(rd.y), az = __builtin_fabsf(rd.z);
    const bool kx = ax >= ay && ax >= az, ky = !kx && ay >= az;
    const float m = kx ? ax : (ky ? ay : az);
    const float dk = kx ? rd.x : (ky ? rd.y : rd.z);
    const float di = kx ? rd.y : (ky ? rd.z : rd.x);     // axis k + 1
    const float dj = kx ? rd.z : (ky ? rd.x : rd.y);     // axis k + 2
    const bool ok = fx >= 0.f && fx < G && fy >= 0.f && fy < G && fz >= 0.f && fz < G &&   // false for NaN
                    __builtin_isfinite(ax + ay + az) && m > 1e-30f;
    const float r = __builtin_amdgcn_rcpf(m);
    constexpr float HB = 0.5f * (float)GRID_B;
    const int bu = __builtin_amdgcn_fmed3f(__builtin_truncf((di * r + 1.f) * HB), 0.f, (float)(GRID_B - 1));
    const int bv = __builtin_amdgcn_fmed3f(__builtin_truncf((dj * r + 1.f) * HB), 0.f, (float)(GRID_B - 1));
    const int face = (kx ? 0 : (ky ? 2 : 4)) + (dk > 0.f ? 1 : 0);
    const int cell = ((int)fz * GRID_G + (int)fy) * GRID_G + (int)fx;
#if PT_GRID_SEP
    // separable table: the (cell, face) row holds the B masks of the first ratio's bins, then the
    // B masks of the second's; the entry is their AND (two independent loads, 2B words per row)
    const int e = ok ? (cell * 6 + face) * (2 * GRID_B) : 0;
    const uint64_t sup = sc.grid[e + (ok ? bu : 0)] & sc.grid[e + (ok ? GRID_B + bv : 0)];
#else
    const int e = ok ? ((cell * 6 + face) * GRID_B + bu) * GRID_B + bv : 0;
    const uint64_t sup = sc.grid[e];
#endif
    return ok ? sup : sc.grid_all;
}
template <bool TIMING = false, bool NEAR_FIRST = false>
PT_DEV void prim_intersect_q(const SceneDev& sc, const DevGeomHot* lgeoms, f3 ro, f3 rd, float& t_min, int& win,
                             f3& seed) {
    uint64_t tc0 = TIMING ? sec_clock() : 0;
    const CullRay cr = cull_ray(ro, rd);
    uint64_t cand = 0;
    t_min = FLT_MAX_;
    win = -1;
    seed = mk(0.f, 0.f, 0.f);
    if (NEAR_FIRST) {
        int first = -1;
        float best = __builtin_inff();
        if (sc.grid) {   // camera rays of a wave share their cell and mostly their bin: a near-uniform loop
            for (uint64_t m = grid_superset(sc, ro, rd); m != 0; m &= m - 1) {
                const int i = __builtin_ctzll(m);
                const float e = cull_entry(sc.geoms[i], cr);
                if (e != __builtin_inff()) {
                    cand |= 1ull << i;
                    if (e < best) {
                        best = e;
                        first = i;
                    }
                }
            }
        } else {
#pragma unroll 4
            for (int i = 0; i < sc.num_geoms; ++i) {
                const float e = cull_entry(sc.geoms[i], cr);
                if (e != __builtin_inff()) {
                    cand |= 1ull << i;
                    if (e < best) {
                        best = e;
                        first = i;
                    }
                }
            }
        }
        if (first >= 0) {
            cand &= ~(1ull << first);
            f3 s;
            const float t = geom_test(lgeoms[first], ro, rd, s);
            if (t > 0.0f && t_min > t) {
                t_min = t;
                win = first;
                seed = s;
            }
        }
        while (__any(cand != 0)) {
            if (cand != 0) {
                const int i = __builtin_ctzll(cand);
                cand &= cand - 1;
                if (!cull_geom(sc.geoms[i], cr, t_min)) {
                    f3 s;
                    const float t = geom_test(lgeoms[i], ro, rd, s);
                    if (t > 0.0f && (t < t_min || (t == t_min && win >= 0 && i < win))) {
                        t_min = t;
                        win = i;
                        seed = s;
                    }
                }
            }
        }
        return;
    }
#pragma unroll 4
    for (int i = 0; i < sc.num_geoms; ++i)
        if (!cull_geom<false>(sc.geoms[i], cr, FLT_MAX_)) cand |= 1ull << i;
    int n_exact = 0, n_iters = 0;
    uint64_t tc1 = 0;
    if (TIMING) {
        tc1 = sec_clock();
        sec_add(SEC_CULL, tc1 - tc0);
        sec_add_lanes(SEC_N_CAND, __builtin_popcountll(cand));
    }
    while (__any(cand != 0)) {
        if (TIMING) n_iters++;
        if (cand != 0) {
            const int i = __builtin_ctzll(cand);
            cand &= cand - 1;
            if (!cull_geom(sc.geoms[i], cr, t_min)) {
                f3 s;
                if (TIMING) n_exact++;
                float t = geom_test(lgeoms[i], ro, rd, s);
                if (t > 0.0f && t_min > t) {
                    t_min = t;
                    win = i;
                    seed = s;
                }
            }
        }
    }
    if (TIMING) {
        sec_add(SEC_EXACT, sec_clock() - tc1);
        sec_add_lanes(SEC_N_EXACT, n_exact);
        sec_add(SEC_N_ITERS, (uint64_t)n_iters);
    }
}
template <bool HAS_BVH, bool TIMING = false, bool BVH_FAST = false, bool NEAR_FIRST = false>
PT_DEV Hit intersect_scene_q(const SceneDev& sc, const DevGeomHot* lgeoms, f3 ro, f3 rd, int* stack) {
    float t_min;
    int win;
    f3 seed;
    prim_intersect_q<TIMING, NEAR_FIRST && !TIMING>(sc, lgeoms, ro, rd, t_min, win, seed);
    if (TIMING) {
        const uint64_t tc2 = sec_clock();
        Hit h = finish_hit<HAS_BVH, BVH_FAST, true>(sc, ro, rd, stack, t_min, win, seed);
        sec_add(SEC_FINISH, sec_clock() - tc2);
        return h;
    }
    return finish_hit<HAS_BVH, BVH_FAST>(sc, ro, rd, stack, t_min, win, seed);
}

// surface attributes of the winner that shading reads only for textured / bump-mapped
// materials (ShadeableIntersection.uv / dpdu / dpdv, pathtrace.cu:439-446): interpolated uv and
// the triangle's tangents for a mesh hit (intersections.cu:207-214), zeros for a primitive
struct HitAttr {
    float u, v;
    f3 dpdu, dpdv;
};
PT_DEV HitAttr hit_attr(const SceneDev& sc, const Hit& h) {
    HitAttr a;
    a.u = 0.0f;
    a.v = 0.0f;
    a.dpdu = mk(0.f, 0.f, 0.f);
    a.dpdv = mk(0.f, 0.f, 0.f);
    if (h.tri >= 0) {
        const DevTriCold& c = sc.cold[h.tri];
        const float w0 = 1.0f - h.u - h.v;
        a.u = (w0 * c.uv0[0] + h.u * c.uv1[0]) + h.v * c.uv2[0];
        a.v = (w0 * c.uv0[1] + h.u * c.uv1[1]) + h.v * c.uv2[1];
        a.dpdu = mk(c.dpdu[0], c.dpdu[1], c.dpdu[2]);
        a.dpdv = mk(c.dpdv[0], c.dpdv[1], c.dpdv[2]);
    }
    return a;
}

// tex2D<float4>(texObjects[id], x, y) (pathtrace.cu:505-519) on the framework's texel store
PT_DEV void tex_fetch(const SceneDev& sc, int id, float x, float y, float out[4]) {
    const int4 ti = sc.texinfo[id];
    pt_tex2d(sc.texels + ti.x, ti.y, ti.z, x, y, out);
}

// computeIntersections for a whole wave at once (VAR_WAVE_REDIST): every lane culls its ray,
// the (lane, candidate geom) pairs of all 64 lanes are listed in LDS in (lane, geom) order and
// the exact tests are dealt out 64 at a time, so a wave runs ceil(pairs / 64) exact-test rounds
// instead of max-over-lanes(candidates).  Each lane then scans its own pairs in geom order with
// the reference's `t > 0 && t_min > t` rule, so the winner (first minimum) is unchanged.  Every
// lane of the wave must call this (uniform control flow); `live` = the lane has a ray.
// candidates the exchanged exact test would certainly reject: a cube the ray leaves through
// on an axis while pointing away from it, which geom_test's slab test always rejects (away_on_axis).  `bounded`: |rd| components <= 1e3
// (away_on_axis' precondition).  Spheres keep theirs: most sphere candidates are rays leaving
// the sphere, whose exact test can round to a self-hit at t ~ 1e-4 (t1 = -b + sqrt(b^2 - ~0) =
// 0), so only the reference arithmetic can reject them (a bounding-ball line test dropped 3 % of
// all pairs and bought nothing).
PT_DEV bool certain_exact_miss(const DevGeomHot& g, f3 ro, f3 rd, bool bounded) {
    const int a = g.away_axis;
    return g.type == PT_CUBE && (unsigned)a < 3u && bounded && away_on_axis(g, a, ro, rd);
}
// !cull_geom<false>(g) for every geom, from the DevCull records (same slab arithmetic as
// cull_geom), as a candidate mask (bit i = geom i), minus the one cube the ray certainly leaves
// (certain_exact_miss).  Records are read four geoms (12 float4, 192 B) at a time through the
// scalar cache, all loads of a group issued before any arithmetic; the host pads the record array
// to a multiple of 4, and bits of pad records are masked off by the (wave-uniform) index test.
// The "away" drop is evaluated for ONE cube per lane: the last kept cube with an away axis whose
// box holds the ray's origin (t0 <= 0: every slab entry behind the origin) -- the surface a
// bounce ray leaves.  A ray outside a cube's box that points away from it on an axis already
// fails the slab test there (axis-aligned boxes), so the drop matters only where the origin is
// inside; a cube it is not applied to stays a candidate and its exact test rejects it (same
// results).  Evaluating the row for every kept cube instead cost each wave ~14 instructions per
// cube, since some lane of the wave keeps nearly every wall.
#ifndef CULL_GROUP
#define CULL_GROUP 4
#endif
#ifndef XSCAN_BALLOT
#define XSCAN_BALLOT 1
#endif
PT_DEV uint64_t cull_candidates(const SceneDev& sc, const DevGeomHot* lg, const CullRay& cr, f3 ro, f3 rd,
                                bool bounded) {
    const float4* rec = reinterpret_cast<const float4*>(sc.cull);
    const int ng = sc.num_geoms;
    uint64_t cand = 0;
    int og = -1;
    for (int i0 = 0; i0 < ng; i0 += CULL_GROUP) {
        float4 R[3 * CULL_GROUP];
#pragma unroll
        for (int k = 0; k < 3 * CULL_GROUP; ++k) R[k] = rec[3 * i0 + k];
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < CULL_GROUP; ++k) {
            const float4 A = R[3 * k], B = R[3 * k + 1], C = R[3 * k + 2];
            const float a0 = __builtin_fmaf(A.x, cr.id.x, -cr.rid.x), b0 = __builtin_fmaf(A.w, cr.id.x, -cr.rid.x);
            const float a1 = __builtin_fmaf(A.y, cr.id.y, -cr.rid.y), b1 = __builtin_fmaf(B.x, cr.id.y, -cr.rid.y);
            const float a2 = __builtin_fmaf(A.z, cr.id.z, -cr.rid.z), b2 = __builtin_fmaf(B.y, cr.id.z, -cr.rid.z);
            const float t0 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(a0, b0), __builtin_fminf(a1, b1)),
                                             __builtin_fmaxf(__builtin_fminf(a2, b2), -1e-2f));
            const float t1 = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(a0, b0), __builtin_fmaxf(a1, b1)),
                                             __builtin_fmaxf(a2, b2));
            const uint32_t slab = (uint32_t)(t1 >= t0) & (uint32_t)(i0 + k < ng);
            const uint32_t row = (uint32_t)(__float_as_int(C.z) != 0);
            og = (slab & row & (uint32_t)(t0 <= 0.0f)) ? i0 + k : og;
            bits |= slab << k;
        }
        cand |= (uint64_t)bits << i0;
    }
    if (og >= 0 && certain_exact_miss(lg[og], ro, rd, bounded)) cand &= ~(1ull << og);
    return cand;
}

PT_DEV uint64_t cull_candidates_grid(const SceneDev& sc, const float4* lc, const CullRay& cr, f3 ro, f3 rd,
                                     bool bounded) {
    uint64_t m = grid_superset(sc, ro, rd);
    uint64_t cand = 0;
    while (m != 0) {   // per lane: the wave runs as many rounds as its largest superset
        const int i = __builtin_ctzll(m);
        m &= m - 1;
        const float4 A = lc[3 * i], B = lc[3 * i + 1], C = lc[3 * i + 2];
        const float a0 = __builtin_fmaf(A.x, cr.id.x, -cr.rid.x), b0 = __builtin_fmaf(A.w, cr.id.x, -cr.rid.x);
        const float a1 = __builtin_fmaf(A.y, cr.id.y, -cr.rid.y), b1 = __builtin_fmaf(B.x, cr.id.y, -cr.rid.y);
        const float a2 = __builtin_fmaf(A.z, cr.id.z, -cr.rid.z), b2 = __builtin_fmaf(B.y, cr.id.z, -cr.rid.z);
        const float t0 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(a0, b0), __builtin_fminf(a1, b1)),
                                         __builtin_fmaxf(__builtin_fminf(a2, b2), -1e-2f));
        const float t1 = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(a0, b0), __builtin_fmaxf(a1, b1)),
                                         __builtin_fmaxf(a2, b2));
        const uint32_t slab = (uint32_t)(t1 >= t0);
        const uint32_t row = (uint32_t)(__float_as_int(C.z) != 0);
        const float qo = (B.z * ro.x + B.w * ro.y) + (C.x * ro.z + C.y * 1.0f);
        const float u = (B.z * rd.x + B.w * rd.y) + C.x * rd.z;
        const uint32_t away = ((uint32_t)(qo > 0.5f) & (uint32_t)(u > 0.0f)) |
                              ((uint32_t)(qo < -0.5f) & (uint32_t)(u < 0.0f));
        const uint32_t keep = slab & ((away & (uint32_t)bounded & row) ^ 1u);
        cand |= (uint64_t)keep << i;
    }
    return cand;
}
// float4s of the block's LDS geom table: the exact tests' DevGeomHot prefix of every geom, then
// (candidate table on) the pre-test's DevCull records
PT_DEV int lds_geom_f4(const SceneDev& sc) {
    return sc.num_geoms * ((int)(sizeof(DevGeomHot) / 16) + (sc.grid ? 3 : 0));
}
// Every load of a thread's share is issued before any of its LDS stores (a 44-geom table with its
// pre-test records is 2 float4 per thread: one L2 round trip, not two).  The caller issues the
// block's path loads before this, so their HBM latency overlaps the table's.
PT_DEV void stage_geoms(const SceneDev& sc, float4* s_dyn) {
    constexpr int HOT4 = (int)(sizeof(DevGeomHot) / 16), GEOM4 = (int)(sizeof(DevGeom) / 16), U = 4;
    const float4* src = reinterpret_cast<const float4*>(sc.geoms);
    const float4* cs = reinterpret_cast<const float4*>(sc.cull);
    const int nh = sc.num_geoms * HOT4;
    const int n = nh + (sc.grid ? 3 * sc.num_geoms : 0);
    auto fetch = [&](int k) { return k < nh ? src[(k / HOT4) * GEOM4 + k % HOT4] : cs[k - nh]; };
    for (int k0 = threadIdx.x; k0 < n; k0 += U * BLOCK) {
        const int k1 = k0 + BLOCK, k2 = k0 + 2 * BLOCK, k3 = k0 + 3 * BLOCK;
        // no branch between the loads (indices past the table re-read its last entry)
        const float4 v0 = fetch(k0), v1 = fetch(min(k1, n - 1)), v2 = fetch(min(k2, n - 1)),
                     v3 = fetch(min(k3, n - 1));
        s_dyn[k0] = v0;
        if (k1 < n) s_dyn[k1] = v1;
        if (k2 < n) s_dyn[k2] = v2;
        if (k3 < n) s_dyn[k3] = v3;
    }
    __syncthreads();
}

constexpr int WCAP = 192;      // pairs per wave held in LDS; more -> per-lane queue fallback
struct WaveLds {
    float ro[3][64], rd[3][64];
    float rt[WCAP], rs[3][WCAP];
    uint16_t task[WCAP];
};
template <bool COUNT = false>
PT_DEV void wave_intersect(const SceneDev& sc, const DevGeomHot* lg, bool live, f3 ro, f3 rd, WaveLds* W,
                           float& t_min, int& win, f3& seed) {
    const int lane = threadIdx.x & 63;
    uint64_t cand = 0;
    CullRay cr;
    if (live) {
        cr = cull_ray(ro, rd);
        // a ray leaving a surface keeps that surface's box as a candidate (its origin sits inside
        // the margin), but geom_test's slab test rejects it ("away", see geom_test): drop such
        // candidates here, with the same arithmetic, so they take no slot in the exact tests
        const bool bounded = __builtin_fabsf(rd.x) <= 1e3f && __builtin_fabsf(rd.y) <= 1e3f &&
                             __builtin_fabsf(rd.z) <= 1e3f;
        cand = cull_candidates(sc, lg, cr, ro, rd, bounded);
    }
    const int cnt = __builtin_popcountll(cand);
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    const int total = __shfl(incl, 63, 64);
    const int excl = incl - cnt;
    t_min = FLT_MAX_;
    win = -1;
    seed = mk(0.f, 0.f, 0.f);
    if (COUNT) {   // tools/section_times.py: exchanged pairs and rounds per wave, sphere pairs
        sec_add(SEC_N_ITERS, (uint64_t)((total + 63) / 64));
        sec_add(SEC_N_EXACT, (uint64_t)total);
        sec_add(SEC_N_BVH_RAYS, 1);                 // waves through the exchange
        int sph = 0;
        for (uint64_t m = cand; m; m &= m - 1) sph += sc.geoms[__builtin_ctzll(m)].type != PT_CUBE;
        sec_add_lanes(SEC_N_CAND, sph);
    }
    if (total > WCAP) {                          // rare: per-lane queue (same results)
        while (__any(cand != 0)) {
            if (cand != 0) {
                const int i = __builtin_ctzll(cand);
                cand &= cand - 1;
                if (!cull_geom(sc.geoms[i], cr, t_min)) {
                    f3 s;
                    const float t = geom_test(lg[i], ro, rd, s);
                    if (t > 0.0f && t_min > t) {
                        t_min = t;
                        win = i;
                        seed = s;
                    }
                }
            }
        }
        return;
    }
    W->ro[0][lane] = ro.x;
    W->ro[1][lane] = ro.y;
    W->ro[2][lane] = ro.z;
    W->rd[0][lane] = rd.x;
    W->rd[1][lane] = rd.y;
    W->rd[2][lane] = rd.z;
    {
        int j = excl;
        for (uint64_t m = cand; m; m &= m - 1) W->task[j++] = (uint16_t)((lane << 8) | __builtin_ctzll(m));
    }
    __builtin_amdgcn_wave_barrier();
    for (int base = 0; base < total; base += 64) {
        const int k = base + lane;
        if (k < total) {
            const int task = W->task[k];
            const int src = task >> 8, gi = task & 255;
            const f3 o = mk(W->ro[0][src], W->ro[1][src], W->ro[2][src]);
            const f3 d = mk(W->rd[0][src], W->rd[1][src], W->rd[2][src]);
            f3 s;
            const float t = geom_test(lg[gi], o, d, s);
            W->rt[k] = t;
            W->rs[0][k] = s.x;
            W->rs[1][k] = s.y;
            W->rs[2][k] = s.z;
        }
    }
    __builtin_amdgcn_wave_barrier();
    for (int j = excl; j < excl + cnt; ++j) {
        const float t = W->rt[j];
        if (t > 0.0f && t_min > t) {
            t_min = t;
            win = W->task[j] & 255;
            seed = mk(W->rs[0][j], W->rs[1][j], W->rs[2][j]);
        }
    }
}

// VAR_BLOCK_REDIST: wave_intersect's exchange across the whole block.  The four waves' (ray,
// geom) pairs form one list in (lane, geom) order; wave w takes entries w*64 + r*256 + lane, so
// the block runs ceil(pairs / 64) wave-rounds of exact tests instead of the sum over its waves
// of ceil(wave pairs / 64) (cornell: 79 pairs per wave on average -> 1.67 rounds each).  Same
// per-lane scan of its own results afterwards, so the winner is unchanged.  Every thread of the
// block must call it.
// 736 pairs (2.9 per lane; cornell averages 0.93 after bounce 0): with cornell's 7-geom table the
// block's LDS is then 20,240 B, so 8 blocks (8 waves per SIMD) fit a CU's 160 KB -- 768 needed
// 20,816 B and held the kernel at 7 whatever its registers.  A capacity chosen per scene at run
// time (so that khaslana's 44-geom table also fits 8 blocks, at 512 pairs) was tried: khaslana
// +-0, cornell +1.8 % from the run-time array offsets (A/B, round 3).  (640 would fit one more
// 44-geom block: khaslana -0.7 %, cornell +0.8 %, round 2.)
#ifndef BCAP_PAIRS
#define BCAP_PAIRS 736
#endif
constexpr int BCAP = BCAP_PAIRS;
struct BlockLds {
    float ro[3][BLOCK], rd[3][BLOCK];
    float rt[BCAP], rs[3][BCAP];
    uint16_t task[BCAP];
    int wsum[BLOCK / 64];
};
// VAR_MAT_GROUP (MATERIAL_SORTING on the fused pipeline, pathtrace.cu:730-735 sorts the whole
// wavefront by materialId before shading): here the block's 256 paths are regrouped by material in
// LDS between intersection and shading, so a wave shades runs of one material.  A counting sort:
// each wave finds the lanes that share its key with one ballot per key bit, the per-(wave, key)
// counts are scanned over the keys by wave 0, and every thread moves its path (+ hit, + queue
// state) to its slot.  Keys 0..MG_KEYS-1: the hit's materialId (a miss is 0, as the reference's
// memset leaves it), MG_KEYS-1 for paths that are not shaded here.  Results do not depend on
// which thread shades a path.
constexpr int MG_KEYS = 64;
constexpr int MG_WORDS = 22;   // exchanged words per path: 15, + 3 for triangle hits, + 4 for the BVH queue
struct MatGroupLds {
    int cnt[BLOCK / 64][MG_KEYS];
    int off[MG_KEYS];
    float x[MG_WORDS][BLOCK];
};
// bytes of MatGroupLds a kernel needs (the exchange array holds only the words it moves)
constexpr size_t mat_group_lds(bool tri, bool split) {
    return sizeof(int) * ((BLOCK / 64) * MG_KEYS + MG_KEYS) + sizeof(float) * BLOCK * (15 + (tri ? 3 : 0) + (split ? 4 : 0));
}
template <bool TRI, bool SPLIT>
PT_DEV void group_by_material(int key, MatGroupLds* S, bool& active, bool& live, bool& queued, PathReg& p, Hit& h,
                              float& qt, int& qw, f3& qs) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint64_t peers = ~0ull;
#pragma unroll
    for (int b = 0; b < 6; ++b) {   // MG_KEYS = 64 keys: 6 bits
        const uint64_t bb = __ballot((key >> b) & 1);
        peers &= ((key >> b) & 1) ? bb : ~bb;
    }
    for (int i = tid; i < (BLOCK / 64) * MG_KEYS; i += BLOCK) (&S->cnt[0][0])[i] = 0;
    __syncthreads();
    const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
    if (below == 0) S->cnt[w][key] = __popcll(peers);
    __syncthreads();
    if (w == 0) {   // exclusive scan over the keys of the block totals
        int t = 0;
#pragma unroll
        for (int i = 0; i < BLOCK / 64; ++i) t += S->cnt[i][lane];
        int incl = t;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        S->off[lane] = incl - t;
    }
    __syncthreads();
    int slot = S->off[key] + below;
    for (int i = 0; i < w; ++i) slot += S->cnt[i][key];
    // rb (0..64: 7 bits) | frame slot (8) | active, live, queued (3) | materialId (< 64: 6) | queued winner + 1 (7)
    // (an inactive lane's path fields are unset: every field is masked to its width)
    const uint32_t packed = ((uint32_t)p.rb & 127u) | (((uint32_t)p.slot & 255u) << 7) | ((active ? 1u : 0u) << 15) |
                            ((live ? 1u : 0u) << 16) | ((queued ? 1u : 0u) << 17) | (((uint32_t)h.mat & 63u) << 18) |
                            (((uint32_t)(qw + 1) & 127u) << 24);
    constexpr int NW = 15 + (TRI ? 3 : 0) + (SPLIT ? 4 : 0);
    float v[NW];
    v[0] = p.o.x; v[1] = p.o.y; v[2] = p.o.z;
    v[3] = p.d.x; v[4] = p.d.y; v[5] = p.d.z;
    v[6] = p.c.x; v[7] = p.c.y; v[8] = p.c.z;
    v[9] = __int_as_float(p.pix); v[10] = __uint_as_float(packed);
    v[11] = h.t; v[12] = h.n.x; v[13] = h.n.y; v[14] = h.n.z;
    if (TRI) { v[15] = __int_as_float(h.tri); v[16] = h.u; v[17] = h.v; }
    if (SPLIT) { v[NW - 4] = qt; v[NW - 3] = qs.x; v[NW - 2] = qs.y; v[NW - 1] = qs.z; }
#pragma unroll
    for (int k = 0; k < NW; ++k) S->x[k][slot] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NW; ++k) v[k] = S->x[k][tid];
    p.o = mk(v[0], v[1], v[2]);
    p.d = mk(v[3], v[4], v[5]);
    p.c = mk(v[6], v[7], v[8]);
    p.pix = __float_as_int(v[9]);
    const uint32_t q = __float_as_uint(v[10]);
    p.rb = (int)(q & 127u);
    p.slot = (int)((q >> 7) & 255u);
    active = ((q >> 15) & 1u) != 0;
    live = ((q >> 16) & 1u) != 0;
    queued = ((q >> 17) & 1u) != 0;
    h.mat = (int)((q >> 18) & 63u);
    qw = (int)((q >> 24) & 127u) - 1;
    h.t = v[11];
    h.n = mk(v[12], v[13], v[14]);
    if (TRI) { h.tri = __float_as_int(v[15]); h.u = v[16]; h.v = v[17]; }
    else { h.tri = -1; h.u = 0.f; h.v = 0.f; }
    if (SPLIT) { qt = v[NW - 4]; qs = mk(v[NW - 3], v[NW - 2], v[NW - 1]); }
}

// lg: the block's LDS geom table (lds_geom_f4)
template <bool TIMING = false>
PT_DEV void block_intersect(const SceneDev& sc, const DevGeomHot* lg, bool live, f3 ro, f3 rd, BlockLds* B,
                            float& t_min, int& win, f3& seed) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t tc0 = TIMING ? sec_clock() : 0;
    uint64_t cand = 0;
    CullRay cr;
    if (live) {
        cr = cull_ray(ro, rd);
        const bool bounded = __builtin_fabsf(rd.x) <= 1e3f && __builtin_fabsf(rd.y) <= 1e3f &&
                             __builtin_fabsf(rd.z) <= 1e3f;
        cand = sc.grid ? cull_candidates_grid(sc, reinterpret_cast<const float4*>(lg + sc.num_geoms), cr, ro, rd,
                                              bounded)
                       : cull_candidates(sc, lg, cr, ro, rd, bounded);
        PT_HOOK(DUP_CULL, sc, lg, ro, rd, bounded);
    }
    if (TIMING && sc.grid) {   // the per-lane superset loop costs a wave its largest superset
        const uint64_t sup = live ? grid_superset(sc, ro, rd) : 0ull;
        int ss = __popcll(sup);
        sec_add_lanes(SEC_N_SUP, ss);
        uint64_t un = sup;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t lo = __shfl_xor((uint32_t)un, off, 64), hi = __shfl_xor((uint32_t)(un >> 32), off, 64);
            un |= ((uint64_t)hi << 32) | lo;
        }
        sec_add(SEC_N_SUP_WUNION, (uint64_t)__popcll(un));
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) ss = max(ss, __shfl_xor(ss, off, 64));
        sec_add(SEC_N_SUP_WMAX, (uint64_t)ss);
    }
    const int cnt = __builtin_popcountll(cand);
    uint64_t tc1 = 0;
    if (TIMING) {
        tc1 = sec_clock();
        sec_add(SEC_CULL, tc1 - tc0);
        sec_add_lanes(SEC_N_CAND, cnt);
    }
#if XSCAN_BALLOT
    // the wave's exclusive prefix sum of cnt, one bit plane at a time (ballot + mbcnt, no LDS
    // round trips); a wave-uniform loop over the planes that are set somewhere (cornell: 2)
    int wexcl = 0, wtot = 0;
    for (int b = 0;; ++b) {
        const uint64_t m = __ballot((cnt >> b) & 1);
        wexcl += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
        wtot += __popcll(m) << b;
        if (!__any(cnt >> (b + 1))) break;
    }
    if (lane == 0) B->wsum[w] = wtot;
#else
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    if (lane == 63) B->wsum[w] = incl;
    const int wexcl = incl - cnt;
#endif
    __syncthreads();
    int woff = 0, total = 0;
#pragma unroll
    for (int i = 0; i < BLOCK / 64; ++i) {
        const int x = B->wsum[i];
        woff += i < w ? x : 0;
        total += x;
    }
    int excl = woff + wexcl;
    // one register: left transparent, the compiler keeps the six scan partials and the four wave
    // sums live across the exact tests and re-adds them afterwards (10 VGPRs at the peak)
    asm volatile("" : "+v"(excl));
    t_min = FLT_MAX_;
    win = -1;
    seed = mk(0.f, 0.f, 0.f);
    if (total > BCAP) {                          // block-uniform, rare: per-lane queue (same results)
        while (__any(cand != 0)) {
            if (cand != 0) {
                const int i = __builtin_ctzll(cand);
                cand &= cand - 1;
                if (!cull_geom(sc.geoms[i], cr, t_min)) {
                    f3 s;
                    const float t = geom_test(lg[i], ro, rd, s);
                    if (t > 0.0f && t_min > t) {
                        t_min = t;
                        win = i;
                        seed = s;
                    }
                }
            }
        }
        return;
    }
    B->ro[0][tid] = ro.x;
    B->ro[1][tid] = ro.y;
    B->ro[2][tid] = ro.z;
    B->rd[0][tid] = rd.x;
    B->rd[1][tid] = rd.y;
    B->rd[2][tid] = rd.z;
    {
        int j = excl;
        if (sc.num_geoms <= 32) {   // uniform: 32-bit mask arithmetic
            for (uint32_t m = (uint32_t)cand; m; m &= m - 1) B->task[j++] = (uint16_t)((tid << 8) | __builtin_ctz(m));
        } else {
            for (uint64_t m = cand; m; m &= m - 1) B->task[j++] = (uint16_t)((tid << 8) | __builtin_ctzll(m));
        }
    }
    __syncthreads();
    for (int k = w * 64 + lane; k < total; k += BLOCK) {
        const int task = B->task[k];
        const int src = task >> 8, gi = task & 255;
        const f3 o = mk(B->ro[0][src], B->ro[1][src], B->ro[2][src]);
        const f3 d = mk(B->rd[0][src], B->rd[1][src], B->rd[2][src]);
        f3 s;
        const float t = geom_test(lg[gi], o, d, s);
        PT_HOOK(DUP_EXACT, lg[gi], o, d);
        B->rt[k] = t;
        B->rs[0][k] = s.x;
        B->rs[1][k] = s.y;
        B->rs[2][k] = s.z;
    }
    __syncthreads();
    for (int j = excl; j < excl + cnt; ++j) {
        const float t = B->rt[j];
        if (t > 0.0f && t_min > t) {
            t_min = t;
            win = B->task[j] & 255;
            seed = mk(B->rs[0][j], B->rs[1][j], B->rs[2][j]);
        }
    }
    if (TIMING) {
        sec_add(SEC_EXACT, sec_clock() - tc1);
        sec_add_lanes(SEC_N_EXACT, cnt);
    }
}

// kernShadeMaterialProper for one live path (pathtrace.cu:521-621), with sampleTexture
// (magenta for an id that names no loaded texture, pathtrace.cu:505-512) and the bump-map
// normal perturbation (pathtrace.cu:579-607).  `attr()` yields the winner's HitAttr; it is
// only evaluated for textured / bump-mapped materials.
// TEX = false (VAR_NO_TEX): the caller guarantees no material has hasTexture or hasBumpMap set,
// so the texture branches below are never taken and are compiled out.
template <bool TEX = true, class AttrFn>
PT_DEV void shade_path(const SceneDev& sc, PathReg& p, const Hit& h, int iter, AttrFn attr) {
    if (h.t > 0.0f) {
        const DevMaterial m = sc.mats[h.mat];
        f3 mcolor = mk(m.color[0], m.color[1], m.color[2]);
        HitAttr ha;
        ha.u = ha.v = 0.0f;
        ha.dpdu = ha.dpdv = mk(0.f, 0.f, 0.f);
        if (TEX && (m.hasTexture | m.hasBumpMap)) ha = attr();
        const float uvx = ha.u, uvy = ha.v;
        if (TEX && m.hasTexture) {
            if (m.textureID < 0 || m.textureID >= sc.num_textures) {
                mcolor = mk(1.0f, 0.0f, 1.0f);
            } else {
                float c[4];
                tex_fetch(sc, m.textureID, uvx, 1.f - uvy, c);
                mcolor = mk(c[0], c[1], c[2]);
            }
        }
        if (m.emittance > 0.0f) {
            p.c = p.c * (mcolor * m.emittance);
            p.rb = 0;
        } else {
            Rng rng = rng_make(iter, p.pix, p.rb);
            f3 intersect = p.o + p.d * h.t;
            f3 shadingNormal = h.n;
            if (TEX && m.hasBumpMap && m.bumpID >= 0 && m.bumpID < sc.num_textures) {
                const f3 ng = h.n;
                const f3 dpdu = ha.dpdu, dpdv = ha.dpdv;
                const int4 ti = sc.texinfo[m.bumpID];
                const float du = 1.0f / float(ti.y);
                const float dv = 1.0f / float(ti.z);
                float t0[4], tu[4], tv[4];
                tex_fetch(sc, m.bumpID, uvx, 1.f - uvy, t0);             // sampleHeight(.., uv)
                tex_fetch(sc, m.bumpID, uvx + du, 1.f - uvy, tu);        // (uv.x + du, uv.y)
                tex_fetch(sc, m.bumpID, uvx, 1.f - (uvy + dv), tv);      // (uv.x, uv.y + dv)
                const float dhdu = (tu[0] - t0[0]) / du;
                const float dhdv = (tv[0] - t0[0]) / dv;
                const float scale = m.bumpScale;
                const f3 dpdu_p = dpdu + ng * (scale * dhdu);
                const f3 dpdv_p = dpdv + ng * (scale * dhdv);
                shadingNormal = normalize(cross(dpdu_p, dpdv_p));
                if (dot(shadingNormal, ng) < 0.0f) shadingNormal = -shadingNormal;
            }
            scatter(p, intersect, shadingNormal, m, mcolor, rng, sc.arg_order);
        }
    } else {
        p.c = mk(0.0f, 0.0f, 0.0f);
        p.rb = 0;
    }
}

}  // namespace ptd
