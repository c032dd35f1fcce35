// pt_runtime.hip — the wavefront path tracer on MI355X: kernels, device buffers, frame loop
// and the C-ABI of include/pt/pathtrace_abi.h.
//
// Two pipelines render bit-identical images (the same per-path functions, pt_kernels.h):
//
//  FUSED (default): one kernel per bounce.  Bounce 0 generates the camera ray in registers;
//    every bounce intersects, shades, adds terminated paths into the image (the reference's
//    finalGather, done at termination — one add per pixel per frame either way) and compacts
//    survivors with a wave ballot + LDS block scan + one atomic per block into one of NSEG
//    output segments (segment = blockIdx % 8, i.e. one per XCD group) — no host round trip,
//    no per-bounce readback of the live count.
//
//  STAGED: one kernel per reference stage — camera, intersect, [material sort], shade,
//    compaction — each a separately testable HIP kernel.  Its compaction is a STABLE
//    partition in three order-independent launches — per-tile alive counts, one single-
//    workgroup scan of the tile counts, scatter (wave ballot/mbcnt within a tile) — the drop-in
//    for thrust::stable_partition(PathAlive) (pathtrace.cu:750-757).
//
// A frame is captured once into a hipGraph and replayed; the iteration number lives in
// device memory (k_frame_begin advances it), so the replay needs no parameter updates.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>   // types only: librccl.so is opened at run time (PT_COMBINE_RCCL)

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pt/pathtrace_abi.h"
#include "pt_kernels.h"
#include "trav_tree.h"

using namespace ptd;

// =============================================================================================
// kernels
// =============================================================================================

// Fold the previous pass's live counts into the running totals, advance (or set) the
// iteration, zero the per-pass counters and start a pass of `batch` frames.  One block.
// `rows`: the counter rows any pass since the last reset of the block wrote (trace depth + 1 at
// most; the rest stay zero), so a frame clears 9 rows of 8 segments at depth 8, not 65.
__global__ void k_frame_begin(FrameCtl* ctl, int set_iter, int local_pixels, int batch, int rows, int plane) {
    int t = threadIdx.x;
    if (ctl->frames > 0) {
        for (int b = t; b < rows; b += blockDim.x) {
            unsigned long long s = 0;
            for (int k = 0; k < NSEG; ++k) s += (unsigned)ctl->cnt[b][k][0];
            ctl->tot[b] += s;
            unsigned long long q = 0, h = 0, hs = 0;
            for (int k = 0; k < NSEG; ++k) {
                q += (unsigned)ctl->qcnt[b][k][0];
                h += (unsigned)ctl->qcnt[b][k][3];
                hs += (unsigned)ctl->qcnt[b][k][4];
            }
            ctl->qtot[b] += q;
            ctl->htot[b] += h;
            ctl->hstk[b] += hs;
        }
    }
    __syncthreads();
    for (int i = t; i < rows * NSEG; i += blockDim.x) (&ctl->cnt[0][0][0])[i * CNT_PAD] = 0;
    for (int i = t; i < rows * NSEG; i += blockDim.x) {
        (&ctl->qcnt[0][0][0])[i * CNT_PAD] = 0;
        (&ctl->qcnt[0][0][0])[i * CNT_PAD + 1] = 0;   // handed-over traversals
        (&ctl->qcnt[0][0][0])[i * CNT_PAD + 2] = 0;   // ... and those taken by k_bvh_tail_trav
        (&ctl->qcnt[0][0][0])[i * CNT_PAD + 3] = 0;   // handed-over traversals stored (stats)
        (&ctl->qcnt[0][0][0])[i * CNT_PAD + 4] = 0;   // ... and their stack entries (stats)
    }
    __syncthreads();
    if (t == 0) {
        ctl->iter = set_iter > 0 ? set_iter : ctl->iter + 1;
        ctl->batch = batch;
        ctl->plane = plane;
        ctl->cnt[0][0][0] = local_pixels * batch;
        ctl->frames += batch;
    }
}

PT_DEV uint64_t lanemask_lt() {
    uint32_t lane = threadIdx.x & 63u;
    return lane == 0 ? 0ull : (~0ull >> (64u - lane));
}
PT_DEV int mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// A pixel receives one contribution per frame (finalGather, pathtrace.cu:217-227, adds every
// path's colour once).  Single-frame pass: add it now.  Pass of F > 1 frames: store it in the
// frame's contribution plane; k_combine adds the planes in frame order afterwards, so the
// image sees the same float additions in the same order as F sequential frames.
PT_DEV void gather_into_image(float* image, const SceneDev& sc, bool to_plane, const PathReg& p) {
    if (to_plane) {
        float* px = sc.contrib + 3 * ((size_t)p.slot * (size_t)(sc.cam.resx * sc.cam.resy) + (size_t)p.pix);
        px[0] = p.c.x;
        px[1] = p.c.y;
        px[2] = p.c.z;
        return;
    }
    float* px = image + 3 * (size_t)p.pix;
    px[0] += p.c.x;
    px[1] += p.c.y;
    px[2] += p.c.z;
}

// end of a pass of F > 1 frames: image += plane 0, += plane 1, ... (local pixels only)
__global__ __launch_bounds__(BLOCK) void k_combine(SceneDev sc, const FrameCtl* ctl, float* __restrict__ image) {
    const int l = blockIdx.x * BLOCK + threadIdx.x;
    if (l >= sc.shard.local_pixels) return;
    const int batch = ctl->batch;
    if (batch <= 1) return;
    const size_t pix = (size_t)shard_pixel(sc, l);
    const size_t plane = (size_t)sc.cam.resx * sc.cam.resy;
    float* px = image + 3 * pix;
    float r = px[0], gch = px[1], b = px[2];
    const float* c = sc.contrib + 3 * pix;
    for (int k = 0; k < batch; ++k, c += 3 * plane) {
        r += c[0];
        gch += c[1];
        b += c[2];
    }
    px[0] = r;
    px[1] = gch;
    px[2] = b;
}

// A speculative single frame (spec_*).  At its end, on its own stream, k_spec_sum forms the image
// the call for its iteration will return: image + its plane (the same float additions, in the same
// order, as its paths' gathers into the image would have made), into a buffer of its own -- so
// that call copies it to the host at once, while k_adopt_frame makes it the image and gives the
// caller's FrameCtl the frame's counters (the previous frame folded into the running totals and
// the speculative frame's live counts in its place, as k_frame_begin and that frame's kernels
// would have left them).  Whole images, as float4 streams (single context, no pixel shards).
__global__ __launch_bounds__(BLOCK) void k_spec_sum(const float* __restrict__ image, const float* __restrict__ plane,
                                                    float* __restrict__ out, int nf) {
    const int i = 4 * (blockIdx.x * BLOCK + threadIdx.x);
    if (i + 3 < nf) {
        float4 x = *reinterpret_cast<const float4*>(image + i);
        const float4 c = *reinterpret_cast<const float4*>(plane + i);
        x.x += c.x;
        x.y += c.y;
        x.z += c.z;
        x.w += c.w;
        *reinterpret_cast<float4*>(out + i) = x;
    } else {
        for (int k = i; k < nf; ++k) out[k] = image[k] + plane[k];
    }
}
__global__ __launch_bounds__(BLOCK) void k_adopt_frame(const float* __restrict__ sum, float* __restrict__ image, int nf,
                                                       FrameCtl* ctl, const FrameCtl* spec, int rows) {
    const int t = threadIdx.x;
    if (blockIdx.x == 0) {   // one thread per (bounce row, segment): all the loads at once
        const bool fold = ctl->frames > 0;
        for (int i = t; i < rows * NSEG; i += BLOCK) {
            int* c = &ctl->cnt[0][0][0] + i * CNT_PAD;
            int* q = &ctl->qcnt[0][0][0] + i * CNT_PAD;
            const int c0 = *c, q0 = q[0], h0 = q[3], hs0 = q[4];
            const int* qs = &spec->qcnt[0][0][0] + i * CNT_PAD;
            const int c1 = (&spec->cnt[0][0][0])[i * CNT_PAD], q1 = qs[0], h1 = qs[3], hs1 = qs[4];
            const int b = i / NSEG;
            if (fold && c0) atomicAdd(&ctl->tot[b], (unsigned long long)(unsigned)c0);
            if (fold && q0) atomicAdd(&ctl->qtot[b], (unsigned long long)(unsigned)q0);
            if (fold && h0) atomicAdd(&ctl->htot[b], (unsigned long long)(unsigned)h0);
            if (fold && hs0) atomicAdd(&ctl->hstk[b], (unsigned long long)(unsigned)hs0);
            *c = c1;
            q[0] = q1;
            q[3] = h1;
            q[4] = hs1;
        }
        __syncthreads();   // every thread read `frames` before it changes
        if (t == 0) {
            ctl->iter = spec->iter;
            ctl->batch = 1;
            ctl->plane = 0;
            ctl->frames += 1;
        }
    }
    const int i = 4 * (blockIdx.x * BLOCK + t);
    if (i + 3 < nf) {
        *reinterpret_cast<float4*>(image + i) = *reinterpret_cast<const float4*>(sum + i);
    } else {
        for (int k = i; k < nf; ++k) image[k] = sum[k];
    }
}

// Multi-device combine (pt_options.num_devices > 1): shard k owns the pixels
// shard_pixel_of(sh_k, W, l), l < sh_k.local_pixels, of every shard image; the first device's
// image receives them after each call.  Plain copies: the image is bit-identical to one device's.
__global__ __launch_bounds__(BLOCK) void k_pack_tile(const float* __restrict__ image, ShardDev sh, int W,
                                                     float* __restrict__ tile) {
    const int l = blockIdx.x * BLOCK + threadIdx.x;
    if (l >= sh.local_pixels) return;
    const size_t pix = 3 * (size_t)shard_pixel_of(sh, W, l);
    tile[3 * (size_t)l] = image[pix];
    tile[3 * (size_t)l + 1] = image[pix + 1];
    tile[3 * (size_t)l + 2] = image[pix + 2];
}
// The whole combine in ONE launch on the first device: every pixel of the frame finds its shard
// from its row band ((y / rows) % n) and copies its float3 from that shard's source -- the shard's
// own image over xGMI peer access (`local` 0: indexed by the global pixel), or the packed tile
// that RCCL / a peer copy brought over (`local` 1: indexed by the shard's local pixel).  All
// shards' reads are in flight together (on N GPUs: every xGMI link at once), instead of one
// launch per shard one after another.  Shard 0's pixels are already in place.
struct GatherSrc {
    const float* src[PT_MAX_DEVICES];
    int local[PT_MAX_DEVICES];
    int n, rows, W, H;
};
__global__ __launch_bounds__(BLOCK) void k_gather_shards(float* __restrict__ image, GatherSrc g) {
    const int pix = blockIdx.x * BLOCK + threadIdx.x;
    if (pix >= g.W * g.H) return;
    const int y = pix / g.W, x = pix - y * g.W;
    const int band = y / g.rows;
    const int k = band % g.n;
    if (k == 0) return;
    const int lrow = (band / g.n) * g.rows + (y - band * g.rows);
    const size_t i = 3 * (size_t)(g.local[k] ? lrow * g.W + x : pix);
    const float* s = g.src[k];
    const float r = s[i], gch = s[i + 1], b = s[i + 2];
    float* px = image + 3 * (size_t)pix;
    px[0] = r;
    px[1] = gch;
    px[2] = b;
}

// --------------------------------------------------------------------------------------------
// FUSED: camera (bounce 0) | load -> intersect -> shade -> gather dead -> compact survivors
// --------------------------------------------------------------------------------------------
// VAR_BVH_SPLIT traversal queue: the path (3 float4 as in PathBuf, C.w = frame slot | (winner
// geom + 1) << 8) and the primitive result it enters traversal with (t_min, normal seed)
struct QueueBuf {
    float4 *A, *B, *C, *D;   // D = t_min | seed.xyz
    int stride;              // entries per queue segment (segment s at s * stride, FrameCtl::qcnt)
};
// Traversals handed from k_bvh_bounce to k_bvh_tail_trav (see trav_run): per entry the queue slot
// and the saved node (trav_saved_node), the best hit so far (the final hit once k_bvh_tail_trav is
// done), and the stack (entry i of e at stack[i * cap + e]).  Segment s (at s * stride; counter
// FrameCtl::qcnt[b][s][1]) holds the rays of k_bvh_bounce's blocks of segment s, so
// k_bvh_tail_shade's survivors fit where theirs would have.
struct TailBuf {
    int2* node;     // queue slot | trav_saved_node
    float4* hit;    // trav_saved_hit
    int* stack;     // the LDS part of the stack (SceneDev::stack_lds entries; deeper ones stay spilled)
    int stride, cap, depth;
};
// queue entry k for path p and its primitive result
PT_DEV void queue_put(const QueueBuf& q, int k, const PathReg& p, float qt, int qw, f3 qs) {
    q.A[k] = make_float4(p.o.x, p.o.y, p.o.z, __int_as_float(p.pix));
    q.B[k] = make_float4(p.d.x, p.d.y, p.d.z, __int_as_float(p.rb));
    q.C[k] = make_float4(p.c.x, p.c.y, p.c.z, __int_as_float(p.slot | ((qw + 1) << 8)));
    q.D[k] = make_float4(qt, qs.x, qs.y, qs.z);
}

// Block-aggregated append of up to two flags: ballot -> per-wave counts -> one atomic per flag
// per block (counters on their own cache lines).  Returns each flagged lane's index.  Every
// thread of the block must call it.
// Slot of the gid-th entry of a segmented buffer: segment s holds entries [segoff[s], segoff[s+1])
// at s * stride.  Resolved once per wave on the scalar unit; per lane only if the wave straddles a
// segment boundary (at most NSEG-1 waves per launch).
PT_DEV int segment_slot(const int* segoff, int gid, int block_start, int stride) {
    const int w0 = block_start + (__builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6) << 6);
    int lo = 0, hi = segoff[1], sb = 0;
#pragma unroll
    for (int k = 1; k < NSEG; ++k)
        if (w0 >= segoff[k]) {
            lo = segoff[k];
            hi = segoff[k + 1];
            sb = k;
        }
    if (w0 + 63 < hi) return sb * stride - lo + gid;
    int sl = 0;
#pragma unroll
    for (int k = 1; k < NSEG; ++k) sl += (gid >= segoff[k]) ? 1 : 0;
    int sofs = 0;
#pragma unroll
    for (int k = 1; k < NSEG; ++k) sofs = (sl == k) ? segoff[k] : sofs;
    return sl * stride + (gid - sofs);
}

template <bool TWO>
PT_DEV void block_append(bool f0, int* ctr0, bool f1, int* ctr1, int& i0, int& i1) {
    __shared__ int s_w[2][BLOCK / 64];
    __shared__ int s_b[2];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t m0 = __ballot(f0);
    const uint64_t m1 = TWO ? __ballot(f1) : 0ull;
    if (lane == 0) {
        s_w[0][w] = __popcll(m0);
        if (TWO) s_w[1][w] = __popcll(m1);
    }
    __syncthreads();
    if (tid < (TWO ? 2 : 1)) {
        int tot = 0;
#pragma unroll
        for (int i = 0; i < BLOCK / 64; ++i) {
            const int c = s_w[tid][i];
            s_w[tid][i] = tot;
            tot += c;
        }
        s_b[tid] = tot ? atomicAdd(tid == 0 ? ctr0 : ctr1, tot) : 0;
        PT_HOOK(ATOMIC_EXTRA, s_b[tid], tid == 0 ? ctr0 : ctr1);
    }
    __syncthreads();
    i0 = s_b[0] + s_w[0][w] + mbcnt(m0);
    i1 = TWO ? s_b[1] + s_w[1][w] + mbcnt(m1) : 0;
}

template <bool FIRST, bool HAS_BVH, int VAR>
__global__ __launch_bounds__(BLOCK) void k_bounce(SceneDev sc, PathBuf in, PathBuf out, FrameCtl* ctl,
                                                  float* __restrict__ image, int bounce, int seg_stride,
                                                  QueueBuf q) {
    // dynamic LDS: [geom table, sc.num_geoms <= LDS_GEOMS, candidate-queue variants]
    //              [HAS_BVH && !SPLIT: traversal stack, stack_depth x BLOCK ints]
    //              [VAR_WAVE_REDIST: one WaveLds per wave]
    extern __shared__ float4 s_dyn[];
    const int iter = ctl->iter;
    const bool to_plane = ctl->batch > 1 || ctl->plane != 0;   // gather into the frame planes
    int n;
    int segoff[NSEG + 1];
    if (FIRST) {
        n = ctl->cnt[0][0][0];          // local_pixels x batch
    } else {
        segoff[0] = 0;
#pragma unroll
        for (int s = 0; s < NSEG; ++s) segoff[s + 1] = segoff[s] + ctl->cnt[bounce][s][0];
        n = segoff[NSEG];
    }
    const int block_start = blockIdx.x * BLOCK;
    if (block_start >= n) return;
    constexpr bool TIMING = (VAR & VAR_SECTION_TIMING) != 0;
    constexpr bool QUEUE = (VAR & VAR_CAND_QUEUE) != 0;
    constexpr bool REDIST = (VAR & VAR_WAVE_REDIST) != 0;
    constexpr bool BVH_FAST = (VAR & VAR_BVH_FAST) != 0;
    // split: the launcher guarantees the pair layout and an LDS geom table (queue or redist)
    constexpr bool SPLIT = HAS_BVH && BVH_FAST && (VAR & VAR_BVH_SPLIT) && (QUEUE || REDIST);
    uint64_t tc = TIMING ? sec_clock() : 0;
    const int tid = threadIdx.x;
    const bool lds_geoms = (QUEUE || REDIST) && sc.num_geoms <= LDS_GEOMS;
    DevGeomHot* s_geoms = reinterpret_cast<DevGeomHot*>(s_dyn);
    int* s_stack = reinterpret_cast<int*>(s_dyn + (lds_geoms ? lds_geom_f4(sc) : 0));
    WaveLds* s_wave_isect =
        reinterpret_cast<WaveLds*>(s_stack + (HAS_BVH && !SPLIT ? sc.stack_depth * BLOCK : 0)) + (tid >> 6);
    const int gid = block_start + tid;
    bool active = gid < n;
    PathReg p;
    p.rb = 0;
    if (active) {
        if (FIRST) {
            const int slot = gid / sc.shard.local_pixels;
            p = camera_ray(sc.cam, iter + slot, sc.trace_depth, shard_pixel(sc, gid - slot * sc.shard.local_pixels));
            p.slot = slot;
        } else {
            p = load_path(in, segment_slot(segoff, gid, block_start, seg_stride));
        }
    }
    // the geom table after the path loads are issued (their latencies overlap); per-lane candidate
    // tests then read their geom from LDS, not L2
    if (lds_geoms) stage_geoms(sc, s_dyn);
    PT_HOOK(STAGE_EXTRA, lds_geoms, sc, s_dyn);
    if (TIMING && active) {
        __builtin_amdgcn_s_waitcnt(0);
        uint64_t t = sec_clock();
        sec_add(SEC_LOAD, t - tc);
        sec_add(SEC_N_WAVES, 1);
        sec_add_lanes(SEC_N_LANES, p.rb > 0 ? 1 : 0);
    }
    bool live = active && p.rb > 0;
    constexpr bool MG = (VAR & VAR_MAT_GROUP) != 0;
    Hit h;
    if (MG) h = Hit{-1.f, mk(0.f, 0.f, 0.f), 0, -1, 0.f, 0.f};
    bool queued = false;
    float qt = 0.f;
    int qw = -1;
    f3 qs = mk(0.f, 0.f, 0.f);
    if (REDIST && lds_geoms) {                     // wave-cooperative: every lane takes part
        if (VAR & VAR_BLOCK_REDIST)
            block_intersect<TIMING>(sc, s_geoms, live, p.o, p.d, reinterpret_cast<BlockLds*>(s_wave_isect - (tid >> 6)),
                                    qt, qw, qs);
        else
            wave_intersect<TIMING>(sc, s_geoms, live, p.o, p.d, s_wave_isect, qt, qw, qs);
    } else if (SPLIT && live) {
        prim_intersect_q<TIMING, FIRST && !TIMING>(sc, s_geoms, p.o, p.d, qt, qw, qs);
    }
    if (live) {
        if (SPLIT) {
            queued = bvh_root_needed(sc, p.o, p.d, qt);
            if (!queued) h = finish_hit<false>(sc, p.o, p.d, s_stack + tid, qt, qw, qs);
        } else if (REDIST && lds_geoms) {
            h = finish_hit<HAS_BVH, BVH_FAST>(sc, p.o, p.d, s_stack + tid, qt, qw, qs);
            PT_HOOK(DUP_HIT, HAS_BVH, BVH_FAST, sc, p.o, p.d, s_stack + tid, qt, qw, qs);
        } else {
            h = lds_geoms ? intersect_scene_q<HAS_BVH, TIMING, BVH_FAST, FIRST>(sc, s_geoms, p.o, p.d, s_stack + tid)
                          : intersect_scene<HAS_BVH, BVH_FAST>(sc, p.o, p.d, s_stack + tid);
        }
        if (!MG && !queued) {
            uint64_t ts = TIMING ? sec_clock() : 0;
            PT_HOOK(DUP_SHADE, (VAR & VAR_NO_TEX) == 0, sc, p, h, iter);
            shade_path<(VAR & VAR_NO_TEX) == 0>(sc, p, h, iter + p.slot, [&]() { return hit_attr(sc, h); });
            if (TIMING) {
                tc = sec_clock();
                sec_add(SEC_SHADE, tc - ts);
            }
        }
    }
    if (MG) {   // MATERIAL_SORTING: regroup the block's paths by material, then shade
        if (SPLIT) {   // the rays queued for the mesh leave first, from their own threads
            int qi, unused;
            block_append<false>(queued, &ctl->qcnt[bounce][blockIdx.x & (NSEG - 1)][0], false, nullptr, qi, unused);
            qi += (blockIdx.x & (NSEG - 1)) * q.stride;
            if (queued) {
                queue_put(q, qi, p, qt, qw, qs);
                active = false;   // handed over to k_bvh_bounce
                live = false;
                queued = false;
            }
        }
        const int key = live ? (h.t > 0.0f ? h.mat : 0) : MG_KEYS - 1;
        MatGroupLds* mg = reinterpret_cast<MatGroupLds*>(s_wave_isect - (tid >> 6));
        group_by_material<HAS_BVH, false>(key, mg, active, live, queued, p, h, qt, qw, qs);
        if (live) shade_path<(VAR & VAR_NO_TEX) == 0>(sc, p, h, iter + p.slot, [&]() { return hit_attr(sc, h); });
    }
    if (TIMING && active) tc = sec_clock();
    const bool surv = active && !queued && p.rb > 0;
    if (active && !queued && !surv) gather_into_image(image, sc, to_plane, p);
    const int lane = tid & 63;
    const int seg = blockIdx.x & (NSEG - 1);
    if (VAR & VAR_WAVE_ATOMIC) {
        // one returning atomic per wave on a counter that owns its cache line; no barrier
        const uint64_t m = __ballot(surv);
        if (m != 0) {
            int base = 0;
            if (lane == 0) base = atomicAdd(&ctl->cnt[bounce + 1][seg][0], __popcll(m));
            base = __shfl(base, 0);
            if (surv) store_path(out, seg * seg_stride + base + mbcnt(m), p);
        }
        if (!SPLIT) return;
        const uint64_t mq = __ballot(queued);
        if (mq != 0) {
            int base = 0;
            if (lane == 0) base = atomicAdd(&ctl->qcnt[bounce][seg][0], __popcll(mq));
            base = __shfl(base, 0);
            if (queued) {
                const int k = seg * q.stride + base + mbcnt(mq);
                queue_put(q, k, p, qt, qw, qs);
            }
        }
        return;
    }
    // block-aggregated compaction (+ the traversal queue): one atomic per counter per block
    int si, qi;
    block_append<SPLIT>(surv, &ctl->cnt[bounce + 1][seg][0], queued, &ctl->qcnt[bounce][seg][0], si, qi);
    if (surv) store_path(out, seg * seg_stride + si, p);
    qi += seg * q.stride;
    if (SPLIT && queued) queue_put(q, qi, p, qt, qw, qs);
    if (TIMING && active) sec_add(SEC_STORE, sec_clock() - tc);
}

// Single-frame passes (the API's pathtrace(), F = 1): bounces `bounce` .. depth-1 of a
// primitive-only scene in ONE launch.  Each block keeps its paths in registers and loops over the
// remaining bounces (block-wide exact-test exchange, shading, gather at termination) until none of
// its paths is alive, with no compaction in between: the late bounces of a lone frame are a few
// thousand waves each, bound by launch and drain latency rather than by work.  Per-path
// arithmetic, RNG keys and the gather are those of k_bounce, so the image is the same bit for
// bit; per-bounce live counts go to the same counters (one atomic per block per bounce).
template <int VAR>
__global__ __launch_bounds__(BLOCK) void k_tail(SceneDev sc, PathBuf in, FrameCtl* ctl, float* __restrict__ image,
                                               int bounce, int seg_stride, int depth) {
    extern __shared__ float4 s_dyn[];
    __shared__ int s_cnt[BLOCK / 64];
    const int iter = ctl->iter;
    const bool to_plane = ctl->batch > 1 || ctl->plane != 0;   // gather into the frame planes
    int segoff[NSEG + 1];
    segoff[0] = 0;
#pragma unroll
    for (int s = 0; s < NSEG; ++s) segoff[s + 1] = segoff[s] + ctl->cnt[bounce][s][0];
    const int n = segoff[NSEG];
    const int block_start = blockIdx.x * BLOCK;
    if (block_start >= n) return;
    const int tid = threadIdx.x, lane = tid & 63;
    DevGeomHot* s_geoms = reinterpret_cast<DevGeomHot*>(s_dyn);
    BlockLds* s_block = reinterpret_cast<BlockLds*>(s_dyn + lds_geom_f4(sc));
    const int gid = block_start + tid;
    const bool active = gid < n;
    PathReg p;
    p.rb = 0;
    if (active) {
        int sl = 0;
#pragma unroll
        for (int k = 1; k < NSEG; ++k) sl += (gid >= segoff[k]) ? 1 : 0;
        int sofs = 0;
#pragma unroll
        for (int k = 1; k < NSEG; ++k) sofs = (sl == k) ? segoff[k] : sofs;
        p = load_path(in, sl * seg_stride + (gid - sofs));
    }
    stage_geoms(sc, s_dyn);   // after the path loads are issued
    const int seg = blockIdx.x & (NSEG - 1);
    for (int b = bounce; b < depth; ++b) {
        const bool live = active && p.rb > 0;
        float qt = 0.f;
        int qw = -1;
        f3 qs = mk(0.f, 0.f, 0.f);
        block_intersect<false>(sc, s_geoms, live, p.o, p.d, s_block, qt, qw, qs);
        if (live) {
            const Hit h = finish_hit<false>(sc, p.o, p.d, nullptr, qt, qw, qs);
            shade_path<(VAR & VAR_NO_TEX) == 0>(sc, p, h, iter + p.slot, [&]() { return hit_attr(sc, h); });
            if (p.rb <= 0) gather_into_image(image, sc, to_plane, p);
        }
        // paths entering bounce b + 1 (k_bounce's survivor count for this bounce)
        const bool surv = live && p.rb > 0;
        const uint64_t m = __ballot(surv);
        if (lane == 0) s_cnt[tid >> 6] = __popcll(m);
        __syncthreads();
        int tot = 0;
#pragma unroll
        for (int i = 0; i < BLOCK / 64; ++i) tot += s_cnt[i];
        if (tid == 0 && tot) atomicAdd(&ctl->cnt[b + 1][seg][0], tot);
        __syncthreads();
        if (tot == 0) break;          // block-uniform
    }
}

// VAR_BVH_SPLIT, second half of a bounce: the queued paths, 64 to a wave, traverse the mesh
// (bvh_intersect_pairs via finish_hit, entering with their primitive winner), are shaded, and
// gathered / compacted into the same output segments as k_bounce (blockIdx % NSEG; the host
// doubles seg_stride so both kernels' survivors fit).
// __launch_bounds__(256, 7): 7 waves per SIMD (<= 72 VGPRs; a few bytes of scratch in the cold
// exact-fallback paths).  Occupancy is what this latency-bound traversal lives on: with the SLP
// vectorizer on (packed-f32 pairs built from duplicated registers) it needed 96 VGPRs for 5
// waves; without it (Makefile) 79 VGPRs natural, and 72 at this bound (bunny 0.489 -> 0.477
// ms/frame); 8 waves (64 VGPRs) spill 100 B
#ifndef BVH_WAVES
#define BVH_WAVES 7
#endif

// after the traversal: the path's other words, the hit, shading (the shared end of k_bvh_bounce
// and k_bvh_tail_shade)
template <int VAR>
PT_DEV void bvh_finish_path(const SceneDev& sc, const QueueBuf& q, int qs, int iter, PathReg& p, const TravState& st) {
    float u = 0.f, v = 0.f;
    int tri = -1;
    const float tb = trav_result(st, u, v, tri);
    // the other words re-read here (L2): reading every word once, before the traversal,
    // keeps 5 more registers live across it -- bunny +6.7 %, khaslana +5.5 % (A/B, round 3)
    const float4 c = q.C[qs], d = q.D[qs];
    p.pix = __float_as_int(q.A[qs].w);
    p.rb = __float_as_int(q.B[qs].w);
    p.c = mk(c.x, c.y, c.z);
    const int cw = __float_as_int(c.w);
    p.slot = cw & 255;
    const int win = (cw >> 8) - 1;
    const Hit h = make_hit(sc, p.d, d.x, win, mk(d.y, d.z, d.w), tb, u, v, tri, sc.hot4);
    shade_path<(VAR & VAR_NO_TEX) == 0>(sc, p, h, iter + p.slot, [&]() { return hit_attr(sc, h); });
}
template <bool COUNT>
PT_DEV void bvh_count_ray(const TravState& st, float t_prim, int n_nodes) {
    if (COUNT) {
        sec_add_lanes(SEC_N_BVH_RAYS, 1);
        const bool hit = st.btri != 0x7fffffff && st.t_hit < t_prim;   // the mesh changes the winner
        sec_add_lanes(SEC_N_BVH_HITS, hit ? 1 : 0);
        sec_add_lanes(SEC_N_MISS_NODES, hit ? 0 : n_nodes);   // (a handed-over ray: its tail's nodes)
    }
}

// hand the calling lanes' traversals (st.cur >= 0) over to k_bvh_tail_trav: one atomic per wave.
// false: the segment is full at this lane's slot -- the caller finishes it itself.  The counter
// still counts it; every slot below min(counter, stride) is written by the lane that reserved it.
PT_DEV bool tail_put(const TailBuf& t, int* ctr, int seg, int qs, const TravState& st, const int* s_stack) {
    const uint64_t m = __ballot(1);
    const int lead = __builtin_ctzll(m);
    int base = 0;
    if ((int)(threadIdx.x & 63) == lead) base = atomicAdd(ctr, __popcll(m));
    const int slot = __builtin_amdgcn_readlane(base, lead) + mbcnt(m);
    if (slot >= t.stride) return false;
    const int e = seg * t.stride + slot;
    t.node[e] = make_int2(qs, trav_saved_node(st));
    t.hit[e] = trav_saved_hit(st);
    for (int i = 0; i < min(st.sp, t.depth); ++i) t.stack[(size_t)i * t.cap + e] = s_stack[i * BLOCK];
    // stats (pt_frame_stats handed_total / handed_stack_total): same-address atomics, one per
    // wave after the compiler's wave reduction, on the counter line the reservation just used
    atomicAdd(ctr + 2, 1);
    atomicAdd(ctr + 3, st.sp);
    return true;
}

template <int VAR, bool QUAD>
__global__ __launch_bounds__(BLOCK, BVH_WAVES) void k_bvh_bounce(SceneDev sc, QueueBuf q, TailBuf tail, int defer,
                                                                 PathBuf out, FrameCtl* ctl, float* __restrict__ image,
                                                                 int bounce, int seg_stride) {
    extern __shared__ float4 s_dyn[];   // traversal stack, stack_depth x BLOCK ints
    int segoff[NSEG + 1];
    segoff[0] = 0;
#pragma unroll
    for (int s = 0; s < NSEG; ++s) segoff[s + 1] = segoff[s] + ctl->qcnt[bounce][s][0];
    const int n = segoff[NSEG];
    const int block_start = blockIdx.x * BLOCK;
    if (block_start >= n) return;
    int* s_stack = reinterpret_cast<int*>(s_dyn);
    const int iter = ctl->iter;
    const bool to_plane = ctl->batch > 1 || ctl->plane != 0;   // gather into the frame planes
    const int tid = threadIdx.x;
    const int gid = block_start + tid;
    const int seg = blockIdx.x & (NSEG - 1);
    const bool active = gid < n;
    bool handed = false;
    const int qs = active ? segment_slot(segoff, gid, block_start, q.stride) : 0;
    PathReg p;
    p.rb = 0;
    if (active) {
        // traversal needs only the ray and its primitive t; the rest of the path is fetched
        // afterwards (fewer registers live across the traversal loop -> occupancy)
        const float4 a = q.A[qs], b = q.B[qs];
        const float t_prim = q.D[qs].x;
        p.o = mk(a.x, a.y, a.z);
        p.d = mk(b.x, b.y, b.z);
        constexpr bool CNT = (VAR & VAR_SECTION_TIMING) != 0;
        int n_nodes = 0, n_tris = 0;
        TravState st;
        trav_begin(sc, st, p.o, p.d, t_prim);
        st.qs = qs;   // deep stack entries spill to the slot's row (SceneDev::spill)
        if (CNT) sec_add_lanes(SEC_N_ROOT_CULLED, st.cur < 0 ? 1 : 0);
        // handed over: the wave's last few traversals go on 64 to a wave (no room: finish here)
        for (int d = defer;; d = 0) {
            trav_run<CNT, QUAD>(sc, st, s_stack + tid, d, n_nodes, n_tris);
            if (st.cur < 0) break;
            if (tail_put(tail, &ctl->qcnt[bounce][seg][1], seg, qs, st, s_stack + tid)) {
                handed = true;
                break;
            }
        }
        if (CNT) {
            sec_add_lanes(SEC_N_NODES, n_nodes);
            sec_add_lanes(SEC_N_TRIS, n_tris);
        }
        if (!handed) {
            bvh_count_ray<CNT>(st, t_prim, n_nodes);
            bvh_finish_path<VAR>(sc, q, qs, iter, p, st);
        }
    }
    const bool surv = active && !handed && p.rb > 0;
    if (active && !handed && !surv) gather_into_image(image, sc, to_plane, p);
    int si, unused;
    block_append<false>(surv, &ctl->cnt[bounce + 1][seg][0], false, nullptr, si, unused);
    if (surv) store_path(out, seg * seg_stride + si, p);
}

// The handed-over traversals, run by a fixed grid of waves that refill their lanes as rays
// finish: whenever `refill` or more of a wave's lanes are idle, it takes that many entries of its
// segment from the segment's counter of taken entries (FrameCtl::qcnt[b][s][2]; one atomic per
// refill), so a wave drains once, when its segment is done, instead of once per 64 rays.
// Traversal only: a finished ray's result (t, u, v, triangle) replaces its saved hit, and
// k_bvh_tail_shade shades the entries in full waves.  No barrier: waves leave on their own.
template <int VAR, bool QUAD>
__global__ __launch_bounds__(BLOCK, BVH_WAVES) void k_bvh_tail_trav(SceneDev sc, QueueBuf q, TailBuf t, FrameCtl* ctl,
                                                                    int bounce, int refill) {
    extern __shared__ float4 s_dyn[];
    int* s_stack = reinterpret_cast<int*>(s_dyn) + threadIdx.x;
    const int seg = blockIdx.x & (NSEG - 1);
    const int n = min(ctl->qcnt[bounce][seg][1], t.stride);
    if (n == 0) return;
    int next = 0;   // the segment's next untaken entry, as of this wave's last refill
    constexpr bool CNT = (VAR & VAR_SECTION_TIMING) != 0;
    int e = -1, qs = 0, n_nodes = 0, n_tris = 0, sp0 = 0;
    bool hit0 = false;
    TravState st;
    st.cur = -1;
    while (true) {
        const uint64_t idle = __ballot(e < 0);
        const int n_idle = __popcll(idle);
        if (next < n && (n_idle >= refill || n_idle == 64)) {
            const int lead = __builtin_ctzll(idle);
            int b0 = 0;
            if ((int)(threadIdx.x & 63) == lead) b0 = atomicAdd(&ctl->qcnt[bounce][seg][2], n_idle);
            next = __builtin_amdgcn_readlane(b0, lead);
            if (e < 0) {
                const int k = next + mbcnt(idle);
                if (k < n) {
                    e = seg * t.stride + k;
                    const int2 nd = t.node[e];
                    qs = nd.x;
                    const float4 a = q.A[qs], b = q.B[qs];
                    trav_resume(st, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), t.hit[e], nd.y, qs);
                    // the LDS part of its stack (spilled entries stay in the slot's row)
                    for (int i = 0; i < min(st.sp, sc.stack_lds); ++i) s_stack[i * BLOCK] = t.stack[(size_t)i * t.cap + e];
                    n_nodes = n_tris = 0;
                    if (CNT) {
                        sp0 = st.sp;
                        hit0 = st.btri != 0x7fffffff;
                    }
                }
            }
            next += n_idle;
        }
        const int lanes = __popcll(__ballot(e >= 0));
        if (lanes == 0) break;   // nothing left in the range
        if (e >= 0) {
            if (CNT) {
                sec_add(SEC_N_BVH_WITERS, 1);
                sec_add(SEC_TAIL_LANES_HIST + (lanes - 1) / 4, 1);
            }
            trav_step<CNT, QUAD>(sc, st, s_stack, n_nodes, n_tris);
            if (st.cur < 0) {
                t.hit[e] = trav_saved_hit(st);
                if (CNT) {
                    sec_add_lanes(SEC_N_NODES, n_nodes);
                    sec_add_lanes(SEC_N_TRIS, n_tris);
                    bvh_count_ray<CNT>(st, q.D[qs].x, n_nodes);
                    const int bk = sp0 < 4 ? sp0 : sp0 < 6 ? 4 : sp0 < 8 ? 5 : sp0 < 12 ? 6 : 7;
                    sec_add_lanes(SEC_TAIL_BY_SP + 2 * bk, 1);
                    sec_add_lanes(SEC_TAIL_BY_SP + 2 * bk + 1, n_nodes);
                    sec_add_lanes(SEC_TAIL_BY_HIT + (hit0 ? 2 : 0), 1);
                    sec_add_lanes(SEC_TAIL_BY_HIT + (hit0 ? 3 : 1), n_nodes);
                }
                e = -1;
            }
        }
    }
}
// ... and their shading, gather and compaction, as k_bvh_bounce's: block b takes the chunks
// j = b / NSEG, + gridDim / NSEG, .. of BLOCK entries of segment s = b % NSEG, survivors to output
// segment s (a grid for the usual counts, not for the capacity: empty blocks cost dispatch time)
template <int VAR>
__global__ __launch_bounds__(BLOCK) void k_bvh_tail_shade(SceneDev sc, QueueBuf q, TailBuf t, PathBuf out, FrameCtl* ctl,
                                                          float* __restrict__ image, int bounce, int seg_stride) {
    const int seg = blockIdx.x & (NSEG - 1);
    const int n = min(ctl->qcnt[bounce][seg][1], t.stride);
    const int iter = ctl->iter;
    const bool to_plane = ctl->batch > 1 || ctl->plane != 0;
    const int tid = threadIdx.x;
    for (int block_start = (blockIdx.x / NSEG) * BLOCK; block_start < n; block_start += (gridDim.x / NSEG) * BLOCK) {
        const bool active = block_start + tid < n;
        PathReg p;
        p.rb = 0;
        if (active) {
            const int e = seg * t.stride + block_start + tid;
            const int qs = t.node[e].x;
            const float4 a = q.A[qs], b = q.B[qs], h = t.hit[e];
            p.o = mk(a.x, a.y, a.z);
            p.d = mk(b.x, b.y, b.z);
            TravState st;
            st.t_hit = h.x;
            st.bu = h.y;
            st.bv = h.z;
            st.btri = __float_as_int(h.w);
            bvh_finish_path<VAR>(sc, q, qs, iter, p, st);
        }
        const bool surv = active && p.rb > 0;
        if (active && !surv) gather_into_image(image, sc, to_plane, p);
        int si, unused;
        block_append<false>(surv, &ctl->cnt[bounce + 1][seg][0], false, nullptr, si, unused);
        if (surv) store_path(out, seg * seg_stride + si, p);
    }
}

// --------------------------------------------------------------------------------------------
// STAGED kernels (single contiguous segment)
// --------------------------------------------------------------------------------------------
struct HitBuf {
    float4* nt;     // surfaceNormal.xyz | t
    int* mat;       // materialId
    float4* uvd0;   // textured scenes only (else null): uv.xy | dpdu.xy
    float4* uvd1;   //                                    dpdu.z | dpdv.xyz
};

__global__ __launch_bounds__(BLOCK) void k_camera(SceneDev sc, PathBuf out, FrameCtl* ctl) {
    int gid = blockIdx.x * BLOCK + threadIdx.x;
    if (gid >= ctl->cnt[0][0][0]) return;
    const int slot = gid / sc.shard.local_pixels;
    PathReg p = camera_ray(sc.cam, ctl->iter + slot, sc.trace_depth, shard_pixel(sc, gid - slot * sc.shard.local_pixels));
    p.slot = slot;
    store_path(out, gid, p);
}

template <bool HAS_BVH, bool BVH_FAST>
__global__ __launch_bounds__(BLOCK) void k_intersect(SceneDev sc, PathBuf in, HitBuf hits, const int* n_ptr) {
    extern __shared__ int s_stack[];
    const int n = *n_ptr;
    int gid = blockIdx.x * BLOCK + threadIdx.x;
    if (blockIdx.x * BLOCK >= n || gid >= n) return;
    float4 a = in.A[gid], b = in.B[gid];
    Hit h = intersect_scene<HAS_BVH, BVH_FAST>(sc, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z), s_stack + threadIdx.x);
    hits.nt[gid] = make_float4(h.n.x, h.n.y, h.n.z, h.t);
    hits.mat[gid] = h.mat;
    if (hits.uvd0) {
        const HitAttr a = hit_attr(sc, h);
        hits.uvd0[gid] = make_float4(a.u, a.v, a.dpdu.x, a.dpdu.y);
        hits.uvd1[gid] = make_float4(a.dpdu.z, a.dpdv.x, a.dpdv.y, a.dpdv.z);
    }
}

// shade (optionally through a material-sorted permutation); terminated paths are gathered
// into the image unless image == nullptr; alive flags feed the compaction kernel.
__global__ __launch_bounds__(BLOCK) void k_shade(SceneDev sc, PathBuf buf, HitBuf hits, const int* perm,
                                                 const int* n_ptr, const FrameCtl* ctl, int iter_override,
                                                 float* image, int* alive) {
    const int n = *n_ptr;
    int j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n) return;
    int i = perm ? perm[j] : j;
    PathReg p = load_path(buf, i);
    if (p.rb <= 0) {                 // pathtrace.cu:535-537
        if (alive) alive[i] = 0;
        return;
    }
    float4 nt = hits.nt[i];
    Hit h;
    h.t = nt.w;
    h.n = mk(nt.x, nt.y, nt.z);
    h.mat = hits.mat[i];
    h.tri = -1;
    h.u = h.v = 0.f;
    const int iter = iter_override > 0 ? iter_override : ctl->iter;
    shade_path(sc, p, h, iter + p.slot, [&]() {
        HitAttr a;
        a.u = a.v = 0.0f;
        a.dpdu = a.dpdv = mk(0.f, 0.f, 0.f);
        if (hits.uvd0) {
            const float4 x = hits.uvd0[i], y = hits.uvd1[i];
            a.u = x.x;
            a.v = x.y;
            a.dpdu = mk(x.z, x.w, y.x);
            a.dpdv = mk(y.y, y.z, y.w);
        }
        return a;
    });
    store_path(buf, i, p);
    if (p.rb <= 0 && image)
        gather_into_image(image, sc, iter_override > 0 ? false : (ctl->batch > 1 || ctl->plane != 0), p);
    if (alive) alive[i] = p.rb > 0;
}

// ---- stable compaction (thrust::stable_partition(PathAlive), pathtrace.cu:750-757) ----
// Reduce-then-scan, three launches with no inter-workgroup waiting (dispatch order on MI355X is
// undefined by contract, and a single-word ticket / hop-by-hop look-back serialises at the
// device-scope atomic rate):
//   k_compact_count   per tile of CTILE items: popcount of ballot(alive) -> tile_cnt[t]
//   k_compact_scan    one workgroup: exclusive scan of tile_cnt -> tile_off, total -> n_out
//   k_compact_scatter per tile: flags + survivor payload loaded together, wave ballot/mbcnt
//                     ranks in item order, stores to tile_off[t] + rank (stable)
constexpr int CITEMS = 4;                       // items per thread (8 spills: measured slower)
constexpr int CTILE_MIN = BLOCK * CITEMS;       // 1024-item tiles (sizes the tile arrays)
constexpr int STILE = BLOCK * 8;                // material-sort tile (2048 items)
constexpr int SCAN_THREADS = 1024;

template <int CITEMS>
__global__ __launch_bounds__(BLOCK) void k_compact_count(const int* __restrict__ alive, const int* n_ptr,
                                                         int* __restrict__ tile_cnt) {
    constexpr int CTILE = BLOCK * CITEMS;
    __shared__ int s_w[BLOCK / 64];
    const int n = *n_ptr;
    const int base = blockIdx.x * CTILE;
    if (base >= n) return;
    const int tid = threadIdx.x;
    int av[CITEMS];
#pragma unroll
    for (int k = 0; k < CITEMS; ++k) av[k] = alive[base + k * BLOCK + tid];   // capacity is tile-padded
    int c = 0;
#pragma unroll
    for (int k = 0; k < CITEMS; ++k) c += __popcll(__ballot((base + k * BLOCK + tid < n) & (av[k] != 0)));
    if ((tid & 63) == 0) s_w[tid >> 6] = c;
    __syncthreads();
    if (tid == 0) {
        int t = 0;
#pragma unroll
        for (int i = 0; i < BLOCK / 64; ++i) t += s_w[i];
        tile_cnt[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(SCAN_THREADS) void k_compact_scan(const int* __restrict__ tile_cnt, const int* n_ptr,
                                                                int* __restrict__ tile_off, int* n_out, int CTILE) {
    __shared__ int s_part[SCAN_THREADS];
    const int n = *n_ptr;
    const int ntiles = (n + CTILE - 1) / CTILE;
    const int per = (ntiles + SCAN_THREADS - 1) / SCAN_THREADS;
    const int tid = threadIdx.x;
    const int lo = tid * per, hi = min(ntiles, lo + per);
    int sum = 0;
    for (int t = lo; t < hi; ++t) sum += tile_cnt[t];
    s_part[tid] = sum;
    __syncthreads();
    for (int off = 1; off < SCAN_THREADS; off <<= 1) {   // Hillis-Steele inclusive scan in LDS
        int v = tid >= off ? s_part[tid - off] : 0;
        __syncthreads();
        s_part[tid] += v;
        __syncthreads();
    }
    int run = tid ? s_part[tid - 1] : 0;
    for (int t = lo; t < hi; ++t) {
        tile_off[t] = run;
        run += tile_cnt[t];
    }
    if (tid == SCAN_THREADS - 1) *n_out = s_part[SCAN_THREADS - 1];
}

// native 4-float vector: arrays of it stay in VGPRs (HIP's float4 is a union wrapper, and
// arrays of it were demoted to LDS/scratch, serialising each item's loads behind a wait)

template <int CITEMS>
__global__ __launch_bounds__(BLOCK) void k_compact_scatter(const float4* __restrict__ inA, const float4* __restrict__ inB,
                                                           const float4* __restrict__ inC, float4* __restrict__ outA,
                                                           float4* __restrict__ outB, float4* __restrict__ outC,
                                                           const int* __restrict__ alive, const int* n_ptr,
                                                           const int* __restrict__ tile_off) {
    constexpr int CTILE = BLOCK * CITEMS;
    __shared__ int s_cnt[CITEMS][BLOCK / 64];
    const int n = *n_ptr;
    const int base = blockIdx.x * CTILE;
    if (base >= n) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const v4f* iA = reinterpret_cast<const v4f*>(inA);
    const v4f* iB = reinterpret_cast<const v4f*>(inB);
    const v4f* iC = reinterpret_cast<const v4f*>(inC);
    bool f[CITEMS];
#pragma unroll
    for (int k = 0; k < CITEMS; ++k) f[k] = (base + k * BLOCK + tid < n) & (alive[base + k * BLOCK + tid] != 0);
    v4f a[CITEMS], b[CITEMS], c[CITEMS];
#pragma unroll
    for (int k = 0; k < CITEMS; ++k) {
        const int idx = base + k * BLOCK + tid;
        if (f[k]) {
            a[k] = __builtin_nontemporal_load(iA + idx);
            b[k] = __builtin_nontemporal_load(iB + idx);
            c[k] = __builtin_nontemporal_load(iC + idx);
        }
    }
    uint64_t m[CITEMS];
#pragma unroll
    for (int k = 0; k < CITEMS; ++k) {
        m[k] = __ballot(f[k]);
        if (lane == 0) s_cnt[k][w] = __popcll(m[k]);
    }
    __syncthreads();
    // exclusive offsets in item order (k-major, then wave): every thread recomputes its own
    int run = tile_off[blockIdx.x];
    int off[CITEMS];
#pragma unroll
    for (int k = 0; k < CITEMS; ++k) {
        int mine = run;
#pragma unroll
        for (int i = 0; i < BLOCK / 64; ++i) {
            const int cnt = s_cnt[k][i];
            mine = (i < w) ? mine + cnt : mine;
            run += cnt;
        }
        off[k] = mine;
    }
    v4f* oA = reinterpret_cast<v4f*>(outA);
    v4f* oB = reinterpret_cast<v4f*>(outB);
    v4f* oC = reinterpret_cast<v4f*>(outC);
#pragma unroll
    for (int k = 0; k < CITEMS; ++k) {
        if (f[k]) {
            const int dst = off[k] + mbcnt(m[k]);
            __builtin_nontemporal_store(a[k], oA + dst);
            __builtin_nontemporal_store(b[k], oB + dst);
            __builtin_nontemporal_store(c[k], oC + dst);
        }
    }
}

// ---- stable counting sort of materialId (MATERIAL_SORTING, pathtrace.cu:730-735) ----
constexpr int MAXMAT = 256;

// per-tile key histogram, tile = STILE items
__global__ __launch_bounds__(BLOCK) void k_sort_hist(const int* __restrict__ keys, const int* n_ptr, int nkeys,
                                                     int* tile_hist) {
    __shared__ int h[MAXMAT];
    const int n = *n_ptr;
    const int tile = blockIdx.x, base = tile * STILE;
    for (int i = threadIdx.x; i < nkeys; i += BLOCK) h[i] = 0;
    __syncthreads();
    if (base < n) {
        for (int k = 0; k < STILE / BLOCK; ++k) {
            int idx = base + k * BLOCK + threadIdx.x;
            if (idx < n) atomicAdd(&h[keys[idx]], 1);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nkeys; i += BLOCK) tile_hist[(size_t)tile * nkeys + i] = h[i];
}

// exclusive scan over (key, tile) in key-major order: one block of SCAN_THREADS, each thread a
// contiguous run of the flattened (key, tile) index space (tile_hist is stored [tile][key]),
// then a block scan of the run sums.  (The earlier one-thread-per-key loop over all tiles ran
// ~780 us at 10k tiles: 5-27 busy threads out of 256.)
__global__ __launch_bounds__(SCAN_THREADS) void k_sort_scan(int* tile_hist, const int* n_ptr, int nkeys) {
    __shared__ int s_part[SCAN_THREADS];
    const int n = *n_ptr;
    const int ntiles = (n + STILE - 1) / STILE;
    const int total = ntiles * nkeys;
    const int per = (total + SCAN_THREADS - 1) / SCAN_THREADS;
    const int tid = threadIdx.x;
    const int lo = min(total, tid * per), hi = min(total, lo + per);
    const int key0 = ntiles ? lo / ntiles : 0, t0 = lo - key0 * ntiles;
    int sum = 0;
    for (int f = lo, key = key0, t = t0; f < hi; ++f) {
        sum += tile_hist[(size_t)t * nkeys + key];
        if (++t == ntiles) { t = 0; ++key; }
    }
    s_part[tid] = sum;
    __syncthreads();
    for (int off = 1; off < SCAN_THREADS; off <<= 1) {   // Hillis-Steele inclusive scan in LDS
        const int v = tid >= off ? s_part[tid - off] : 0;
        __syncthreads();
        s_part[tid] += v;
        __syncthreads();
    }
    int run = tid ? s_part[tid - 1] : 0;
    for (int f = lo, key = key0, t = t0; f < hi; ++f) {
        const size_t at = (size_t)t * nkeys + key;
        const int c = tile_hist[at];
        tile_hist[at] = run;
        run += c;
        if (++t == ntiles) { t = 0; ++key; }
    }
}

// stable scatter: rank among equal keys = earlier items of the tile (item order k-major, wave,
// lane) — peers found with one ballot per key bit
__global__ __launch_bounds__(BLOCK) void k_sort_scatter(const int* __restrict__ keys, const int* n_ptr, int nkeys,
                                                        int key_bits, const int* tile_off, int* perm) {
    __shared__ int run[MAXMAT];           // items of each key already placed in this tile
    __shared__ int wcnt[BLOCK / 64][MAXMAT];
    const int n = *n_ptr;
    const int tile = blockIdx.x, base = tile * STILE;
    if (base >= n) return;
    const int tid = threadIdx.x, w = tid >> 6;
    for (int i = tid; i < nkeys; i += BLOCK) run[i] = 0;
    __syncthreads();
    for (int k = 0; k < STILE / BLOCK; ++k) {
        int idx = base + k * BLOCK + tid;
        bool valid = idx < n;
        int key = valid ? keys[idx] : 0;
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < key_bits; ++b) {
            uint64_t bb = __ballot(valid && ((key >> b) & 1));
            peers &= ((key >> b) & 1) ? bb : ~bb;
        }
        for (int i = tid; i < (BLOCK / 64) * MAXMAT; i += BLOCK) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        // the lowest lane of each peer group publishes the group size for its wave
        if (valid && mbcnt(peers) == 0) wcnt[w][key] = __popcll(peers);
        __syncthreads();
        if (valid) {
            int r = run[key] + mbcnt(peers);
            for (int ww = 0; ww < w; ++ww) r += wcnt[ww][key];
            perm[tile_off[(size_t)tile * nkeys + key] + r] = idx;
        }
        __syncthreads();
        for (int key2 = tid; key2 < nkeys; key2 += BLOCK) {
            int s = 0;
            for (int ww = 0; ww < BLOCK / 64; ++ww) s += wcnt[ww][key2];
            run[key2] += s;
        }
        __syncthreads();
    }
}

// sendImageToPBO (pathtrace.cu:59-80)
__global__ void k_to_pbo(const float* __restrict__ image, pt_uchar4* pbo, int n, int iter) {
    int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    int c[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double d = (double)(image[3 * (size_t)i + k] / (float)iter) * 255.0;
        int v = (d != d) ? 0 : (d >= 2147483647.0 ? 2147483647 : (d <= -2147483648.0 ? (-2147483647 - 1) : (int)d));
        c[k] = v < 0 ? 0 : (v > 255 ? 255 : v);
    }
    pt_uchar4 o;
    o.x = (uint8_t)c[0];
    o.y = (uint8_t)c[1];
    o.z = (uint8_t)c[2];
    o.w = 0;
    pbo[i] = o;
}

__global__ void k_rng(const int* iid, int m, int n, float* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    Rng r = rng_make(iid[3 * i], iid[3 * i + 1], iid[3 * i + 2]);
    for (int k = 0; k < n; ++k) out[(size_t)i * n + k] = u01(r);
}

// =============================================================================================
// host runtime
// =============================================================================================
namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define RC(x)                      \
    do {                           \
        int rc_ = (x);             \
        if (rc_ != PT_OK) return rc_; \
    } while (0)
#define HIPCHK(expr)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return fail(PT_E_HIP, "%s:%d: %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
    } while (0)

template <class T>
int dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) return PT_OK;
    HIPCHK(hipMalloc((void**)p, n * sizeof(T)));
    return PT_OK;
}

constexpr int MAXF = 256;                   // frames per pass, upper bound (slot: 8 bits of a queue entry)
// auto F: up to ~84M paths at bounce 0 -> 800x800: F = 128, 1600x1600: F = 32.  A/B (ms/frame):
// cornell 800^2 F = 8 0.0992, 16 0.0949 (0.0937), 32 0.0921; bunny 800^2 F = 8 0.685, 16 0.633;
// khaslana 1600^2 F = 2 2.52, 4 1.95 (1.93), 8 1.66 (earlier kernels: F = 1 0.214, 2 0.161,
// 4 0.137, 8 0.129).  Round 2 (tools/autof_ab.sh, target 21M / 42M / 84M paths): khaslana
// 1600^2 d12 1.38 / 1.27 / 1.23, bunny 0.397 / 0.388 / 0.391, cornell flat.  ~16 GB of path
// buffers + 5.2 GB traversal queue at 1600^2, F = 32 (of 288 GB).
constexpr int64_t AUTO_BATCH_PATHS = 84000000;

// Tuning and test knobs (tools, A/B runs, tests).  Every one is read from the environment in ONE
// place, read_tuning(), when pt_init builds a context -- never on a hot call -- and none changes a
// result (the tests run each one against the oracle).  INTEGRATION.md §4 lists them.
struct Tuning {
    size_t bounce_lds_pad = 0, bvh_lds_pad = 0;   // PT_BOUNCE_LDS_PAD / PT_BVH_LDS_PAD: unused LDS (occupancy A/B)
    bool sections_skip_camera = false;              // PT_SECTIONS_SKIP_CAMERA: camera bounce out of the counters
    bool tail_off = false;                          // PT_TAIL=0: no k_tail launch
    bool tail_any_batch = false;                    // PT_TAIL_BATCH=1: k_tail for multi-frame passes too
    int tail_from = 0;                              // PT_TAIL_FROM: k_tail's first bounce (0: depth / 2)
    int64_t auto_paths = 0;                         // PT_AUTO_PATHS: auto pass size in paths (0: AUTO_BATCH_PATHS)
    bool f1_graph = false;                          // PT_F1_GRAPH=1: single-frame passes through a graph
    bool multi_f1_direct = false;                   // PT_MULTI_F1_DIRECT=1: shards' single frames launched directly
    int bvh_tail_lanes = -1;                        // PT_BVH_TAIL_LANES (0..56; 0: no hand-over; -1: by tree size)
    int bvh_tail_chunks = 0;                        // PT_BVH_TAIL_CHUNKS: capped hand-over buffers (tests)
    int tail_refill = 16;                           // PT_BVH_TAIL_REFILL (1..64 idle lanes)
    int tail_trav_blocks = 224;                     // PT_BVH_TAIL_TRAV_BLOCKS per segment
    int tail_shade_blocks = 512;                    // PT_BVH_TAIL_SHADE_BLOCKS per segment (0: one per chunk)
    bool combine_force_staged = false;              // PT_COMBINE_FORCE_STAGED=1: peer shards via packed tiles
    bool bvh_tree_ref = false;                      // PT_BVH_TREE=ref: the reference's hierarchy, no SAH tree
    bool bvh_tree_info = false;                     // PT_BVH_TREE_INFO: print the traversal tree's shape
    int bvh_max_height = -1;                        // PT_BVH_MAX_HEIGHT: SAH tree height bound (0: none; -1: the
                                                    // height whose LDS stack still admits BVH_WAVES blocks per CU)
    int bvh_quad = 1;                               // PT_BVH_QUAD: the traversal kernels on 4-wide records (1) or on
                                                    // the pairs (0) (A/B: 262k -7.6 %, 1.0M -8.7 %, bunny -5.0 %,
                                                    // khaslana -1.9 %; profiles/r06_ab_four_wide.json)
    int bvh_stack_lds = 0;                          // PT_BVH_STACK_LDS: traversal stack entries kept in LDS by the split
                                                    // kernels, deeper ones spilled to a row per queue slot (0: all)
    int bvh_bfs_levels = 12;                        // PT_BVH_BFS_LEVELS: SAH pairs numbered breadth-first over
                                                    // this many levels, each subtree below in preorder
                                                    // (A/B: 262k -1.0 %, 1.0M -1.4 %, bunny +-0 vs all
                                                    // breadth-first; profiles/r06_ab_pair_numbering.json)
    int grid = -1;                                  // PT_GRID: 0 no candidate table, 1 also for small scenes
    bool speculate = true;                          // PT_SPECULATE=0: initial state of pt_set_speculation
    int band_copy = -1;                             // PT_BAND_COPY: several devices' host copy split over the
                                                    // shards (1), one copy from the first device (0), or
                                                    // split only when every shard has a device of its own (-1)
};
Tuning read_tuning() {
    auto num = [](const char* name, long dflt) {
        const char* e = getenv(name);
        return e && *e ? atol(e) : dflt;
    };
    Tuning t;
    t.bounce_lds_pad = (size_t)std::max(0L, num("PT_BOUNCE_LDS_PAD", 0));
    t.bvh_lds_pad = (size_t)std::max(0L, num("PT_BVH_LDS_PAD", 0));
    t.sections_skip_camera = getenv("PT_SECTIONS_SKIP_CAMERA") != nullptr;
    t.tail_off = num("PT_TAIL", 1) == 0;
    t.tail_any_batch = num("PT_TAIL_BATCH", 0) != 0;
    t.tail_from = (int)num("PT_TAIL_FROM", 0);
    t.auto_paths = num("PT_AUTO_PATHS", 0);
    t.f1_graph = num("PT_F1_GRAPH", 0) != 0;
    t.multi_f1_direct = num("PT_MULTI_F1_DIRECT", 0) != 0;
    t.bvh_tail_lanes = (int)std::min(56L, std::max(-1L, num("PT_BVH_TAIL_LANES", -1)));
    t.bvh_tail_chunks = (int)std::max(0L, num("PT_BVH_TAIL_CHUNKS", 0));
    t.tail_refill = (int)std::max(1L, std::min(64L, num("PT_BVH_TAIL_REFILL", 16)));
    t.tail_trav_blocks = (int)std::max(1L, num("PT_BVH_TAIL_TRAV_BLOCKS", 224));
    t.tail_shade_blocks = (int)std::max(0L, num("PT_BVH_TAIL_SHADE_BLOCKS", 512));
    t.combine_force_staged = num("PT_COMBINE_FORCE_STAGED", 0) != 0;
    const char* tree = getenv("PT_BVH_TREE");
    t.bvh_tree_ref = tree && strcmp(tree, "ref") == 0;
    t.bvh_tree_info = getenv("PT_BVH_TREE_INFO") != nullptr;
    t.bvh_bfs_levels = (int)std::max(0L, num("PT_BVH_BFS_LEVELS", 12));
    t.bvh_max_height = (int)std::max(-1L, num("PT_BVH_MAX_HEIGHT", -1));
    t.bvh_quad = num("PT_BVH_QUAD", 1) != 0 ? 1 : 0;
    t.bvh_stack_lds = (int)std::max(0L, num("PT_BVH_STACK_LDS", 0));
    t.grid = (int)num("PT_GRID", -1);
    t.speculate = num("PT_SPECULATE", 1) != 0;
    t.band_copy = (int)std::max(-1L, std::min(1L, num("PT_BAND_COPY", -1)));
    return t;
}

struct State {
    bool inited = false;
    Tuning tune;
    pt_options opts{};
    int device = 0;
    hipStream_t stream = nullptr;
    SceneDev sc{};
    int width = 0, height = 0, pixels_total = 0, local_pixels = 0;
    // per-pass buffers are sized lazily (ensure_frames): a caller that only ever traces single
    // frames (the drop-in pathtrace(), the viewer) holds one frame's worth, not a whole pass's
    int seg_stride = 0, capacity = 0;
    int alloc_frames = 0;            // frames per pass the path buffers / queue / planes hold now
    bool staged_alloc = false;       // hit / alive / permutation / tile buffers at `capacity`
    int num_tex = 0;
    bool has_bvh = false;
    int stack_depth = 0;
    int pair_depth = 0;              // entries the pair traversal needs: height of its hierarchy + 1
    size_t bvh_lds = 0;
    // device buffers
    DevGeom* d_geoms = nullptr;
    DevCull* d_cull = nullptr;
    DevMaterial* d_mats = nullptr;
    float4* d_node_aux = nullptr;
    DevNode* d_nodes = nullptr;
    DevTriHot* d_hot = nullptr;
    DevPair* d_pairs = nullptr;
    float4* d_quads = nullptr;       // the 4-wide layout (SceneDev::quads), trees past the L2
    DevTriHot* d_hot4 = nullptr;
    float4* d_leaf9 = nullptr;
    DevTriCold* d_cold = nullptr;
    float4* d_path[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};
    float4* d_hit_nt = nullptr;
    int* d_hit_mat = nullptr;
    float4* d_hit_uvd0 = nullptr;    // textured scenes only
    float4* d_hit_uvd1 = nullptr;
    uint32_t* d_texels = nullptr;
    int4* d_texinfo = nullptr;
    int* d_alive = nullptr;
    int* d_perm = nullptr;
    int* d_tile_hist = nullptr;
    int* d_tile_cnt = nullptr;
    int* d_tile_off = nullptr;
    float* d_image = nullptr;
    FrameCtl* d_ctl = nullptr;
    float* d_contrib = nullptr;      // passes of F > 1 frames: F planes of pixels_total float3
    unsigned long long* d_grid = nullptr;   // the pre-test's candidate table (build_candidate_table)
    int batch = 1;                   // frames per pass (pt_options.frames_per_pass, resolved)
    bool split = false;              // VAR_BVH_SPLIT active (fused, fast BVH on the pair layout)
    bool no_tex = false;             // no textured / bump-mapped material (VAR_NO_TEX kernels)
    QueueBuf queue{};                // its traversal queue (capacity: one pass's paths)
    TailBuf tail{};                  // the traversals k_bvh_bounce hands to k_bvh_tail_trav
    int tail_lanes = 0;              // bvh_tail_lanes()
    int tail_refill = 16, tail_trav_blocks = 224, tail_shade_blocks = 512;   // PT_BVH_TAIL_REFILL / _TRAV_BLOCKS / _SHADE_BLOCKS
    int tail_depth = 0;              // stack entries per handed-over traversal
    // one captured pass per pass size (1..MAXF frames)
    hipGraph_t graph[MAXF + 1] = {};
    hipGraphExec_t graph_exec[MAXF + 1] = {};
    int last_iter = 0;
    int dev_iter = 0;                // FrameCtl::iter after the passes queued so far (0 after a reset)
    int ctl_rows = 1;                // counter rows k_frame_begin folds / clears (max trace depth + 1)
    int frames_done = 0;
    int32_t* traced_depth = nullptr;
    int* h_cnt = nullptr;            // page-locked copy of the live counters (TracedDepth, frame_depth_*)
    // single-frame speculation (pt_trace, spec_*): frame N + 1 traced into a plane of its own on a
    // second stream while frame N's image crosses PCIe to the caller
    hipStream_t spec_stream = nullptr;
    hipEvent_t spec_ev_in = nullptr;      // gp->stream: what the speculative frame follows
    hipEvent_t spec_ev_done = nullptr;    // spec_stream: the speculative frame is finished
    FrameCtl* d_ctl_spec = nullptr;       // its own counters (d_ctl keeps the caller's frame)
    float* d_spec_plane = nullptr;        // its contributions, one float3 per pixel
    float* d_spec_sum[2] = {nullptr, nullptr};   // image + plane, formed at its end (alternating)
    int spec_sum_idx = 0;                 // the buffer the pending speculative frame writes
    hipStream_t copy_stream = nullptr;    // the host copy of a taken-over frame's image
    hipStream_t band_stream = nullptr;    // several devices: the host copy of this shard's row bands
    hipEvent_t band_ready = nullptr;      // ... what it follows (the shard's frame)
    hipGraph_t spec_graph = nullptr;      // its pass, captured once (released with the pass graphs)
    hipGraphExec_t spec_exec = nullptr;
    int spec_iter = 0;                    // iteration of the queued speculative frame (0: none)
    int64_t spec_launched = 0, spec_adopted = 0;   // speculated frames queued / taken over (pt_debug_spec_counts)
    int spec_dev_iter = 0;                // d_ctl_spec->iter after the speculative frames queued so far
    int key_bits = 1;
    bool multi = false;              // a shard context of a multi-device pt_init
};
State g_primary;                 // the process's context (shard 0 of a multi-device context)
State* gp = &g_primary;          // the context the host runtime works on now (see ShardScope)
int ensure_frames(int frames);

// Host <-> device copies and memsets of the runtime, ordered on the library's stream and
// completed before returning.  gp->stream is a non-blocking stream: the legacy null stream that
// plain hipMemset / hipMemcpy use does not order against it, so a memset of FrameCtl could land
// after a kernel enqueued behind it on gp->stream (pt_test_camera saw a zeroed path count).
hipError_t smemset(void* p, int v, size_t n) {
    hipError_t e = hipMemsetAsync(p, v, n, gp->stream);
    return e != hipSuccess ? e : hipStreamSynchronize(gp->stream);
}
hipError_t smemcpy(void* dst, const void* src, size_t n, hipMemcpyKind kind) {
    hipError_t e = hipMemcpyAsync(dst, src, n, kind, gp->stream);
    return e != hipSuccess ? e : hipStreamSynchronize(gp->stream);
}

PathBuf pathbuf(int i) { return PathBuf{gp->d_path[i][0], gp->d_path[i][1], gp->d_path[i][2]}; }

// zero the frame control block (counters, totals, the device iteration)
int ctl_reset() {
    const hipError_t e = smemset(gp->d_ctl, 0, sizeof(FrameCtl));
    if (e != hipSuccess) return fail(PT_E_HIP, "FrameCtl reset: %s", hipGetErrorString(e));
    gp->dev_iter = 0;
    return PT_OK;
}

// pt_profile_frames: every kernel of the frame is launched with hipExtLaunchKernel's start/stop
// events, which take their timestamps from that dispatch packet itself -- the kernel's own
// execution time, independent of how far ahead of the GPU the host is.
struct ProfRec {
    int kind;            // -1 frame begin, 0 camera, 1 intersect, 2 shade, 3 compact scatter,
                         // 4 material sort, 5 compact count+scan, 100+b fused bounce b,
                         // 200+b its split BVH traversal kernel, 300+b k_tail from bounce b
    hipEvent_t start, stop;
};
// The per-dispatch events skip the system-scope fence a default event performs when it is
// recorded: that fence writes back and invalidates L2 around every profiled kernel, which made
// the eager replay's k_bounce launches ~18 % longer than the same launches in the timed graph
// replay (rocprofv3 kernel trace, cornell 800^2 F = 20: 0.221 vs 0.188 ms per launch).  The
// kernels run on one stream and are ordered by it; no host reads their results through these
// events.
constexpr unsigned PROF_EVENT_FLAGS = hipEventDisableSystemFence;
std::vector<ProfRec>* g_prof = nullptr;
std::vector<hipEvent_t> g_prof_pool;   // events created before the profiled run (no host-side
size_t g_prof_next = 0;                // event creation between the timed launches)

hipEvent_t prof_event() {
    if (g_prof_next < g_prof_pool.size()) return g_prof_pool[g_prof_next++];
    hipEvent_t e = nullptr;
    (void)hipEventCreateWithFlags(&e, PROF_EVENT_FLAGS);
    g_prof_pool.push_back(e);
    g_prof_next = g_prof_pool.size();
    return e;
}

template <class K, class... A>
void launch(int kind, K kernel, dim3 grid, dim3 block, uint32_t lds, A... args) {
    if (g_prof) {
        ProfRec r{kind, prof_event(), prof_event()};
        hipExtLaunchKernelGGL(kernel, grid, block, lds, gp->stream, r.start, r.stop, 0, args...);
        g_prof->push_back(r);
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, gp->stream, args...);
    }
}
int nblocks(int n) { return (n + BLOCK - 1) / BLOCK; }

int spec_worker_idle();
void release_graph() {
    if (gp->spec_exec) {   // the launcher may still be queueing it, the stream still running it
        (void)spec_worker_idle();
        (void)hipStreamSynchronize(gp->spec_stream);
        (void)hipGraphExecDestroy(gp->spec_exec);
    }
    if (gp->spec_graph) (void)hipGraphDestroy(gp->spec_graph);
    gp->spec_exec = nullptr;
    gp->spec_graph = nullptr;
    for (int f = 0; f <= MAXF; ++f) {
        if (gp->graph_exec[f]) (void)hipGraphExecDestroy(gp->graph_exec[f]);
        if (gp->graph[f]) (void)hipGraphDestroy(gp->graph[f]);
        gp->graph_exec[f] = nullptr;
        gp->graph[f] = nullptr;
    }
}

// bytes of the block's LDS geom table (lds_geom_f4 on the device)
size_t geom_table_lds() {
    return (sizeof(DevGeomHot) + (gp->sc.grid ? sizeof(DevCull) : 0)) * (size_t)gp->sc.num_geoms;
}

// device-side counter of the input of bounce b in the staged pipeline
const int* staged_count(int b) { return &gp->d_ctl->cnt[b][0][0]; }

template <bool FIRST, bool HAS_BVH, int VAR>
void launch_bounce_t(dim3 grid, PathBuf in, PathBuf out, int b) {
    constexpr bool SPLIT = HAS_BVH && (VAR & VAR_BVH_SPLIT);
    const bool lds = (VAR & (VAR_CAND_QUEUE | VAR_WAVE_REDIST)) && gp->sc.num_geoms <= LDS_GEOMS;
    const size_t geom_lds = lds ? geom_table_lds() : 0;
    // the exchange's region: block_intersect's BlockLds, or one WaveLds per wave (wave_intersect)
    const size_t redist_lds = (VAR & VAR_WAVE_REDIST) && lds
                                  ? ((VAR & VAR_BLOCK_REDIST) ? sizeof(BlockLds) : sizeof(WaveLds) * (BLOCK / 64))
                                  : 0;
    const size_t stack_lds = HAS_BVH && !SPLIT ? gp->bvh_lds : 0;
    // VAR_MAT_GROUP's exchange reuses the exact-test exchange's region (it runs after it)
    const size_t xchg_lds = (VAR & VAR_MAT_GROUP) ? std::max(redist_lds, mat_group_lds(HAS_BVH, false)) : redist_lds;
    // tools: unused LDS added to k_bounce / the traversal kernel (occupancy A/B)
    const size_t bounce_pad = gp->tune.bounce_lds_pad;
    launch(100 + b, k_bounce<FIRST, HAS_BVH, VAR>, grid, dim3(BLOCK), geom_lds + stack_lds + xchg_lds + bounce_pad, gp->sc,
           in, out, gp->d_ctl, gp->d_image, b, gp->seg_stride, gp->queue);
    const size_t lds_pad = gp->tune.bvh_lds_pad;
    if (SPLIT) {
        const size_t stack_bytes = (size_t)gp->sc.stack_lds * BLOCK * sizeof(int);
        // the handed-over stacks were sized for the pair tree of the allocation (ensure_frames)
        if (gp->tail_lanes > 0 && gp->sc.stack_lds > gp->tail_depth) gp->tail_lanes = 0;
        if (gp->sc.quads)   // the 4-wide layout (trees past the L2)
            launch(200 + b, k_bvh_bounce<VAR, true>, grid, dim3(BLOCK), stack_bytes + lds_pad, gp->sc, gp->queue,
                   gp->tail, gp->tail_lanes, out, gp->d_ctl, gp->d_image, b, gp->seg_stride);
        else
            launch(200 + b, k_bvh_bounce<VAR, false>, grid, dim3(BLOCK), stack_bytes + lds_pad, gp->sc, gp->queue,
                   gp->tail, gp->tail_lanes, out, gp->d_ctl, gp->d_image, b, gp->seg_stride);
        if (gp->tail_lanes > 0) {   // the handed-over rays: refilling waves, then their shading
            if (gp->sc.quads)
                launch(400 + b, k_bvh_tail_trav<VAR, true>, dim3(NSEG * gp->tail_trav_blocks), dim3(BLOCK), stack_bytes,
                       gp->sc, gp->queue, gp->tail, gp->d_ctl, b, gp->tail_refill);
            else
                launch(400 + b, k_bvh_tail_trav<VAR, false>, dim3(NSEG * gp->tail_trav_blocks), dim3(BLOCK), stack_bytes,
                       gp->sc, gp->queue, gp->tail, gp->d_ctl, b, gp->tail_refill);
            const int per_seg = gp->tail_shade_blocks > 0 ? std::min(gp->tail_shade_blocks, nblocks(gp->tail.stride))
                                                          : nblocks(gp->tail.stride);
            launch(400 + b, k_bvh_tail_shade<VAR>, dim3(NSEG * per_seg), dim3(BLOCK), 0, gp->sc,
                   gp->queue, gp->tail, out, gp->d_ctl, gp->d_image, b, gp->seg_stride);
        }
    }
}
template <bool FIRST, bool HAS_BVH>
void launch_bounce_v(int var, dim3 grid, PathBuf in, PathBuf out, int b) {
    switch (var) {
#ifdef PT_VAR_PROBE   // tools: register-pressure probes compile only the default variants
        case 154: launch_bounce_t<FIRST, HAS_BVH, 154>(grid, in, out, b); break;
        case 186: launch_bounce_t<FIRST, HAS_BVH, 186>(grid, in, out, b); break;
#else
        case 0: launch_bounce_t<FIRST, HAS_BVH, 0>(grid, in, out, b); break;
        case 1: launch_bounce_t<FIRST, HAS_BVH, 1>(grid, in, out, b); break;
        case 2: launch_bounce_t<FIRST, HAS_BVH, 2>(grid, in, out, b); break;
        case 6: launch_bounce_t<FIRST, HAS_BVH, 6>(grid, in, out, b); break;
        case 10: launch_bounce_t<FIRST, HAS_BVH, 10>(grid, in, out, b); break;
        case 18: launch_bounce_t<FIRST, HAS_BVH, 18>(grid, in, out, b); break;
        case 26: launch_bounce_t<FIRST, HAS_BVH, 26>(grid, in, out, b); break;
        case 22: launch_bounce_t<FIRST, HAS_BVH, 22>(grid, in, out, b); break;
        case 50: launch_bounce_t<FIRST, HAS_BVH, 50>(grid, in, out, b); break;
        case 58: launch_bounce_t<FIRST, HAS_BVH, 58>(grid, in, out, b); break;
        case 54: launch_bounce_t<FIRST, HAS_BVH, 54>(grid, in, out, b); break;   // split + section counters
        case 30: launch_bounce_t<FIRST, HAS_BVH, 30>(grid, in, out, b); break;   // redist + pair counters
        case 154: launch_bounce_t<FIRST, HAS_BVH, 154>(grid, in, out, b); break;
        case 186: launch_bounce_t<FIRST, HAS_BVH, 186>(grid, in, out, b); break;
        case 190: launch_bounce_t<FIRST, HAS_BVH, 190>(grid, in, out, b); break;   // 186 + section counters
        case 158: launch_bounce_t<FIRST, HAS_BVH, 158>(grid, in, out, b); break;   // 154 + section counters
        case 666: launch_bounce_t<FIRST, HAS_BVH, 666>(grid, in, out, b); break;   // 154 + material grouping
        case 530: launch_bounce_t<FIRST, HAS_BVH, 530>(grid, in, out, b); break;   // camera bounce of 666
        case 698: launch_bounce_t<FIRST, HAS_BVH, 698>(grid, in, out, b); break;   // 186 + material grouping
        case 562: launch_bounce_t<FIRST, HAS_BVH, 562>(grid, in, out, b); break;   // camera bounce of 698
#endif
        // the same without texture fetches (VAR_NO_TEX: no textured / bump-mapped material)
        case 1024 + 18: launch_bounce_t<FIRST, HAS_BVH, 1024 + 18>(grid, in, out, b); break;
        case 1024 + 22: launch_bounce_t<FIRST, HAS_BVH, 1024 + 22>(grid, in, out, b); break;
        case 1024 + 50: launch_bounce_t<FIRST, HAS_BVH, 1024 + 50>(grid, in, out, b); break;
        case 1024 + 54: launch_bounce_t<FIRST, HAS_BVH, 1024 + 54>(grid, in, out, b); break;
        case 1024 + 154: launch_bounce_t<FIRST, HAS_BVH, 1024 + 154>(grid, in, out, b); break;
        case 1024 + 158: launch_bounce_t<FIRST, HAS_BVH, 1024 + 158>(grid, in, out, b); break;
        case 1024 + 186: launch_bounce_t<FIRST, HAS_BVH, 1024 + 186>(grid, in, out, b); break;
        case 1024 + 190: launch_bounce_t<FIRST, HAS_BVH, 1024 + 190>(grid, in, out, b); break;
#ifndef PT_VAR_PROBE
        case 1024 + 530: launch_bounce_t<FIRST, HAS_BVH, 1024 + 530>(grid, in, out, b); break;
        case 1024 + 562: launch_bounce_t<FIRST, HAS_BVH, 1024 + 562>(grid, in, out, b); break;
        case 1024 + 666: launch_bounce_t<FIRST, HAS_BVH, 1024 + 666>(grid, in, out, b); break;
        case 1024 + 698: launch_bounce_t<FIRST, HAS_BVH, 1024 + 698>(grid, in, out, b); break;
#endif
        default: launch_bounce_t<FIRST, HAS_BVH, 3>(grid, in, out, b); break;   // unreachable: pt_init checks
    }
}
bool variant_compiled(int v);
// the fused kernel's template variant for a bounce: the requested bits minus what this bounce /
// scene does not use
int effective_variant(bool first, int var) {
    var &= ~(VAR_BVH_NODES | VAR_NO_TEX);   // host-only bits (layout choice; texture-free build: below)
    // camera rays of neighbouring pixels share their candidates: redistribution only costs there
    // (A/B: bounce 0 0.164 -> 0.174 ms, bounces 1-7 ~6 % faster)
    if (first) var &= ~(VAR_WAVE_REDIST | VAR_BLOCK_REDIST);
    // tools: PT_SECTIONS_SKIP_CAMERA=1 leaves the camera bounce out of the section counters
    if (first && gp->tune.sections_skip_camera) var &= ~VAR_SECTION_TIMING;
    if (!gp->split) var &= ~VAR_BVH_SPLIT;
    // the texture-free build exists for the default variants (and their section-counter and
    // material-grouping forms); other variants keep the texture code
    if (gp->no_tex && variant_compiled(var | VAR_NO_TEX)) var |= VAR_NO_TEX;
    return var;
}
// variants instantiated in launch_bounce_v (pt_init refuses others instead of running a
// different kernel than asked for)
bool variant_compiled(int v) {
    static const int k[] = {0, 1, 2, 6, 10, 18, 22, 26, 30, 50, 54, 58, 154, 158, 186, 190, 530, 562, 666, 698};
    static const int kt[] = {18, 22, 50, 54, 154, 158, 186, 190, 530, 562, 666, 698};   // also with VAR_NO_TEX
    const int* b = (v & VAR_NO_TEX) ? kt : k;
    const int n = (v & VAR_NO_TEX) ? (int)(sizeof kt / sizeof kt[0]) : (int)(sizeof k / sizeof k[0]);
    for (int i = 0; i < n; ++i)
        if (b[i] == (v & ~VAR_NO_TEX)) return true;
    return false;
}
void launch_bounce(bool first, bool bvh, int var, dim3 grid, PathBuf in, PathBuf out, int b) {
    var = effective_variant(first, var);
    if (first) {
        if (bvh) launch_bounce_v<true, true>(var, grid, in, out, b);
        else launch_bounce_v<true, false>(var, grid, in, out, b);
    } else {
        if (bvh) launch_bounce_v<false, true>(var, grid, in, out, b);
        else launch_bounce_v<false, false>(var, grid, in, out, b);
    }
}

// stable compaction of the n_in paths of `pi` into `po` (three launches, see k_compact_*)
template <int CITEMS>
void launch_compact(PathBuf pi, PathBuf po, const int* n_in, int* n_out, int npaths) {
    constexpr int CTILE = BLOCK * CITEMS;
    const int ntiles = (npaths + CTILE - 1) / CTILE;
    launch(5, k_compact_count<CITEMS>, dim3(ntiles), dim3(BLOCK), 0, (const int*)gp->d_alive, n_in, gp->d_tile_cnt);
    launch(5, k_compact_scan, dim3(1), dim3(SCAN_THREADS), 0, (const int*)gp->d_tile_cnt, n_in, gp->d_tile_off, n_out,
           CTILE);
    launch(3, k_compact_scatter<CITEMS>, dim3(ntiles), dim3(BLOCK), 0, (const float4*)pi.A, (const float4*)pi.B,
           (const float4*)pi.C, po.A, po.B, po.C, (const int*)gp->d_alive, n_in, (const int*)gp->d_tile_off);
}

// Enqueue one pass's kernels (everything after k_frame_begin) on gp->stream: `batch` frames
// traced together as one wavefront of local_pixels x batch paths.
// single-frame passes of primitive-only scenes run bounces tail_from() .. depth-1 as one k_tail
// launch (PT_TAIL=0 turns it off for A/B); 0: no tail launch
int tail_from(int batch) {
    const int depth = gp->sc.trace_depth;
    const bool lds = gp->sc.num_geoms <= LDS_GEOMS;
    if (gp->tune.tail_off || (batch != 1 && !gp->tune.tail_any_batch) || gp->has_bvh || !lds || depth < 3 ||
        (effective_variant(false, gp->opts.variant) & ~VAR_NO_TEX) !=
            (VAR_CAND_QUEUE | VAR_WAVE_REDIST | VAR_BVH_FAST | VAR_BLOCK_REDIST))
        return 0;
    const int from = gp->tune.tail_from;
    return std::min(depth - 1, std::max(1, from > 0 ? from : depth / 2));
}

int enqueue_pass_body(int batch) {
    const int depth = gp->sc.trace_depth;
    const int npaths = gp->local_pixels * batch;
    const int nb = nblocks(npaths);
    const int nbounces = std::max(1, depth);
    if (gp->opts.pipeline == PT_PIPELINE_FUSED) {
        const int t = tail_from(batch);
        for (int b = 0; b < (t ? t : nbounces); ++b) {
            PathBuf in = pathbuf(b & 1), out = pathbuf((b + 1) & 1);
            launch_bounce(b == 0, gp->has_bvh, gp->opts.variant & ~VAR_BVH_NODES, dim3(nb), in, out, b);
            HIPCHK(hipGetLastError());
        }
        if (t) {
            constexpr int V = VAR_CAND_QUEUE | VAR_WAVE_REDIST | VAR_BVH_FAST | VAR_BLOCK_REDIST;
            const size_t lds = geom_table_lds() + sizeof(BlockLds);
            if (gp->no_tex)
                launch(300 + t, k_tail<V | VAR_NO_TEX>, dim3(nb), dim3(BLOCK), lds, gp->sc, pathbuf(t & 1), gp->d_ctl,
                       gp->d_image, t, gp->seg_stride, depth);
            else
                launch(300 + t, k_tail<V>, dim3(nb), dim3(BLOCK), lds, gp->sc, pathbuf(t & 1), gp->d_ctl, gp->d_image, t,
                       gp->seg_stride, depth);
            HIPCHK(hipGetLastError());
        }
        return PT_OK;
    }
    // STAGED (k_combine after the pass is enqueued by enqueue_pass)
    // STAGED
    launch(0, k_camera, dim3(nb), dim3(BLOCK), 0, gp->sc, pathbuf(0), gp->d_ctl);
    HIPCHK(hipGetLastError());
    const int stiles = (npaths + STILE - 1) / STILE;   // material-sort tiles
    int cur = 0;
    for (int b = 0; b < nbounces; ++b) {
        // compaction off: paths never move, every bounce sees all of them (pathtrace.cu:690)
        const int* n_in = gp->opts.stream_compaction ? staged_count(b) : staged_count(0);
        HitBuf hits{gp->d_hit_nt, gp->d_hit_mat, gp->d_hit_uvd0, gp->d_hit_uvd1};
        if (gp->has_bvh && (gp->opts.variant & VAR_BVH_FAST))
            launch(1, k_intersect<true, true>, dim3(nb), dim3(BLOCK), gp->bvh_lds, gp->sc, pathbuf(cur), hits, n_in);
        else if (gp->has_bvh)
            launch(1, k_intersect<true, false>, dim3(nb), dim3(BLOCK), gp->bvh_lds, gp->sc, pathbuf(cur), hits, n_in);
        else
            launch(1, k_intersect<false, false>, dim3(nb), dim3(BLOCK), 0, gp->sc, pathbuf(cur), hits, n_in);
        HIPCHK(hipGetLastError());
        const int* perm = nullptr;
        if (gp->opts.material_sort) {
            const int nk = std::max(1, gp->sc.num_mats);
            launch(4, k_sort_hist, dim3(stiles), dim3(BLOCK), 0, (const int*)gp->d_hit_mat, n_in, nk, gp->d_tile_hist);
            launch(4, k_sort_scan, dim3(1), dim3(SCAN_THREADS), 0, gp->d_tile_hist, n_in, nk);
            launch(4, k_sort_scatter, dim3(stiles), dim3(BLOCK), 0, (const int*)gp->d_hit_mat, n_in, nk, gp->key_bits,
                   (const int*)gp->d_tile_hist, gp->d_perm);
            HIPCHK(hipGetLastError());
            perm = gp->d_perm;
        }
        launch(2, k_shade, dim3(nb), dim3(BLOCK), 0, gp->sc, pathbuf(cur), hits, perm, n_in, (const FrameCtl*)gp->d_ctl,
               0, gp->d_image, gp->opts.stream_compaction ? gp->d_alive : (int*)nullptr);
        HIPCHK(hipGetLastError());
        if (gp->opts.stream_compaction) {
            PathBuf pi = pathbuf(cur), po = pathbuf(cur ^ 1);
            int* n_out = &gp->d_ctl->cnt[b + 1][0][0];
            launch_compact<CITEMS>(pi, po, n_in, n_out, npaths);
            HIPCHK(hipGetLastError());
            cur ^= 1;
        }
    }
    return PT_OK;
}

int enqueue_pass(int set_iter, int batch, int plane = 0) {
    gp->ctl_rows = std::max(gp->ctl_rows, std::min(MAXB + 1, gp->sc.trace_depth + 1));
    launch(-1, k_frame_begin, dim3(1), dim3(256), 0, gp->d_ctl, set_iter, gp->local_pixels, batch, gp->ctl_rows, plane);
    HIPCHK(hipGetLastError());
    RC(enqueue_pass_body(batch));
    if (batch > 1) {
        launch(6, k_combine, dim3(nblocks(gp->local_pixels)), dim3(BLOCK), 0, gp->sc, (const FrameCtl*)gp->d_ctl,
               gp->d_image);
        HIPCHK(hipGetLastError());
    }
    return PT_OK;
}

int build_graph(int batch) {
    HIPCHK(hipStreamBeginCapture(gp->stream, hipStreamCaptureModeThreadLocal));
    int rc = enqueue_pass(0, batch);
    hipGraph_t gr = nullptr;
    hipError_t e = hipStreamEndCapture(gp->stream, &gr);
    if (rc != PT_OK) return rc;
    HIPCHK(e);
    gp->graph[batch] = gr;
    HIPCHK(hipGraphInstantiate(&gp->graph_exec[batch], gr, nullptr, nullptr, 0));
    return PT_OK;
}

// one pass: frames iter .. iter + batch - 1
int run_pass(int iter, int batch) {
    RC(ensure_frames(batch));
    // a single-frame pass (the API's pathtrace(), one call per frame) is launched directly: its six
    // kernels run back to back either way, and a graph launch costs the host ~10 us more before
    // its first kernel starts (tools/api_trace.py; PT_F1_GRAPH=1 keeps the graph, A/B)
    // Shards of a multi-device context replay their single-frame pass as a graph too: there the
    // host walks the shards one after another, and one graph launch per shard costs the host less
    // than six kernel launches (tools/multi_probe.py enqueue_us_per_shard)
    if (gp->opts.use_graph && (batch > 1 || gp->tune.f1_graph || (gp->multi && !gp->tune.multi_f1_direct))) {
        if (!gp->graph_exec[batch]) RC(build_graph(batch));
        // the graph's k_frame_begin advances the device iteration by one: preset iter - 1 (stream-
        // ordered) unless the last pass left it there -- main.cpp's pathtrace(pbo, 0, ++iteration)
        // calls then launch the graph alone
        if (gp->dev_iter != iter - 1) HIPCHK(hipMemsetD32Async((hipDeviceptr_t)&gp->d_ctl->iter, iter - 1, 1, gp->stream));
        HIPCHK(hipGraphLaunch(gp->graph_exec[batch], gp->stream));
    } else {
        RC(enqueue_pass(iter, batch));
    }
    gp->dev_iter = iter;
    gp->last_iter = iter + batch - 1;
    gp->frames_done += batch;
    return PT_OK;
}
int run_frame(int iter) { return run_pass(iter, 1); }

// ---- single-frame speculation -----------------------------------------------------------------
// main.cpp calls pathtrace(pbo, frame, ++iteration) every frame and copies the 7.68 MB image to
// pageable host memory each time (pathtrace.cu:783): on MI355X that copy (~0.15 ms over PCIe) is
// longer than the frame's kernels (~0.12 ms).  So once frame N is traced, frame N + 1 is traced
// at once on a second stream -- into a plane of its own with a FrameCtl of its own, the accumulated
// image untouched -- while frame N's image is copied out.  At its end the frame forms image +
// plane into a sum buffer (k_spec_sum: the same additions as the frame's own gathers); the call for
// iteration N + 1 then copies that sum out while k_adopt_frame makes it the image and takes over
// the frame's counters, bit for bit what tracing it then would have produced.
// Any call that could make it differ (another iteration, a camera or depth change, multi-frame
// passes, the test and profiling entry points) first waits for it and drops it (spec_cancel).
// Only calls that copy the image out start one.  PT_SPECULATE=0 turns it off.  One device
// context, fused pipeline.
// The speculative frame is queued by a launcher thread: the copy into the caller's pageable memory
// holds the calling thread for its whole ~0.14 ms, so the frame must be queued before it -- and
// queueing it on the calling thread (event wait + graph launch, ~20 us of host time) delayed the
// copy by as much.  The caller records spec_ev_in, hands the launcher {stream, graph, events,
// iteration preset} and goes straight on to the copy; everything that later touches the speculative
// stream, its events or its graph waits for the launcher first (spec_worker_idle).
// One launch: {device, stream, events, graph, iteration preset, k_spec_sum's buffers}.  A call of a
// context of several devices posts one per shard together; the launcher queues them in order.
struct SpecTask {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_in = nullptr, ev_done = nullptr;
    hipGraphExec_t exec = nullptr;
    int* iter_ptr = nullptr;
    int preset = -1;                 // < 0: the iteration is already right
    const float* image = nullptr;    // k_spec_sum: image + plane -> sum
    const float* plane = nullptr;
    float* sum = nullptr;
    int nf = 0;
};
// Threading: the launcher thread only ever touches the HIP objects of the tasks handed to it (by
// value) and its own current device (hipSetDevice is per host thread); it never reads the
// runtime's process-global context (gp, M) nor calls RCCL.  The caller waits for it (idle) before
// it touches a posted task's stream, events or graph again.
struct SpecLauncher {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    bool task = false, busy = false, stop = false;
    hipError_t err = hipSuccess;
    SpecTask tasks[PT_MAX_DEVICES];
    int ntasks = 0;

    static hipError_t launch_one(const SpecTask& t) {
        hipError_t e = hipSetDevice(t.device);
        if (e == hipSuccess) e = hipStreamWaitEvent(t.stream, t.ev_in, 0);
        if (e == hipSuccess && t.preset >= 0) e = hipMemsetD32Async((hipDeviceptr_t)t.iter_ptr, t.preset, 1, t.stream);
        if (e == hipSuccess) e = hipGraphLaunch(t.exec, t.stream);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_spec_sum, dim3(nblocks((t.nf + 3) / 4)), dim3(BLOCK), 0, t.stream, t.image, t.plane,
                               t.sum, t.nf);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipEventRecord(t.ev_done, t.stream);
        return e;
    }
    void run() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return task || stop; });
            if (stop) return;
            task = false;
            SpecTask ts[PT_MAX_DEVICES];
            const int n = ntasks;
            for (int i = 0; i < n; ++i) ts[i] = tasks[i];
            lk.unlock();
            hipError_t e = hipSuccess;
            for (int i = 0; i < n && e == hipSuccess; ++i) e = launch_one(ts[i]);
            lk.lock();
            if (e != hipSuccess) err = e;
            busy = false;
            cv.notify_all();
        }
    }
    void post(const SpecTask* t, int n) {
        std::lock_guard<std::mutex> lk(mu);
        if (!th.joinable()) th = std::thread([this] { run(); });
        for (int i = 0; i < n; ++i) tasks[i] = t[i];
        ntasks = n;
        task = busy = true;
        cv.notify_all();
    }
    hipError_t idle() {   // wait until the posted launches are queued; their error, once
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !busy; });
        const hipError_t e = err;
        err = hipSuccess;
        return e;
    }
    void join() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
            cv.notify_all();
        }
        if (th.joinable()) th.join();
        stop = false;
    }
    ~SpecLauncher() { join(); }   // a process that exits without pt_free: an idle thread, stopped
};
SpecLauncher g_spec_launcher;

// ---- several devices: the host copy split over the shards' own links --------------------------
// main.cpp's pathtrace() copies the whole image to pageable host memory every call
// (pathtrace.cu:783).  From one device that copy crosses one PCIe link (~0.14 ms at 800^2, longer
// than the frame).  With several devices each shard copies its own row bands from its own device,
// so the devices' links run side by side.  A copy into pageable memory holds the thread that
// issues it until it is done, so shard k's copy is issued by helper thread k (shard 0's by the
// caller).  The helpers keep INTEGRATION.md's threading rules: a helper gets copied values only
// (its shard's device and band stream, the event the caller recorded after the shard's frame, the
// two image bases and the band geometry), calls nothing but those HIP copies, and the call waits
// for every helper before it returns.
struct BandCopy {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ready = nullptr;
    const char* src = nullptr;     // a full-size image on the shard's device (same layout as dst)
    char* dst = nullptr;           // the caller's host image
    size_t first = 0, pitch = 0, width = 0, height = 0;   // `height` bands of `width` bytes, `pitch` apart
    size_t tail_off = 0, tail_bytes = 0;                 // a shorter last band (0 bytes: none)
    hipError_t run() const {
        hipError_t e = hipSetDevice(device);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, ready, 0);
        if (e == hipSuccess && height > 0)
            e = hipMemcpy2DAsync(dst + first, pitch, src + first, pitch, width, height, hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess && tail_bytes > 0)
            e = hipMemcpyAsync(dst + tail_off, src + tail_off, tail_bytes, hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        return e;
    }
};
struct CopyHelper {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    bool task = false, busy = false, stop = false;
    hipError_t err = hipSuccess;
    BandCopy job;
    void run_loop() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return task || stop; });
            if (stop) return;
            task = false;
            const BandCopy j = job;
            lk.unlock();
            const hipError_t e = j.run();
            lk.lock();
            err = e;
            busy = false;
            cv.notify_all();
        }
    }
    void post(const BandCopy& j) {
        std::lock_guard<std::mutex> lk(mu);
        if (!th.joinable()) th = std::thread([this] { run_loop(); });
        job = j;
        task = busy = true;
        cv.notify_all();
    }
    hipError_t wait() {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !busy; });
        const hipError_t e = err;
        err = hipSuccess;
        return e;
    }
    void join() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
            cv.notify_all();
        }
        if (th.joinable()) th.join();
        stop = false;
    }
    ~CopyHelper() { join(); }
};
CopyHelper g_copy_helpers[PT_MAX_DEVICES];

// the current shard's row bands of `src` (a full-size image on its device: its own pixels are
// final) into the host image, after the work queued so far on `after`
int band_prepare(BandCopy& b, float* host, const float* src, hipStream_t after) {
    if (!gp->band_stream) {
        HIPCHK(hipStreamCreateWithFlags(&gp->band_stream, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&gp->band_ready, hipEventDisableTiming));
    }
    HIPCHK(hipEventRecord(gp->band_ready, after));
    const ShardDev& sd = gp->sc.shard;
    const size_t W = (size_t)gp->width, H = (size_t)gp->height, R = (size_t)std::max(1, sd.rows);
    const size_t N = (size_t)std::max(1, sd.count), k = (size_t)sd.rank, row = 3 * sizeof(float) * W;
    const size_t nb = (H + R - 1) / R;                   // bands of the image; shard k has k, k + N, ..
    size_t mine = k < nb ? (nb - 1 - k) / N + 1 : 0;
    b = BandCopy();
    b.device = gp->device;
    b.stream = gp->band_stream;
    b.ready = gp->band_ready;
    b.src = reinterpret_cast<const char*>(src);
    b.dst = reinterpret_cast<char*>(host);
    b.width = R * row;
    b.pitch = N * R * row;
    b.first = k * R * row;
    if (mine > 0 && (nb - 1) % N == k && H % R != 0) {   // the image's last band is shorter and ours
        --mine;
        b.tail_off = (nb - 1) * R * row;
        b.tail_bytes = (H - (nb - 1) * R) * row;
    }
    b.height = mine;
    return PT_OK;
}
int spec_worker_idle() {
    HIPCHK(g_spec_launcher.idle());
    return PT_OK;
}

// the calling context (g_primary): one device context, or the shards of a multi-device one (each
// speculates its own pixels); not a pixel shard of a one-process-per-GPU job (its caller combines)
bool spec_enabled() {
    return g_primary.tune.speculate && gp == &g_primary && gp->opts.pipeline == PT_PIPELINE_FUSED &&
           (gp->multi || gp->sc.shard.mode != PT_SHARD_PIXELS);
}
int spec_cancel() {
    if (gp->spec_iter == 0) return PT_OK;
    // the stream is drained even when the launcher reports an error: the launch may have failed
    // after the graph was queued (k_spec_sum, the event), and the graph uses the pass buffers the
    // caller's next work on gp->stream overwrites.  spec_iter is cleared once it is drained.
    const hipError_t le = g_spec_launcher.idle();
    const hipError_t se = hipStreamSynchronize(gp->spec_stream);
    gp->spec_iter = 0;
    HIPCHK(le);
    HIPCHK(se);
    return PT_OK;
}
void spec_release() {
    (void)g_spec_launcher.idle();
    if (gp == &g_primary) g_spec_launcher.join();
    if (gp->spec_stream) (void)hipStreamSynchronize(gp->spec_stream);
    // the speculated frame's graph goes with its stream (release_graph would otherwise sync a
    // stream that no longer exists before destroying it)
    if (gp->spec_exec) (void)hipGraphExecDestroy(gp->spec_exec);
    if (gp->spec_graph) (void)hipGraphDestroy(gp->spec_graph);
    gp->spec_exec = nullptr;
    gp->spec_graph = nullptr;
    if (gp->spec_ev_in) (void)hipEventDestroy(gp->spec_ev_in);
    if (gp->spec_ev_done) (void)hipEventDestroy(gp->spec_ev_done);
    if (gp->spec_stream) (void)hipStreamDestroy(gp->spec_stream);
    if (gp->d_ctl_spec) (void)hipFree(gp->d_ctl_spec);
    if (gp->d_spec_plane) (void)hipFree(gp->d_spec_plane);
    for (float*& p : gp->d_spec_sum)
        if (p) (void)hipFree(p), p = nullptr;
    if (gp->copy_stream) (void)hipStreamSynchronize(gp->copy_stream), (void)hipStreamDestroy(gp->copy_stream);
    gp->copy_stream = nullptr;
    gp->spec_stream = nullptr;
    gp->spec_ev_in = gp->spec_ev_done = nullptr;
    gp->d_ctl_spec = nullptr;
    gp->d_spec_plane = nullptr;
    gp->spec_iter = 0;
    gp->spec_dev_iter = 0;
}
// frame `iter` of the current context on its speculation stream, behind everything queued on
// gp->stream so far: the launch is described in `t` (posted by the caller, with the other shards')
int spec_prepare(int iter, SpecTask& t) {
    if (!gp->spec_stream) {
        HIPCHK(hipStreamCreateWithFlags(&gp->spec_stream, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&gp->spec_ev_in, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&gp->spec_ev_done, hipEventDisableTiming));
        HIPCHK(hipMalloc((void**)&gp->d_ctl_spec, sizeof(FrameCtl)));
        HIPCHK(hipMemsetAsync(gp->d_ctl_spec, 0, sizeof(FrameCtl), gp->spec_stream));
        HIPCHK(hipMalloc((void**)&gp->d_spec_plane, sizeof(float) * 3 * (size_t)gp->pixels_total));
        for (float*& p : gp->d_spec_sum) HIPCHK(hipMalloc((void**)&p, sizeof(float) * 3 * (size_t)gp->pixels_total));
        HIPCHK(hipStreamCreateWithFlags(&gp->copy_stream, hipStreamNonBlocking));
    }
    if (!gp->spec_exec) {   // captured once (released with the pass graphs: camera, depth, buffers)
        hipStream_t main_stream = gp->stream;
        FrameCtl* main_ctl = gp->d_ctl;
        float* main_contrib = gp->sc.contrib;
        gp->stream = gp->spec_stream;
        gp->d_ctl = gp->d_ctl_spec;
        gp->sc.contrib = gp->d_spec_plane;
        hipError_t e = hipStreamBeginCapture(gp->spec_stream, hipStreamCaptureModeThreadLocal);
        const int rc = e == hipSuccess ? enqueue_pass(0, 1, 1) : PT_OK;   // iteration: the device's + 1
        hipGraph_t gr = nullptr;
        if (e == hipSuccess) e = hipStreamEndCapture(gp->spec_stream, &gr);
        gp->stream = main_stream;
        gp->d_ctl = main_ctl;
        gp->sc.contrib = main_contrib;
        RC(rc);
        HIPCHK(e);
        gp->spec_graph = gr;
        HIPCHK(hipGraphInstantiate(&gp->spec_exec, gr, nullptr, nullptr, 0));
    }
    // behind gp->stream's work so far, as ONE graph launch queued by the launcher thread, so that
    // the image copy the caller queues next starts at once.  The captured k_frame_begin advances the
    // speculative FrameCtl's iteration by one: it is preset only when the last speculative frame was
    // not iter - 1 (consecutive calls launch the graph alone)
    HIPCHK(hipEventRecord(gp->spec_ev_in, gp->stream));
    gp->spec_sum_idx ^= 1;   // the other buffer: the one the caller may still be copying from is kept
    t.device = gp->device;
    t.stream = gp->spec_stream;
    t.ev_in = gp->spec_ev_in;
    t.ev_done = gp->spec_ev_done;
    t.exec = gp->spec_exec;
    t.iter_ptr = &gp->d_ctl_spec->iter;
    t.preset = gp->spec_dev_iter != iter - 1 ? iter - 1 : -1;
    t.image = gp->d_image;
    t.plane = gp->d_spec_plane;
    t.sum = gp->d_spec_sum[gp->spec_sum_idx];
    t.nf = 3 * gp->pixels_total;
    gp->spec_dev_iter = iter;
    gp->spec_iter = iter;
    gp->spec_launched += 1;
    return PT_OK;
}
// the call for the speculative frame's iteration: take it over on gp->stream
// on gp->stream (its image and counters) -- and, when the caller copies the image out, the copy
// stream waits for it too: the copy reads the finished sum at once, beside k_adopt_frame
int spec_adopt(bool copy_out) {
    const int iter = gp->spec_iter;
    hipError_t e = g_spec_launcher.idle();   // spec_ev_done recorded
    if (e == hipSuccess) e = hipStreamWaitEvent(gp->stream, gp->spec_ev_done, 0);
    if (e == hipSuccess && copy_out) e = hipStreamWaitEvent(gp->copy_stream, gp->spec_ev_done, 0);
    if (e != hipSuccess) {   // dropped: a retried call for this iteration traces it afresh
        (void)hipStreamSynchronize(gp->spec_stream);
        gp->spec_iter = 0;
        HIPCHK(e);
    }
    const int nf = 3 * gp->pixels_total;
    launch(7, k_adopt_frame, dim3(nblocks((nf + 3) / 4)), dim3(BLOCK), 0, (const float*)gp->d_spec_sum[gp->spec_sum_idx],
           gp->d_image, nf, gp->d_ctl, (const FrameCtl*)gp->d_ctl_spec, gp->ctl_rows);
    HIPCHK(hipGetLastError());
    gp->spec_iter = 0;
    gp->dev_iter = iter;
    gp->last_iter = iter;
    gp->frames_done += 1;
    gp->spec_adopted += 1;
    return PT_OK;
}

// frames of the next pass when `remaining` frames are left: the passes of a run are balanced
// (100 frames at F = 32 -> 4 x 25, not 32 + 32 + 32 + 4: a small last pass runs its launches
// with a fraction of the paths in flight at nearly full per-launch cost)
int pass_frames(int remaining) {
    const int passes = (remaining + gp->batch - 1) / gp->batch;
    return (remaining + passes - 1) / passes;
}

// max DFS stack the reference traversal can reach on this tree (no culling)
int bvh_max_stack(const pt_bvh_node* nodes, int n) {
    if (n <= 0) return 0;
    std::vector<int> st;
    st.push_back(0);
    size_t mx = 1;
    std::vector<char> seen(n, 0);
    while (!st.empty()) {
        int i = st.back();
        st.pop_back();
        if (i < 0 || i >= n || seen[i]) continue;
        seen[i] = 1;
        const pt_bvh_node& nd = nodes[i];
        if (nd.triCount > 0 && nd.start >= 0) continue;
        if (nd.left >= 0) st.push_back(nd.left);
        if (nd.right >= 0) st.push_back(nd.right);
        mx = std::max(mx, st.size());
    }
    return (int)mx;
}

// levels of the tree below node 0 (root = 1); -1 for a malformed tree (a child out of range or
// reached twice).  The near-first traversals (VAR_BVH_FAST) push at most one entry per level.
int bvh_height(const pt_bvh_node* nodes, int n) {
    if (n <= 0) return 0;
    std::vector<std::pair<int, int>> st{{0, 1}};
    std::vector<char> seen(n, 0);
    int h = 0;
    while (!st.empty()) {
        const int i = st.back().first, d = st.back().second;
        st.pop_back();
        if (i < 0 || i >= n || seen[i]) return -1;
        seen[i] = 1;
        h = std::max(h, d);
        const pt_bvh_node& nd = nodes[i];
        if (nd.triCount > 0 && nd.start >= 0) continue;
        if (nd.left >= 0) st.push_back({nd.left, d + 1});
        if (nd.right >= 0) st.push_back({nd.right, d + 1});
    }
    return h;
}

// The pre-test's candidate table (SceneDev::grid, read by grid_superset): GRID_G^3 origin cells
// over the scene x 6 dominant-axis faces x GRID_B^2 bins of the two other direction ratios
// (d_i / |d_k| in [-1, 1]).  Entry bit g is set when SOME ray with its origin in the cell and its
// direction in the bin can reach geom g's conservative world box at a nonnegative distance --
// interval arithmetic in double along the dominant axis (the distance interval tau) and then on
// the other two axes (origin interval + ratio interval x tau interval), a superset of the real
// condition.  Every exact hit point lies in that box (the pre-test's premise, cull_geom), so a geom
// outside the entry cannot be hit.  The cells are grown by far more than the device's float
// cell computation can be off, the bins likewise for its rcp-based ratio, the boxes by 1e-6 of
// the scene.  The two ratio axes are bounded independently, so an entry is the AND of one mask
// per bin of each: with PT_GRID_SEP the table holds those 2 GRID_B masks per (cell, face) and the
// device ANDs them (the same entries in 2 / GRID_B of the words).  Returns false (no table) for
// scenes whose geom boxes are not finite.
bool build_candidate_table(const std::vector<DevCull>& culls, int ng, const pt_vec3& cam,
                           std::vector<unsigned long long>& table, float lo_out[3], float inv_out[3]) {
    double lo[3] = {cam.x, cam.y, cam.z}, hi[3] = {cam.x, cam.y, cam.z};
    for (int g = 0; g < ng; ++g)
        for (int a = 0; a < 3; ++a) {
            if (!(std::fabs(culls[g].lo[a]) < 1e17f && std::fabs(culls[g].hi[a]) < 1e17f)) return false;
            lo[a] = std::min(lo[a], (double)culls[g].lo[a]);
            hi[a] = std::max(hi[a], (double)culls[g].hi[a]);
        }
    double ext = 1.0;
    for (int a = 0; a < 3; ++a) ext = std::max({ext, std::fabs(lo[a]), std::fabs(hi[a])});
    double cs[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] -= 1e-3 * ext;
        hi[a] += 1e-3 * ext;
        lo_out[a] = (float)lo[a];
        lo[a] = lo_out[a];                                  // the device's origin of the cells
        inv_out[a] = (float)(GRID_G / (hi[a] - lo[a]));
        cs[a] = 1.0 / (double)inv_out[a];                   // the device's cell size
    }
    const double cm = 1e-6 * ext, bin_eps = 1e-5;
    const int G = GRID_G, B = GRID_B;
    table.assign((size_t)G * G * G * 6 * (PT_GRID_SEP ? 2 * B : B * B), 0ull);
    std::vector<double> ta(ng), tb(ng);
    std::vector<unsigned long long> mi(B), mj(B);
    for (int cz = 0; cz < G; ++cz)
        for (int cy = 0; cy < G; ++cy)
            for (int cx = 0; cx < G; ++cx) {
                const int c[3] = {cx, cy, cz};
                double cl[3], ch[3];
                for (int a = 0; a < 3; ++a) {
                    cl[a] = lo[a] + c[a] * cs[a] - (1e-4 * cs[a] + cm);
                    ch[a] = lo[a] + (c[a] + 1) * cs[a] + (1e-4 * cs[a] + cm);
                }
                const int cell = (cz * G + cy) * G + cx;
                for (int face = 0; face < 6; ++face) {
                    const int k = face / 2, i = (k + 1) % 3, j = (k + 2) % 3;
                    const double s = (face & 1) ? 1.0 : -1.0;
                    unsigned long long mk_ = 0;
                    for (int g = 0; g < ng; ++g) {   // distance along axis k to reach the box's k-slab
                        const double bl = culls[g].lo[k] - cm, bh = culls[g].hi[k] + cm;
                        double a0 = s > 0 ? bl - ch[k] : cl[k] - bh, a1 = s > 0 ? bh - cl[k] : ch[k] - bl;
                        a0 = std::max(a0, -cm);
                        ta[g] = a0;
                        tb[g] = a1;
                        if (a1 >= a0) mk_ |= 1ull << g;
                    }
                    for (int axis = 0; axis < 2; ++axis) {
                        const int a = axis == 0 ? i : j;
                        std::vector<unsigned long long>& m = axis == 0 ? mi : mj;
                        for (int b = 0; b < B; ++b) {
                            const double r0 = (b == 0 ? -1.0 : -1.0 + 2.0 * b / B) - bin_eps;
                            const double r1 = (b == B - 1 ? 1.0 : -1.0 + 2.0 * (b + 1) / B) + bin_eps;
                            unsigned long long bits = 0;
                            for (int g = 0; g < ng; ++g) {
                                if (!((mk_ >> g) & 1)) continue;
                                const double p[4] = {r0 * ta[g], r0 * tb[g], r1 * ta[g], r1 * tb[g]};
                                const double pl = std::min({p[0], p[1], p[2], p[3]});
                                const double ph = std::max({p[0], p[1], p[2], p[3]});
                                if (cl[a] + pl <= (double)culls[g].hi[a] + cm && ch[a] + ph >= (double)culls[g].lo[a] - cm)
                                    bits |= 1ull << g;
                            }
                            m[b] = bits;
                        }
                    }
                    if (PT_GRID_SEP) {   // the device ANDs the two bins' masks
                        unsigned long long* row = &table[((size_t)cell * 6 + face) * 2 * B];
                        for (int b = 0; b < B; ++b) {
                            row[b] = mi[b];
                            row[B + b] = mj[b];
                        }
                        continue;
                    }
                    unsigned long long* row = &table[((size_t)cell * 6 + face) * B * B];
                    for (int bu = 0; bu < B; ++bu)
                        for (int bv = 0; bv < B; ++bv) row[bu * B + bv] = mi[bu] & mj[bv];
                }
            }
    return true;
}

// Every inner node's box contains both children's boxes and every leaf's box contains its
// triangles' vertices, with ordered (non-NaN) bounds -- true of every tree scene.cpp:428-441
// builds (each box is the min / max over its own triangles).  The reference then visits a leaf
// iff the leaf's own box passes, which is what a different hierarchy above the
// leaves and the certified t-culls need.  Called after the structural checks (children and
// triIndices in range).
bool bvh_boxes_nested(const pt_scene_view& s) {
    auto inside = [](const pt_vec3& lo, const pt_vec3& hi, const pt_vec3& a, const pt_vec3& b) {
        return lo.x <= a.x && lo.y <= a.y && lo.z <= a.z && b.x <= hi.x && b.y <= hi.y && b.z <= hi.z;
    };
    for (int i = 0; i < s.num_bvh_nodes; ++i) {
        const pt_bvh_node& nd = s.bvh_nodes[i];
        if (nd.triCount > 0 && nd.start >= 0) {
            for (int k = 0; k < nd.triCount; ++k) {
                const int64_t j = (int64_t)nd.start + k;
                if (j >= s.num_tri_indices) return false;
                const int ti = s.tri_indices[j];
                if (ti < 0 || ti >= s.num_triangles) return false;
                const pt_triangle& t = s.triangles[ti];
                for (const pt_vertex* v : {&t.v1, &t.v2, &t.v3})
                    if (!inside(nd.aabb.min, nd.aabb.max, v->position, v->position)) return false;
            }
            continue;
        }
        for (int c : {nd.left, nd.right}) {
            if (c < 0) continue;
            if (c >= s.num_bvh_nodes) return false;
            const pt_bvh_node& ch = s.bvh_nodes[c];
            if (!inside(nd.aabb.min, nd.aabb.max, ch.aabb.min, ch.aabb.max)) return false;
        }
    }
    return true;
}

template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

// staged-pipeline buffers (hits, alive flags, permutation, tile counts): the staged pipeline and
// the pt_test_* entry points use them; the fused pipeline never does
void free_staged_buffers() {
    dfree(gp->d_hit_nt);
    dfree(gp->d_hit_mat);
    dfree(gp->d_hit_uvd0);
    dfree(gp->d_hit_uvd1);
    dfree(gp->d_alive);
    dfree(gp->d_perm);
    dfree(gp->d_tile_hist);
    dfree(gp->d_tile_cnt);
    dfree(gp->d_tile_off);
    gp->staged_alloc = false;
}
void free_pass_buffers() {
    free_staged_buffers();
    for (int i = 0; i < 2; ++i)
        for (int k = 0; k < 3; ++k) dfree(gp->d_path[i][k]);
    dfree(gp->queue.A);
    dfree(gp->queue.B);
    dfree(gp->queue.C);
    dfree(gp->queue.D);
    dfree(gp->tail.node);
    dfree(gp->tail.hit);
    dfree(gp->tail.stack);
    gp->tail.stride = gp->tail.cap = 0;
    dfree(gp->sc.spill);
    dfree(gp->d_contrib);
    gp->sc.contrib = nullptr;
    gp->alloc_frames = 0;
    gp->seg_stride = 0;
    gp->capacity = 0;
}

// output segment s receives the survivors of the chunks c = s (mod NSEG): of k_bounce's, and in
// split mode also of k_bvh_bounce's (its chunks of the queue) -- twice the room then
int seg_stride_for(int frames) {
    const int nb = nblocks(std::max(1, gp->local_pixels * frames));
    return ((nb + NSEG - 1) / NSEG) * BLOCK * (gp->split ? 2 : 1);
}
// entries per traversal-queue segment: the rays of its k_bounce blocks (blockIdx % NSEG)
int q_stride_for(int frames) {
    const int nb = nblocks(std::max(1, gp->local_pixels * frames));
    return ((nb + NSEG - 1) / NSEG) * BLOCK;
}
// k_bvh_bounce hands a wave's traversals to k_bvh_tail_trav once no more than this many of its lanes
// are still traversing (PT_BVH_TAIL_LANES, 0: never; at most 56).  By default 32, and 48 for trees
// of 65,536 refs or more (stack entries with refs wider than 16 bits): deeper traversals diverge
// more, so handing over earlier pays (A/B on the 4-wide records, profiles/r06_ab_tail_lanes_four_wide.json:
// bunny / khaslana best at 32, the 262k stand-in at 48, 3.5 % below 32)
int bvh_tail_lanes() {
    if (gp->tune.bvh_tail_lanes >= 0) return gp->tune.bvh_tail_lanes;
    return 32 - gp->sc.ref_shift > 16 ? 48 : 32;
}
// entries per tail segment: what k_bvh_bounce can hand over, `lanes` per wave of its blocks of one
// segment.  Tools: PT_BVH_TAIL_CHUNKS=c caps it at c blocks' worth; a lane that finds its segment
// full then finishes its ray itself (tail_put).  A cap measured slower at every size tried:
// bunny's passes hand over ~20 % of 128 frames' queued rays (DESIGN Appendix A).
int tail_stride(int frames, int lanes) {
    const int chunks = gp->tune.bvh_tail_chunks;
    const int nb = nblocks(std::max(1, gp->local_pixels * frames));
    const int s = ((nb + NSEG - 1) / NSEG) * (BLOCK / 64) * lanes;
    return chunks > 0 ? std::min(s, chunks * BLOCK) : s;
}
// paths a pass of `frames` frames needs room for, tile-padded (kernels may read a whole tile)
int capacity_for(int frames) {
    const int c = std::max(seg_stride_for(frames) * NSEG, gp->local_pixels * frames);
    return ((c + STILE - 1) / STILE) * STILE;
}
// device bytes of the per-pass buffers for `frames` frames (auto F is capped by free memory)
size_t pass_bytes(int frames, bool staged) {
    const size_t cap = (size_t)capacity_for(frames);
    size_t b = 2 * 3 * sizeof(float4) * cap;                                     // path ping-pong
    if (gp->split) b += (4 * sizeof(float4) + sizeof(int) * gp->sc.spill_stride) * (size_t)q_stride_for(frames) * NSEG;   // traversal queue (+ stack spill rows)
    if (gp->split && bvh_tail_lanes() > 0)   // handed-over traversals
        b += (sizeof(int2) + sizeof(float4) + sizeof(int) * std::max(1, gp->sc.stack_lds)) * NSEG *
             (size_t)tail_stride(frames, bvh_tail_lanes());
    if (frames > 1) b += 3 * sizeof(float) * (size_t)gp->pixels_total * frames;      // contribution planes
    if (staged) b += cap * (sizeof(float4) + 3 * sizeof(int) + (gp->num_tex ? 2 * sizeof(float4) : 0));
    return b;
}

// Path buffers, traversal queue and contribution planes for passes of up to `frames` frames.
// Grows only; captured pass graphs hold the old pointers, so they are released on growth.
int ensure_frames(int frames) {
    frames = std::max(1, frames);
    if (frames <= gp->alloc_frames) return PT_OK;
    const bool staged = gp->staged_alloc || gp->opts.pipeline == PT_PIPELINE_STAGED;
    // a captured pass may still be running (pt_trace_frames does not wait): drain the stream
    // before its graph and the buffers it reads go away
    HIPCHK(hipStreamSynchronize(gp->stream));
    release_graph();
    free_pass_buffers();
    gp->seg_stride = seg_stride_for(frames);
    gp->capacity = capacity_for(frames);
    for (int i = 0; i < 2; ++i)
        for (int k = 0; k < 3; ++k) RC(dalloc(&gp->d_path[i][k], (size_t)gp->capacity));
    if (gp->split) {   // NSEG queue segments, each room for the queued rays of its k_bounce blocks
        gp->queue.stride = q_stride_for(frames);
        const size_t qn = (size_t)gp->queue.stride * NSEG;
        RC(dalloc(&gp->queue.A, qn));
        RC(dalloc(&gp->queue.B, qn));
        RC(dalloc(&gp->queue.C, qn));
        RC(dalloc(&gp->queue.D, qn));
        gp->tail_lanes = bvh_tail_lanes();
        gp->tail_refill = gp->tune.tail_refill;
        gp->tail_trav_blocks = gp->tune.tail_trav_blocks;
        gp->tail_shade_blocks = gp->tune.tail_shade_blocks;
        // stack entries past the LDS part: one row per queue slot (rare: deep stacks only)
        if (gp->sc.spill_stride > 0) RC(dalloc(&gp->sc.spill, qn * (size_t)gp->sc.spill_stride));
        if (gp->tail_lanes > 0) {   // a wave hands over at most tail_lanes rays
            gp->tail_depth = std::max(1, gp->sc.stack_lds);
            TailBuf& t = gp->tail;
            t.stride = tail_stride(frames, gp->tail_lanes);
            t.cap = t.stride * NSEG;
            t.depth = gp->tail_depth;
            RC(dalloc(&t.node, (size_t)t.cap));
            RC(dalloc(&t.hit, (size_t)t.cap));
            RC(dalloc(&t.stack, (size_t)t.cap * gp->tail_depth));
        }
    }
    if (frames > 1) RC(dalloc(&gp->d_contrib, (size_t)gp->pixels_total * 3 * frames));
    gp->sc.contrib = gp->d_contrib;
    gp->alloc_frames = frames;
    if (staged) {
        RC(dalloc(&gp->d_hit_nt, (size_t)gp->capacity));
        RC(dalloc(&gp->d_hit_mat, (size_t)gp->capacity));
        if (gp->num_tex) {
            RC(dalloc(&gp->d_hit_uvd0, (size_t)gp->capacity));
            RC(dalloc(&gp->d_hit_uvd1, (size_t)gp->capacity));
        }
        RC(dalloc(&gp->d_alive, (size_t)gp->capacity));
        RC(dalloc(&gp->d_perm, (size_t)gp->capacity));
        const int ntiles = (gp->capacity + CTILE_MIN - 1) / CTILE_MIN + 1;
        RC(dalloc(&gp->d_tile_hist, (size_t)ntiles * std::max(1, gp->sc.num_mats)));
        RC(dalloc(&gp->d_tile_cnt, (size_t)ntiles));
        RC(dalloc(&gp->d_tile_off, (size_t)ntiles));
        gp->staged_alloc = true;
    }
    return PT_OK;
}
// the staged buffers at the current capacity (the pt_test_* entry points under the fused pipeline)
int ensure_staged() {
    if (gp->staged_alloc) return PT_OK;
    const int f = std::max(1, gp->alloc_frames);
    gp->alloc_frames = 0;              // re-size everything with the staged buffers included
    gp->staged_alloc = true;
    return ensure_frames(f);
}
// a pt_test_* call on n paths: room for n (up to what a pass of gp->batch frames holds) + staged buffers
int ensure_test_paths(int64_t n) {
    const int64_t most = capacity_for(gp->batch);
    if (n < 0 || n > most) return fail(PT_E_INVALID, "n out of range (capacity %lld)", (long long)most);
    RC(ensure_staged());
    const int frames = (int)std::min<int64_t>(gp->batch, std::max<int64_t>(1, (n + gp->local_pixels - 1) / gp->local_pixels));
    RC(ensure_frames(frames));
    if (n > gp->capacity) return fail(PT_E_INVALID, "n out of range (capacity %d)", gp->capacity);
    return PT_OK;
}

void free_all() {
    spec_release();
    if (gp->band_stream) (void)hipStreamSynchronize(gp->band_stream), (void)hipStreamDestroy(gp->band_stream);
    if (gp->band_ready) (void)hipEventDestroy(gp->band_ready);
    gp->band_stream = nullptr;
    gp->band_ready = nullptr;
    release_graph();
    free_pass_buffers();
    void* ptrs[] = {gp->d_geoms, gp->d_cull, gp->d_mats, gp->d_nodes, gp->d_node_aux, gp->d_hot, gp->d_pairs, gp->d_quads, gp->d_hot4,
                    gp->d_leaf9, gp->d_cold, gp->d_texels, gp->d_texinfo, gp->d_image, gp->d_ctl, gp->d_grid};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (gp->stream) (void)hipStreamDestroy(gp->stream);
    if (gp->h_cnt) (void)hipHostFree(gp->h_cnt);
    int32_t* td = gp->traced_depth;
    *gp = State();
    gp->traced_depth = td;
}

template <class T>
int upload(T* d, const T* h, size_t n) {
    if (n) HIPCHK(smemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice));
    return PT_OK;
}

CamDev to_camdev(const pt_camera& c) {
    CamDev d;
    d.resx = c.resolution.x;
    d.resy = c.resolution.y;
    d.position = f3{c.position.x, c.position.y, c.position.z};
    d.view = f3{c.view.x, c.view.y, c.view.z};
    d.up = f3{c.up.x, c.up.y, c.up.z};
    d.right = f3{c.right.x, c.right.y, c.right.z};
    d.plx = c.pixelLength.x;
    d.ply = c.pixelLength.y;
    d.aperture = c.aperture;
    d.focalDist = c.focalDist;
    return d;
}

// AoS (reference layout) <-> SoA wavefront
void paths_to_soa(const pt_path_segment* p, int64_t n, std::vector<float4>& A, std::vector<float4>& B,
                  std::vector<float4>& C) {
    A.resize(n);
    B.resize(n);
    C.resize(n);
    for (int64_t i = 0; i < n; ++i) {
        int32_t pix = p[i].pixelIndex, rb = p[i].remainingBounces;
        float fp, fr;
        memcpy(&fp, &pix, 4);
        memcpy(&fr, &rb, 4);
        A[i] = make_float4(p[i].ray.origin.x, p[i].ray.origin.y, p[i].ray.origin.z, fp);
        B[i] = make_float4(p[i].ray.direction.x, p[i].ray.direction.y, p[i].ray.direction.z, fr);
        C[i] = make_float4(p[i].color.x, p[i].color.y, p[i].color.z, 0.f);
    }
}
void soa_to_paths(const std::vector<float4>& A, const std::vector<float4>& B, const std::vector<float4>& C,
                  int64_t n, pt_path_segment* p) {
    for (int64_t i = 0; i < n; ++i) {
        p[i].ray.origin = pt_vec3{A[i].x, A[i].y, A[i].z};
        p[i].ray.direction = pt_vec3{B[i].x, B[i].y, B[i].z};
        p[i].color = pt_vec3{C[i].x, C[i].y, C[i].z};
        memcpy(&p[i].pixelIndex, &A[i].w, 4);
        memcpy(&p[i].remainingBounces, &B[i].w, 4);
    }
}

int upload_paths(int buf, const pt_path_segment* paths, int64_t n) {
    std::vector<float4> A, B, C;
    paths_to_soa(paths, n, A, B, C);
    HIPCHK(smemcpy(gp->d_path[buf][0], A.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    HIPCHK(smemcpy(gp->d_path[buf][1], B.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    HIPCHK(smemcpy(gp->d_path[buf][2], C.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    return PT_OK;
}
int download_paths(int buf, int64_t n, pt_path_segment* out) {
    std::vector<float4> A(n), B(n), C(n);
    HIPCHK(smemcpy(A.data(), gp->d_path[buf][0], n * sizeof(float4), hipMemcpyDeviceToHost));
    HIPCHK(smemcpy(B.data(), gp->d_path[buf][1], n * sizeof(float4), hipMemcpyDeviceToHost));
    HIPCHK(smemcpy(C.data(), gp->d_path[buf][2], n * sizeof(float4), hipMemcpyDeviceToHost));
    soa_to_paths(A, B, C, n, out);
    return PT_OK;
}
int set_count(int slot, int value) {
    HIPCHK(smemcpy(&gp->d_ctl->cnt[slot][0][0], &value, sizeof(int), hipMemcpyHostToDevice));
    return PT_OK;
}

int need_init() { return gp->inited ? PT_OK : fail(PT_E_STATE, "pt_init has not been called"); }

// ---------------------------------------------------------------------------------------------
// Several GPUs behind one pathtrace() (pt_options.num_devices > 1; SURVEY §8b: the split is
// internal to the boundary).  Shard k is a whole context of its own (State: device, stream,
// scene copy, pass buffers, full-size image of which it writes only its pixels) tracing the
// interleaved row bands (y / rows) % N == k; pixels are independent (the RNG is keyed by pixel,
// iteration and depth), so the shards need no exchange while tracing.  After every call the
// first device's image receives every shard's pixels: a pull kernel over xGMI peer access (or a
// packed tile + hipMemcpyPeerAsync without it), or one RCCL group of send / recv.
// ---------------------------------------------------------------------------------------------
struct Rccl {   // librccl.so, opened at the first pt_init that asks for it (the library is ~570 MB)
    void* h = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
};
Rccl g_rccl;

int rccl_open() {
    if (g_rccl.h) return PT_OK;
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return fail(PT_E_UNSUPPORTED, "PT_COMBINE_RCCL: cannot load librccl.so: %s", dlerror());
    Rccl r;
    r.h = h;
#define PT_RCCL_SYM(f)                                                             \
    r.f = reinterpret_cast<decltype(r.f)>(dlsym(h, "nccl" #f));                    \
    if (!r.f) {                                                                    \
        dlclose(h);                                                                \
        return fail(PT_E_UNSUPPORTED, "PT_COMBINE_RCCL: librccl.so lacks nccl" #f); \
    }
    PT_RCCL_SYM(CommInitAll)
    PT_RCCL_SYM(CommDestroy)
    PT_RCCL_SYM(GroupStart)
    PT_RCCL_SYM(GroupEnd)
    PT_RCCL_SYM(Send)
    PT_RCCL_SYM(Recv)
    PT_RCCL_SYM(GetErrorString)
#undef PT_RCCL_SYM
    g_rccl = r;
    return PT_OK;
}
#define NCCLCHK(expr)                                                                                   \
    do {                                                                                                \
        ncclResult_t r_ = (expr);                                                                       \
        if (r_ != ncclSuccess)                                                                          \
            return fail(PT_E_HIP, "%s:%d: %s: %s", __FILE__, __LINE__, #expr, g_rccl.GetErrorString(r_)); \
    } while (0)

struct Multi {
    int n = 0;                                     // shard contexts (0: single-context mode)
    State* shard[PT_MAX_DEVICES] = {};             // shard[0] == &g_primary
    int combine = PT_COMBINE_PEER;
    hipEvent_t done[PT_MAX_DEVICES] = {};          // shard k's queued work (its stream, its device)
    hipEvent_t pulled = nullptr;                   // the first device finished reading the shards
    bool direct[PT_MAX_DEVICES] = {};              // PEER: the first device reads shard k's image itself
    float* tile[PT_MAX_DEVICES] = {};              // shard k's packed pixels on its device (RCCL, staged peer)
    float* recv[PT_MAX_DEVICES] = {};              // the same on the first device
    // RCCL: one communicator rank per distinct device, each with its own stream
    int ndist = 0;
    int dist_dev[PT_MAX_DEVICES] = {};
    int dist_of[PT_MAX_DEVICES] = {};              // shard k -> index of its device in dist_dev
    ncclComm_t comm[PT_MAX_DEVICES] = {};
    hipStream_t cstream[PT_MAX_DEVICES] = {};
    hipEvent_t cdone[PT_MAX_DEVICES] = {};
    bool band_copy = false;                        // the host copy split over the shards (pt_trace)
};
Multi M;

int nshards() { return M.n > 1 ? M.n : 1; }
State* shard_ctx(int k) { return M.n > 1 ? M.shard[k] : &g_primary; }

// the host runtime works on one shard (its context and its device) until the scope ends
struct ShardScope {
    State* prev;
    int prev_dev = 0;
    explicit ShardScope(State* s) : prev(gp) {
        (void)hipGetDevice(&prev_dev);
        gp = s;
        (void)hipSetDevice(s->device);
    }
    ~ShardScope() {
        gp = prev;
        (void)hipSetDevice(prev_dev);
    }
};

// frame `iter` speculated by every shard of the calling context, as one post to the launcher
int spec_launch(int iter) {
    RC(spec_worker_idle());   // the launcher is done with the previous launches (events, graphs)
    SpecTask ts[PT_MAX_DEVICES];
    for (int k = 0; k < nshards(); ++k) {
        ShardScope sc(shard_ctx(k));
        RC(spec_prepare(iter, ts[k]));
    }
    g_spec_launcher.post(ts, nshards());
    return PT_OK;
}
// every shard's speculated frame waited for and dropped
int spec_cancel_all() {
    for (int k = 0; k < nshards(); ++k) {
        ShardScope sc(shard_ctx(k));
        RC(spec_cancel());
    }
    return PT_OK;
}
int need_single(const char* what) {
    if (M.n > 1) return fail(PT_E_UNSUPPORTED, "%s: one device context only (pt_options.num_devices > 1)", what);
    return spec_cancel();   // the test / profiling entry points use the path buffers themselves
}

void multi_release() {
    if (M.n <= 1) return;
    int entry_dev = 0;
    (void)hipGetDevice(&entry_dev);
    for (int i = 0; i < M.ndist; ++i) {
        (void)hipSetDevice(M.dist_dev[i]);
        if (M.comm[i] && g_rccl.CommDestroy) (void)g_rccl.CommDestroy(M.comm[i]);
        if (M.cdone[i]) (void)hipEventDestroy(M.cdone[i]);
        if (M.cstream[i]) (void)hipStreamDestroy(M.cstream[i]);
    }
    for (int k = 0; k < M.n; ++k) {
        State* s = M.shard[k];
        if (!s) continue;
        (void)hipSetDevice(s->device);
        if (M.done[k]) (void)hipEventDestroy(M.done[k]);
        if (M.tile[k]) (void)hipFree(M.tile[k]);
    }
    (void)hipSetDevice(M.shard[0] ? M.shard[0]->device : 0);
    for (int k = 0; k < M.n; ++k)
        if (M.recv[k]) (void)hipFree(M.recv[k]);
    if (M.pulled) (void)hipEventDestroy(M.pulled);
    (void)hipSetDevice(entry_dev);
}

// events, peer access, tiles and (RCCL) communicators once every shard is initialised
int multi_setup() {
    State* p = M.shard[0];
    ShardScope entry(p);   // restores the caller's device and context last
    for (int k = 0; k < M.n; ++k) {
        ShardScope sc(M.shard[k]);
        HIPCHK(hipEventCreateWithFlags(&M.done[k], hipEventDisableTiming));
    }
    {
        ShardScope sc(p);
        HIPCHK(hipEventCreateWithFlags(&M.pulled, hipEventDisableTiming));
    }
    // tools / tests: PT_COMBINE_FORCE_STAGED=1 sends every PEER shard through its packed tile and a
    // hipMemcpyPeerAsync (the branch taken without peer access), also when the shards share a device
    const bool force_staged = p->tune.combine_force_staged;
    for (int k = 1; k < M.n; ++k) {
        State* s = M.shard[k];
        const size_t bytes = 3 * sizeof(float) * (size_t)std::max(1, s->local_pixels);
        bool direct = M.combine == PT_COMBINE_PEER && s->device == p->device && !force_staged;
        if (M.combine == PT_COMBINE_PEER && !direct && !force_staged) {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, p->device, s->device) == hipSuccess && can) {
                ShardScope sc(p);
                const hipError_t e = hipDeviceEnablePeerAccess(s->device, 0);
                if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) direct = true;
                (void)hipGetLastError();
            }
        }
        M.direct[k] = direct;
        if (!direct) {   // packed tiles: RCCL, or peer copies without peer access
            {
                ShardScope sc(s);
                RC(dalloc(&M.tile[k], bytes / sizeof(float)));
            }
            ShardScope sc(p);
            RC(dalloc(&M.recv[k], bytes / sizeof(float)));
        }
    }
    // the host copy of single-frame calls split over the shards' own links: by default only when
    // every shard has a device of its own (shards sharing a device share its link, and the split
    // then only adds the helper hand-offs: tools/multi_probe.py on one GPU)
    {
        bool distinct = true;
        for (int a = 0; a < M.n; ++a)
            for (int b = a + 1; b < M.n; ++b) distinct = distinct && M.shard[a]->device != M.shard[b]->device;
        M.band_copy = p->tune.band_copy > 0 || (p->tune.band_copy < 0 && distinct);
    }
    if (M.combine != PT_COMBINE_RCCL) return PT_OK;
    RC(rccl_open());
    for (int k = 0; k < M.n; ++k) {
        int i = 0;
        while (i < M.ndist && M.dist_dev[i] != M.shard[k]->device) ++i;
        if (i == M.ndist) M.dist_dev[M.ndist++] = M.shard[k]->device;
        M.dist_of[k] = i;
    }
    NCCLCHK(g_rccl.CommInitAll(M.comm, M.ndist, M.dist_dev));
    for (int i = 0; i < M.ndist; ++i) {
        HIPCHK(hipSetDevice(M.dist_dev[i]));
        HIPCHK(hipStreamCreateWithFlags(&M.cstream[i], hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&M.cdone[i], hipEventDisableTiming));
    }
    HIPCHK(hipSetDevice(p->device));
    return PT_OK;
}

// k_gather_shards' shard layout (sources filled in by the caller)
GatherSrc gather_src(int W, int H) {
    GatherSrc g{};
    g.n = M.n;
    g.rows = std::max(1, M.shard[0]->sc.shard.rows);
    g.W = W;
    g.H = H;
    return g;
}

// every shard's pixels into the first device's image, ordered after the work queued so far on
// every shard's stream; the shards' next work waits until the first device has read them
int multi_combine() {
    if (M.n <= 1) return PT_OK;
    State* p = M.shard[0];
    ShardScope entry(p);   // restores the caller's device and context last
    const int W = p->width;
    for (int k = 1; k < M.n; ++k) {
        State* s = M.shard[k];
        ShardScope sc(s);
        if (!M.direct[k]) {
            hipLaunchKernelGGL(k_pack_tile, dim3(nblocks(s->local_pixels)), dim3(BLOCK), 0, s->stream, s->d_image,
                               s->sc.shard, W, M.tile[k]);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipEventRecord(M.done[k], s->stream));
    }
    if (M.combine == PT_COMBINE_RCCL) {
        const int d0 = M.dist_of[0];
        {   // the first device's receive buffers are free once its earlier unpacks ran
            ShardScope sc(p);
            HIPCHK(hipEventRecord(M.done[0], p->stream));
        }
        for (int k = 0; k < M.n; ++k) {
            HIPCHK(hipSetDevice(M.dist_dev[M.dist_of[k]]));
            HIPCHK(hipStreamWaitEvent(M.cstream[M.dist_of[k]], M.done[k], 0));
        }
        NCCLCHK(g_rccl.GroupStart());
        for (int k = 1; k < M.n; ++k) {
            const size_t cnt = 3 * (size_t)M.shard[k]->local_pixels;
            const int dk = M.dist_of[k];
            NCCLCHK(g_rccl.Send(M.tile[k], cnt, ncclFloat32, d0, M.comm[dk], M.cstream[dk]));
            NCCLCHK(g_rccl.Recv(M.recv[k], cnt, ncclFloat32, dk, M.comm[d0], M.cstream[d0]));
        }
        NCCLCHK(g_rccl.GroupEnd());
        for (int i = 0; i < M.ndist; ++i) {
            HIPCHK(hipSetDevice(M.dist_dev[i]));
            HIPCHK(hipEventRecord(M.cdone[i], M.cstream[i]));
        }
        for (int k = 1; k < M.n; ++k) {   // a tile is rewritten only after its send completed
            ShardScope sc(M.shard[k]);
            HIPCHK(hipStreamWaitEvent(M.shard[k]->stream, M.cdone[M.dist_of[k]], 0));
        }
        ShardScope sc(p);
        HIPCHK(hipStreamWaitEvent(p->stream, M.cdone[d0], 0));
        // every shard's own work too (its TracedDepth counter copy is queued before done[k]):
        // once the first device's stream has drained, so has every shard's frame
        for (int k = 1; k < M.n; ++k) HIPCHK(hipStreamWaitEvent(p->stream, M.done[k], 0));
        GatherSrc g = gather_src(W, p->height);
        for (int k = 1; k < M.n; ++k) {
            g.src[k] = M.recv[k];
            g.local[k] = 1;
        }
        hipLaunchKernelGGL(k_gather_shards, dim3(nblocks(p->pixels_total)), dim3(BLOCK), 0, p->stream, p->d_image, g);
        HIPCHK(hipGetLastError());
        return PT_OK;
    }
    ShardScope sc(p);
    GatherSrc g = gather_src(W, p->height);
    for (int k = 1; k < M.n; ++k) {
        State* s = M.shard[k];
        HIPCHK(hipStreamWaitEvent(p->stream, M.done[k], 0));
        if (M.direct[k]) {   // read in place over peer access
            g.src[k] = s->d_image;
            g.local[k] = 0;
        } else {             // packed tile, copied to the first device
            HIPCHK(hipMemcpyPeerAsync(M.recv[k], p->device, M.tile[k], s->device,
                                      3 * sizeof(float) * (size_t)s->local_pixels, p->stream));
            g.src[k] = M.recv[k];
            g.local[k] = 1;
        }
    }
    hipLaunchKernelGGL(k_gather_shards, dim3(nblocks(p->pixels_total)), dim3(BLOCK), 0, p->stream, p->d_image, g);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(M.pulled, p->stream));
    for (int k = 1; k < M.n; ++k) {   // a shard's image changes again only after it was read
        ShardScope s2(M.shard[k]);
        HIPCHK(hipStreamWaitEvent(M.shard[k]->stream, M.pulled, 0));
    }
    return PT_OK;
}

// GuiDataContainer::TracedDepth of the last single-frame pass of the current context: the loop
// stops after bounce k when no path is left alive, or at traceDepth (pathtrace.cu:759-770).
// Two halves so that no call waits twice: frame_depth_enqueue queues the copy of the frame's live
// counters into page-locked host memory on the context's stream (behind the frame, before the
// caller's one synchronisation), frame_depth_read reads them after it.
int frame_depth_enqueue() {
    if (!gp->opts.stream_compaction) return PT_OK;
    const size_t n = (size_t)std::max(1, gp->sc.trace_depth) * NSEG * CNT_PAD;
    if (!gp->h_cnt) HIPCHK(hipHostMalloc((void**)&gp->h_cnt, sizeof(int) * (size_t)(MAXB + 1) * NSEG * CNT_PAD));
    HIPCHK(hipMemcpyAsync(gp->h_cnt, &gp->d_ctl->cnt[0][0][0], n * sizeof(int), hipMemcpyDeviceToHost, gp->stream));
    return PT_OK;
}
int frame_depth_read() {
    int depth = std::max(1, gp->sc.trace_depth);
    if (!gp->opts.stream_compaction || !gp->h_cnt) return depth;
    for (int k = 1; k < depth; ++k) {
        int64_t live = 0;
        for (int q = 0; q < NSEG; ++q) live += gp->h_cnt[((size_t)k * NSEG + q) * CNT_PAD];
        if (live == 0) return k;
    }
    return depth;
}

}  // namespace

// =============================================================================================
// C-ABI
// =============================================================================================
extern "C" {

int32_t pt_abi_version(void) { return PT_ABI_VERSION; }
const char* pt_last_error(void) { return g_err.c_str(); }

void pt_default_options(pt_options* o) {
    memset(o, 0, sizeof(*o));
    o->stream_compaction = 1;
    o->material_sort = 0;
    o->bvh = 1;
    o->arg_order = 0;
    o->pipeline = PT_PIPELINE_FUSED;
    o->use_graph = 1;
    o->device = 0;
    o->shard_mode = PT_SHARD_NONE;
    o->shard_rank = 0;
    o->shard_count = 1;
    o->shard_rows = 8;
    o->block_size = BLOCK;
    // fastest in the in-process A/B (tools/ab_variants.py); every variant is bit-identical
    o->variant = VAR_CAND_QUEUE | VAR_WAVE_REDIST | VAR_BVH_FAST | VAR_BVH_SPLIT | VAR_BLOCK_REDIST;
    o->frames_per_pass = 0;        // auto
    // several GPUs behind one pathtrace(): the drop-in and pt_render reach it through the environment
    o->num_devices = 0;
    for (int k = 0; k < PT_MAX_DEVICES; ++k) o->device_ids[k] = k;
    if (const char* e = getenv("PT_DEVICES")) {
        if (strchr(e, ',')) {
            int n = 0;
            for (const char* c = e; *c && n < PT_MAX_DEVICES;) {
                char* end = nullptr;
                const long v = strtol(c, &end, 10);
                if (end == c) break;
                o->device_ids[n++] = (int32_t)v;
                c = *end == ',' ? end + 1 : end;
                if (*end != ',') break;
            }
            o->num_devices = n;
        } else {
            o->num_devices = (int32_t)std::min<long>(PT_MAX_DEVICES, std::max<long>(0, strtol(e, nullptr, 10)));
        }
    }
    o->combine = PT_COMBINE_PEER;
    if (const char* e = getenv("PT_COMBINE")) o->combine = strcmp(e, "rccl") == 0 ? PT_COMBINE_RCCL : PT_COMBINE_PEER;
}

int32_t pt_init_data_container(int32_t* traced_depth) {
    gp->traced_depth = traced_depth;
    return PT_OK;
}

int32_t pt_free(void) {
    gp = &g_primary;
    if (M.n > 1) {
        multi_release();
        for (int k = M.n - 1; k >= 1; --k) {
            if (!M.shard[k]) continue;
            {   // whatever a shard allocated, also when its init_one failed part-way (inited false):
                // free_all releases only the buffers and stream that exist
                ShardScope sc(M.shard[k]);
                free_all();
            }
            delete M.shard[k];
        }
    }
    M = Multi();
    for (CopyHelper& h : g_copy_helpers) h.join();
    free_all();   // also resets g_primary's sizes (alloc_frames, capacity, ...) after a failed init
    return PT_OK;
}

// frames per pass when pt_options.frames_per_pass == 0: enough paths in flight to fill the
// chip in the late, mostly-terminated bounces (~84M paths at bounce 0), at most MAXF
int auto_batch(int local_pixels) {
    const int64_t target = gp->tune.auto_paths > 0 ? gp->tune.auto_paths : AUTO_BATCH_PATHS;
    int f = 1;
    while (f * 2 <= MAXF && (int64_t)local_pixels * f * 2 <= target) f *= 2;
    return f;
}

// one context (gp): the whole pathtraceInit for one device, or for shard k of a multi-device
// context; `share` contexts live on this device (auto F divides its free memory among them)
static int32_t init_one(const pt_scene_view* s, pt_options o, int share) {
    if (o.block_size != BLOCK) return fail(PT_E_UNSUPPORTED, "block_size must be %d", BLOCK);
    const int W = s->camera.resolution.x, H = s->camera.resolution.y;
    if (W <= 0 || H <= 0) return fail(PT_E_INVALID, "bad resolution %dx%d", W, H);
    if (s->trace_depth > MAXB) return fail(PT_E_UNSUPPORTED, "trace depth %d > %d", s->trace_depth, MAXB);
    if (s->num_geoms < 0 || s->num_materials < 0 || s->num_triangles < 0 || s->num_bvh_nodes < 0)
        return fail(PT_E_INVALID, "negative counts");
    if (s->num_materials > MAXMAT) return fail(PT_E_UNSUPPORTED, "more than %d materials", MAXMAT);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(PT_E_NODEVICE, "no HIP device visible");
    if (o.device < 0 || o.device >= ndev) return fail(PT_E_INVALID, "device %d out of range", o.device);
    HIPCHK(hipSetDevice(o.device));
    gp->opts = o;
    gp->device = o.device;
    gp->tune = read_tuning();
    HIPCHK(hipStreamCreateWithFlags(&gp->stream, hipStreamNonBlocking));
    gp->width = W;
    gp->height = H;
    gp->pixels_total = W * H;
    // shard
    ShardDev sh{};
    sh.mode = o.shard_mode == PT_SHARD_PIXELS && o.shard_count > 1 ? 1 : 0;
    sh.rank = o.shard_rank;
    sh.count = std::max(1, o.shard_count);
    sh.rows = std::max(1, o.shard_rows);
    if (sh.mode == 1) {
        if (o.shard_rank < 0 || o.shard_rank >= o.shard_count) return fail(PT_E_INVALID, "bad shard rank");
        int rows = 0;
        for (int y = 0; y < H; ++y) rows += ((y / sh.rows) % sh.count) == sh.rank;
        sh.local_pixels = rows * W;
    } else {
        sh.local_pixels = gp->pixels_total;
    }
    gp->local_pixels = sh.local_pixels;
    if (o.frames_per_pass < 0 || o.frames_per_pass > MAXF)
        return fail(PT_E_INVALID, "frames_per_pass must be 0 (auto) .. %d", MAXF);

    // ---- scene -> device records ----
    std::vector<DevGeom> geoms(s->num_geoms);
    for (int i = 0; i < s->num_geoms; ++i) {
        const pt_geom& gg = s->geoms[i];
        DevGeom& d = geoms[i];
        memset(&d, 0, sizeof d);
        for (int c = 0; c < 4; ++c)
            for (int r = 0; r < 3; ++r) {
                d.inv[c * 3 + r] = gg.inverseTransform.m[c][r];
                d.fwd[c * 3 + r] = gg.transform.m[c][r];
                d.itr[c * 3 + r] = gg.invTranspose.m[c][r];
            }
        d.type = gg.type;
        d.materialid = gg.materialid;
        // away_on_axis pre-test: the object axis of smallest world scale (a wall's thin axis,
        // the face a ray leaving it crosses); only when the inverse matrix is bounded so that
        // dot(u, u) < inf is guaranteed for |rd| components <= 1e3
        d.away_axis = -1;
        if (gg.type == PT_CUBE) {
            double big = 0.0;
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < 3; ++r) big = std::max(big, std::fabs((double)gg.inverseTransform.m[c][r]));
            if (big <= 1e12) {
                double best = 1e300;
                for (int a = 0; a < 3; ++a) {
                    const double len = std::sqrt((double)gg.transform.m[a][0] * gg.transform.m[a][0] +
                                                 (double)gg.transform.m[a][1] * gg.transform.m[a][1] +
                                                 (double)gg.transform.m[a][2] * gg.transform.m[a][2]);
                    if (len < best) {
                        best = len;
                        d.away_axis = a;
                    }
                }
            }
        }
    }
    // conservative world boxes for cull_geom: the transformed unit cube (contains the radius-0.5
    // sphere too), grown by a margin far above every rounding the exact test can make (1e-3 of
    // the largest half extent + 1e-3 absolute; object-space pull-back is 1e-4 times the scale)
    // and above the cull's own fma/rcp error for ray origins anywhere in the scene (1e-6 of the
    // scene extent), then rounded outward.
    {
        double extent = std::max({std::fabs((double)s->camera.position.x), std::fabs((double)s->camera.position.y),
                                  std::fabs((double)s->camera.position.z), 1.0});
        std::vector<float> bc(3 * (size_t)s->num_geoms), bh(3 * (size_t)s->num_geoms);
        std::vector<char> fin(s->num_geoms);
        for (int i = 0; i < s->num_geoms; ++i) {
            DevGeom& d = geoms[i];
            float hmax = 0.f;
            for (int r = 0; r < 3; ++r) {
                bc[3 * i + r] = d.fwd[9 + r];
                bh[3 * i + r] = 0.5f * (std::fabs(d.fwd[r]) + std::fabs(d.fwd[3 + r]) + std::fabs(d.fwd[6 + r]));
                hmax = std::max(hmax, bh[3 * i + r]);
            }
            for (int r = 0; r < 3; ++r) bh[3 * i + r] += 1e-3f * hmax + 1e-3f * std::max(1.0f, hmax);
            fin[i] = std::isfinite(hmax) && std::isfinite(bc[3 * i]) && std::isfinite(bc[3 * i + 1]) &&
                     std::isfinite(bc[3 * i + 2]) && hmax < 1e17f;
            if (fin[i])
                for (int r = 0; r < 3; ++r)
                    extent = std::max(extent, std::fabs((double)bc[3 * i + r]) + (double)bh[3 * i + r]);
        }
        for (int t = 0; t < s->num_triangles; ++t) {
            const pt_vertex* v[3] = {&s->triangles[t].v1, &s->triangles[t].v2, &s->triangles[t].v3};
            for (auto* x : v) {
                double m = std::max({std::fabs((double)x->position.x), std::fabs((double)x->position.y),
                                     std::fabs((double)x->position.z)});
                if (std::isfinite(m)) extent = std::max(extent, m);
            }
        }
        const float emargin = (float)std::min(1e-6 * extent, 1e17);
        for (int i = 0; i < s->num_geoms; ++i) {
            DevGeom& d = geoms[i];
            for (int r = 0; r < 3; ++r) {
                if (!fin[i]) {   // degenerate transform: a box that never culls
                    d.box_lo[r] = -1e18f;
                    d.box_hi[r] = 1e18f;
                    continue;
                }
                const float h = bh[3 * i + r] + emargin;
                d.box_lo[r] = std::nextafter(bc[3 * i + r] - h, -INFINITY);
                d.box_hi[r] = std::nextafter(bc[3 * i + r] + h, INFINITY);
            }
        }
    }
    // padded to a multiple of CULL_GROUP records (cull_candidates reads that many at a time; pad
    // bits are masked)
    std::vector<DevCull> culls((std::max(1, s->num_geoms) + CULL_GROUP - 1) / CULL_GROUP * CULL_GROUP);
    for (DevCull& c : culls) memset(&c, 0, sizeof c);
    for (int i = 0; i < s->num_geoms; ++i) {
        const DevGeom& d = geoms[i];
        DevCull& c = culls[i];
        memset(&c, 0, sizeof c);
        for (int r = 0; r < 3; ++r) {
            c.lo[r] = d.box_lo[r];
            c.hi[r] = d.box_hi[r];
        }
        const int a = d.away_axis;
        if (d.type == PT_CUBE && a >= 0 && a < 3) {
            for (int k = 0; k < 4; ++k) c.row[k] = d.inv[3 * k + a];
            c.has_row = 1;
        }
    }
    std::vector<DevMaterial> mats(std::max(1, s->num_materials));
    for (int i = 0; i < s->num_materials; ++i) {
        const pt_material& m = s->materials[i];
        DevMaterial& d = mats[i];
        memset(&d, 0, sizeof d);
        d.color[0] = m.color.x;
        d.color[1] = m.color.y;
        d.color[2] = m.color.z;
        d.emittance = m.emittance;
        d.hasReflective = m.hasReflective;
        d.hasRefractive = m.hasRefractive;
        d.roughness = m.roughness;
        d.metallic = m.metallic;
        d.ior = m.indexOfRefraction;
        d.hasTexture = m.hasTexture ? 1 : 0;
        d.textureID = m.textureID;
        d.hasBumpMap = m.hasBumpMap ? 1 : 0;
        d.bumpID = m.bumpID;
        d.bumpScale = m.bumpScale;
    }
    // no material samples a texture or bump map: the fused kernels' texture-free build (VAR_NO_TEX)
    gp->no_tex = true;
    for (int i = 0; i < s->num_materials; ++i)
        if (s->materials[i].hasTexture || s->materials[i].hasBumpMap) gp->no_tex = false;
    // BVH: only when the reference would traverse it (BVH_ACCELERATION and a non-empty tree)
    gp->has_bvh = o.bvh && s->num_bvh_nodes > 0 && s->num_triangles > 0;
    std::vector<DevNode> nodes;
    std::vector<float4> node_aux;
    std::vector<DevTriHot> hot;
    std::vector<DevTriCold> cold;
    std::vector<DevPair> pairs;      // VAR_BVH_FAST layout (empty: tree not representable)
    std::vector<float4> quads;       // its 4-wide form (8 float4 per record; empty: not built)
    int quad_stack = 0;              // stack entries the 4-wide traversal can need
    std::vector<DevTriHot> hot4;
    std::vector<float4> leaf9;
    int pair_root_ref = 0, pair_count = 0, pair_ref_shift = 16;

    float4 pair_root_lo{}, pair_root_hi{};
    double cull_extent = 1.0;
    if (gp->has_bvh) {
        nodes.resize(s->num_bvh_nodes);
        for (int i = 0; i < s->num_bvh_nodes; ++i) {
            const pt_bvh_node& nd = s->bvh_nodes[i];
            bool leaf = nd.triCount > 0 && nd.start >= 0;
            int a = leaf ? nd.start : nd.left;
            int b = leaf ? -(nd.triCount + 2) : (nd.right >= 0 ? nd.right : -1);
            if (leaf && (int64_t)nd.start + nd.triCount > s->num_tri_indices)
                return fail(PT_E_INVALID, "BVH leaf %d indexes past triIndices", i);
            if (!leaf && (nd.left >= s->num_bvh_nodes || nd.right >= s->num_bvh_nodes))
                return fail(PT_E_INVALID, "BVH node %d child out of range", i);
            float fa, fb;
            memcpy(&fa, &a, 4);
            memcpy(&fb, &b, 4);
            nodes[i].lo = make_float4(nd.aabb.min.x, nd.aabb.min.y, nd.aabb.min.z, fa);
            nodes[i].hi = make_float4(nd.aabb.max.x, nd.aabb.max.y, nd.aabb.max.z, fb);
        }
        // per-node culling bounds and the reference's DFS visit rank (push left, push right, pop)
        node_aux.assign(s->num_bvh_nodes, make_float4(0.f, 0.f, 0.f, 0.f));
        {
            double extent = std::max({1.0, std::fabs((double)s->camera.position.x),
                                      std::fabs((double)s->camera.position.y), std::fabs((double)s->camera.position.z)});
            for (int t = 0; t < s->num_triangles; ++t) {
                const pt_vertex* v[3] = {&s->triangles[t].v1, &s->triangles[t].v2, &s->triangles[t].v3};
                for (auto* x : v)
                    extent = std::max({extent, std::fabs((double)x->position.x), std::fabs((double)x->position.y),
                                       std::fabs((double)x->position.z)});
            }
            for (int i = 0; i < s->num_geoms; ++i)   // hit points on primitives are ray origins too
                for (int r = 0; r < 3; ++r)
                    extent = std::max(extent, std::fabs((double)geoms[i].box_lo[r]) + std::fabs((double)geoms[i].box_hi[r]));
            cull_extent = extent;
            std::vector<double> smax(s->num_bvh_nodes, -1.0);
            // bottom-up max edge: children have larger indices than parents in the reference build,
            // but compute it by explicit post-order to accept any valid tree
            std::vector<int> order, st{0};
            std::vector<char> seen(s->num_bvh_nodes, 0);
            while (!st.empty()) {
                int n = st.back();
                st.pop_back();
                if (n < 0 || n >= s->num_bvh_nodes || seen[n]) continue;
                seen[n] = 1;
                order.push_back(n);
                const pt_bvh_node& nd = s->bvh_nodes[n];
                if (!(nd.triCount > 0 && nd.start >= 0)) {
                    if (nd.left >= 0) st.push_back(nd.left);
                    if (nd.right >= 0) st.push_back(nd.right);
                }
            }
            for (size_t k = order.size(); k-- > 0;) {
                const int n = order[k];
                const pt_bvh_node& nd = s->bvh_nodes[n];
                double m = 0.0;
                if (nd.triCount > 0 && nd.start >= 0) {
                    for (int i = 0; i < nd.triCount; ++i) {
                        const int ti = s->tri_indices[nd.start + i];
                        if (ti < 0 || ti >= s->num_triangles) continue;   // rejected below
                        const pt_triangle& t = s->triangles[ti];
                        const double e1 = std::hypot((double)t.v2.position.x - t.v1.position.x,
                                                     (double)t.v2.position.y - t.v1.position.y,
                                                     (double)t.v2.position.z - t.v1.position.z);
                        const double e2 = std::hypot((double)t.v3.position.x - t.v1.position.x,
                                                     (double)t.v3.position.y - t.v1.position.y,
                                                     (double)t.v3.position.z - t.v1.position.z);
                        m = std::max({m, e1, e2});
                    }
                } else {
                    if (nd.left >= 0) m = std::max(m, smax[nd.left]);
                    if (nd.right >= 0) m = std::max(m, smax[nd.right]);
                }
                smax[n] = m;
                const double sx = m * 1.01 + 1e-30;
                const double c = 64.0 * std::ldexp(1.0, -24) * sx * sx / 1e-5;
                node_aux[n].x = (float)std::min(c * 1.01, 1e30);
                node_aux[n].y = (float)std::min(sx, 1e30);
                node_aux[n].w = (float)std::min(c * extent * 1.01, 1e30);
            }
            // reference visit rank
            int rank = 0;
            st.assign(1, 0);
            std::fill(seen.begin(), seen.end(), 0);
            while (!st.empty()) {
                int n = st.back();
                st.pop_back();
                if (n < 0 || n >= s->num_bvh_nodes) continue;
                int r = rank++;
                float fr;
                memcpy(&fr, &r, 4);
                node_aux[n].z = fr;
                const pt_bvh_node& nd = s->bvh_nodes[n];
                if (!(nd.triCount > 0 && nd.start >= 0) && !seen[n]) {
                    seen[n] = 1;
                    if (nd.left >= 0) st.push_back(nd.left);
                    if (nd.right >= 0) st.push_back(nd.right);
                }
            }
        }
        hot.resize(s->num_tri_indices);
        for (int k = 0; k < s->num_tri_indices; ++k) {
            int ti = s->tri_indices[k];
            if (ti < 0 || ti >= s->num_triangles) return fail(PT_E_INVALID, "triIndices[%d] out of range", k);
            const pt_triangle& t = s->triangles[ti];
            float fti;
            memcpy(&fti, &ti, 4);
            hot[k].a = make_float4(t.v1.position.x, t.v1.position.y, t.v1.position.z, t.v2.position.x);
            hot[k].b = make_float4(t.v2.position.y, t.v2.position.z, t.v3.position.x, t.v3.position.y);
            hot[k].c = make_float4(t.v3.position.z, fti, 0.f, 0.f);
        }
        cold.resize(s->num_triangles);
        for (int i = 0; i < s->num_triangles; ++i) {
            const pt_triangle& t = s->triangles[i];
            DevTriCold& c = cold[i];
            memset(&c, 0, sizeof c);
            const pt_vertex* v[3] = {&t.v1, &t.v2, &t.v3};
            float* ns[3] = {c.n0, c.n1, c.n2};
            float* uvs[3] = {c.uv0, c.uv1, c.uv2};
            for (int k = 0; k < 3; ++k) {
                ns[k][0] = v[k]->normal.x;
                ns[k][1] = v[k]->normal.y;
                ns[k][2] = v[k]->normal.z;
                uvs[k][0] = v[k]->uv.x;
                uvs[k][1] = v[k]->uv.y;
            }
            c.dpdu[0] = t.dpdu.x; c.dpdu[1] = t.dpdu.y; c.dpdu[2] = t.dpdu.z;
            c.dpdv[0] = t.dpdv.x; c.dpdv[1] = t.dpdv.y; c.dpdv[2] = t.dpdv.z;
            c.materialID = t.materialID;
            if (t.materialID < 0 || t.materialID >= std::max(1, s->num_materials))
                return fail(PT_E_INVALID, "triangle %d material %d out of range", i, t.materialID);
        }
        // traversal stack (LDS, MAXSTACK entries per lane at most).  The reference-order DFS needs
        // bvh_max_stack entries -- more than 64 overflows the reference's own int stack[64]
        // (intersections.cu:167), so such a tree is refused rather than traversed differently.
        // The near-first traversals need up to height + 1; a tree too deep (or malformed) for
        // that keeps the reference-order traversal.  No push is ever dropped.
        const int ref_stack = bvh_max_stack(s->bvh_nodes, s->num_bvh_nodes);
        if (ref_stack > MAXSTACK)
            return fail(PT_E_UNSUPPORTED, "BVH needs a %d-entry traversal stack; the reference's holds %d "
                        "(intersections.cu:167)", ref_stack, MAXSTACK);
        const int tree_height = bvh_height(s->bvh_nodes, s->num_bvh_nodes);
        // the near-first traversals (pair layout, SAH hierarchy, certified t-culls) rely on the
        // boxes being nested as scene.cpp:428-441 builds them; a caller-supplied tree that is not
        // keeps the reference-order traversal, which assumes nothing
        if (tree_height < 0 || tree_height + 1 > MAXSTACK || !bvh_boxes_nested(*s)) {
            o.variant &= ~(VAR_BVH_FAST | VAR_BVH_SPLIT);
            gp->opts.variant = o.variant;
        }
        gp->stack_depth = std::max(2, ref_stack);
        if (o.variant & VAR_BVH_FAST) gp->stack_depth = std::max(gp->stack_depth, tree_height + 1);
        // VAR_BVH_FAST pair layout (DevPair): walk the tree in the reference's visit order
        // (push left, push right, pop -> right subtree first), numbering internal nodes (pairs)
        // and leaves (4-slot triangle groups).  Any tree this layout cannot hold exactly -- a
        // missing child, a node reached twice, a leaf of more than 4 triangles, 2^24 refs or more
        // (pack_ref's widest ref field) or a deeper tree than the stack -- keeps the node-array
        // traversal.
        {
            const int nn = s->num_bvh_nodes;
            std::vector<int> id(nn, -1);
            std::vector<char> is_leaf(nn, 0);
            std::vector<std::pair<int, int>> st{{0, 1}};
            int P = 0, L = 0, height = 0;
            bool ok = true;
            std::vector<int> leaf_nodes;
            while (!st.empty() && ok) {
                const int n = st.back().first, d = st.back().second;
                st.pop_back();
                if (n < 0 || n >= nn || id[n] >= 0) { ok = false; break; }
                height = std::max(height, d);
                const pt_bvh_node& nd = s->bvh_nodes[n];
                if (nd.triCount > 0 && nd.start >= 0) {
                    if (nd.triCount > 4) ok = false;
                    is_leaf[n] = 1;
                    id[n] = L++;
                    leaf_nodes.push_back(n);
                } else {
                    if (nd.left < 0 || nd.right < 0) { ok = false; break; }
                    id[n] = P++;
                    st.push_back({nd.left, d + 1});
                    st.push_back({nd.right, d + 1});
                }
            }
            if (ok) {   // internal refs breadth-first: the top levels share a few cache lines
                std::vector<int> fifo{0};
                int k = 0;
                for (size_t h = 0; h < fifo.size(); ++h) {
                    const int n = fifo[h];
                    if (is_leaf[n]) continue;
                    id[n] = k++;
                    fifo.push_back(s->bvh_nodes[n].left);
                    fifo.push_back(s->bvh_nodes[n].right);
                }
            }
            ok = ok && (int64_t)P + L < (1 << 24) && height + 1 <= MAXSTACK && !(o.variant & VAR_BVH_NODES);
            if (ok) {
                auto ref = [&](int n) { return is_leaf[n] ? P + id[n] : id[n]; };
                // cull_threshold_packed's constants for a child of cull size s (same c0 and E as
                // SceneDev::cull_c0 / cull_E below), evaluated in double and rounded up
                const float c0f = (float)(64.0 * std::ldexp(1.0, -24) / 1e-5 * 1.01 * (1.0 + 1e-5));
                const float Ef = (float)(cull_extent * (1.0 + 1e-5));
                auto pack_cull = [&](float sf) {
                    auto up16 = [](double v) -> uint32_t {
                        if (!(v >= 0.0)) v = HUGE_VAL;                  // NaN: never cull
                        float f = (float)v;
                        if ((double)f < v) f = std::nextafter(f, HUGE_VALF);
                        uint32_t b;
                        memcpy(&b, &f, 4);
                        if (b & 0xffffu) b = (b & 0xffff0000u) + 0x10000u;   // up to 16 bits (inf stays inf)
                        return b >> 16;
                    };
                    const double sd = sf, c = sd * sd * (double)c0f;
                    const double A = c * sd * 1.002 + c * (double)Ef * (1.0 + 1e-6);
                    const double d = 1.0 - (1.0 - 1e-6) / (1.0 + 2.0 * c + 2e-6);
                    const uint32_t w = (up16(A) << 16) | up16(d);
                    float f;
                    memcpy(&f, &w, 4);
                    return f;
                };
                // The hierarchy above the reference's leaves (trav_tree.h): a binned-SAH tree over
                // them, its inner boxes the unions of their leaves' boxes, unless a leaf box has a
                // NaN / infinite bound (the containment argument needs ordered bounds), the union
                // differs from the reference root box, or the tree would not fit the stack.
                // PT_BVH_TREE=ref (tools, A/B) keeps the reference's own hierarchy.
                std::vector<pth::TravInner> tt;
                int th = 0;
                bool sah = !gp->tune.bvh_tree_ref && L >= 2;
                if (sah) {
                    std::vector<float> llo(3 * (size_t)L), lhi(3 * (size_t)L), ls(L);
                    for (int k = 0; k < L; ++k) {
                        const DevNode& nd = nodes[leaf_nodes[k]];
                        llo[3 * k] = nd.lo.x; llo[3 * k + 1] = nd.lo.y; llo[3 * k + 2] = nd.lo.z;
                        lhi[3 * k] = nd.hi.x; lhi[3 * k + 1] = nd.hi.y; lhi[3 * k + 2] = nd.hi.z;
                        ls[k] = node_aux[leaf_nodes[k]].y;
                    }
                    // the traversal kernels keep one stack entry per tree level in LDS (BLOCK x 4 B each):
                    // a tree of height h needs (h + 1) KB per block, so the height is bounded to what
                    // still lets BVH_WAVES blocks share a CU's 160 KB (21 levels; the 262k / 1.0M
                    // stand-ins' SAH trees are 24 / 26 high unbounded: 6 / 5 blocks)
                    const int hmax = gp->tune.bvh_max_height > 0 ? gp->tune.bvh_max_height
                                     : gp->tune.bvh_max_height == 0
                                         ? (1 << 30)
                                         : (int)(163840 / ((size_t)BVH_WAVES * BLOCK * sizeof(int))) - 1;
                    sah = pth::build_sah_tree(llo, lhi, ls, tt, th, gp->tune.bvh_bfs_levels, hmax) && th + 1 <= MAXSTACK &&
                          (int64_t)tt.size() + L < (1 << 24);
                    if (sah) {   // the union of the leaves is the reference root box, bit for bit
                        const pth::TravChild& a = tt[0].c[0];
                        const pth::TravChild& b = tt[0].c[1];
                        const float r[6] = {nodes[0].lo.x, nodes[0].lo.y, nodes[0].lo.z,
                                            nodes[0].hi.x, nodes[0].hi.y, nodes[0].hi.z};
                        for (int ax = 0; ax < 3; ++ax)
                            sah = sah && std::min(a.lo[ax], b.lo[ax]) == r[ax] && std::max(a.hi[ax], b.hi[ax]) == r[3 + ax];
                    }
                }
                if (sah) {
                    P = (int)tt.size();
                    pairs.resize(P);
                    for (int i = 0; i < P; ++i) {
                        DevPair& pr = pairs[i];
                        float4* lo[2] = {&pr.l_lo, &pr.r_lo};
                        float4* hi[2] = {&pr.l_hi, &pr.r_hi};
                        for (int k = 0; k < 2; ++k) {
                            const pth::TravChild& c = tt[i].c[k];
                            const int rf = c.leaf ? P + c.ref : c.ref;
                            float frf;
                            memcpy(&frf, &rf, 4);
                            *lo[k] = make_float4(c.lo[0], c.lo[1], c.lo[2], frf);
                            *hi[k] = make_float4(c.hi[0], c.hi[1], c.hi[2], pack_cull(c.s));
                        }
                    }
                    gp->stack_depth = std::max(gp->stack_depth, th + 1);
                    gp->pair_depth = th + 1;
                    // the 4-wide form of the same hierarchy: record q holds the children of binary
                    // node n, an inner child replaced by its own two children (two levels per
                    // record, one 128-B line); quad 0 is the root's.  Inner refs breadth-first over
                    // the top levels, preorder below, as the pairs (PT_BVH_BFS_LEVELS / 2 levels).
                    const bool quad_on = gp->tune.bvh_quad > 0;
                    if (quad_on) {
                        std::vector<pth::QuadRecord> qr;
                        int qneed = 0;
                        pth::build_quad_records(tt, std::max(0, gp->tune.bvh_bfs_levels / 2), qr, qneed);
                        // the hand-over saves the stack depth in 7 bits (trav_saved_node): deeper
                        // worst cases (trees far past the height bound) keep the pairs
                        if (qneed + 1 > 96) qr.clear();
                        const int Q = (int)qr.size();
                        quads.assign(8 * (size_t)Q, make_float4(0.f, 0.f, 0.f, 0.f));
                        for (int q = 0; q < Q; ++q) {
                            float4* R = &quads[8 * (size_t)q];
                            float* f[8] = {&R[0].x, &R[1].x, &R[2].x, &R[3].x, &R[4].x, &R[5].x, &R[6].x, &R[7].x};
                            for (int i = 0; i < 4; ++i) {
                                int rf = -1;   // no child
                                if (i < qr[q].n) {
                                    const pth::TravChild& c = qr[q].c[i];
                                    for (int a = 0; a < 3; ++a) {
                                        f[a][i] = c.lo[a];
                                        f[3 + a][i] = c.hi[a];
                                    }
                                    rf = c.leaf ? Q + c.ref : c.ref;
                                    f[7][i] = pack_cull(c.s);
                                }
                                memcpy(&f[6][i], &rf, 4);
                            }
                        }
                        quad_stack = Q > 0 ? qneed + 1 : 0;
                        gp->stack_depth = std::max(gp->stack_depth, quad_stack);
                        gp->pair_depth = std::max(gp->pair_depth, quad_stack);   // the push bound covers both
                        if (gp->tune.bvh_tree_info)
                            fprintf(stderr, "pt_init: 4-wide records %d (pairs %d), stack %d entries\n", Q, P, quad_stack);
                    }
                    if (gp->tune.bvh_tree_info)
                        fprintf(stderr, "pt_init: SAH traversal tree over %d reference leaves, height %d (reference %d)\n", L,
                                th, height);
                }
                pairs.resize(std::max(1, P));
                for (int n = 0; n < nn && !sah; ++n) {
                    if (id[n] < 0 || is_leaf[n]) continue;
                    const pt_bvh_node& nd = s->bvh_nodes[n];
                    DevPair& pr = pairs[id[n]];
                    const int kids[2] = {nd.left, nd.right};
                    float4* lo[2] = {&pr.l_lo, &pr.r_lo};
                    float4* hi[2] = {&pr.l_hi, &pr.r_hi};
                    for (int k = 0; k < 2; ++k) {
                        const int c = kids[k];
                        const int rf = ref(c);
                        float frf;
                        memcpy(&frf, &rf, 4);
                        *lo[k] = make_float4(nodes[c].lo.x, nodes[c].lo.y, nodes[c].lo.z, frf);
                        *hi[k] = make_float4(nodes[c].hi.x, nodes[c].hi.y, nodes[c].hi.z, pack_cull(node_aux[c].y));
                    }
                }
                hot4.assign(4 * (size_t)L, DevTriHot{});
                for (int k = 0; k < L; ++k) {
                    const pt_bvh_node& nd = s->bvh_nodes[leaf_nodes[k]];
                    for (int i = 0; i < nd.triCount; ++i) hot4[4 * (size_t)k + i] = hot[nd.start + i];
                    const int cnt = nd.triCount;
                    memcpy(&hot4[4 * (size_t)k].c.z, &cnt, 4);
                }
                // trav_step's leaf records: component k of the 4 slots in one float4, positions
                // as v0 and the float edges v1 - v0, v2 - v0 (tri_test's own first rounding)
                leaf9.assign(9 * (size_t)L, make_float4(0.f, 0.f, 0.f, 0.f));
                for (int k = 0; k < L; ++k)
                    for (int i = 0; i < 4; ++i) {
                        const DevTriHot& h = hot4[4 * (size_t)k + i];
                        const float v0[3] = {h.a.x, h.a.y, h.a.z}, v1[3] = {h.a.w, h.b.x, h.b.y},
                                    v2[3] = {h.b.z, h.b.w, h.c.x};
                        float comp9[9];
                        for (int a = 0; a < 3; ++a) {
                            comp9[a] = v0[a];
                            comp9[3 + a] = v1[a] - v0[a];
                            comp9[6 + a] = v2[a] - v0[a];
                        }
                        for (int m = 0; m < 9; ++m) (&leaf9[9 * (size_t)k + m].x)[i] = comp9[m];
                    }
                if (!sah) gp->pair_depth = height + 1;
                pair_root_ref = sah ? 0 : ref(0);
                pair_root_lo = make_float4(nodes[0].lo.x, nodes[0].lo.y, nodes[0].lo.z, 0.f);
                pair_root_hi = make_float4(nodes[0].hi.x, nodes[0].hi.y, nodes[0].hi.z, node_aux[0].y);
                pair_count = P;
                // stack entries: as few ref bits as the P + L refs need, the rest for the cull T
                int rb = 2;
                while (((int64_t)1 << rb) < (int64_t)P + L) ++rb;
                pair_ref_shift = 32 - rb;
            }
        }
        gp->bvh_lds = (size_t)gp->stack_depth * BLOCK * sizeof(int);
    }
    for (int i = 0; i < s->num_geoms; ++i)
        if (s->geoms[i].materialid < 0 || s->geoms[i].materialid >= std::max(1, s->num_materials))
            return fail(PT_E_INVALID, "geom %d material %d out of range", i, s->geoms[i].materialid);
    // VAR_BVH_SPLIT needs the pair layout, the fast traversal and an LDS geom table
    gp->split = gp->has_bvh && !pairs.empty() && o.pipeline == PT_PIPELINE_FUSED && (o.variant & VAR_BVH_SPLIT) &&
              (o.variant & VAR_BVH_FAST) && (o.variant & (VAR_CAND_QUEUE | VAR_WAVE_REDIST)) &&
              s->num_geoms <= LDS_GEOMS;
    // MATERIAL_SORTING on the fused pipeline: the block-local regrouping by material (VAR_MAT_GROUP;
    // keys are the material ids, at most MG_KEYS - 1 of them), for the kernel variants built with it
    if (o.material_sort && o.pipeline == PT_PIPELINE_FUSED && s->num_materials <= MG_KEYS - 1 &&
        variant_compiled(effective_variant(true, o.variant | VAR_MAT_GROUP)) &&
        variant_compiled(effective_variant(false, o.variant | VAR_MAT_GROUP))) {
        o.variant |= VAR_MAT_GROUP;
        gp->opts.variant = o.variant;
    }
    if (o.pipeline == PT_PIPELINE_FUSED) {
        for (int first = 0; first < 2; ++first) {
            const int v = effective_variant(first != 0, o.variant);
            if (v != 3 && !variant_compiled(v))
                return fail(PT_E_UNSUPPORTED, "variant %d (effective %d for the %s bounce) is not compiled in", o.variant,
                            v, first ? "camera" : "later");
        }
    }
    gp->num_tex = (s->num_textures > 0 && s->textures) ? s->num_textures : 0;
    gp->sc.num_mats = s->num_materials;
    // frames per pass: as asked, or auto (~84M paths), halved while the per-pass buffers would
    // take more than half of the device memory free now.  Buffers are allocated when a pass of
    // that size is first traced or prepared (ensure_frames), not here.
    if (o.frames_per_pass > 0) {
        gp->batch = o.frames_per_pass;
    } else {
        gp->batch = auto_batch(gp->local_pixels);
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
            while (gp->batch > 1 && pass_bytes(gp->batch, o.pipeline == PT_PIPELINE_STAGED) > free_b / (2 * (size_t)share))
                gp->batch /= 2;
    }
    if ((int64_t)gp->local_pixels * gp->batch > (1 << 28)) return fail(PT_E_UNSUPPORTED, "wavefront too large");

    RC(dalloc(&gp->d_geoms, geoms.size()));
    RC(dalloc(&gp->d_mats, mats.size()));
    RC(upload(gp->d_geoms, geoms.data(), geoms.size()));
    RC(dalloc(&gp->d_cull, culls.size()));
    // the pre-test's candidate table, for scenes whose flat pre-test is long (A/B: PT_GRID=0 off,
    // PT_GRID=1 also for scenes under GRID_MIN_GEOMS)
    std::vector<unsigned long long> grid;
    float grid_lo[3] = {0.f, 0.f, 0.f}, grid_inv[3] = {0.f, 0.f, 0.f};
    {
        const int grid_env = gp->tune.grid;
        const int grid_min = grid_env == 1 ? 2 : GRID_MIN_GEOMS;
        if (grid_env != 0 && s->num_geoms >= grid_min && s->num_geoms <= LDS_GEOMS &&
            build_candidate_table(culls, s->num_geoms, s->camera.position, grid, grid_lo, grid_inv)) {
            RC(dalloc(&gp->d_grid, grid.size()));
            RC(upload(gp->d_grid, grid.data(), grid.size()));
        }
    }
    RC(upload(gp->d_cull, culls.data(), culls.size()));
    RC(upload(gp->d_mats, mats.data(), mats.size()));
    if (gp->has_bvh) {
        RC(dalloc(&gp->d_nodes, nodes.size()));
        RC(dalloc(&gp->d_node_aux, node_aux.size()));
        RC(upload(gp->d_node_aux, node_aux.data(), node_aux.size()));
        RC(dalloc(&gp->d_hot, hot.size()));
        RC(dalloc(&gp->d_cold, cold.size()));
        RC(upload(gp->d_nodes, nodes.data(), nodes.size()));
        RC(upload(gp->d_hot, hot.data(), hot.size()));
        RC(upload(gp->d_cold, cold.data(), cold.size()));
        if (!pairs.empty()) {
            RC(dalloc(&gp->d_pairs, pairs.size()));
            RC(upload(gp->d_pairs, pairs.data(), pairs.size()));
            RC(dalloc(&gp->d_hot4, hot4.size()));
            RC(upload(gp->d_hot4, hot4.data(), hot4.size()));
            RC(dalloc(&gp->d_leaf9, leaf9.size()));
            RC(upload(gp->d_leaf9, leaf9.data(), leaf9.size()));
            if (!quads.empty()) {
                RC(dalloc(&gp->d_quads, quads.size()));
                RC(upload(gp->d_quads, quads.data(), quads.size()));
            }
        }
    }
    // textures (pathtrace.cu:169-201): RGBA8 texels of every texture in one buffer
    int num_tex = 0;
    if (s->num_textures > 0 && s->textures) {
        std::vector<int4> info(s->num_textures);
        size_t total = 0;
        for (int i = 0; i < s->num_textures; ++i) {
            const pt_texture& t = s->textures[i];
            if (t.width <= 0 || t.height <= 0 || !t.data || t.channels != 4)
                return fail(PT_E_INVALID, "texture %d: need RGBA8 data (channels 4)", i);
            info[i] = make_int4((int)total, t.width, t.height, 0);
            total += (size_t)t.width * t.height;
        }
        if (total > (size_t)INT32_MAX) return fail(PT_E_UNSUPPORTED, "texture data too large");
        RC(dalloc(&gp->d_texels, total));
        RC(dalloc(&gp->d_texinfo, info.size()));
        for (int i = 0; i < s->num_textures; ++i) {
            const pt_texture& t = s->textures[i];
            HIPCHK(smemcpy(gp->d_texels + info[i].x, t.data, (size_t)t.width * t.height * 4, hipMemcpyHostToDevice));
        }
        RC(upload(gp->d_texinfo, info.data(), info.size()));
        num_tex = s->num_textures;
    }
    RC(dalloc(&gp->d_image, (size_t)gp->pixels_total * 3));
    HIPCHK(smemset(gp->d_image, 0, sizeof(float) * 3 * (size_t)gp->pixels_total));
    RC(dalloc(&gp->d_ctl, 1));
    RC(ctl_reset());
    gp->key_bits = 1;
    while ((1 << gp->key_bits) < std::max(2, s->num_materials)) gp->key_bits++;

    SceneDev& sc = gp->sc;
    sc.geoms = gp->d_geoms;
    sc.cull = gp->d_cull;
    sc.mats = gp->d_mats;
    sc.nodes = gp->d_nodes;
    sc.node_aux = gp->d_node_aux;
    sc.hot = gp->d_hot;
    sc.cold = gp->d_cold;
    sc.num_geoms = s->num_geoms;
    sc.num_mats = s->num_materials;
    sc.num_nodes = gp->has_bvh ? s->num_bvh_nodes : 0;
    sc.num_tris = s->num_triangles;
    sc.trace_depth = s->trace_depth;
    sc.arg_order = o.arg_order;
    sc.use_bvh = gp->has_bvh ? 1 : 0;
    sc.stack_depth = gp->stack_depth;
    // the pair traversal pushes at most one entry per level of its hierarchy (never more than the
    // stack_depth the other traversals size their stacks for); k_bvh_bounce's LDS stack is sized
    // by it
    sc.pair_stack_depth = gp->pair_depth > 0 ? std::min(gp->pair_depth, gp->stack_depth) : gp->stack_depth;
    // the split kernels' LDS stack: all of it, or its first bvh_stack_lds entries and a spill row per
    // queue slot for the rest
    sc.stack_lds = gp->split && gp->tune.bvh_stack_lds > 0 ? std::min(gp->tune.bvh_stack_lds, sc.pair_stack_depth)
                                                           : sc.pair_stack_depth;
    sc.spill_stride = sc.pair_stack_depth - sc.stack_lds;
    sc.spill = nullptr;   // allocated with the traversal queue (ensure_frames)
    sc.cam = to_camdev(s->camera);
    sc.shard = sh;
    sc.contrib = gp->d_contrib;
    sc.texels = gp->d_texels;
    sc.texinfo = gp->d_texinfo;
    sc.num_textures = num_tex;
    sc.pairs = gp->d_pairs;
    sc.hot4 = gp->d_hot4;
    sc.leaf9 = gp->d_leaf9;
    sc.num_pairs = pair_count;
    sc.quads = gp->split ? gp->d_quads : nullptr;   // the 4-wide records serve the traversal kernels only
    sc.num_quads = (int)(quads.size() / 8);
    sc.root_ref = pair_root_ref;
    sc.ref_shift = pair_ref_shift;
    sc.root_lo = pair_root_lo;
    sc.root_hi = pair_root_hi;
    // node_aux's c = 64 2^-24 sx^2 / 1e-5, stored x 1.01, and cE = c x extent x 1.01: the same
    // bounds from s = sx on the device, rounded up
    sc.cull_c0 = (float)(64.0 * std::ldexp(1.0, -24) / 1e-5 * 1.01 * (1.0 + 1e-5));
    sc.cull_E = (float)(cull_extent * (1.0 + 1e-5));
    sc.grid = gp->d_grid;
    sc.grid_all = s->num_geoms >= 64 ? ~0ull : ((1ull << s->num_geoms) - 1);
    for (int a = 0; a < 3; ++a) {
        sc.grid_lo[a] = grid_lo[a];
        sc.grid_inv[a] = grid_inv[a];
    }
    RC(ensure_frames(1));            // one frame's wavefront now; larger passes grow it on first use
    gp->inited = true;
    HIPCHK(hipDeviceSynchronize());
    return PT_OK;
}

int32_t pt_init(const pt_scene_view* s, const pt_options* opts_in) {
    if (!s) return fail(PT_E_INVALID, "scene is NULL");
    pt_free();
    pt_options o;
    if (opts_in) o = *opts_in;
    else pt_default_options(&o);
    if (o.num_devices < 0 || o.num_devices > PT_MAX_DEVICES)
        return fail(PT_E_INVALID, "num_devices must be 0 .. %d", PT_MAX_DEVICES);
    if (o.num_devices <= 1) {
        const int rc = init_one(s, o, 1);
        if (rc != PT_OK) free_all();   // whatever was allocated before the failure
        return rc;
    }
    const int n = o.num_devices;
    if (o.shard_mode != PT_SHARD_NONE)
        return fail(PT_E_INVALID, "num_devices > 1 splits the frame itself; shard_mode must be PT_SHARD_NONE");
    if (o.combine != PT_COMBINE_PEER && o.combine != PT_COMBINE_RCCL) return fail(PT_E_INVALID, "bad combine");
    const int H = s->camera.resolution.y, rows = std::max(1, o.shard_rows);
    if (H > 0 && (H + rows - 1) / rows < n)
        return fail(PT_E_INVALID, "%d shards but only %d row bands of %d rows", n, (H + rows - 1) / rows, rows);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(PT_E_NODEVICE, "no HIP device visible");
    for (int k = 0; k < n; ++k)
        if (o.device_ids[k] < 0 || o.device_ids[k] >= ndev)
            return fail(PT_E_INVALID, "device_ids[%d] = %d out of range (%d devices)", k, o.device_ids[k], ndev);
    M.n = n;
    M.combine = o.combine;
    int rc = PT_OK;
    for (int k = 0; k < n && rc == PT_OK; ++k) {
        M.shard[k] = k == 0 ? &g_primary : new State();
        pt_options ok = o;
        ok.num_devices = 1;
        ok.device = o.device_ids[k];
        ok.shard_mode = PT_SHARD_PIXELS;
        ok.shard_rank = k;
        ok.shard_count = n;
        ok.shard_rows = rows;
        int share = 0;
        for (int j = 0; j < n; ++j) share += o.device_ids[j] == o.device_ids[k];
        ShardScope sc(M.shard[k]);
        rc = init_one(s, ok, share);
        gp->multi = true;
    }
    if (rc == PT_OK) rc = multi_setup();
    if (rc != PT_OK) {
        const std::string err = g_err;
        pt_free();
        g_err = err;
        return rc;
    }
    HIPCHK(hipSetDevice(g_primary.device));
    return PT_OK;
}

int32_t pt_set_camera(const pt_camera* c) {
    RC(need_init());
    if (!c || c->resolution.x != gp->width || c->resolution.y != gp->height)
        return fail(PT_E_INVALID, "camera resolution must match pt_init");
    const CamDev nc = to_camdev(*c);
    for (int k = 0; k < nshards(); ++k) {
        ShardScope sc(shard_ctx(k));
        if (memcmp(&nc, &gp->sc.cam, sizeof nc) != 0) {
            RC(spec_cancel());                          // traced with the old camera
            HIPCHK(hipStreamSynchronize(gp->stream));   // a replayed pass may still hold the graph
            gp->sc.cam = nc;
            release_graph();   // kernel arguments changed
        }
    }
    return PT_OK;
}

int32_t pt_set_trace_depth(int32_t depth) {
    RC(need_init());
    if (depth < 0 || depth > MAXB) return fail(PT_E_UNSUPPORTED, "trace depth %d not in 0 .. %d", depth, MAXB);
    for (int k = 0; k < nshards(); ++k) {
        ShardScope sc(shard_ctx(k));
        if (gp->sc.trace_depth != depth) {
            RC(spec_cancel());
            HIPCHK(hipStreamSynchronize(gp->stream));
            gp->sc.trace_depth = depth;
            release_graph();   // the bounce count is baked into the captured passes
        }
    }
    return PT_OK;
}

int32_t pt_debug_spec_counts(int64_t* launched, int64_t* adopted) {
    RC(need_init());
    int64_t l = 0, a = 0;
    for (int k = 0; k < nshards(); ++k) {
        l += shard_ctx(k)->spec_launched;
        a += shard_ctx(k)->spec_adopted;
    }
    if (launched) *launched = l;
    if (adopted) *adopted = a;
    return PT_OK;
}

int32_t pt_set_speculation(int32_t enabled) {
    RC(need_init());
    State* p = &g_primary;
    if (!enabled) RC(spec_cancel_all());
    p->tune.speculate = enabled != 0;
    return PT_OK;
}

int32_t pt_trace(pt_uchar4* pbo, int32_t frame, int32_t iteration, float* host_image) {
    (void)frame;   // unused by the reference too (pathtrace.cu:639)
    RC(need_init());
    if (iteration <= 0) return fail(PT_E_INVALID, "iteration is 1-based (main.cpp:458), got %d", iteration);
    // speculate only for callers that copy the image out (main.cpp's pathtrace() always does): a
    // call without the copy has nothing for the next frame to overlap with.  Several devices: every
    // shard speculates its own pixels; the call for N + 1 takes each shard's frame over, then
    // combines as usual (the host copy reads the combined image, so it waits for the combine)
    const bool spec = spec_enabled() && (host_image != nullptr || gp->spec_iter == iteration);
    const bool single = M.n <= 1;
    const bool bands_on = !single && M.band_copy && host_image;
    bool adopted = false;
    const int sum_idx = gp->spec_sum_idx;   // the taken-over frame's image, before the next launch flips it
    BandCopy bands[PT_MAX_DEVICES];
    for (int k = 0; k < nshards(); ++k) {
        ShardScope sc(shard_ctx(k));
        if (spec && gp->spec_iter == iteration) {
            adopted = true;
            const float* sum = gp->d_spec_sum[gp->spec_sum_idx];
            RC(spec_adopt(host_image != nullptr && single));   // traced already, during the previous call's copy
            // several devices: this shard's bands of the finished sum (the speculative stream has it)
            if (bands_on) RC(band_prepare(bands[k], host_image, sum, gp->spec_stream));
        } else {
            RC(spec_cancel());
            RC(run_frame(iteration));
            if (bands_on) RC(band_prepare(bands[k], host_image, gp->d_image, gp->stream));
        }
        if (g_primary.traced_depth) RC(frame_depth_enqueue());   // read after the one sync below
    }
    RC(multi_combine());
    if (pbo) {
        hipLaunchKernelGGL(k_to_pbo, dim3(nblocks(gp->pixels_total)), dim3(BLOCK), 0, gp->stream, gp->d_image, pbo,
                           gp->pixels_total, iteration);
        HIPCHK(hipGetLastError());
    }
    // the next frame, on the second stream, while this one's image is copied out (queued before
    // the copy: a copy into pageable memory may hold the host until it is done)
    if (spec && host_image && iteration < INT32_MAX) RC(spec_launch(iteration + 1));
    if (bands_on) {
        // every shard's row bands from its own device, side by side (shard 0's on this thread)
        for (int k = 1; k < nshards(); ++k) g_copy_helpers[k].post(bands[k]);
        hipError_t e = bands[0].run();
        for (int k = 1; k < nshards(); ++k) {
            const hipError_t ek = g_copy_helpers[k].wait();
            if (e == hipSuccess) e = ek;
        }
        HIPCHK(hipSetDevice(g_primary.device));
        HIPCHK(e);
    } else if (host_image) {
        // the caller's pageable memory, as cudaMemcpy(state.image) (pathtrace.cu:783).  It is not
        // page-locked: a registration would outlive a caller that frees the buffer and gets a new
        // one at the same address, and on MI355X the pageable copy runs at the pinned rate anyway
        // (tools/copy_probe.py: 7.68 MB in 0.145 ms either way)
        const size_t bytes = sizeof(float) * 3 * (size_t)gp->pixels_total;
        if (adopted && single)   // the speculated frame's finished sum, on the copy stream (it waited for it)
            HIPCHK(hipMemcpyAsync(host_image, gp->d_spec_sum[sum_idx], bytes, hipMemcpyDeviceToHost, gp->copy_stream));
        else
            HIPCHK(hipMemcpyAsync(host_image, gp->d_image, bytes, hipMemcpyDeviceToHost, gp->stream));
    }
    // one wait: the first device's stream waited for every shard's frame (multi_combine), and each
    // shard queued its counter copy before that
    HIPCHK(hipStreamSynchronize(gp->stream));
    if (adopted && single && host_image) HIPCHK(hipStreamSynchronize(gp->copy_stream));
    if (gp->traced_depth) {
        // GuiDataContainer::TracedDepth = the bounces the frame ran (pathtrace.cu:759-770); with
        // shards, the frame ran as long as its longest shard
        int depth = 0;
        for (int k = 0; k < nshards(); ++k) {
            ShardScope sc(shard_ctx(k));
            depth = std::max(depth, frame_depth_read());
        }
        *gp->traced_depth = depth;
    }
    return PT_OK;
}

int32_t pt_trace_frames(int32_t first_iteration, int32_t count) {
    RC(need_init());
    RC(spec_cancel_all());
    if (first_iteration <= 0 || count < 0) return fail(PT_E_INVALID, "bad iteration range");
    // passes of gp->batch frames (bit-identical to frame-by-frame: k_combine keeps the order);
    // every shard's passes are queued before the combine, so the devices trace concurrently
    for (int k = 0; k < nshards(); ++k) {
        ShardScope sc(shard_ctx(k));
        for (int i = 0; i < count;) {
            const int f = pass_frames(count - i);
            RC(run_pass(first_iteration + i, f));
            i += f;
        }
    }
    return count > 0 ? multi_combine() : PT_OK;
}

int32_t pt_prepare_frames(int32_t count) {
    RC(need_init());
    RC(spec_cancel_all());
    if (count < 0) return fail(PT_E_INVALID, "bad count");
    for (int k = 0; k < nshards(); ++k) {
        ShardScope sc(shard_ctx(k));
        RC(ensure_frames(count > 0 ? pass_frames(count) : 1));   // the largest pass of the run comes first
        if (!gp->opts.use_graph) continue;
        // the pass sizes pt_trace_frames(., count) will replay
        for (int i = 0; i < count;) {
            const int f = pass_frames(count - i);
            if (!gp->graph_exec[f]) RC(build_graph(f));
            i += f;
        }
    }
    return PT_OK;
}

int32_t pt_synchronize(void) {
    RC(need_init());
    HIPCHK(g_spec_launcher.idle());
    for (int k = 0; k < nshards(); ++k) {   // speculated frames (their streams stay valid)
        State* s = shard_ctx(k);
        if (!s->spec_stream) continue;
        ShardScope sc(s);
        HIPCHK(hipStreamSynchronize(s->spec_stream));
    }
    for (int k = nshards() - 1; k >= 0; --k) {
        ShardScope sc(shard_ctx(k));
        HIPCHK(hipStreamSynchronize(gp->stream));
    }
    return PT_OK;
}

int32_t pt_get_image(float* host_out, int64_t n_floats) {
    RC(need_init());
    if (!host_out || n_floats < (int64_t)gp->pixels_total * 3) return fail(PT_E_INVALID, "image buffer too small");
    HIPCHK(hipStreamSynchronize(gp->stream));
    HIPCHK(smemcpy(host_out, gp->d_image, sizeof(float) * 3 * (size_t)gp->pixels_total, hipMemcpyDeviceToHost));
    return PT_OK;
}

int32_t pt_get_image_device(void** device_ptr, int64_t* n_floats) {
    RC(need_init());
    // the caller may write through the pointer before the next pt_trace: a speculated next frame
    // summed from the image as it is now would then overwrite that write, so it is dropped here
    RC(spec_cancel_all());
    HIPCHK(hipStreamSynchronize(gp->stream));
    if (device_ptr) *device_ptr = gp->d_image;
    if (n_floats) *n_floats = (int64_t)gp->pixels_total * 3;
    return PT_OK;
}

int32_t pt_set_image(const float* host_in, int64_t n_floats) {
    RC(need_init());
    RC(spec_cancel_all());   // its image + plane was formed from the image being replaced
    if (!host_in || n_floats != (int64_t)gp->pixels_total * 3) return fail(PT_E_INVALID, "image size mismatch");
    for (int k = 0; k < nshards(); ++k) {   // each shard keeps accumulating into its own pixels of it
        ShardScope sc(shard_ctx(k));
        HIPCHK(hipStreamSynchronize(gp->stream));
        HIPCHK(smemcpy(gp->d_image, host_in, sizeof(float) * (size_t)n_floats, hipMemcpyHostToDevice));
    }
    return PT_OK;
}

// device buffers for callers without the HIP headers (the headless viewer's PBO, ctypes)
int32_t pt_device_alloc(int64_t bytes, void** out) {
    if (!out || bytes <= 0) return fail(PT_E_INVALID, "pt_device_alloc: bad argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(PT_E_NODEVICE, "no HIP device visible");
    HIPCHK(hipMalloc(out, (size_t)bytes));
    return PT_OK;
}

int32_t pt_device_free(void* p) {
    if (p) HIPCHK(hipFree(p));
    return PT_OK;
}

int32_t pt_device_read(void* host_dst, const void* device_src, int64_t bytes) {
    if (!host_dst || !device_src || bytes < 0) return fail(PT_E_INVALID, "pt_device_read: bad argument");
    if (gp->stream) HIPCHK(hipStreamSynchronize(gp->stream));
    HIPCHK(smemcpy(host_dst, device_src, (size_t)bytes, hipMemcpyDeviceToHost));
    return PT_OK;
}

static int32_t frame_stats(pt_frame_stats* out);   // the current context's (below)

int32_t pt_get_frame_stats(pt_frame_stats* out) {
    RC(need_init());
    if (!out) return fail(PT_E_INVALID, "NULL");
    RC(frame_stats(out));
    for (int k = 1; k < nshards(); ++k) {   // shards: the counts of every shard's pixels
        pt_frame_stats s;
        {
            ShardScope sc(shard_ctx(k));
            RC(frame_stats(&s));
        }
        out->pixels += s.pixels;
        out->segments += s.segments;
        out->segments_total += s.segments_total;
        for (int b = 0; b < 64; ++b) out->live[b] += s.live[b];
        for (int b = 0; b <= MAXB; ++b) {
            out->live_total[b] += s.live_total[b];
            out->queued_total[b] += s.queued_total[b];
            out->handed_total[b] += s.handed_total[b];
            out->handed_stack_total[b] += s.handed_stack_total[b];
        }
    }
    return PT_OK;
}

static int32_t frame_stats(pt_frame_stats* out) {
    HIPCHK(hipStreamSynchronize(gp->stream));
    FrameCtl ctl;
    HIPCHK(smemcpy(&ctl, gp->d_ctl, sizeof ctl, hipMemcpyDeviceToHost));
    memset(out, 0, sizeof(*out));
    out->iteration = ctl.iter;
    out->bounces = std::max(1, gp->sc.trace_depth);
    out->pixels = gp->local_pixels;
    for (int b = 0; b < out->bounces; ++b) {
        int64_t s = 0;
        if (gp->opts.pipeline == PT_PIPELINE_STAGED && !gp->opts.stream_compaction) {
            s = b == 0 ? ctl.cnt[0][0][0] : -1;   // no compaction: the live count is never formed
        } else {
            for (int k = 0; k < NSEG; ++k) s += ctl.cnt[b][k][0];
        }
        out->live[b] = s;
        if (s > 0) out->segments += s;
    }
    out->frames_total = (int64_t)ctl.frames;
    out->frames_per_pass = gp->batch;
    out->last_pass_frames = ctl.batch;
    for (int b = 0; b <= MAXB; ++b) {
        int64_t cur = 0;
        for (int k = 0; k < NSEG; ++k) cur += ctl.cnt[b][k][0];
        out->live_total[b] = (int64_t)ctl.tot[b] + (ctl.frames > 0 ? cur : 0);
        int64_t q = 0;
        for (int k = 0; k < NSEG; ++k) q += ctl.qcnt[b][k][0];
        out->queued_total[b] = (int64_t)ctl.qtot[b] + (ctl.frames > 0 ? q : 0);
        int64_t h = 0, hs = 0;
        for (int k = 0; k < NSEG; ++k) {
            h += ctl.qcnt[b][k][3];
            hs += ctl.qcnt[b][k][4];
        }
        out->handed_total[b] = (int64_t)ctl.htot[b] + (ctl.frames > 0 ? h : 0);
        out->handed_stack_total[b] = (int64_t)ctl.hstk[b] + (ctl.frames > 0 ? hs : 0);
        if (b < out->bounces) out->segments_total += out->live_total[b];
    }
    return PT_OK;
}

int32_t pt_reset_stats(void) {
    RC(need_init());
    for (int k = 0; k < nshards(); ++k) {
        ShardScope sc(shard_ctx(k));
        HIPCHK(hipStreamSynchronize(gp->stream));
        RC(ctl_reset());
    }
    return PT_OK;
}

// ---------------------------------------------------------------------------------------------
// test entry points
// ---------------------------------------------------------------------------------------------
int32_t pt_test_camera(int32_t iteration, pt_path_segment* out, int64_t n) {
    RC(need_init());
    RC(need_single("pt_test_camera"));
    if (!out || n < gp->local_pixels) return fail(PT_E_INVALID, "output too small");
    RC(ensure_frames(1));
    RC(ctl_reset());
    hipLaunchKernelGGL(k_frame_begin, dim3(1), dim3(256), 0, gp->stream, gp->d_ctl, iteration, gp->local_pixels, 1,
                       gp->ctl_rows, 0);
    hipLaunchKernelGGL(k_camera, dim3(nblocks(gp->local_pixels)), dim3(BLOCK), 0, gp->stream, gp->sc, pathbuf(0), gp->d_ctl);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(gp->stream));
    release_graph();
    RC(download_paths(0, gp->local_pixels, out));
    RC(ctl_reset());
    return PT_OK;
}

int32_t pt_test_intersect(const pt_path_segment* paths, int64_t n, pt_shadeable_isect* isects) {
    RC(need_init());
    RC(need_single("pt_test_intersect"));
    RC(ensure_test_paths(n));
    if (n == 0) return PT_OK;
    RC(upload_paths(0, paths, n));
    RC(set_count(0, (int)n));
    // uv / dpdu / dpdv are kept by the production pipelines only for textured scenes (nothing else
    // reads them); this entry point returns the reference's whole record, so mesh scenes without
    // textures get temporary attribute buffers, released on every return path
    struct TmpAttr {
        float4* p[2] = {nullptr, nullptr};
        ~TmpAttr() {
            for (float4* x : p)
                if (x) (void)hipFree(x);
        }
    } tmp;
    float4 *uvd0 = gp->d_hit_uvd0, *uvd1 = gp->d_hit_uvd1;
    if (!uvd0 && gp->has_bvh) {
        RC(dalloc(&tmp.p[0], (size_t)n));
        RC(dalloc(&tmp.p[1], (size_t)n));
        uvd0 = tmp.p[0];
        uvd1 = tmp.p[1];
    }
    HitBuf hits{gp->d_hit_nt, gp->d_hit_mat, uvd0, uvd1};
    if (gp->has_bvh && (gp->opts.variant & VAR_BVH_FAST))
        hipLaunchKernelGGL((k_intersect<true, true>), dim3(nblocks((int)n)), dim3(BLOCK), gp->bvh_lds, gp->stream, gp->sc,
                           pathbuf(0), hits, staged_count(0));
    else if (gp->has_bvh)
        hipLaunchKernelGGL((k_intersect<true, false>), dim3(nblocks((int)n)), dim3(BLOCK), gp->bvh_lds, gp->stream, gp->sc,
                           pathbuf(0), hits, staged_count(0));
    else
        hipLaunchKernelGGL((k_intersect<false, false>), dim3(nblocks((int)n)), dim3(BLOCK), 0, gp->stream, gp->sc,
                           pathbuf(0), hits, staged_count(0));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(gp->stream));
    std::vector<float4> nt(n);
    std::vector<int> mat(n);
    HIPCHK(smemcpy(nt.data(), gp->d_hit_nt, n * sizeof(float4), hipMemcpyDeviceToHost));
    HIPCHK(smemcpy(mat.data(), gp->d_hit_mat, n * sizeof(int), hipMemcpyDeviceToHost));
    std::vector<float4> a0, a1;
    if (uvd0) {
        a0.resize(n);
        a1.resize(n);
        HIPCHK(smemcpy(a0.data(), uvd0, n * sizeof(float4), hipMemcpyDeviceToHost));
        HIPCHK(smemcpy(a1.data(), uvd1, n * sizeof(float4), hipMemcpyDeviceToHost));
    }
    for (int64_t i = 0; i < n; ++i) {
        memset(&isects[i], 0, sizeof(pt_shadeable_isect));
        isects[i].t = nt[i].w;
        isects[i].surfaceNormal = pt_vec3{nt[i].x, nt[i].y, nt[i].z};
        isects[i].materialId = mat[i];
        if (uvd0 && nt[i].w > 0.0f) {   // uv / dpdu / dpdv as the reference writes them (zero for primitives)
            isects[i].uv = pt_vec2{a0[i].x, a0[i].y};
            isects[i].dpdu = pt_vec3{a0[i].z, a0[i].w, a1[i].x};
            isects[i].dpdv = pt_vec3{a1[i].y, a1[i].z, a1[i].w};
        }
    }
    release_graph();
    RC(ctl_reset());
    return PT_OK;
}

int32_t pt_test_shade(int32_t iteration, const pt_shadeable_isect* isects, pt_path_segment* paths, int64_t n) {
    RC(need_init());
    RC(need_single("pt_test_shade"));
    RC(ensure_test_paths(n));
    if (n == 0) return PT_OK;
    RC(upload_paths(0, paths, n));
    RC(set_count(0, (int)n));
    std::vector<float4> nt(n);
    std::vector<int> mat(n);
    for (int64_t i = 0; i < n; ++i) {
        nt[i] = make_float4(isects[i].surfaceNormal.x, isects[i].surfaceNormal.y, isects[i].surfaceNormal.z,
                            isects[i].t);
        mat[i] = isects[i].materialId;
        if (isects[i].t > 0.0f && (mat[i] < 0 || mat[i] >= std::max(1, gp->sc.num_mats)))
            return fail(PT_E_INVALID, "materialId %d out of range", mat[i]);
    }
    HIPCHK(smemcpy(gp->d_hit_nt, nt.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    HIPCHK(smemcpy(gp->d_hit_mat, mat.data(), n * sizeof(int), hipMemcpyHostToDevice));
    if (gp->d_hit_uvd0) {
        std::vector<float4> a0(n), a1(n);
        for (int64_t i = 0; i < n; ++i) {
            const pt_shadeable_isect& x = isects[i];
            a0[i] = make_float4(x.uv.x, x.uv.y, x.dpdu.x, x.dpdu.y);
            a1[i] = make_float4(x.dpdu.z, x.dpdv.x, x.dpdv.y, x.dpdv.z);
        }
        HIPCHK(smemcpy(gp->d_hit_uvd0, a0.data(), n * sizeof(float4), hipMemcpyHostToDevice));
        HIPCHK(smemcpy(gp->d_hit_uvd1, a1.data(), n * sizeof(float4), hipMemcpyHostToDevice));
    }
    HitBuf hits{gp->d_hit_nt, gp->d_hit_mat, gp->d_hit_uvd0, gp->d_hit_uvd1};
    hipLaunchKernelGGL(k_shade, dim3(nblocks((int)n)), dim3(BLOCK), 0, gp->stream, gp->sc, pathbuf(0), hits,
                       (const int*)nullptr, staged_count(0), (const FrameCtl*)gp->d_ctl, iteration, (float*)nullptr,
                       (int*)nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(gp->stream));
    release_graph();
    RC(download_paths(0, n, paths));
    RC(ctl_reset());
    return PT_OK;
}

int32_t pt_test_compact(const pt_path_segment* paths, int64_t n, pt_path_segment* out, int64_t* alive_out) {
    RC(need_init());
    RC(need_single("pt_test_compact"));
    RC(ensure_test_paths(n));
    RC(upload_paths(0, paths, n));
    std::vector<int> al(std::max<int64_t>(1, n));
    for (int64_t i = 0; i < n; ++i) al[i] = paths[i].remainingBounces > 0;   // PathAlive
    if (n) HIPCHK(smemcpy(gp->d_alive, al.data(), n * sizeof(int), hipMemcpyHostToDevice));
    RC(ctl_reset());
    RC(set_count(0, (int)n));
    if (n > 0) {   // the pipeline's launch sequence
        launch_compact<CITEMS>(pathbuf(0), pathbuf(1), staged_count(0), &gp->d_ctl->cnt[1][0][0], (int)n);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(gp->stream));
    int na = 0;
    HIPCHK(smemcpy(&na, &gp->d_ctl->cnt[1][0][0], sizeof(int), hipMemcpyDeviceToHost));
    if (alive_out) *alive_out = na;
    release_graph();
    RC(download_paths(1, na, out));
    RC(ctl_reset());
    return PT_OK;
}

int32_t pt_test_sort(const pt_shadeable_isect* isects, int64_t n, int32_t* perm) {
    RC(need_init());
    RC(need_single("pt_test_sort"));
    RC(ensure_test_paths(n));
    if (n == 0) return PT_OK;
    const int nk = std::max(1, gp->sc.num_mats);
    std::vector<int> mat(n);
    for (int64_t i = 0; i < n; ++i) {
        mat[i] = isects[i].materialId;
        if (mat[i] < 0 || mat[i] >= nk) return fail(PT_E_INVALID, "materialId %d out of range", mat[i]);
    }
    HIPCHK(smemcpy(gp->d_hit_mat, mat.data(), n * sizeof(int), hipMemcpyHostToDevice));
    RC(set_count(0, (int)n));
    const int ntiles = (int)((n + STILE - 1) / STILE);
    hipLaunchKernelGGL(k_sort_hist, dim3(ntiles), dim3(BLOCK), 0, gp->stream, gp->d_hit_mat, staged_count(0), nk,
                       gp->d_tile_hist);
    hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(SCAN_THREADS), 0, gp->stream, gp->d_tile_hist, staged_count(0), nk);
    hipLaunchKernelGGL(k_sort_scatter, dim3(ntiles), dim3(BLOCK), 0, gp->stream, gp->d_hit_mat, staged_count(0), nk,
                       gp->key_bits, gp->d_tile_hist, gp->d_perm);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(gp->stream));
    HIPCHK(smemcpy(perm, gp->d_perm, n * sizeof(int), hipMemcpyDeviceToHost));
    release_graph();
    RC(ctl_reset());
    return PT_OK;
}

int32_t pt_test_rng(const int32_t* iid, int64_t m, int32_t n, float* out) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(PT_E_NODEVICE, "no HIP device visible");
    if (m <= 0 || n <= 0) return PT_OK;
    int* d_iid = nullptr;
    float* d_out = nullptr;
    HIPCHK(hipMalloc(&d_iid, sizeof(int) * 3 * m));
    HIPCHK(hipMalloc(&d_out, sizeof(float) * m * n));
    HIPCHK(smemcpy(d_iid, iid, sizeof(int) * 3 * m, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_rng, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, 0, d_iid, (int)m, n, d_out);
    HIPCHK(hipGetLastError());
    HIPCHK(smemcpy(out, d_out, sizeof(float) * m * n, hipMemcpyDeviceToHost));
    (void)hipFree(d_iid);
    (void)hipFree(d_out);
    return PT_OK;
}

int32_t pt_test_pbo(const float* image, int64_t n, int32_t iteration, pt_uchar4* pbo) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(PT_E_NODEVICE, "no HIP device visible");
    if (n <= 0) return PT_OK;
    float* d_img = nullptr;
    pt_uchar4* d_pbo = nullptr;
    HIPCHK(hipMalloc(&d_img, sizeof(float) * 3 * n));
    HIPCHK(hipMalloc(&d_pbo, sizeof(pt_uchar4) * n));
    HIPCHK(smemcpy(d_img, image, sizeof(float) * 3 * n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_to_pbo, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, 0, d_img, d_pbo, (int)n,
                       iteration);
    HIPCHK(hipGetLastError());
    HIPCHK(smemcpy(pbo, d_pbo, sizeof(pt_uchar4) * n, hipMemcpyDeviceToHost));
    (void)hipFree(d_img);
    (void)hipFree(d_pbo);
    return PT_OK;
}

int32_t pt_debug_section_counters(uint64_t* out, int32_t n, int32_t reset) {
    RC(need_init());
    if (!out || n < 0 || n > SEC_SLOTS) return fail(PT_E_INVALID, "bad arguments");
    HIPCHK(hipStreamSynchronize(gp->stream));
    unsigned long long tmp[SEC_SLOTS];
    HIPCHK(hipMemcpyFromSymbolAsync(tmp, HIP_SYMBOL(g_sections), sizeof tmp, 0, hipMemcpyDeviceToHost, gp->stream));
    HIPCHK(hipStreamSynchronize(gp->stream));
    for (int i = 0; i < n; ++i) out[i] = tmp[i];
    if (reset) {
        memset(tmp, 0, sizeof tmp);
        HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_sections), tmp, sizeof tmp, 0, hipMemcpyHostToDevice, gp->stream));
        HIPCHK(hipStreamSynchronize(gp->stream));
    }
    return PT_OK;
}

int32_t pt_profile_frames(int32_t first_iteration, int32_t count, pt_kernel_times* out) {
    RC(need_init());
    RC(need_single("pt_profile_frames"));
    if (!out || count <= 0) return fail(PT_E_INVALID, "bad arguments");
    memset(out, 0, sizeof(*out));
    RC(ensure_frames(pass_frames(count)));
    // the same passes as pt_trace_frames, launched eagerly with per-dispatch start/stop events,
    // no host synchronisation until the end; stream-level events around the whole run
    std::vector<ProfRec> rec;
    std::vector<size_t> pass_start;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    {   // every kernel of every pass gets a start and a stop event, created up front
        const int passes = (count + gp->batch - 1) / gp->batch;
        const size_t need = 2 * (size_t)passes * (size_t)(4 * std::max(1, gp->sc.trace_depth) + 8);
        while (g_prof_pool.size() < need) {
            hipEvent_t e = nullptr;
            HIPCHK(hipEventCreateWithFlags(&e, PROF_EVENT_FLAGS));
            g_prof_pool.push_back(e);
        }
        g_prof_next = 0;
    }
    HIPCHK(hipEventRecord(e0, gp->stream));
    g_prof = &rec;
    int rc = PT_OK;
    for (int i = 0; i < count && rc == PT_OK;) {
        const int f = pass_frames(count - i);
        pass_start.push_back(rec.size());
        rc = enqueue_pass(first_iteration + i, f);
        gp->dev_iter = first_iteration + i;
        gp->frames_done += f;
        gp->last_iter = first_iteration + i + f - 1;
        i += f;
    }
    g_prof = nullptr;
    (void)hipEventRecord(e1, gp->stream);
    hipError_t se = hipStreamSynchronize(gp->stream);
    const int passes = (int)pass_start.size();
    double bounce_ms[MAXB] = {0}, bvh_ms[MAXB] = {0};
    double compact_ms = 0, isect_ms = 0, shade_ms = 0, cam_ms = 0, sort_ms = 0, scan_ms = 0, comb_ms = 0, tail_ms = 0;
    int tail_from = 0;
    float frame_ms = 0;
    if (rc == PT_OK && se == hipSuccess) {
        (void)hipEventElapsedTime(&frame_ms, e0, e1);
        for (int f = 0; f < passes; ++f) {
            size_t a = pass_start[f], b = (f + 1 < passes) ? pass_start[f + 1] : rec.size();
            int bi = 0;
            for (size_t i = a; i < b; ++i) {
                float ms = 0;
                (void)hipEventElapsedTime(&ms, rec[i].start, rec[i].stop);
                int k = rec[i].kind;
                if (k >= 400) { bounce_ms[k - 400] += ms; bvh_ms[k - 400] += ms; }   // k_bvh_tail_trav / _shade
                else if (k >= 300) { tail_ms += ms; tail_from = k - 300; }
                else if (k >= 200) { bounce_ms[k - 200] += ms; bvh_ms[k - 200] += ms; }
                else if (k >= 100) bounce_ms[k - 100] += ms;
                else if (k == 0) cam_ms += ms;
                else if (k == 1) isect_ms += ms;
                else if (k == 2) shade_ms += ms;
                else if (k == 3) { compact_ms += ms; if (bi < MAXB) bounce_ms[bi++] += ms; }
                else if (k == 5) scan_ms += ms;
                else if (k == 4) sort_ms += ms;
                else if (k == 6) comb_ms += ms;
            }
        }
    }
    for (auto e : g_prof_pool) (void)hipEventDestroy(e);
    g_prof_pool.clear();
    g_prof_next = 0;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    RC(rc);
    HIPCHK(se);
    out->frames = count;
    out->passes = passes;
    out->frame_ms = frame_ms / count;
    for (int b = 0; b < MAXB; ++b) {
        out->bounce_ms[b] = (float)(bounce_ms[b] / passes);
        out->bvh_ms[b] = (float)(bvh_ms[b] / passes);
    }
    out->combine_ms = (float)(comb_ms / count);
    out->compact_ms = (float)(compact_ms / count);
    out->intersect_ms = (float)(isect_ms / count);
    out->shade_ms = (float)(shade_ms / count);
    out->camera_ms = (float)(cam_ms / count);
    out->sort_ms = (float)(sort_ms / count);
    out->compact_scan_ms = (float)(scan_ms / count);
    out->tail_ms = (float)(tail_ms / passes);
    out->tail_from = tail_from;
    return PT_OK;
}

}  // extern "C"
