// pt_bvh_build.hip — the reference's host BVH builder (scene.cpp:428-525) on the GPU, producing
// the SAME bvhNodes and triIndices bit for bit (the traversal's exact-t tie
// order depends on that layout, so a different tree would not be a drop-in).
//
// The reference recursion, per node over its triangle range [start, end):
//   bounds   = fold of glm::min / glm::max over v1, v2, v3 of every triangle, in range order
//              (glm 0.9.6: min(x, y) = x < y ? x : y -- ties go to the later element, which
//              decides the sign of a zero bound, and a NaN coordinate resets the fold)
//   leaf     if end - start <= 4
//   axis     from the centroid bounds' extent (y if it beats x and z, then z if it beats x)
//   split    0.5f * (cmin[axis] + cmax[axis])
//   partition: the in-place swap loop `if (c < split) swap(idx[i], idx[mid++])` (Lomuto)
//   median fallback when one side is empty; children: left (preorder next), then right
//
// GPU formulation, level by level (all nodes of one depth at once; a node's range is cut into
// pieces of 4096 triangles, one workgroup per piece, so the top levels fill the chip too):
//   * bounds: each thread folds a contiguous chunk in order into a summary (value, "holds a
//     NaN"), and chunks are joined pairwise in order (stride doubling).  The join is
//     associative, so the result equals the sequential fold, signed zeros and NaNs included;
//   * the swap loop has a closed form.  The k-th "less" element (in range order) lands at
//     start + k.  A "not less" element is moved only by a swap: the one at position p (which
//     is mid at that moment) jumps to the index of the (p - start)-th less element.  So its final
//     slot is the fixed point of J(p) = lessIdx[p - start] for p < start + nLess, J(p) = p
//     beyond -- resolved by grid-wide pointer jumping (ceil(log2 len) + 1 rounds).  (Checked against the loop itself on 20k random
//     sequences while deriving it; the GPU result is checked against host/scene.cpp's
//     sequential builder in tests/test_gpu_parity.py::test_gpu_bvh_build_bitexact.)
//   * node numbering is the reference's preorder; it needs the subtree sizes, so the host keeps
//     the (small) tree skeleton, one download per level, and numbers the nodes at the end;
//   * a node of at most SUBT triangles is not split by the levels: it becomes a subtree root, and
//     k_subtree finishes every such subtree (one wave each, LDS-resident) in a single launch.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <chrono>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "pt/pathtrace_abi.h"

namespace {

constexpr int BT = 256;   // threads per workgroup

// glm 0.9.6 (func_common.inl:409-435): min(x, y) = x < y ? x : y, max(x, y) = x > y ? x : y.
// Folded as acc = min(acc, v): ties go to the LATER element (the sign of a zero bound), and a
// NaN element replaces the running value, which the next element then replaces in turn.
__device__ __forceinline__ float glm_min(float acc, float v) { return acc < v ? acc : v; }
__device__ __forceinline__ float glm_max(float acc, float v) { return acc > v ? acc : v; }

// summary of folding one contiguous run of elements, combinable in order:
//   empty       no element yet
//   reset       the run holds a NaN: its result no longer depends on what came before it
//   val         the fold of the run (from its first element, or from after its last NaN)
struct Fold {
    float val;
    int flags;   // bit 0: empty, bit 1: reset
};
template <bool MIN>
__device__ __forceinline__ void fold_push(Fold& f, float v) {
    if (f.flags & 1) f.val = v;
    else f.val = MIN ? glm_min(f.val, v) : glm_max(f.val, v);
    f.flags = (f.flags & ~1) | (v != v ? 2 : 0) | (f.flags & 2);
}
template <bool MIN>
__device__ __forceinline__ Fold fold_join(Fold a, Fold b) {   // a precedes b
    if (b.flags & 1) return a;
    if (a.flags & 1) return b;
    if (b.flags & 2) return b;
    return Fold{MIN ? glm_min(a.val, b.val) : glm_max(a.val, b.val), a.flags};
}
// the reference's fold starts from AABB's default FLT_MAX / -FLT_MAX (sceneStructs.h:91-92)
template <bool MIN>
__device__ __forceinline__ float fold_final(Fold f) {
    const float init = MIN ? FLT_MAX : -FLT_MAX;
    if (f.flags & 1) return init;
    if (f.flags & 2) return f.val;
    return MIN ? glm_min(init, f.val) : glm_max(init, f.val);
}

__device__ __forceinline__ const float* tri_f(const pt_triangle* t, int i) {
    return reinterpret_cast<const float*>(t + i);
}
// float offsets inside pt_triangle (scene_structs.h): v1.position 1, v2.position 10, v3.position 19, centroid 27
constexpr int OFF_V[3] = {1, 10, 19};
constexpr int OFF_C = 27;

// ---- level kernels.  A node's triangle range is cut into pieces of up to PIECE elements, so a
// large node (the top levels) is spread over many workgroups. ----
constexpr int PIECE = 4096;

struct Piece {
    int seg;              // index of the node (segment) in this level's list
    int start, end;       // element range of the piece
};

__device__ __forceinline__ bool is_min_comp(int k) { return k < 3 || (k >= 6 && k < 9); }

// fold of one piece (12 components: node min.xyz max.xyz, centroid min.xyz max.xyz), threads fold
// contiguous sub-ranges in order, then join in order
__global__ __launch_bounds__(BT) void k_piece_fold(const pt_triangle* __restrict__ tris, const int* __restrict__ idx,
                                                   const Piece* __restrict__ pieces, float* __restrict__ pv,
                                                   int* __restrict__ pf) {
    __shared__ float rv[12][BT];
    __shared__ int rf[12][BT];
    const Piece pc = pieces[blockIdx.x];
    const int len = pc.end - pc.start;
    const int chunk = (len + BT - 1) / BT;
    const int a = pc.start + threadIdx.x * chunk;
    const int b = min(pc.end, a + chunk);
    Fold f[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) f[k] = Fold{0.f, 1};
    for (int i = a; i < b; ++i) {
        const float* t = tri_f(tris, idx[i]);
        // UpdateNodeBounds: per component, min / max over v1, v2, v3 of each triangle in order
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                fold_push<true>(f[k], t[OFF_V[q] + k]);
                fold_push<false>(f[3 + k], t[OFF_V[q] + k]);
            }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            fold_push<true>(f[6 + k], t[OFF_C + k]);
            fold_push<false>(f[9 + k], t[OFF_C + k]);
        }
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        rv[k][threadIdx.x] = f[k].val;
        rf[k][threadIdx.x] = f[k].flags;
    }
    __syncthreads();
    // in-order pairwise join: slot i covers sub-ranges [i, i + 2s) after the step of stride s
    for (int s = 1; s < BT; s <<= 1) {
        const int i = threadIdx.x;
        if ((i & (2 * s - 1)) == 0) {
#pragma unroll
            for (int k = 0; k < 12; ++k) {
                const Fold x{rv[k][i], rf[k][i]}, y{rv[k][i + s], rf[k][i + s]};
                const Fold z = is_min_comp(k) ? fold_join<true>(x, y) : fold_join<false>(x, y);
                rv[k][i] = z.val;
                rf[k][i] = z.flags;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 12) {
        pv[12 * blockIdx.x + threadIdx.x] = rv[threadIdx.x][0];
        pf[12 * blockIdx.x + threadIdx.x] = rf[threadIdx.x][0];
    }
}

// join the pieces of each node in order and apply the fold's FLT_MAX / -FLT_MAX start
__global__ void k_seg_fold(const int* __restrict__ first_piece, const float* __restrict__ pv,
                           const int* __restrict__ pf, float* __restrict__ out, int nseg) {
    const int s = blockIdx.x * 4 + (threadIdx.x >> 4), k = threadIdx.x & 15;
    if (s >= nseg || k >= 12) return;
    Fold z{0.f, 1};
    for (int p = first_piece[s]; p < first_piece[s + 1]; ++p) {
        const Fold y{pv[12 * p + k], pf[12 * p + k]};
        z = is_min_comp(k) ? fold_join<true>(z, y) : fold_join<false>(z, y);
    }
    out[12 * s + k] = is_min_comp(k) ? fold_final<true>(z) : fold_final<false>(z);
}

struct Split {
    int axis;
    float split;
};

// the swap partition, step 1: per piece of a split node, flag the "less" elements and count them
__global__ __launch_bounds__(BT) void k_piece_count(const pt_triangle* __restrict__ tris, const int* __restrict__ idx,
                                                    const Piece* __restrict__ pieces, const Split* __restrict__ splits,
                                                    unsigned char* __restrict__ less, int* __restrict__ cnt) {
    __shared__ int red[BT];
    const Piece pc = pieces[blockIdx.x];
    const Split sp = splits[pc.seg];
    int c = 0;
    for (int p = pc.start + (int)threadIdx.x; p < pc.end; p += BT) {
        const bool l = tri_f(tris, idx[p])[OFF_C + sp.axis] < sp.split;
        less[p] = l ? 1 : 0;
        c += l ? 1 : 0;
    }
    red[threadIdx.x] = c;
    __syncthreads();
    for (int s = BT / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) cnt[blockIdx.x] = red[0];
}

// step 2: per split node, the exclusive scan of its pieces' counts (pieces of a node are
// consecutive) and the node's "less" total
__global__ void k_seg_scan(const int* __restrict__ first_piece, int* __restrict__ cnt_to_off, int* __restrict__ nless,
                           int nseg) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    int run = 0;
    for (int p = first_piece[s]; p < first_piece[s + 1]; ++p) {
        const int c = cnt_to_off[p];
        cnt_to_off[p] = run;
        run += c;
    }
    nless[s] = run;
}

// step 3: the k-th "less" element of the node lands at start + k; J[start + k] = its position
// (the slot the "not less" element sitting at start + k is swapped out to)
__global__ __launch_bounds__(BT) void k_piece_place(const int* __restrict__ idx_in, int* __restrict__ idx_out,
                                                    const Piece* __restrict__ pieces, const int* __restrict__ seg_start,
                                                    const unsigned char* __restrict__ less, const int* __restrict__ off,
                                                    int* __restrict__ J) {
    __shared__ int scan[BT];
    const Piece pc = pieces[blockIdx.x];
    const int len = pc.end - pc.start;
    const int chunk = (len + BT - 1) / BT;
    const int a = pc.start + threadIdx.x * chunk;
    const int b = min(pc.end, a + chunk);
    int c = 0;
    for (int i = a; i < b; ++i) c += less[i];
    scan[threadIdx.x] = c;
    __syncthreads();
    for (int s = 1; s < BT; s <<= 1) {   // inclusive Hillis-Steele scan
        const int x = (int)threadIdx.x >= s ? scan[threadIdx.x - s] : 0;
        __syncthreads();
        scan[threadIdx.x] += x;
        __syncthreads();
    }
    int r = seg_start[pc.seg] + off[blockIdx.x] + scan[threadIdx.x] - c;
    for (int i = a; i < b; ++i)
        if (less[i]) {
            idx_out[r] = idx_in[i];
            J[r] = i;
            ++r;
        }
}

__global__ void k_fill(int* __restrict__ J, unsigned char* __restrict__ less, int n) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) {
        J[p] = p;
        less[p] = 0;
    }
}
// the chain J(p) = position of the (p - start)-th less element, for p < start + nless; J(p) = p
// beyond.  Positions rise along a chain, so ceil(log2 len) + 1 jumping rounds reach the ends.
__global__ void k_jump(const int* __restrict__ J, int* __restrict__ Jn, int n) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) Jn[p] = J[J[p]];
}
// every "not less" element (and every element of a leaf) goes to the end of its chain
__global__ void k_scatter_rest(const int* __restrict__ idx_in, int* __restrict__ idx_out, const int* __restrict__ J,
                               const unsigned char* __restrict__ less, int n) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n && !less[p]) idx_out[J[p]] = idx_in[p];
}

// split decisions (scene.cpp:484-499) on the device, one thread per node of the level: the axis from
// the centroid extent, the midpoint; the node's bounds are kept for the host's node records (allb),
// its range start for the partition kernels
__global__ void k_split(const float* __restrict__ bounds, const Piece* __restrict__ pieces, const int* __restrict__ first,
                        Split* __restrict__ splits, int* __restrict__ sstart, float* __restrict__ allb, int nseg) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nseg) return;
    const float* b = bounds + 12 * (size_t)k;
    const float ex = b[9] - b[6], ey = b[10] - b[7], ez = b[11] - b[8];
    int axis = 0;
    if (ey > ex && ey > ez) axis = 1;
    if (ez > ex) axis = 2;
    splits[k] = Split{axis, 0.5f * (b[6 + axis] + b[9 + axis])};
    sstart[k] = pieces[first[k]].start;
    for (int c = 0; c < 6; ++c) allb[6 * (size_t)k + c] = b[c];
}

// the swap partition of a node that fits one workgroup (<= PIECE triangles: every node of the lower
// levels), in place: the less elements' ranks by a block scan of contiguous chunks, the not-less
// elements' chains by in-place pointer jumping in LDS
__global__ __launch_bounds__(BT) void k_node_partition(const pt_triangle* __restrict__ tris, int* __restrict__ idx,
                                                       const Piece* __restrict__ pieces, const Split* __restrict__ splits,
                                                       int* __restrict__ nless) {
    __shared__ int sidx[PIECE];
    __shared__ int sout[PIECE];
    __shared__ short J[PIECE];
    __shared__ int scan[BT];
    const Piece pc = pieces[blockIdx.x];   // one piece = the whole node
    const Split sp = splits[blockIdx.x];
    const int len = pc.end - pc.start;
    const int tid = threadIdx.x;
    for (int i = tid; i < len; i += BT) {
        sidx[i] = idx[pc.start + i];
        J[i] = (short)i;
    }
    __syncthreads();
    const int chunk = (len + BT - 1) / BT;
    const int a = tid * chunk, b = min(len, a + chunk);
    int c = 0;
    for (int i = a; i < b; ++i) c += tri_f(tris, sidx[i])[OFF_C + sp.axis] < sp.split ? 1 : 0;
    scan[tid] = c;
    __syncthreads();
    for (int d = 1; d < BT; d <<= 1) {   // inclusive Hillis-Steele scan
        const int x = tid >= d ? scan[tid - d] : 0;
        __syncthreads();
        scan[tid] += x;
        __syncthreads();
    }
    int rank = scan[tid] - c;
    for (int i = a; i < b; ++i)
        if (tri_f(tris, sidx[i])[OFF_C + sp.axis] < sp.split) {   // the k-th less element lands at k; the
            sout[rank] = sidx[i];                                 // not-less element at k jumps to i
            J[rank] = (short)i;
            ++rank;
        }
    __syncthreads();
    while (true) {
        int changed = 0;
        for (int i = tid; i < len; i += BT) {
            const int j = J[i], jj = J[j];
            if (jj != j) {
                J[i] = (short)jj;
                changed = 1;
            }
        }
        if (!__syncthreads_or(changed)) break;
    }
    for (int i = a; i < b; ++i)
        if (!(tri_f(tris, sidx[i])[OFF_C + sp.axis] < sp.split)) sout[J[i]] = sidx[i];
    __syncthreads();
    for (int i = tid; i < len; i += BT) idx[pc.start + i] = sout[i];
    if (tid == 0) nless[blockIdx.x] = scan[BT - 1];
}

// ---- subtrees: a node of <= SUBT triangles is finished, with every node below it, in one launch
// (the level loop above would spend ~10 more levels of launches and host round trips on them), one
// wave per subtree root, its triangles' vertices and centroids staged in LDS:
//   1. the wave walks the nodes of more than SMALLT triangles depth-first, all 64 lanes on one node:
//      the bounds fold (lanes fold contiguous chunks in order, joined in lane order), the split
//      decision, and the swap partition in closed form (the less elements' ranks by an in-order
//      scan, the chains of the not-less elements by in-place pointer jumping in LDS);
//   2. each node of at most SMALLT triangles below them is a small subtree, built by ONE lane with
//      the reference's own sequential loops (many small subtrees at once, one per lane);
//   3. lane 0 numbers the whole subtree in the reference's preorder (the large nodes' skeleton,
//      each small subtree a block of its size), and the records are written in place. ----
constexpr int SUBT = 512;
constexpr int SMALLT = 48;
constexpr int SUB_LANES = 64;

struct SubRoot {
    int start, end;       // triangle range (positions in idx)
    int out;              // first slot of its output nodes (at most 2 (end - start) - 1)
};
struct SubLds {
    float e[12][SUBT];               // per local element: v1.xyz v2.xyz v3.xyz centroid.xyz
    int tri[SUBT];                   // local element -> triangle index
    unsigned short pos[SUBT];        // position (relative to the subtree start) -> local element
    unsigned short tmp[SUBT];        // partition scratch
    short jump[SUBT];                // partition chains
    short stk[SUBT][4];              // large nodes pending as right children: start, end, parent
    short bl[SUBT], br[SUBT];        // large node -> children: >= 0 large node, < 0: -(small + 1)
    short bfinal[SUBT];              // large node -> preorder id
    short ss[SUBT], st[SUBT];        // small subtree -> element range
    short ssize[SUBT], sbase[SUBT];  // small subtree -> node count, preorder id of its root
    short lstk[SUB_LANES][SMALLT][3];   // per-lane stacks of the small builds
};

__device__ __forceinline__ Fold shfl_fold(Fold f, int src_delta) {
    Fold o;
    o.val = __shfl_down(f.val, src_delta, SUB_LANES);
    o.flags = __shfl_down(f.flags, src_delta, SUB_LANES);
    return o;
}

// in-order join of the lanes' folds (lane i joins lane i + d, d = 1, 2, 4, ...), finished with the
// reference's FLT_MAX / -FLT_MAX start and broadcast from lane 0
__device__ __forceinline__ void sub_fold_join(Fold (&f)[12], int lane, float (&fin)[12]) {
    for (int d = 1; d < SUB_LANES; d <<= 1) {
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            const Fold y = shfl_fold(f[k], d);
            if ((lane & (2 * d - 1)) == 0 && lane + d < SUB_LANES)
                f[k] = is_min_comp(k) ? fold_join<true>(f[k], y) : fold_join<false>(f[k], y);
        }
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const float v = is_min_comp(k) ? fold_final<true>(f[k]) : fold_final<false>(f[k]);
        fin[k] = __shfl(v, 0, SUB_LANES);
    }
}
// scene.cpp:484-499: the split axis from the centroid extent (y if it beats x and z, then z if it beats x)
__device__ __forceinline__ int sub_axis(float ex, float ey, float ez) {
    int axis = 0;
    if (ey > ex && ey > ez) axis = 1;
    if (ez > ex) axis = 2;
    return axis;
}

__global__ __launch_bounds__(SUB_LANES) void k_subtree(const pt_triangle* __restrict__ tris, int* __restrict__ idx,
                                                      const SubRoot* __restrict__ roots, pt_bvh_node* __restrict__ out,
                                                      pt_bvh_node* __restrict__ scratch, int* __restrict__ out_count) {
    extern __shared__ float4 sub_smem[];
    SubLds& L = *reinterpret_cast<SubLds*>(sub_smem);
    const SubRoot r = roots[blockIdx.x];
    const int m = r.end - r.start;
    const int lane = threadIdx.x;
    for (int e = lane; e < m; e += SUB_LANES) {
        const int ti = idx[r.start + e];
        const float* t = tri_f(tris, ti);
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int k = 0; k < 3; ++k) L.e[3 * q + k][e] = t[OFF_V[q] + k];
#pragma unroll
        for (int k = 0; k < 3; ++k) L.e[9 + k][e] = t[OFF_C + k];
        L.tri[e] = ti;
        L.pos[e] = (unsigned short)e;
    }
    __syncthreads();
    // scratch: 3 slots per triangle -- the large nodes' records (at most m) at 3 start, then room for
    // 2 (t - s) - 1 records of each small subtree [s, t) at 3 start + m + 2 s
    pt_bvh_node* big = scratch + 3 * (size_t)r.start;
    pt_bvh_node* smallrec = big + m;
    // ---- 1. the large nodes, depth-first, the whole wave on each ----
    int nb = 0, ns = 0;
    if (m <= SMALLT) {
        if (lane == 0) {
            L.ss[0] = 0;
            L.st[0] = (short)m;
        }
        ns = 1;
    } else {
        int sp = 0, s = 0, t = m, parent = -1, side = 0;
        while (true) {
            const int id = nb++;
            if (parent >= 0 && lane == 0) (side ? L.br : L.bl)[parent] = (short)id;
            const int len = t - s;
            const int chunk = (len + SUB_LANES - 1) / SUB_LANES;
            const int a = s + lane * chunk, b = min(t, a + chunk);
            Fold f[12];
#pragma unroll
            for (int k = 0; k < 12; ++k) f[k] = Fold{0.f, 1};
            for (int p = a; p < b; ++p) {
                const int e = L.pos[p];
#pragma unroll
                for (int q = 0; q < 3; ++q)
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        fold_push<true>(f[k], L.e[3 * q + k][e]);
                        fold_push<false>(f[3 + k], L.e[3 * q + k][e]);
                    }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    fold_push<true>(f[6 + k], L.e[9 + k][e]);
                    fold_push<false>(f[9 + k], L.e[9 + k][e]);
                }
            }
            float fin[12];
            sub_fold_join(f, lane, fin);
            if (lane == 0) {
                pt_bvh_node& nd = big[id];
                nd.aabb.min = pt_vec3{fin[0], fin[1], fin[2]};
                nd.aabb.max = pt_vec3{fin[3], fin[4], fin[5]};
                nd.left = -1;
                nd.right = -1;
                nd.start = -1;
                nd.triCount = 0;
            }
            const int axis = sub_axis(fin[9] - fin[6], fin[10] - fin[7], fin[11] - fin[8]);
            const float cmin = axis == 0 ? fin[6] : axis == 1 ? fin[7] : fin[8];
            const float cmax = axis == 0 ? fin[9] : axis == 1 ? fin[10] : fin[11];
            const float split = 0.5f * (cmin + cmax);
            const float* cen = L.e[9 + axis];
            // ranks of the less elements in position order: per-lane counts of its chunk, then an
            // exclusive scan over the lanes
            int c = 0;
            for (int p = a; p < b; ++p) c += cen[L.pos[p]] < split ? 1 : 0;
            int incl = c;
            for (int d = 1; d < SUB_LANES; d <<= 1) {
                const int y = __shfl_up(incl, d, SUB_LANES);
                if (lane >= d) incl += y;
            }
            const int nless = __shfl(incl, SUB_LANES - 1, SUB_LANES);
            for (int p = s + lane; p < t; p += SUB_LANES) L.jump[p] = (short)p;
            __syncthreads();
            int rank = incl - c;
            for (int p = a; p < b; ++p) {
                const int e = L.pos[p];
                if (cen[e] < split) {   // the k-th less element lands at s + k; the not-less element
                    L.tmp[s + rank] = (unsigned short)e;   // sitting at s + k jumps to its position p
                    L.jump[s + rank] = (short)p;
                    ++rank;
                }
            }
            __syncthreads();
            // chains: a not-less element at p ends at the fixed point of jump (positions rise along it)
            while (true) {
                bool changed = false;
                for (int p = s + lane; p < t; p += SUB_LANES) {
                    const int j = L.jump[p], jj = L.jump[j];
                    if (jj != j) {
                        L.jump[p] = (short)jj;
                        changed = true;
                    }
                }
                __syncthreads();
                if (!__any(changed)) break;
            }
            for (int p = s + lane; p < t; p += SUB_LANES) {
                const int e = L.pos[p];
                if (!(cen[e] < split)) L.tmp[L.jump[p]] = (unsigned short)e;
            }
            __syncthreads();
            for (int p = s + lane; p < t; p += SUB_LANES) L.pos[p] = L.tmp[p];
            int mid = s + nless;
            if (mid == s || mid == t) mid = (s + t) / 2;   // scene.cpp:513-515
            // children: a small one is deferred to step 2, a large right one waits on the stack
            if (t - mid <= SMALLT) {
                if (lane == 0) {
                    L.ss[ns] = (short)mid;
                    L.st[ns] = (short)t;
                    L.br[id] = (short)-(ns + 1);
                }
                ++ns;
            } else {
                if (lane == 0) {
                    L.stk[sp][0] = (short)mid;
                    L.stk[sp][1] = (short)t;
                    L.stk[sp][2] = (short)id;
                }
                ++sp;
            }
            if (mid - s <= SMALLT) {
                if (lane == 0) {
                    L.ss[ns] = (short)s;
                    L.st[ns] = (short)mid;
                    L.bl[id] = (short)-(ns + 1);
                }
                ++ns;
            } else {
                t = mid;
                parent = id;
                side = 0;
                __syncthreads();
                continue;
            }
            __syncthreads();
            if (sp == 0) break;
            --sp;
            s = L.stk[sp][0];
            t = L.stk[sp][1];
            parent = L.stk[sp][2];
            side = 1;
            __syncthreads();
        }
    }
    __syncthreads();
    // ---- 2. small subtrees: one lane each, the reference's recursion (scene.cpp:459-525) verbatim ----
    for (int k = lane; k < ns; k += SUB_LANES) {
        const int s0 = L.ss[k], t0 = L.st[k];
        pt_bvh_node* rec = smallrec + 2 * s0;   // room for 2 (t0 - s0) - 1 nodes
        int cnt = 0, sp = 0, s = s0, t = t0, parent = -1;
        while (true) {
            const int id = cnt++;
            if (parent >= 0) rec[parent].right = id;
            float bmin[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, bmax[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
            for (int p = s; p < t; ++p) {   // UpdateNodeBounds
                const int e = L.pos[p];
#pragma unroll
                for (int q = 0; q < 3; ++q)
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        bmin[c] = glm_min(bmin[c], L.e[3 * q + c][e]);
                        bmax[c] = glm_max(bmax[c], L.e[3 * q + c][e]);
                    }
            }
            pt_bvh_node nd;
            nd.aabb.min = pt_vec3{bmin[0], bmin[1], bmin[2]};
            nd.aabb.max = pt_vec3{bmax[0], bmax[1], bmax[2]};
            nd.left = -1;
            nd.right = -1;
            const int len = t - s;
            if (len <= 4) {
                nd.start = r.start + s;
                nd.triCount = len;
                rec[id] = nd;
                if (sp == 0) break;
                --sp;
                s = L.lstk[lane][sp][0];
                t = L.lstk[lane][sp][1];
                parent = L.lstk[lane][sp][2];
                continue;
            }
            float cmin[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, cmax[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
            for (int p = s; p < t; ++p) {
                const int e = L.pos[p];
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    cmin[c] = glm_min(cmin[c], L.e[9 + c][e]);
                    cmax[c] = glm_max(cmax[c], L.e[9 + c][e]);
                }
            }
            const int axis = sub_axis(cmax[0] - cmin[0], cmax[1] - cmin[1], cmax[2] - cmin[2]);
            const float split = 0.5f * (cmin[axis] + cmax[axis]);
            const float* cen = L.e[9 + axis];
            int mid = s;
            for (int p = s; p < t; ++p) {   // the swap loop
                const int e = L.pos[p];
                if (cen[e] < split) {
                    L.pos[p] = L.pos[mid];
                    L.pos[mid] = (unsigned short)e;
                    ++mid;
                }
            }
            if (mid == s || mid == t) mid = (s + t) / 2;
            nd.left = id + 1;
            nd.start = -1;
            nd.triCount = 0;
            rec[id] = nd;
            L.lstk[lane][sp][0] = (short)mid;
            L.lstk[lane][sp][1] = (short)t;
            L.lstk[lane][sp][2] = (short)id;
            ++sp;
            t = mid;
            parent = -1;
        }
        L.ssize[k] = (short)cnt;
    }
    __syncthreads();
    // ---- 3. preorder numbering (lane 0): the large skeleton depth-first, a small subtree a block ----
    if (lane == 0) {
        int f = 0;
        if (nb == 0) {
            L.sbase[0] = 0;
            f = L.ssize[0];
        } else {
            int sp = 0, code = 0;
            while (true) {
                if (code >= 0) {
                    L.bfinal[code] = (short)f++;
                    L.stk[sp][0] = L.br[code];   // right after the left subtree
                    ++sp;
                    code = L.bl[code];
                    continue;
                }
                const int k = -code - 1;
                L.sbase[k] = (short)f;
                f += L.ssize[k];
                if (sp == 0) break;
                code = L.stk[--sp][0];
            }
        }
        out_count[blockIdx.x] = f;
    }
    __syncthreads();
    // ---- 4. records at their preorder ids, children relocated ----
    pt_bvh_node* o = out + r.out;
    for (int b = lane; b < nb; b += SUB_LANES) {
        pt_bvh_node nd = big[b];
        const int cl = L.bl[b], cr = L.br[b];
        nd.left = cl >= 0 ? L.bfinal[cl] : L.sbase[-cl - 1];
        nd.right = cr >= 0 ? L.bfinal[cr] : L.sbase[-cr - 1];
        o[L.bfinal[b]] = nd;
    }
    for (int k = 0; k < ns; ++k) {
        const int base = L.sbase[k], n = L.ssize[k];
        const pt_bvh_node* rec = smallrec + 2 * L.ss[k];
        for (int i = lane; i < n; i += SUB_LANES) {
            pt_bvh_node nd = rec[i];
            if (nd.left >= 0) nd.left += base;
            if (nd.right >= 0) nd.right += base;
            o[base + i] = nd;
        }
    }
    for (int p = lane; p < m; p += SUB_LANES) idx[r.start + p] = L.tri[L.pos[p]];
}

std::string g_err;

#define BCHK(x)                                                                            \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            g_err = std::string(#x) + ": " + hipGetErrorString(e_);                           \
            rc = PT_E_HIP;                                                                   \
            goto done;                                                                       \
        }                                                                                    \
    } while (0)

struct TreeNode {   // host skeleton, breadth-first
    int start, end;
    int left = -1, right = -1;   // skeleton indices
    float b[6];                  // node bounds
};

}  // namespace

extern "C" const char* pt_bvh_build_last_error(void) { return g_err.c_str(); }

// scene.cpp:445-525 on the current HIP device.  nodes: capacity 2n - 1 (a binary tree whose
// leaves hold >= 1 triangle); *num_nodes receives the count.  tri_indices: n entries.
// Nodes of more than SUBT triangles are split level by level (all nodes of a level at once, pieces
// of PIECE triangles per workgroup); every node of at most SUBT triangles becomes a subtree root,
// finished with its whole subtree by k_subtree in one launch after the levels.
extern "C" int32_t pt_bvh_build(const pt_triangle* tris, int32_t n, pt_bvh_node* nodes, int32_t cap,
                                int32_t* num_nodes, int32_t* tri_indices) {
    int32_t rc = PT_OK;
    pt_triangle* d_tris = nullptr;
    int *d_idx = nullptr, *d_idx2 = nullptr, *d_J = nullptr, *d_Jn = nullptr;
    unsigned char* d_less = nullptr;
    // per-level scratch, grown on demand
    Piece* d_pieces = nullptr;
    int *d_first = nullptr, *d_pf = nullptr, *d_cnt = nullptr, *d_nless = nullptr, *d_sstart = nullptr;
    float *d_pv = nullptr, *d_bounds = nullptr;
    Split* d_splits = nullptr;
    SubRoot* d_subs = nullptr;
    pt_bvh_node* d_subnodes = nullptr;
    pt_bvh_node* d_subscratch = nullptr;
    int* d_lvl = nullptr;        // one level's pieces + first-piece table
    size_t lvl_cap = 0;
    float* d_allb = nullptr;     // bounds (6 floats) of every node the level loop split, in level order
    size_t allb_cap = 0, allb_used = 0;
    std::vector<int> lvl_nodes;  // their skeleton indices, same order
    int* d_subcount = nullptr;
    size_t piece_cap = 0, seg_cap = 0;
    const bool timing = getenv("PT_BVH_TIMING") != nullptr;   // per-level times on stderr (tools)
    auto clk = [] { return std::chrono::steady_clock::now(); };
    std::chrono::steady_clock::time_point t_start = clk();
    int dev_count = 0;
    std::vector<TreeNode> tree;
    std::vector<int> level;   // skeleton indices of the current level's nodes of > SUBT triangles
    std::vector<int> sub_of;  // skeleton index -> subtree number (-1: split by the level loop)
    std::vector<SubRoot> subs;
    std::vector<int> sub_node;   // subtree number -> skeleton index
    std::vector<int> pre;
    const unsigned gn = (unsigned)((n + BT - 1) / BT);
    if (n < 0 || !num_nodes || (n > 0 && (!tris || !nodes || !tri_indices))) {
        g_err = "bad arguments";
        return PT_E_INVALID;
    }
    *num_nodes = 0;
    if (n == 0) return PT_OK;   // buildBVH returns before the recursion (scene.cpp:451)
    if (cap < 2 * n - 1) {
        g_err = "node capacity must be >= 2 n - 1";
        return PT_E_INVALID;
    }
    if (hipGetDeviceCount(&dev_count) != hipSuccess || dev_count <= 0) {
        (void)hipGetLastError();
        g_err = "no HIP device visible";
        return PT_E_NODEVICE;
    }
    BCHK(hipMalloc(&d_tris, sizeof(pt_triangle) * (size_t)n));
    BCHK(hipMalloc(&d_idx, sizeof(int) * (size_t)n));
    BCHK(hipMalloc(&d_idx2, sizeof(int) * (size_t)n));
    BCHK(hipMalloc(&d_J, sizeof(int) * (size_t)n));
    BCHK(hipMalloc(&d_Jn, sizeof(int) * (size_t)n));
    BCHK(hipMalloc(&d_less, (size_t)n));
    BCHK(hipMemcpy(d_tris, tris, sizeof(pt_triangle) * (size_t)n, hipMemcpyHostToDevice));
    {
        std::vector<int> iota(n);
        for (int i = 0; i < n; ++i) iota[i] = i;
        BCHK(hipMemcpy(d_idx, iota.data(), sizeof(int) * (size_t)n, hipMemcpyHostToDevice));
    }
    tree.reserve(2 * (size_t)n);
    t_start = clk();
    {   // a node enters the level loop or, at most SUBT triangles, becomes a subtree root
        int outs = 0;
        auto add = [&](int st, int en) {
            const int ti = (int)tree.size();
            tree.push_back(TreeNode{st, en});
            sub_of.push_back(-1);
            if (en - st <= SUBT) {
                sub_of[ti] = (int)subs.size();
                subs.push_back(SubRoot{st, en, outs});
                sub_node.push_back(ti);
                outs += 2 * (en - st) - 1;
            } else {
                level.push_back(ti);
            }
            return ti;
        };
        add(0, n);
        while (!level.empty()) {
            auto t_lv = clk();
            const int S = (int)level.size();
            std::vector<Piece> pieces;
            std::vector<int> first(S + 1);
            for (int k = 0; k < S; ++k) {
                first[k] = (int)pieces.size();
                const TreeNode& t = tree[level[k]];
                for (int a = t.start; a < t.end; a += PIECE) pieces.push_back(Piece{k, a, std::min(t.end, a + PIECE)});
            }
            first[S] = (int)pieces.size();
            if (pieces.size() > piece_cap) {
                (void)hipFree(d_pv);
                (void)hipFree(d_pf);
                (void)hipFree(d_cnt);
                d_pv = nullptr;
                d_pf = nullptr;
                d_cnt = nullptr;
                piece_cap = std::max(pieces.size(), 2 * piece_cap);
                BCHK(hipMalloc(&d_pv, sizeof(float) * 12 * piece_cap));
                BCHK(hipMalloc(&d_pf, sizeof(int) * 12 * piece_cap));
                BCHK(hipMalloc(&d_cnt, sizeof(int) * piece_cap));
            }
            if ((size_t)S + 1 > seg_cap) {
                (void)hipFree(d_bounds);
                (void)hipFree(d_nless);
                (void)hipFree(d_sstart);
                (void)hipFree(d_splits);
                d_bounds = nullptr;
                d_nless = nullptr;
                d_sstart = nullptr;
                d_splits = nullptr;
                seg_cap = std::max<size_t>(S + 1, 2 * seg_cap);
                BCHK(hipMalloc(&d_bounds, sizeof(float) * 12 * seg_cap));
                BCHK(hipMalloc(&d_nless, sizeof(int) * seg_cap));
                BCHK(hipMalloc(&d_sstart, sizeof(int) * seg_cap));
                BCHK(hipMalloc(&d_splits, sizeof(Split) * seg_cap));
            }
            {   // pieces and per-node first piece in one upload
                std::vector<int> up(3 * pieces.size() + S + 1);
                memcpy(up.data(), pieces.data(), sizeof(Piece) * pieces.size());
                memcpy(up.data() + 3 * pieces.size(), first.data(), sizeof(int) * (S + 1));
                if (up.size() > lvl_cap) {
                    (void)hipFree(d_lvl);
                    d_lvl = nullptr;
                    lvl_cap = std::max(up.size(), 2 * lvl_cap);
                    BCHK(hipMalloc(&d_lvl, sizeof(int) * lvl_cap));
                }
                BCHK(hipMemcpy(d_lvl, up.data(), sizeof(int) * up.size(), hipMemcpyHostToDevice));
                d_pieces = reinterpret_cast<Piece*>(d_lvl);
                d_first = d_lvl + 3 * pieces.size();
            }
            if (allb_used + S > allb_cap) {   // node bounds of every level, downloaded once at the end
                float* nb = nullptr;
                const size_t cap2 = std::max<size_t>(allb_used + S, 2 * allb_cap);
                BCHK(hipMalloc(&nb, sizeof(float) * 6 * cap2));
                if (allb_used) BCHK(hipMemcpy(nb, d_allb, sizeof(float) * 6 * allb_used, hipMemcpyDeviceToDevice));
                (void)hipFree(d_allb);
                d_allb = nb;
                allb_cap = cap2;
            }
            hipLaunchKernelGGL(k_piece_fold, dim3((unsigned)pieces.size()), dim3(BT), 0, 0, d_tris, d_idx, d_pieces,
                               d_pv, d_pf);
            hipLaunchKernelGGL(k_seg_fold, dim3((unsigned)((S + 3) / 4)), dim3(64), 0, 0, d_first, d_pv, d_pf, d_bounds,
                               S);
            hipLaunchKernelGGL(k_split, dim3((unsigned)((S + 63) / 64)), dim3(64), 0, 0, d_bounds, d_pieces, d_first,
                               d_splits, d_sstart, d_allb + 6 * allb_used, S);
            BCHK(hipGetLastError());
            int maxlen = 0;
            for (int k = 0; k < S; ++k) {
                lvl_nodes.push_back(level[k]);
                maxlen = std::max(maxlen, tree[level[k]].end - tree[level[k]].start);
            }
            allb_used += S;
            const unsigned np = (unsigned)pieces.size();
            const bool local = maxlen <= PIECE;   // every node of the level fits one workgroup
            if (local) {
                hipLaunchKernelGGL(k_node_partition, dim3(np), dim3(BT), 0, 0, d_tris, d_idx, d_pieces, d_splits, d_nless);
            } else {
                hipLaunchKernelGGL(k_fill, dim3(gn), dim3(BT), 0, 0, d_J, d_less, n);
                hipLaunchKernelGGL(k_piece_count, dim3(np), dim3(BT), 0, 0, d_tris, d_idx, d_pieces, d_splits, d_less,
                                   d_cnt);
                hipLaunchKernelGGL(k_seg_scan, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, 0, d_first, d_cnt,
                                   d_nless, S);
                hipLaunchKernelGGL(k_piece_place, dim3(np), dim3(BT), 0, 0, d_idx, d_idx2, d_pieces, d_sstart, d_less,
                                   d_cnt, d_J);
                int rounds = 1;
                while ((1 << (rounds - 1)) < maxlen) ++rounds;   // ceil(log2 maxlen) + 1
                for (int r = 0; r < rounds; ++r) {
                    hipLaunchKernelGGL(k_jump, dim3(gn), dim3(BT), 0, 0, d_J, d_Jn, n);
                    std::swap(d_J, d_Jn);
                }
                hipLaunchKernelGGL(k_scatter_rest, dim3(gn), dim3(BT), 0, 0, d_idx, d_idx2, d_J, d_less, n);
            }
            BCHK(hipGetLastError());
            std::vector<int> nl(S);
            BCHK(hipMemcpy(nl.data(), d_nless, sizeof(int) * S, hipMemcpyDeviceToHost));
            if (!local) std::swap(d_idx, d_idx2);
            std::vector<int> cur;
            cur.swap(level);
            for (int k = 0; k < S; ++k) {   // children in level order
                const int ti = cur[k];
                const int st = tree[ti].start, en = tree[ti].end;
                int mid = st + nl[k];
                if (mid == st || mid == en) mid = (st + en) / 2;   // scene.cpp:513-515
                const int l = add(st, mid);
                const int r = add(mid, en);
                tree[ti].left = l;
                tree[ti].right = r;
            }
            if (timing) {
                BCHK(hipDeviceSynchronize());
                const double ms = std::chrono::duration<double, std::milli>(clk() - t_lv).count();
                std::fprintf(stderr, "pt_bvh_build level: %d nodes split, %.3f ms\n", S, ms);
            }
        }
        // every subtree in one launch
        const int NS = (int)subs.size();
        const size_t lds = sizeof(SubLds);
        BCHK(hipFuncSetAttribute((const void*)k_subtree, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        BCHK(hipMalloc(&d_subs, sizeof(SubRoot) * NS));
        BCHK(hipMalloc(&d_subnodes, sizeof(pt_bvh_node) * (size_t)outs));
        BCHK(hipMalloc(&d_subcount, sizeof(int) * NS));
        BCHK(hipMalloc(&d_subscratch, sizeof(pt_bvh_node) * 3 * (size_t)n));
        BCHK(hipMemcpy(d_subs, subs.data(), sizeof(SubRoot) * NS, hipMemcpyHostToDevice));
        auto t_sub = clk();
        hipLaunchKernelGGL(k_subtree, dim3((unsigned)NS), dim3(SUB_LANES), lds, 0, d_tris, d_idx, d_subs, d_subnodes,
                           d_subscratch, d_subcount);
        BCHK(hipGetLastError());
        std::vector<pt_bvh_node> sn(outs);
        std::vector<int> scount(NS);
        BCHK(hipMemcpy(sn.data(), d_subnodes, sizeof(pt_bvh_node) * (size_t)outs, hipMemcpyDeviceToHost));
        BCHK(hipMemcpy(scount.data(), d_subcount, sizeof(int) * NS, hipMemcpyDeviceToHost));
        BCHK(hipMemcpy(tri_indices, d_idx, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost));
        if (allb_used) {
            std::vector<float> ab(6 * allb_used);
            BCHK(hipMemcpy(ab.data(), d_allb, sizeof(float) * 6 * allb_used, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < allb_used; ++i) memcpy(tree[lvl_nodes[i]].b, &ab[6 * i], 6 * sizeof(float));
        }
        if (timing)
            std::fprintf(stderr, "pt_bvh_build %d subtrees %.3f ms, total %.3f ms\n", NS,
                         std::chrono::duration<double, std::milli>(clk() - t_sub).count(),
                         std::chrono::duration<double, std::milli>(clk() - t_start).count());
        // preorder numbering (the reference pushes a node, then recurses left, then right); a
        // subtree root stands for its whole subtree, numbered in preorder by k_subtree
        const int T = (int)tree.size();
        std::vector<int> size(T, 1);
        for (int i = T - 1; i >= 0; --i) {
            if (sub_of[i] >= 0) size[i] = scount[sub_of[i]];
            else if (tree[i].left >= 0) size[i] = 1 + size[tree[i].left] + size[tree[i].right];
        }
        pre.assign(T, 0);
        for (int i = 0; i < T; ++i)   // parents precede children in creation order
            if (sub_of[i] < 0 && tree[i].left >= 0) {
                pre[tree[i].left] = pre[i] + 1;
                pre[tree[i].right] = pre[i] + 1 + size[tree[i].left];
            }
        int total = 0;
        for (int i = 0; i < T; ++i) {
            if (sub_of[i] >= 0) {
                const SubRoot& sr = subs[sub_of[i]];
                const int base = pre[i];
                for (int k = 0; k < size[i]; ++k) {
                    pt_bvh_node nd = sn[sr.out + k];
                    if (nd.left >= 0) nd.left += base;
                    if (nd.right >= 0) nd.right += base;
                    nodes[base + k] = nd;
                }
                total += size[i];
                continue;
            }
            pt_bvh_node& o = nodes[pre[i]];
            o.aabb.min = pt_vec3{tree[i].b[0], tree[i].b[1], tree[i].b[2]};
            o.aabb.max = pt_vec3{tree[i].b[3], tree[i].b[4], tree[i].b[5]};
            o.left = pre[tree[i].left];
            o.right = pre[tree[i].right];
            o.start = -1;
            o.triCount = 0;
            ++total;
        }
        *num_nodes = total;
    }
done:
    for (void* q : {(void*)d_tris, (void*)d_idx, (void*)d_idx2, (void*)d_J, (void*)d_Jn, (void*)d_less,
                    (void*)d_pf, (void*)d_cnt, (void*)d_nless, (void*)d_sstart,
                    (void*)d_pv, (void*)d_bounds, (void*)d_splits, (void*)d_subs, (void*)d_subnodes, (void*)d_subcount,
                    (void*)d_subscratch, (void*)d_lvl, (void*)d_allb})
        (void)hipFree(q);
    return rc;
}
