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
//     the (small) tree skeleton, one download per level, and numbers the nodes at the end.
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

// ---- small nodes (<= SMALL triangles: the bulk of the lower levels): one thread each, the
// reference's sequential loops verbatim ----
constexpr int SMALL = 256;

struct SmallSeg {
    int slot;             // index of the node in this level's list (bounds slot)
    int start, end;
};

__global__ void k_small_bounds(const pt_triangle* __restrict__ tris, const int* __restrict__ idx,
                               const SmallSeg* __restrict__ segs, float* __restrict__ out, int nseg) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    const SmallSeg sg = segs[s];
    float v[12];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        v[k] = FLT_MAX;
        v[3 + k] = -FLT_MAX;
        v[6 + k] = FLT_MAX;
        v[9 + k] = -FLT_MAX;
    }
    for (int i = sg.start; i < sg.end; ++i) {   // UpdateNodeBounds (scene.cpp:429-442), then the centroid loop
        const float* t = tri_f(tris, idx[i]);
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                v[k] = glm_min(v[k], t[OFF_V[q] + k]);
                v[3 + k] = glm_max(v[3 + k], t[OFF_V[q] + k]);
            }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            v[6 + k] = glm_min(v[6 + k], t[OFF_C + k]);
            v[9 + k] = glm_max(v[9 + k], t[OFF_C + k]);
        }
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) out[12 * sg.slot + k] = v[k];
}

// the swap loop itself (scene.cpp:503-511) on one small split node; its elements are marked done
// (less = 2) so the grid-wide scatter leaves them alone
__global__ void k_small_partition(const pt_triangle* __restrict__ tris, const int* __restrict__ idx_in,
                                  int* __restrict__ idx_out, const SmallSeg* __restrict__ segs,
                                  const Split* __restrict__ splits, unsigned char* __restrict__ less,
                                  int* __restrict__ nless, int nseg) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    const SmallSeg sg = segs[s];
    const Split sp = splits[s];
    for (int i = sg.start; i < sg.end; ++i) {
        idx_out[i] = idx_in[i];
        less[i] = 2;
    }
    int mid = sg.start;
    for (int i = sg.start; i < sg.end; ++i) {
        const int ti = idx_out[i];
        if (tri_f(tris, ti)[OFF_C + sp.axis] < sp.split) {
            idx_out[i] = idx_out[mid];
            idx_out[mid] = ti;
            mid++;
        }
    }
    nless[s] = mid - sg.start;
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

std::string g_err;

#define BCHK(x)                                                                              \
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
    size_t piece_cap = 0, seg_cap = 0, small_cap = 0;
    const bool timing = getenv("PT_BVH_TIMING") != nullptr;   // per-level times on stderr (tools)
    auto clk = [] { return std::chrono::steady_clock::now(); };
    std::chrono::steady_clock::time_point t_start = clk();
    SmallSeg* d_small = nullptr;
    Split* d_ssplit = nullptr;
    int* d_snless = nullptr;
    int dev_count = 0;
    std::vector<TreeNode> tree;
    std::vector<int> level;   // skeleton indices of the current level
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
    tree.push_back(TreeNode{0, n});
    tree.reserve(2 * (size_t)n);
    level.push_back(0);
    t_start = clk();
    while (!level.empty()) {
        auto t_lv = clk();
        const int S = (int)level.size();
        // pieces of every node of the level, in node order
        std::vector<Piece> pieces;
        std::vector<int> first(S + 1);
        std::vector<SmallSeg> small;
        for (int k = 0; k < S; ++k) {
            first[k] = (int)pieces.size();
            const TreeNode& t = tree[level[k]];
            if (t.end - t.start <= SMALL) {
                small.push_back(SmallSeg{k, t.start, t.end});
                continue;
            }
            for (int a = t.start; a < t.end; a += PIECE) pieces.push_back(Piece{k, a, std::min(t.end, a + PIECE)});
        }
        first[S] = (int)pieces.size();
        if (pieces.size() > piece_cap) {
            (void)hipFree(d_pieces);
            (void)hipFree(d_pv);
            (void)hipFree(d_pf);
            (void)hipFree(d_cnt);
            d_pieces = nullptr;
            d_pv = nullptr;
            d_pf = nullptr;
            d_cnt = nullptr;
            piece_cap = std::max(pieces.size(), 2 * piece_cap);
            BCHK(hipMalloc(&d_pieces, sizeof(Piece) * piece_cap));
            BCHK(hipMalloc(&d_pv, sizeof(float) * 12 * piece_cap));
            BCHK(hipMalloc(&d_pf, sizeof(int) * 12 * piece_cap));
            BCHK(hipMalloc(&d_cnt, sizeof(int) * piece_cap));
        }
        if (small.size() > small_cap) {
            (void)hipFree(d_small);
            (void)hipFree(d_ssplit);
            (void)hipFree(d_snless);
            d_small = nullptr;
            d_ssplit = nullptr;
            d_snless = nullptr;
            small_cap = std::max(small.size(), 2 * small_cap);
            BCHK(hipMalloc(&d_small, sizeof(SmallSeg) * small_cap));
            BCHK(hipMalloc(&d_ssplit, sizeof(Split) * small_cap));
            BCHK(hipMalloc(&d_snless, sizeof(int) * small_cap));
        }
        if ((size_t)S + 1 > seg_cap) {
            (void)hipFree(d_first);
            (void)hipFree(d_bounds);
            (void)hipFree(d_nless);
            (void)hipFree(d_sstart);
            (void)hipFree(d_splits);
            d_first = nullptr;
            d_bounds = nullptr;
            d_nless = nullptr;
            d_sstart = nullptr;
            d_splits = nullptr;
            seg_cap = std::max<size_t>(S + 1, 2 * seg_cap);
            BCHK(hipMalloc(&d_first, sizeof(int) * seg_cap));
            BCHK(hipMalloc(&d_bounds, sizeof(float) * 12 * seg_cap));
            BCHK(hipMalloc(&d_nless, sizeof(int) * seg_cap));
            BCHK(hipMalloc(&d_sstart, sizeof(int) * seg_cap));
            BCHK(hipMalloc(&d_splits, sizeof(Split) * seg_cap));
        }
        if (!pieces.empty()) {
            BCHK(hipMemcpy(d_pieces, pieces.data(), sizeof(Piece) * pieces.size(), hipMemcpyHostToDevice));
            BCHK(hipMemcpy(d_first, first.data(), sizeof(int) * (S + 1), hipMemcpyHostToDevice));
            hipLaunchKernelGGL(k_piece_fold, dim3((unsigned)pieces.size()), dim3(BT), 0, 0, d_tris, d_idx, d_pieces,
                               d_pv, d_pf);
            hipLaunchKernelGGL(k_seg_fold, dim3((unsigned)((S + 3) / 4)), dim3(64), 0, 0, d_first, d_pv, d_pf, d_bounds,
                               S);
        }
        if (!small.empty()) {   // after k_seg_fold, which writes the empty fold into small nodes' slots
            BCHK(hipMemcpy(d_small, small.data(), sizeof(SmallSeg) * small.size(), hipMemcpyHostToDevice));
            hipLaunchKernelGGL(k_small_bounds, dim3((unsigned)((small.size() + 63) / 64)), dim3(64), 0, 0, d_tris,
                               d_idx, d_small, d_bounds, (int)small.size());
        }
        BCHK(hipGetLastError());
        std::vector<float> bounds(12 * (size_t)S);
        BCHK(hipMemcpy(bounds.data(), d_bounds, sizeof(float) * 12 * S, hipMemcpyDeviceToHost));
        // split decisions (scene.cpp:466-499) on the host: a few float ops per node
        std::vector<int> split_nodes;                 // skeleton indices of the nodes that split
        std::vector<Split> splits;
        std::vector<Piece> spieces;                   // their pieces, seg = index into split_nodes
        std::vector<int> sfirst{0}, sstart;
        std::vector<int> small_nodes;                 // small nodes that split (thread per node)
        std::vector<SmallSeg> ssegs;
        std::vector<Split> ssplits;
        for (int k = 0; k < S; ++k) {
            TreeNode& t = tree[level[k]];
            memcpy(t.b, &bounds[12 * (size_t)k], 6 * sizeof(float));
            if (t.end - t.start <= 4) continue;
            const float* cmin = &bounds[12 * (size_t)k + 6];
            const float* cmax = &bounds[12 * (size_t)k + 9];
            const float ex = cmax[0] - cmin[0], ey = cmax[1] - cmin[1], ez = cmax[2] - cmin[2];
            int axis = 0;
            if (ey > ex && ey > ez) axis = 1;
            if (ez > ex) axis = 2;
            if (t.end - t.start <= SMALL) {
                small_nodes.push_back(level[k]);
                ssegs.push_back(SmallSeg{k, t.start, t.end});
                ssplits.push_back(Split{axis, 0.5f * (cmin[axis] + cmax[axis])});
                continue;
            }
            const int si = (int)split_nodes.size();
            split_nodes.push_back(level[k]);
            splits.push_back(Split{axis, 0.5f * (cmin[axis] + cmax[axis])});
            sstart.push_back(t.start);
            for (int p = first[k]; p < first[k + 1]; ++p) spieces.push_back(Piece{si, pieces[p].start, pieces[p].end});
            sfirst.push_back((int)spieces.size());
        }
        const int SS = (int)split_nodes.size();
        hipLaunchKernelGGL(k_fill, dim3(gn), dim3(BT), 0, 0, d_J, d_less, n);
        std::vector<int> snl(small_nodes.size());
        if (!small_nodes.empty()) {
            BCHK(hipMemcpy(d_small, ssegs.data(), sizeof(SmallSeg) * ssegs.size(), hipMemcpyHostToDevice));
            BCHK(hipMemcpy(d_ssplit, ssplits.data(), sizeof(Split) * ssplits.size(), hipMemcpyHostToDevice));
            hipLaunchKernelGGL(k_small_partition, dim3((unsigned)((ssegs.size() + 63) / 64)), dim3(64), 0, 0, d_tris,
                               d_idx, d_idx2, d_small, d_ssplit, d_less, d_snless, (int)ssegs.size());
            BCHK(hipGetLastError());
            BCHK(hipMemcpy(snl.data(), d_snless, sizeof(int) * snl.size(), hipMemcpyDeviceToHost));
        }
        std::vector<int> nl(SS);
        if (SS > 0) {
            int maxlen = 0;
            for (int k = 0; k < SS; ++k) maxlen = std::max(maxlen, tree[split_nodes[k]].end - tree[split_nodes[k]].start);
            BCHK(hipMemcpy(d_pieces, spieces.data(), sizeof(Piece) * spieces.size(), hipMemcpyHostToDevice));
            BCHK(hipMemcpy(d_first, sfirst.data(), sizeof(int) * (SS + 1), hipMemcpyHostToDevice));
            BCHK(hipMemcpy(d_splits, splits.data(), sizeof(Split) * SS, hipMemcpyHostToDevice));
            BCHK(hipMemcpy(d_sstart, sstart.data(), sizeof(int) * SS, hipMemcpyHostToDevice));
            const unsigned np = (unsigned)spieces.size();
            hipLaunchKernelGGL(k_piece_count, dim3(np), dim3(BT), 0, 0, d_tris, d_idx, d_pieces, d_splits, d_less,
                               d_cnt);
            hipLaunchKernelGGL(k_seg_scan, dim3((unsigned)((SS + 255) / 256)), dim3(256), 0, 0, d_first, d_cnt, d_nless,
                               SS);
            hipLaunchKernelGGL(k_piece_place, dim3(np), dim3(BT), 0, 0, d_idx, d_idx2, d_pieces, d_sstart, d_less,
                               d_cnt, d_J);
            int rounds = 1;
            while ((1 << (rounds - 1)) < maxlen) ++rounds;   // ceil(log2 maxlen) + 1
            for (int r = 0; r < rounds; ++r) {
                hipLaunchKernelGGL(k_jump, dim3(gn), dim3(BT), 0, 0, d_J, d_Jn, n);
                std::swap(d_J, d_Jn);
            }
            BCHK(hipGetLastError());
            BCHK(hipMemcpy(nl.data(), d_nless, sizeof(int) * SS, hipMemcpyDeviceToHost));
        }
        hipLaunchKernelGGL(k_scatter_rest, dim3(gn), dim3(BT), 0, 0, d_idx, d_idx2, d_J, d_less, n);
        BCHK(hipGetLastError());
        std::swap(d_idx, d_idx2);
        // children in level order (big and small split nodes are interleaved in the level)
        std::vector<int> next;
        next.reserve(2 * (split_nodes.size() + small_nodes.size()));
        size_t ib = 0, is = 0;
        while (ib < split_nodes.size() || is < small_nodes.size()) {
            const bool big = is >= small_nodes.size() || (ib < split_nodes.size() && split_nodes[ib] < small_nodes[is]);
            const int ti = big ? split_nodes[ib] : small_nodes[is];
            const int nlk = big ? nl[ib++] : snl[is++];
            const int st = tree[ti].start, en = tree[ti].end;
            int mid = st + nlk;
            if (mid == st || mid == en) mid = (st + en) / 2;   // scene.cpp:513-515
            const int l = (int)tree.size();
            tree.push_back(TreeNode{st, mid});
            tree.push_back(TreeNode{mid, en});
            tree[ti].left = l;
            tree[ti].right = l + 1;
            next.push_back(l);
            next.push_back(l + 1);
        }
        level.swap(next);
        if (timing) {
            BCHK(hipDeviceSynchronize());
            const double ms = std::chrono::duration<double, std::milli>(clk() - t_lv).count();
            std::fprintf(stderr, "pt_bvh_build level: %zu nodes (%d split, %zu small) %.3f ms\n", (size_t)S, SS,
                         small_nodes.size(), ms);
        }
    }
    BCHK(hipDeviceSynchronize());
    if (timing)
        std::fprintf(stderr, "pt_bvh_build levels total %.3f ms\n",
                     std::chrono::duration<double, std::milli>(clk() - t_start).count());
    BCHK(hipMemcpy(tri_indices, d_idx, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost));
    {
        // preorder numbering (the reference pushes a node, then recurses left, then right)
        const int T = (int)tree.size();
        std::vector<int> size(T, 1);
        for (int i = T - 1; i >= 0; --i)
            if (tree[i].left >= 0) size[i] = 1 + size[tree[i].left] + size[tree[i].right];
        pre.assign(T, 0);
        for (int i = 0; i < T; ++i)   // parents precede children in breadth-first order
            if (tree[i].left >= 0) {
                pre[tree[i].left] = pre[i] + 1;
                pre[tree[i].right] = pre[i] + 1 + size[tree[i].left];
            }
        for (int i = 0; i < T; ++i) {
            pt_bvh_node& o = nodes[pre[i]];
            o.aabb.min = pt_vec3{tree[i].b[0], tree[i].b[1], tree[i].b[2]};
            o.aabb.max = pt_vec3{tree[i].b[3], tree[i].b[4], tree[i].b[5]};
            if (tree[i].left >= 0) {
                o.left = pre[tree[i].left];
                o.right = pre[tree[i].right];
                o.start = -1;
                o.triCount = 0;
            } else {
                o.left = -1;
                o.right = -1;
                o.start = tree[i].start;
                o.triCount = tree[i].end - tree[i].start;
            }
        }
        *num_nodes = T;
    }
done:
    for (void* q : {(void*)d_tris, (void*)d_idx, (void*)d_idx2, (void*)d_J, (void*)d_Jn, (void*)d_less,
                    (void*)d_pieces, (void*)d_first, (void*)d_pf, (void*)d_cnt, (void*)d_nless, (void*)d_sstart,
                    (void*)d_pv, (void*)d_bounds, (void*)d_splits, (void*)d_small, (void*)d_ssplit, (void*)d_snless})
        (void)hipFree(q);
    return rc;
}
