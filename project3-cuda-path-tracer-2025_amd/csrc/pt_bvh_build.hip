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
// GPU formulation, level by level (all nodes of one depth at once, one workgroup per node):
//   * bounds: each thread folds a contiguous chunk in order into a summary (value, "holds a
//     NaN"), and chunks are joined pairwise in order (stride doubling).  The join is
//     associative, so the result equals the sequential fold, signed zeros and NaNs included;
//   * the swap loop has a closed form.  The k-th "less" element (in range order) lands at
//     start + k.  A "not less" element is moved only by a swap: the one at position p (which
//     is mid at that moment) jumps to the index of the (p - start)-th less element.  So its final
//     slot is the fixed point of J(p) = lessIdx[p - start] for p < start + nLess, J(p) = p
//     beyond -- resolved by pointer jumping.  (Checked against the loop itself on 20k random
//     sequences while deriving it; the GPU result is checked against host/scene.cpp's
//     sequential builder in tests/test_gpu_parity.py::test_gpu_bvh_build_bitexact.)
//   * node numbering is the reference's preorder; it needs the subtree sizes, so the host keeps
//     the (small) tree skeleton, one download per level, and numbers the nodes at the end.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pt/pathtrace_abi.h"

namespace {

constexpr int BT = 256;   // threads per workgroup

struct Seg {
    int start, end;       // triangle range
    int axis;             // split axis (build kernel output)
    float split;          // split position
};

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

// node bounds + centroid bounds of one segment; out[12 * s]: min.xyz max.xyz cmin.xyz cmax.xyz
__global__ __launch_bounds__(BT) void k_seg_bounds(const pt_triangle* __restrict__ tris, const int* __restrict__ idx,
                                                   const Seg* __restrict__ segs, float* __restrict__ out) {
    __shared__ float rv[12][BT];
    __shared__ int rf[12][BT];
    const Seg sg = segs[blockIdx.x];
    const int len = sg.end - sg.start;
    const int chunk = (len + BT - 1) / BT;
    const int a = sg.start + threadIdx.x * chunk;
    const int b = min(sg.end, a + chunk);
    Fold f[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) f[k] = Fold{0.f, 1};
    for (int i = a; i < b; ++i) {
        const float* t = tri_f(tris, idx[i]);
        // UpdateNodeBounds order: min over v1, v2, v3 then max over v1, v2, v3 (per component
        // these are independent folds, each in element order)
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
    // in-order pairwise join: slot i covers chunks [i, i + 2s) after the step of stride s
    for (int s = 1; s < BT; s <<= 1) {
        const int i = threadIdx.x;
        if ((i & (2 * s - 1)) == 0) {
#pragma unroll
            for (int k = 0; k < 12; ++k) {
                const Fold x{rv[k][i], rf[k][i]}, y{rv[k][i + s], rf[k][i + s]};
                const bool mn = (k < 3) || (k >= 6 && k < 9);
                const Fold z = mn ? fold_join<true>(x, y) : fold_join<false>(x, y);
                rv[k][i] = z.val;
                rf[k][i] = z.flags;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < 12) {
        const int k = threadIdx.x;
        const Fold z{rv[k][0], rf[k][0]};
        const bool mn = (k < 3) || (k >= 6 && k < 9);
        out[12 * blockIdx.x + k] = mn ? fold_final<true>(z) : fold_final<false>(z);
    }
}

// the swap-partition of one segment (closed form, see the header): idx_in -> idx_out on
// [start, end); nless[s] = number of "less" elements.  J / Jn: pointer-jumping scratch.
__global__ __launch_bounds__(BT) void k_seg_partition(const pt_triangle* __restrict__ tris, const int* __restrict__ idx_in,
                                                      int* __restrict__ idx_out, const Seg* __restrict__ segs,
                                                      int* __restrict__ J, int* __restrict__ Jn, int* __restrict__ nless) {
    __shared__ int scan[BT];
    __shared__ int changed;
    const Seg sg = segs[blockIdx.x];
    const int len = sg.end - sg.start;
    const int chunk = (len + BT - 1) / BT;
    const int a = sg.start + threadIdx.x * chunk;
    const int b = min(sg.end, a + chunk);
    auto less = [&](int p) { return tri_f(tris, idx_in[p])[OFF_C + sg.axis] < sg.split; };
    int cnt = 0;
    for (int i = a; i < b; ++i) cnt += less(i) ? 1 : 0;
    scan[threadIdx.x] = cnt;
    __syncthreads();
    for (int s = 1; s < BT; s <<= 1) {   // inclusive scan (Hillis-Steele)
        const int x = threadIdx.x >= s ? scan[threadIdx.x - s] : 0;
        __syncthreads();
        scan[threadIdx.x] += x;
        __syncthreads();
    }
    const int total = scan[BT - 1];
    int r = scan[threadIdx.x] - cnt;   // rank of this chunk's first "less" element
    // the k-th less element lands at start + k; J[start + k] = its position (the hop target of
    // the element the swap at that moment moves out of slot start + k)
    for (int i = a; i < b; ++i) {
        if (less(i)) {
            idx_out[sg.start + r] = idx_in[i];
            J[sg.start + r] = i;
            ++r;
        }
    }
    __syncthreads();
    const int lim = sg.start + total;
    for (int p = sg.start + (int)threadIdx.x; p < sg.end; p += BT)
        if (p >= lim) J[p] = p;
    __threadfence_block();
    __syncthreads();
    // pointer jumping to the fixed point: every chain ends in a slot >= start + total
    int* cur = J;
    int* nxt = Jn;
    for (;;) {
        if (threadIdx.x == 0) changed = 0;
        __syncthreads();
        for (int p = sg.start + (int)threadIdx.x; p < sg.end; p += BT) {
            const int j = cur[p];
            const int jj = cur[j];
            nxt[p] = jj;
            if (jj != j) changed = 1;
        }
        __threadfence_block();
        __syncthreads();
        int* t = cur;
        cur = nxt;
        nxt = t;
        if (!changed) break;
        __syncthreads();
    }
    for (int i = a; i < b; ++i)
        if (!less(i)) idx_out[cur[i]] = idx_in[i];
    if (threadIdx.x == 0) nless[blockIdx.x] = total;
}

// leaf segments keep their order
__global__ __launch_bounds__(BT) void k_seg_copy(const int* __restrict__ idx_in, int* __restrict__ idx_out,
                                                 const Seg* __restrict__ segs) {
    const Seg sg = segs[blockIdx.x];
    for (int p = sg.start + (int)threadIdx.x; p < sg.end; p += BT) idx_out[p] = idx_in[p];
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
    int *d_idx = nullptr, *d_idx2 = nullptr, *d_J = nullptr, *d_Jn = nullptr, *d_nl = nullptr;
    Seg* d_segs = nullptr;
    float* d_bounds = nullptr;
    int dev_count = 0;
    std::vector<TreeNode> tree;
    std::vector<int> level;   // skeleton indices of the current level
    std::vector<int> pre;
    size_t seg_cap = 0;
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
    BCHK(hipMemcpy(d_tris, tris, sizeof(pt_triangle) * (size_t)n, hipMemcpyHostToDevice));
    {
        std::vector<int> iota(n);
        for (int i = 0; i < n; ++i) iota[i] = i;
        BCHK(hipMemcpy(d_idx, iota.data(), sizeof(int) * (size_t)n, hipMemcpyHostToDevice));
    }
    tree.push_back(TreeNode{0, n});
    level.push_back(0);
    while (!level.empty()) {
        const size_t S = level.size();
        if (S > seg_cap) {
            (void)hipFree(d_segs);
            (void)hipFree(d_bounds);
            (void)hipFree(d_nl);
            d_segs = nullptr;
            d_bounds = nullptr;
            d_nl = nullptr;
            seg_cap = std::max<size_t>(S, 2 * seg_cap);
            BCHK(hipMalloc(&d_segs, sizeof(Seg) * seg_cap));
            BCHK(hipMalloc(&d_bounds, sizeof(float) * 12 * seg_cap));
            BCHK(hipMalloc(&d_nl, sizeof(int) * seg_cap));
        }
        std::vector<Seg> segs(S);
        for (size_t s = 0; s < S; ++s) segs[s] = Seg{tree[level[s]].start, tree[level[s]].end, 0, 0.f};
        BCHK(hipMemcpy(d_segs, segs.data(), sizeof(Seg) * S, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_seg_bounds, dim3((unsigned)S), dim3(BT), 0, 0, d_tris, d_idx, d_segs, d_bounds);
        BCHK(hipGetLastError());
        std::vector<float> bounds(12 * S);
        BCHK(hipMemcpy(bounds.data(), d_bounds, sizeof(float) * 12 * S, hipMemcpyDeviceToHost));
        // split decisions (scene.cpp:466-499) on the host: a few float ops per node
        std::vector<Seg> split, leaf;
        std::vector<int> split_node;
        for (size_t s = 0; s < S; ++s) {
            TreeNode& t = tree[level[s]];
            memcpy(t.b, &bounds[12 * s], 6 * sizeof(float));
            if (t.end - t.start <= 4) {
                leaf.push_back(segs[s]);
                continue;
            }
            const float* cmin = &bounds[12 * s + 6];
            const float* cmax = &bounds[12 * s + 9];
            const float ex = cmax[0] - cmin[0], ey = cmax[1] - cmin[1], ez = cmax[2] - cmin[2];
            int axis = 0;
            if (ey > ex && ey > ez) axis = 1;
            if (ez > ex) axis = 2;
            const float sp = 0.5f * (cmin[axis] + cmax[axis]);
            split.push_back(Seg{t.start, t.end, axis, sp});
            split_node.push_back(level[s]);
        }
        std::vector<Seg> all(split);
        all.insert(all.end(), leaf.begin(), leaf.end());
        BCHK(hipMemcpy(d_segs, all.data(), sizeof(Seg) * all.size(), hipMemcpyHostToDevice));
        if (!split.empty())
            hipLaunchKernelGGL(k_seg_partition, dim3((unsigned)split.size()), dim3(BT), 0, 0, d_tris, d_idx, d_idx2,
                               d_segs, d_J, d_Jn, d_nl);
        if (!leaf.empty())
            hipLaunchKernelGGL(k_seg_copy, dim3((unsigned)leaf.size()), dim3(BT), 0, 0, d_idx, d_idx2,
                               d_segs + split.size());
        BCHK(hipGetLastError());
        std::vector<int> nl(split.size());
        if (!split.empty()) BCHK(hipMemcpy(nl.data(), d_nl, sizeof(int) * split.size(), hipMemcpyDeviceToHost));
        std::swap(d_idx, d_idx2);
        std::vector<int> next;
        for (size_t k = 0; k < split.size(); ++k) {
            const int ti = split_node[k];
            const int st = tree[ti].start, en = tree[ti].end;
            int mid = st + nl[k];
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
    }
    BCHK(hipDeviceSynchronize());
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
    (void)hipFree(d_tris);
    (void)hipFree(d_idx);
    (void)hipFree(d_idx2);
    (void)hipFree(d_J);
    (void)hipFree(d_Jn);
    (void)hipFree(d_segs);
    (void)hipFree(d_bounds);
    (void)hipFree(d_nl);
    return rc;
}
