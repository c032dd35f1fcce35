// trav_tree.h — the traversal hierarchy the GPU walks above the reference's BVH leaves.
//
// The reference visits a BVH leaf iff the leaf's OWN box passes aabbIntersectionTest: every node box
// is the min / max over its triangles (scene.cpp:428-441), so an ancestor's box contains the leaf's,
// and aabbIntersectionTest is monotone in the box bounds.  The hierarchy ABOVE the
// leaves therefore decides nothing but cost: any tree whose inner boxes contain their leaves' boxes,
// walked with the reference's exact box decision, visits exactly the reference's leaves (minus the
// certified t-culls).  The reference's own hierarchy is a midpoint split on the "longest" centroid
// axis with its z-over-y quirk (scene.cpp:493-498); this builds a surface-area-heuristic tree over
// the reference's leaves instead (binned SAH, 32 bins per axis), whose leaves are exactly the
// reference's leaves, with their exact boxes and their reference visit-order numbering (the tie rule).
#pragma once

#include <vector>

namespace pth {

struct TravChild {
    float lo[3], hi[3];   // inner child: union of its leaves' boxes; leaf child: the reference box
    int ref;              // inner child: index of its TravInner; leaf child: the leaf's id
    bool leaf;
    float s;              // largest cull size (node_aux .y) of the leaves below
};
struct TravInner {
    TravChild c[2];
};

// Binned-SAH tree over `n` leaves (boxes lo/hi as 3 floats each, cull sizes s).  Inner nodes are
// numbered breadth-first over the top `bfs_levels` levels, then each subtree below them in
// depth-first preorder (so a subtree's nodes share cache lines; a large value: breadth-first
// throughout, 0: preorder throughout); the root is inner node 0 (n >= 2).  `height`: levels of
// inner nodes plus the leaf level.  Returns false for n < 2 or for a box with a NaN / infinite
// coordinate (the containment argument needs ordered, finite bounds): the caller keeps the
// reference hierarchy.  `max_height` bounds `height`: where a SAH split would leave a child no room
// for a balanced subtree below the bound, the split is the median one (the traversal stack, one
// entry per level, lives in LDS, whose size sets the traversal kernels' occupancy); a bound below
// 1 + ceil(log2 n) is raised to it.
bool build_sah_tree(const std::vector<float>& leaf_lo, const std::vector<float>& leaf_hi,
                    const std::vector<float>& leaf_s, std::vector<TravInner>& out, int& height,
                    int bfs_levels = 1 << 30, int max_height = 1 << 30);

// The 4-wide form of a tree from build_sah_tree: record q holds the children of one binary inner
// node, an inner child replaced by its own two children (two levels per record: 2 to 4 children).
// Record 0 is the root's.  Records are numbered breadth-first over the top `bfs_levels` levels and
// in preorder below; a child is a record (`leaf` false, `ref` its index) or a leaf (`ref` its id).
// `stack_need`: the most stack entries a depth-first walk that pushes every child but the one it
// continues with can hold (the sum of children - 1 along a path).
struct QuadRecord {
    TravChild c[4];
    int n;   // children in use
};
void build_quad_records(const std::vector<TravInner>& tree, int bfs_levels, std::vector<QuadRecord>& out,
                        int& stack_need);

}  // namespace pth
