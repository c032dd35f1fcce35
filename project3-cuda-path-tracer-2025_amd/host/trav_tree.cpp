// trav_tree.cpp — binned-SAH traversal hierarchy over the reference's BVH leaves (trav_tree.h).
#include "trav_tree.h"

#include <algorithm>
#include <cmath>
#include <numeric>

namespace pth {
namespace {

constexpr int BINS = 32;

struct Box {
    double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    void grow(const float* l, const float* h) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], (double)l[a]);
            hi[a] = std::max(hi[a], (double)h[a]);
        }
    }
    void grow(const Box& b) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b.lo[a]);
            hi[a] = std::max(hi[a], b.hi[a]);
        }
    }
    double area() const {
        if (!(hi[0] >= lo[0])) return 0.0;
        const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return x * y + y * z + z * x;
    }
};

struct Tmp {
    int kid[2];   // >= 0: Tmp index; < 0: -(leaf + 1)
    float lo[3], hi[3];
    float s;
};

int ceil_log2(int c) {
    int h = 0;
    while ((1 << h) < c) ++h;
    return h;
}

}  // namespace

bool build_sah_tree(const std::vector<float>& leaf_lo, const std::vector<float>& leaf_hi,
                    const std::vector<float>& leaf_s, std::vector<TravInner>& out, int& height, int bfs_levels,
                    int max_height) {
    const int n = (int)leaf_s.size();
    out.clear();
    height = 0;
    if (n < 2 || (int)leaf_lo.size() != 3 * n || (int)leaf_hi.size() != 3 * n) return false;
    for (int i = 0; i < 3 * n; ++i)
        if (!std::isfinite(leaf_lo[i]) || !std::isfinite(leaf_hi[i]) || leaf_lo[i] > leaf_hi[i]) return false;
    std::vector<double> cen(3 * (size_t)n);
    for (int i = 0; i < 3 * n; ++i) cen[i] = 0.5 * ((double)leaf_lo[i] + (double)leaf_hi[i]);

    std::vector<int> idx(n);
    std::iota(idx.begin(), idx.end(), 0);
    std::vector<Tmp> T;
    T.reserve(n);
    struct Work {
        int begin, end, parent, side, depth;
    };
    max_height = std::max(max_height, 1 + ceil_log2(n));
    std::vector<Work> st{{0, n, -1, 0, 1}};
    while (!st.empty()) {
        const Work w = st.back();
        st.pop_back();
        int code;
        if (w.end - w.begin == 1) {
            code = -(idx[w.begin] + 1);
            height = std::max(height, w.depth);
        } else {
            // centroid bounds
            double cl[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, ch[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
            for (int i = w.begin; i < w.end; ++i)
                for (int a = 0; a < 3; ++a) {
                    cl[a] = std::min(cl[a], cen[3 * (size_t)idx[i] + a]);
                    ch[a] = std::max(ch[a], cen[3 * (size_t)idx[i] + a]);
                }
            double best = HUGE_VAL;
            int bax = -1, bsplit = -1;
            for (int a = 0; a < 3; ++a) {
                const double ext = ch[a] - cl[a];
                if (!(ext > 0.0)) continue;
                Box bb[BINS];
                int bc[BINS] = {0};
                for (int i = w.begin; i < w.end; ++i) {
                    const int k = idx[i];
                    const int b = std::min(BINS - 1, (int)((cen[3 * (size_t)k + a] - cl[a]) / ext * BINS));
                    bc[b]++;
                    bb[b].grow(&leaf_lo[3 * (size_t)k], &leaf_hi[3 * (size_t)k]);
                }
                double rarea[BINS];
                int rcnt[BINS];
                Box r;
                int rc = 0;
                for (int b = BINS - 1; b > 0; --b) {
                    r.grow(bb[b]);
                    rc += bc[b];
                    rarea[b] = r.area();
                    rcnt[b] = rc;
                }
                Box l;
                int lc = 0;
                for (int b = 0; b < BINS - 1; ++b) {   // split after bin b
                    l.grow(bb[b]);
                    lc += bc[b];
                    if (lc == 0 || rcnt[b + 1] == 0) continue;
                    const double c = l.area() * lc + rarea[b + 1] * rcnt[b + 1];
                    if (c < best) {
                        best = c;
                        bax = a;
                        bsplit = b;
                    }
                }
            }
            int mid;
            if (bax < 0) {   // every centroid equal: halve in index order
                mid = w.begin + (w.end - w.begin) / 2;
            } else {
                const double ext = ch[bax] - cl[bax];
                auto left = [&](int k) {
                    return std::min(BINS - 1, (int)((cen[3 * (size_t)k + bax] - cl[bax]) / ext * BINS)) <= bsplit;
                };
                mid = (int)(std::stable_partition(idx.begin() + w.begin, idx.begin() + w.end, left) - idx.begin());
                if (mid == w.begin || mid == w.end) mid = w.begin + (w.end - w.begin) / 2;
            }
            // height bound: a child of c leaves needs ceil(log2 c) more levels at best; a split that
            // leaves a child no room becomes the median split on the same axis (by centroid, ties by
            // leaf id), which keeps every subtree within the bound from here on
            const int big = std::max(mid - w.begin, w.end - mid);
            if (w.depth + 1 + ceil_log2(big) > max_height) {
                const int a = bax >= 0 ? bax : 0;
                mid = w.begin + (w.end - w.begin) / 2;
                std::nth_element(idx.begin() + w.begin, idx.begin() + mid, idx.begin() + w.end, [&](int x, int y) {
                    const double cx = cen[3 * (size_t)x + a], cy = cen[3 * (size_t)y + a];
                    return cx < cy || (cx == cy && x < y);
                });
            }
            code = (int)T.size();
            T.push_back(Tmp{});
            st.push_back({mid, w.end, code, 1, w.depth + 1});
            st.push_back({w.begin, mid, code, 0, w.depth + 1});
        }
        if (w.parent >= 0) T[w.parent].kid[w.side] = code;
    }
    // boxes and cull sizes bottom-up (children are created after their parent)
    auto child_box = [&](int code, float* lo, float* hi, float& s) {
        if (code < 0) {
            const int k = -code - 1;
            for (int a = 0; a < 3; ++a) {
                lo[a] = leaf_lo[3 * (size_t)k + a];
                hi[a] = leaf_hi[3 * (size_t)k + a];
            }
            s = leaf_s[k];
        } else {
            for (int a = 0; a < 3; ++a) {
                lo[a] = T[code].lo[a];
                hi[a] = T[code].hi[a];
            }
            s = T[code].s;
        }
    };
    for (int i = (int)T.size() - 1; i >= 0; --i) {
        float l0[3], h0[3], l1[3], h1[3], s0, s1;
        child_box(T[i].kid[0], l0, h0, s0);
        child_box(T[i].kid[1], l1, h1, s1);
        for (int a = 0; a < 3; ++a) {
            T[i].lo[a] = std::min(l0[a], l1[a]);   // exact: min / max of finite floats
            T[i].hi[a] = std::max(h0[a], h1[a]);
        }
        T[i].s = std::max(s0, s1);
    }
    // numbering: breadth-first over the top bfs_levels levels (they share a few cache lines), then
    // every subtree below them in preorder -- T's own order (a parent is created before its
    // children, a left subtree before its right one), so a subtree is one contiguous range of T
    std::vector<int> order{0}, bfs(T.size(), -1), depth(T.size(), 0), roots;
    bfs[0] = 0;
    for (size_t h = 0; h < order.size(); ++h) {
        const int n = order[h];
        if (depth[n] >= bfs_levels) {   // a subtree root: numbered below
            roots.push_back(n);
            continue;
        }
        for (int k : T[n].kid)
            if (k >= 0) {
                depth[k] = depth[n] + 1;
                order.push_back(k);
            }
    }
    if (!roots.empty()) {
        order.erase(std::remove_if(order.begin(), order.end(), [&](int n) { return depth[n] >= bfs_levels; }),
                    order.end());
        for (int r : roots) {   // preorder of r's subtree: T[r .. r + size)
            std::vector<int> st{r};
            while (!st.empty()) {
                const int n = st.back();
                st.pop_back();
                order.push_back(n);
                if (T[n].kid[1] >= 0) st.push_back(T[n].kid[1]);
                if (T[n].kid[0] >= 0) st.push_back(T[n].kid[0]);
            }
        }
    }
    for (size_t h = 0; h < order.size(); ++h) bfs[order[h]] = (int)h;
    out.resize(T.size());
    for (size_t h = 0; h < order.size(); ++h) {
        const Tmp& t = T[order[h]];
        for (int c = 0; c < 2; ++c) {
            TravChild& ch = out[h].c[c];
            child_box(t.kid[c], ch.lo, ch.hi, ch.s);
            ch.leaf = t.kid[c] < 0;
            ch.ref = ch.leaf ? -t.kid[c] - 1 : bfs[t.kid[c]];
        }
    }
    return true;
}

void build_quad_records(const std::vector<TravInner>& tt, int bfs_levels, std::vector<QuadRecord>& out,
                        int& stack_need) {
    out.clear();
    stack_need = 0;
    if (tt.empty()) return;
    const int P = (int)tt.size();
    auto kids = [&](int n, TravChild* k4) {
        int k = 0;
        for (int c = 0; c < 2; ++c) {
            const TravChild& ch = tt[n].c[c];
            if (ch.leaf) {
                k4[k++] = ch;
            } else {
                k4[k++] = tt[ch.ref].c[0];
                k4[k++] = tt[ch.ref].c[1];
            }
        }
        return k;
    };
    // the binary nodes that head a record, breadth-first: the root and every inner child of a record
    std::vector<int> head{0}, depth{0}, qid(P, -1);
    qid[0] = 0;
    for (size_t h = 0; h < head.size(); ++h) {
        TravChild k4[4];
        const int nk = kids(head[h], k4);
        for (int i = 0; i < nk; ++i)
            if (!k4[i].leaf) {
                qid[k4[i].ref] = (int)head.size();
                head.push_back(k4[i].ref);
                depth.push_back(depth[h] + 1);
            }
    }
    const int Q = (int)head.size();
    const int qlev = std::max(0, bfs_levels);
    std::vector<int> order, num(Q, -1);
    std::vector<int> roots;
    for (int h = 0; h < Q; ++h) {
        if (depth[h] < qlev) order.push_back(h);
        else if (depth[h] == qlev) roots.push_back(h);
    }
    for (int r : roots) {   // each subtree below the breadth-first levels in preorder
        std::vector<int> st{r};
        while (!st.empty()) {
            const int h = st.back();
            st.pop_back();
            order.push_back(h);
            TravChild k4[4];
            const int nk = kids(head[h], k4);
            for (int i = nk - 1; i >= 0; --i)
                if (!k4[i].leaf) st.push_back(qid[k4[i].ref]);
        }
    }
    for (int i = 0; i < (int)order.size(); ++i) num[order[i]] = i;
    out.assign(Q, QuadRecord{});
    std::vector<int> need(Q, 0);
    for (int h = Q - 1; h >= 0; --h) {   // a record's children come after it breadth-first
        QuadRecord& R = out[num[h]];
        R.n = kids(head[h], R.c);
        int deeper = 0;
        for (int i = 0; i < R.n; ++i)
            if (!R.c[i].leaf) {
                const int ch = qid[R.c[i].ref];
                deeper = std::max(deeper, need[ch]);
                R.c[i].ref = num[ch];
            }
        need[h] = (R.n - 1) + deeper;
    }
    stack_need = need[0];
}

}  // namespace pth
