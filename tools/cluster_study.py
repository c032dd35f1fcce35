"""How much of the fused kernel's candidate pre-test a wave could skip (CPU study, oracle rays).

For every bounce >= 1 of a few frames of a scene (the oracle's per-bounce path dumps, live paths in
order, 64 to a wave), count per wave:
  flat      : geoms tested (every geom, what cull_candidates does today)
  clustered : cluster boxes tested + the geoms of every cluster that some lane's ray passes
with the pre-test's slab rule (t1 >= max(t0, -0.01)) on world boxes.  Clusters: greedy spatial
grouping of the geoms' boxes.  Waves either in path order or after regrouping each 256-path block
by the ray direction's dominant axis (6 classes).

    python tools/cluster_study.py [--scene cornell_obj_khaslana] [--res 160] [--frames 2]
    python tools/cluster_study.py --tree [...]     # per-lane tree over the geoms' boxes (below)
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402


def world_boxes(sc):
    lo, hi = [], []
    for g in sc.geoms:
        M = np.array(g["transform"], np.float64).T      # glm column-major -> row-major
        c = np.array([[x, y, z, 1.0] for x in (-.5, .5) for y in (-.5, .5) for z in (-.5, .5)])
        w = (M @ c.T).T[:, :3]
        lo.append(w.min(0)); hi.append(w.max(0))
    return np.array(lo), np.array(hi)


def passes(o, d, lo, hi):
    """[nrays, nboxes] pre-test pass mask."""
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = np.clip(1.0 / d, -1e20, 1e20)
    a = (lo[None, :, :] - o[:, None, :]) * inv[:, None, :]
    b = (hi[None, :, :] - o[:, None, :]) * inv[:, None, :]
    t0 = np.maximum(np.minimum(a, b).max(2), -1e-2)
    t1 = np.maximum(a, b).min(2)
    return t1 >= t0


def clusters(lo, hi, k):
    """greedy: repeatedly merge the pair whose union box grows the least (surface area)."""
    groups = [[i] for i in range(len(lo))]
    blo, bhi = [lo[i].copy() for i in range(len(lo))], [hi[i].copy() for i in range(len(lo))]
    def area(l, h):
        e = np.maximum(h - l, 0)
        return e[0] * e[1] + e[1] * e[2] + e[2] * e[0]
    while len(groups) > k:
        best = None
        for i in range(len(groups)):
            for j in range(i + 1, len(groups)):
                l, h = np.minimum(blo[i], blo[j]), np.maximum(bhi[i], bhi[j])
                c = area(l, h) - area(blo[i], bhi[i]) - area(blo[j], bhi[j])
                if best is None or c < best[0]:
                    best = (c, i, j, l, h)
        _, i, j, l, h = best
        groups[i] += groups[j]; blo[i], bhi[i] = l, h
        del groups[j], blo[j], bhi[j]
    return groups, np.array(blo), np.array(bhi)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell_obj_khaslana")
    ap.add_argument("--res", type=int, default=160)
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--clusters", default="4,6,8,12")
    args = ap.parse_args()
    sc = O.load_scene(os.path.join(REPO, "scenes", args.scene + ".json"), res=(args.res, args.res))
    lo, hi = world_boxes(sc)
    ng = len(lo)
    rays = []
    r = O.Renderer(sc, O.options(trig_mode=1))
    for it in range(1, args.frames + 1):
        _, dump = r.trace(it, dump=True)
        for b in range(1, sc.trace_depth):
            p = dump[b][dump[b]["remainingBounces"] > 0]
            if len(p):
                rays.append((p["origin"].astype(np.float64), p["direction"].astype(np.float64)))
    print(f"{args.scene}: {ng} geoms, {sum(len(o) for o, _ in rays)} bounce>=1 rays")
    for k in [int(x) for x in args.clusters.split(",")]:
        groups, clo, chi = clusters(lo, hi, k)
        for sort in (False, True):
            flat = clus = waves = 0
            for o, d in rays:
                if sort:   # regroup each 256-ray block by dominant direction axis
                    key = np.argmax(np.abs(d), 1) * 2 + (d[np.arange(len(d)), np.argmax(np.abs(d), 1)] > 0)
                    idx = np.concatenate([s + np.argsort(key[s:s + 256], kind="stable") for s in range(0, len(d), 256)])
                    o, d = o[idx], d[idx]
                cp = passes(o, d, clo, chi)
                for w in range(0, len(o), 64):
                    waves += 1
                    flat += ng
                    need = cp[w:w + 64].any(0)
                    clus += k + sum(len(groups[c]) for c in range(k) if need[c])
            print(f"  clusters {k:2d} {'sorted' if sort else 'order '}: geom tests per wave flat {flat / waves:.1f}, "
                  f"clustered {clus / waves:.1f} ({clus / flat:.2f}x)")


if __name__ == "__main__" and "--tree" not in sys.argv:
    main()


# ---------------------------------------------------------------------------------------------
# a per-lane tree over the geoms' boxes instead of the flat pre-test.
# Each lane walks its own binary tree (near-first is irrelevant without a t bound: the pre-test
# has no exact hit to cull with, so a lane visits every node its infinite ray passes); the wave
# runs as long as its slowest lane.  Counted: node (box) tests per lane, the wave-max per wave,
# for a tree over all geoms and for "large boxes flat + tree over the rest".
# ---------------------------------------------------------------------------------------------
def sah_tree(lo, hi, ids):
    """binary SAH tree (object split over centroid-sorted prefixes) -> nested tuples"""
    if len(ids) == 1:
        return ids[0]
    def area(l, h):
        e = np.maximum(h - l, 0)
        return e[0] * e[1] + e[1] * e[2] + e[2] * e[0]
    best = None
    for ax in range(3):
        order = sorted(ids, key=lambda i: lo[i][ax] + hi[i][ax])
        for s in range(1, len(order)):
            L, R = order[:s], order[s:]
            c = (area(lo[L].min(0), hi[L].max(0)) * len(L) + area(lo[R].min(0), hi[R].max(0)) * len(R))
            if best is None or c < best[0]:
                best = (c, L, R)
    return (sah_tree(lo, hi, best[1]), sah_tree(lo, hi, best[2]))


def tree_boxes(t, lo, hi, out):
    if isinstance(t, tuple):
        a = tree_boxes(t[0], lo, hi, out)
        b = tree_boxes(t[1], lo, hi, out)
        box = (np.minimum(a[0], b[0]), np.maximum(a[1], b[1]))
    else:
        box = (lo[t], hi[t])
    out.append((t, box))
    return box


def lane_visits(t, o, d, lo, hi):
    """node tests per ray of a per-lane DFS of tree t (every node whose box the ray passes)"""
    nodes = []
    tree_boxes(t, lo, hi, nodes)
    box_of = {id(n): b for n, b in nodes}
    visits = np.zeros(len(o), np.int64)
    def walk(n, mask):
        # mask: rays that reached node n (the parent's box passed): they test n's box
        visits[mask] += 1
        l, h = box_of[id(n)] if isinstance(n, tuple) else (lo[n], hi[n])
        p = np.zeros(len(o), bool)
        p[mask] = passes(o[mask], d[mask], l[None], h[None])[:, 0]
        if isinstance(n, tuple) and p.any():
            walk(n[0], p)
            walk(n[1], p)
    walk(t, np.ones(len(o), bool))
    return visits


def tree_study(sc, rays, lo, hi):
    ng = len(lo)
    ext = (hi - lo).max(1)
    big = [i for i in range(ng) if ext[i] > 0.5 * ext.max()]
    rest = [i for i in range(ng) if i not in big]
    o = np.concatenate([x for x, _ in rays])
    d = np.concatenate([y for _, y in rays])
    full = sah_tree(lo, hi, list(range(ng)))
    part = sah_tree(lo, hi, rest) if len(rest) > 1 else None
    v_full = lane_visits(full, o, d, lo, hi)
    v_part = len(big) + (lane_visits(part, o, d, lo, hi) if part is not None else 0)
    cand = passes(o, d, lo, hi).sum(1)
    for name, v in (("tree over all geoms", v_full), (f"{len(big)} large flat + tree over {len(rest)}", v_part)):
        wmax = [v[w:w + 64].max() for w in range(0, len(v), 64)]
        print(f"  {name}: box tests per lane mean {v.mean():.1f}, wave-max mean {np.mean(wmax):.1f} "
              f"(flat: {ng} per lane; boxes passed per ray {cand.mean():.2f})")


def tree_main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell_obj_khaslana")
    ap.add_argument("--res", type=int, default=160)
    ap.add_argument("--frames", type=int, default=2)
    args, _ = ap.parse_known_args()
    sc = O.load_scene(os.path.join(REPO, "scenes", args.scene + ".json"), res=(args.res, args.res))
    lo, hi = world_boxes(sc)
    rays = []
    r = O.Renderer(sc, O.options(trig_mode=1))
    for it in range(1, args.frames + 1):
        _, dump = r.trace(it, dump=True)
        for b in range(1, sc.trace_depth):
            p = dump[b][dump[b]["remainingBounces"] > 0]
            if len(p):
                rays.append((p["origin"].astype(np.float64), p["direction"].astype(np.float64)))
    print(f"{args.scene}: {len(lo)} geoms, {sum(len(o) for o, _ in rays)} bounce>=1 rays (per-lane tree study)")
    tree_study(sc, rays, lo, hi)


if __name__ == "__main__" and "--tree" in sys.argv:
    sys.argv.remove("--tree")
    tree_main()
