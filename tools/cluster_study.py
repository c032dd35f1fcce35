"""How much of the fused kernel's candidate pre-test a wave could skip (CPU study, oracle rays).

For every bounce >= 1 of a few frames of a scene (the oracle's per-bounce path dumps, live paths in
order, 64 to a wave), count per wave:
  flat      : geoms tested (every geom, what cull_candidates does today)
  clustered : cluster boxes tested + the geoms of every cluster that some lane's ray passes
with the pre-test's slab rule (t1 >= max(t0, -0.01)) on world boxes.  Clusters: greedy spatial
grouping of the geoms' boxes.  Waves either in path order or after regrouping each 256-path block
by the ray direction's dominant axis (6 classes).

    python tools/cluster_study.py [--scene cornell_obj_khaslana] [--res 160] [--frames 2]
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


if __name__ == "__main__":
    main()
