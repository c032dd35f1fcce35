"""Shared helpers of the reference pins (TEST INFRASTRUCTURE).

Used by oracle/ref_pins/make_ref_fixtures.py (which runs the reference's own code, built into
oracle/_ref/ by oracle/ref_pins/make_fixtures.sh, and writes tests/golden/ref_pin.json) and by the
tests that check the oracle, the C++ scene loader and the HIP kernels against that fixture.

* Packed dtypes: the field streams oracle/ref_pins/ref_harness.cpp writes — every field of the
  reference structs (sceneStructs.h:18-165) in declaration order, without padding bytes.
* `rays(scene_kind, n, targets, eye)`: deterministic probe rays, generated from an integer hash
  with float32 arithmetic only, so this container and the GPU box produce identical bytes.
* `digest(arr)`: sha256 of the packed bytes with every float NaN canonicalised (the reference's
  x86 build and the GPU may produce NaNs of different sign/payload; their value is the same).
"""
from __future__ import annotations

import hashlib

import numpy as np

V3 = ("<f4", (3,))
P_VERTEX = np.dtype([("materialID", "<i4"), ("position",) + V3, ("normal",) + V3, ("uv", "<f4", (2,))])
P_GEOM = np.dtype([("type", "<i4"), ("materialid", "<i4"), ("translation",) + V3, ("rotation",) + V3,
                   ("scale",) + V3, ("transform", "<f4", (4, 4)), ("inverseTransform", "<f4", (4, 4)),
                   ("invTranspose", "<f4", (4, 4))])
P_MATERIAL = np.dtype([("color",) + V3, ("spec_exponent", "<f4"), ("spec_color",) + V3, ("hasReflective", "<f4"),
                       ("hasRefractive", "<f4"), ("roughness", "<f4"), ("metallic", "<f4"),
                       ("indexOfRefraction", "<f4"), ("emittance", "<f4"), ("hasTexture", "u1"),
                       ("textureID", "<i4"), ("hasBumpMap", "u1"), ("bumpID", "<i4"), ("bumpScale", "<f4")])
P_TRIANGLE = np.dtype([("v1", P_VERTEX), ("v2", P_VERTEX), ("v3", P_VERTEX), ("centroid",) + V3,
                       ("materialID", "<i4"), ("dpdu",) + V3, ("dpdv",) + V3])
P_BVHNODE = np.dtype([("min",) + V3, ("max",) + V3, ("left", "<i4"), ("right", "<i4"), ("start", "<i4"),
                      ("triCount", "<i4")])
P_CAMERA = np.dtype([("resolution", "<i4", (2,)), ("position",) + V3, ("lookAt",) + V3, ("view",) + V3,
                     ("up",) + V3, ("right",) + V3, ("fov", "<f4", (2,)), ("pixelLength", "<f4", (2,)),
                     ("aperture", "<f4"), ("focalDist", "<f4")])
P_PATH = np.dtype([("origin",) + V3, ("direction",) + V3, ("color",) + V3, ("pixelIndex", "<i4"),
                   ("remainingBounces", "<i4")])
P_ISECT = np.dtype([("t", "<f4"), ("surfaceNormal",) + V3, ("materialId", "<i4"), ("uv", "<f4", (2,)),
                    ("dpdu",) + V3, ("dpdv",) + V3])
# per (ray, geom): box / sphere test result (ref_harness prims)
P_PRIM = np.dtype([("t", "<f4"), ("point",) + V3, ("normal",) + V3, ("outside", "<i4")])
# per (ray, triangle): intersectTriangle (ref_harness tris)
P_TRI = np.dtype([("hit", "<i4"), ("t", "<f4"), ("u", "<f4"), ("v", "<f4")])

TRIS_K = 48   # triangles / BVH nodes probed per ray by `ref_harness tris`


def pack(arr: np.ndarray, packed: np.dtype) -> np.ndarray:
    """Copy a (possibly padded) structured array into the packed dtype, field by field."""
    out = np.zeros(arr.shape, packed)
    for name in packed.names:
        src = name
        if src not in arr.dtype.names:
            raise KeyError(name)
        sub = packed.fields[name][0]
        if sub.names:
            out[name] = pack(arr[src], sub)
        else:
            out[name] = arr[src]
    return out


def _canon(a: np.ndarray) -> np.ndarray:
    """NaN-canonicalised copy (structured: per float field)."""
    a = np.array(a, copy=True)
    if a.dtype.names:
        for n in a.dtype.names:
            a[n] = _canon(a[n])
        return a
    if a.dtype.kind == "f":
        a[np.isnan(a)] = np.float32(np.nan)
    return a


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(_canon(a)).tobytes()).hexdigest()


# ---------------------------------------------------------------------------------------------
# probe rays
# ---------------------------------------------------------------------------------------------
def _hash(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def _u(seed: int, n: int, k: int) -> np.ndarray:
    """(n, k) floats in [0, 1): 24-bit hashes scaled exactly."""
    i = np.arange(n * k, dtype=np.uint64).astype(np.uint32) + np.uint32((seed * 0x9E3779B9) & 0xFFFFFFFF)
    h = _hash(_hash(i) ^ np.uint32(seed & 0xFFFFFFFF))
    return ((h >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)).reshape(n, k)


def _normalize(d: np.ndarray) -> np.ndarray:
    d = d.astype(np.float32)
    ln = np.sqrt((d * d).sum(axis=1, dtype=np.float32)).astype(np.float32)
    ln[ln == 0] = np.float32(1)
    return (d / ln[:, None]).astype(np.float32)


def rays(n: int, seed: int, targets: np.ndarray, eye=(0.0, 5.0, 10.5),
         lo=(-5.6, -0.6, -5.6), hi=(5.6, 10.6, 11.0)) -> np.ndarray:
    """n probe rays (PathSegment records).  Mix: random origin/direction, aimed at `targets`
    (geom centres, triangle vertices / edge midpoints / centroids), axis-aligned, near-axis (a
    component below aabbIntersectionTest's 1e-5 threshold, or exactly +-0), camera-like from
    `eye`, and a few degenerate rays (NaN / inf / zero direction)."""
    f32 = np.float32
    lo, hi, eye = np.array(lo, f32), np.array(hi, f32), np.array(eye, f32)
    u = _u(seed, n, 8)
    org = (lo + u[:, 0:3] * (hi - lo)).astype(f32)
    d = (u[:, 3:6] * f32(2) - f32(1)).astype(f32)
    kind = (u[:, 6] * f32(20)).astype(np.int32)
    pick = (u[:, 7] * f32(max(1, len(targets)))).astype(np.int64)
    out = np.zeros(n, P_PATH)
    dirs = _normalize(d)
    if len(targets):
        tg = targets[np.minimum(pick, len(targets) - 1)].astype(f32)
        aim = _normalize(tg - org)
        sel = (kind >= 8) & (kind < 14)                       # 30 %: aimed
        dirs[sel] = aim[sel]
    ax = (kind == 14) | (kind == 15)                          # 10 %: axis-aligned
    axis = (u[:, 3] * f32(3)).astype(np.int64) % 3
    sgn = np.where(u[:, 4] < f32(0.5), f32(-1), f32(1))
    a = np.zeros((n, 3), f32)
    a[np.arange(n), axis] = sgn
    dirs[ax] = a[ax]
    near = kind == 16                                         # 5 %: tiny / signed-zero components
    tiny = np.where(u[:, 5] < f32(0.5), f32(3e-6), f32(-0.0))
    dn = dirs.copy()
    dn[np.arange(n), axis] = tiny
    dirs[near] = _normalize(dn)[near]
    cam = (kind == 17) | (kind == 18)                         # 10 %: from the eye
    org[cam] = eye + (u[cam, 0:3] - f32(0.5)) * f32(0.04)
    back = np.stack([lo[0] + u[:, 3] * (hi[0] - lo[0]), lo[1] + u[:, 4] * (hi[1] - lo[1]),
                     np.full(n, lo[2], f32)], axis=1).astype(f32)
    dirs[cam] = _normalize(back - org)[cam]
    out["origin"] = org
    out["direction"] = dirs
    # kind 19 (5 %): degenerate rays, cycling through the cases
    deg = np.flatnonzero(kind == 19)
    for j, i in enumerate(deg):
        c = j % 5
        if c == 0:
            out["direction"][i] = (np.nan, 0.0, 1.0)
        elif c == 1:
            out["direction"][i] = (0.0, 0.0, 0.0)
        elif c == 2:
            out["origin"][i] = (np.inf, 5.0, 0.0)
        elif c == 3:
            out["direction"][i] = (-0.0, -1.0, -0.0)
        else:
            out["origin"][i] = (0.0, 5.0, 1e30)
    out["color"] = 1.0
    out["pixelIndex"] = np.arange(n, dtype=np.int32)
    out["remainingBounces"] = 8
    return out


def scene_targets(geoms: np.ndarray, triangles: np.ndarray) -> np.ndarray:
    """Aim points: geom centres plus, for meshes, triangle vertices, edge midpoints and centroids."""
    pts = [np.asarray(geoms["translation"], np.float32).reshape(-1, 3)]
    if len(triangles):
        p1 = np.asarray(triangles["v1"]["position"], np.float32)
        p2 = np.asarray(triangles["v2"]["position"], np.float32)
        p3 = np.asarray(triangles["v3"]["position"], np.float32)
        mid = ((p1 + p2) * np.float32(0.5)).astype(np.float32)
        pts += [p1, mid, np.asarray(triangles["centroid"], np.float32)]
    return np.concatenate(pts).astype(np.float32)


# scenes whose intersections are pinned (primitives only / meshes with the synthetic stand-ins)
ISECT_SCENES = ["cornell", "cornell_glass_test", "cornell_microfacet_test", "cornell_reflective_test",
                "cornell_transmissive_test", "cornell_multiple_glass", "sphere", "cornell_obj_bnnuy",
                "cornell_obj_khaslana", "cornell_obj_phatphuck_texture_test", "cornell_obj_phainon_halo",
                "cornell_obj_cyrene", "cornell_obj_phainon"]   # 262k / 1.0M-triangle stand-ins
ISECT_RAYS = 4096


def png_input():
    """37x23 float image for the saveImage / savePNG pin: values across the [0, 1] clamp, NaN,
    +-inf and negatives; accumulated over 3 iterations."""
    w, h = 37, 23
    u = _u(77, w * h, 3)
    img = (u * np.float32(4.5) - np.float32(0.5)).astype(np.float32)
    img[5, 0] = np.nan
    img[6, 1] = np.inf
    img[7, 2] = -np.inf
    img[8] = (3.0, 3.0, 3.0)
    img[9] = (2.9999998, 0.0, 765.0 / 255.0)
    return w, h, 3, img


def png_input_large():
    """320x200 float image with smooth gradients, flat regions and repeated tiles, so the
    encoder's long matches, 32 KiB window, hash-chain trimming and every filter type are used;
    accumulated over 5 iterations."""
    w, h = 320, 200
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    r = (x / np.float32(w)) * np.float32(5)
    g = np.where((x.astype(np.int32) // 16 + y.astype(np.int32) // 16) % 2 == 0, np.float32(2.5), np.float32(0.7))
    b = (np.sin(x * np.float32(0.05)) * np.cos(y * np.float32(0.07)) * np.float32(3) + np.float32(2)).astype(np.float32)
    noise = _u(5, w * h, 1).reshape(h, w) * np.float32(0.4)
    img = np.stack([r + noise * (y > 100), g, b], axis=-1).astype(np.float32).reshape(-1, 3)
    return w, h, 5, img
