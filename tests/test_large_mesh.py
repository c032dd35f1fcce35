"""Meshes past the 65,535-ref pair layout of rounds 2-5 (VERDICT r05 "What's missing" 1).

The reference names meshes far larger than bunny / khaslana (scenes/cornell_obj_cyrene.json:266,
cornell_obj_phainon*.json; README.md:206 times cyrene at 282 ms/frame).  Their OBJ files are not in
the checkout, so tools/make_synthetic_meshes.py writes stand-ins at the same paths: cyrene.obj
262,208 triangles (173,591 reference BVH nodes), phainon.obj 1,001,884 triangles (661,995 nodes).

The pair layout (DevPair records, the k_bounce -> k_bvh_bounce traversal queue and the hand-over
to k_bvh_tail_trav) now holds trees of up to 2^24 refs: a stack entry is [ref | T field] with as
few ref bits as the tree needs (pack_ref, pt_kernels.h) and the cull threshold T in the rest,
rounded down.  These tests check that those scenes take that path (rays are queued) and that it is
bit-exact against the oracle (the reference's DFS order) -- images, per-bounce live counts, the
hand-over at its extremes -- and that the full intersection records equal the reference's own
intersections.cu (tests/golden/ref_pin.json, made by oracle/ref_pins/make_ref_fixtures.py).
"""
import json
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN, scene_path

BIT = dict(trig_mode=1, arg_order=0)
LARGE = [("cornell_obj_cyrene", (64, 64)), ("cornell_obj_phainon", (48, 48))]


def _eq(x, y):
    return np.asarray(x).tobytes() == np.asarray(y).tobytes()


# ---- the stack entry's T field (host restatement of pack_ref / unpack_T; CPU) ----
T_BIAS = 0x37000000


def _bits(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def _flt(b):
    return struct.unpack("<f", struct.pack("<I", b & 0xffffffff))[0]


def _pack_T(T, S):
    u = min(max(_bits(T), T_BIAS), T_BIAS + 0x3fffffff) - T_BIAS
    return u >> (30 - S)


def _unpack_T(field, S):
    return _flt((field << (30 - S)) + T_BIAS)


@pytest.mark.parametrize("S", [8, 10, 12, 14, 16, 20, 30])
def test_stack_entry_threshold_rounds_down(S):
    """For every ref width the decoded cull threshold never exceeds the true one (a cull may only
    be lost, never added), except below 2^-17, where it decodes to 2^-17: a cull there needs
    t_best < 2^-17 < 1e-5, when no triangle can be accepted (tri_test_e rejects t <= 1e-5)."""
    rng = np.random.default_rng(S)
    vals = np.concatenate([np.float32(2.0) ** rng.uniform(-30, 120, 4000).astype(np.float32),
                           np.array([0.0, 1e-5, 2.0 ** -17, 1.0, 3.4e38, np.inf], np.float32)])
    worst = 0.0
    for T in vals.astype(np.float32):
        T = float(T)
        d = _unpack_T(_pack_T(T, S), S)
        if T >= 2.0 ** -17:
            assert d <= T, (S, T, d)
            if T < 2.0 ** 110:
                worst = max(worst, 1.0 - d / T)
        else:
            assert d == 2.0 ** -17 and d < 1e-5
    # the relative loss is bounded by the mantissa bits the field keeps (S - 7)
    assert worst < 2.0 ** -(S - 7) + 1e-12, (S, worst)
    # the field fits S bits, so refs of 32 - S bits fit beside it
    assert _pack_T(3.4e38, S) < (1 << S)


def test_large_mesh_fixtures_present():
    """The reference's own intersections.cu has been run on both stand-ins (ref_pin.json)."""
    with open(os.path.join(GOLDEN, "ref_pin.json")) as f:
        fx = json.load(f)
    for name, _ in LARGE:
        counts = fx["scenes"][name]["counts"]
        assert counts["triangles"] > 250000 and counts["bvhNodes"] > 65535
        assert fx["isect"][name]["hits"] > 1000


# ---- GPU ----
@pytest.mark.gpu
@pytest.mark.parametrize("name,res", LARGE)
def test_large_mesh_fast_path_bitexact(name, res, oracle, ptamd):
    """Multi-frame pass + single API frames on the split traversal (queue + hand-over), bit-exact."""
    a = oracle.load_scene(scene_path(name), res=res)
    b = ptamd.SceneFile(scene_path(name), res=res)
    assert len(b.triangles) > 250000 and len(b.bvh_nodes) > 65535
    r = oracle.Renderer(a, oracle.options(**BIT))
    tr = ptamd.PathTracer(b)
    try:
        segs = 0
        for it in range(1, 5):
            segs += int(np.maximum(r.trace(it), 0).sum())
        tr.trace_frames(1, 4)
        st = tr.stats()
        assert sum(st["queued_total"]) > 0, "the mesh rays did not take the traversal queue"
        assert _eq(tr.image(), r.image), name
        assert st["segments_total"] == segs
        for it in (5, 6):
            live = r.trace(it)
            tr.trace(it, copy_image=True)
            assert tr.stats()["live"][:a.trace_depth] == [int(x) if x >= 0 else 0 for x in live][:a.trace_depth]
        assert _eq(tr.image(), r.image), name
    finally:
        tr.free()


@pytest.mark.gpu
@pytest.mark.parametrize("lanes,refill,chunks", [(56, 1, 0), (32, 64, 1)])
def test_large_mesh_hand_over_extremes(lanes, refill, chunks, oracle, ptamd, monkeypatch):
    """Hand-over at its extremes on the 262k-triangle tree: 24-bit node refs saved and resumed."""
    monkeypatch.setenv("PT_BVH_TAIL_LANES", str(lanes))
    monkeypatch.setenv("PT_BVH_TAIL_REFILL", str(refill))
    monkeypatch.setenv("PT_BVH_TAIL_CHUNKS", str(chunks))
    name, res = LARGE[0]
    a = oracle.load_scene(scene_path(name), res=res)
    b = ptamd.SceneFile(scene_path(name), res=res)
    r = oracle.Renderer(a, oracle.options(**BIT))
    tr = ptamd.PathTracer(b)
    try:
        for it in range(1, 4):
            r.trace(it)
        tr.trace_frames(1, 3)
        assert _eq(tr.image(), r.image), (lanes, refill, chunks)
    finally:
        tr.free()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [None, 26, 250])
@pytest.mark.parametrize("name", [n for n, _ in LARGE])
def test_large_mesh_intersections_match_reference(name, variant, ptamd):
    """Full 52-B intersection records on 4096 probe rays (axis / NaN / inf rays, vertex and edge
    ties) equal the reference's own computeIntersections: default variant (pair layout), the
    pair traversal without the queue (26), and the node-array traversal (250)."""
    import refpins as R
    with open(os.path.join(GOLDEN, "ref_pin.json")) as f:
        ref = json.load(f)["isect"][name]
    b = ptamd.SceneFile(scene_path(name), res=(96, 96))
    raw = ptamd.SceneFile(scene_path(name), viewer_camera=False)
    rays = R.rays(R.ISECT_RAYS, seed=len(name), targets=R.scene_targets(raw.geoms, raw.triangles))
    assert R.digest(rays) == ref["rays_sha256"]
    tr = ptamd.PathTracer(b, **({} if variant is None else {"variant": variant}))
    got = tr.test_intersect(rays.astype(ptamd.PATH))
    tr.free()
    assert int((got["t"] > 0).sum()) == ref["hits"]
    assert R.digest(R.pack(got, R.P_ISECT)) == ref["isect_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("levels", [0, 8])
def test_pair_numbering_does_not_change_results(levels, oracle, ptamd, monkeypatch):
    """PT_BVH_BFS_LEVELS: the SAH pairs numbered breadth-first over the top levels and in preorder
    below (0: preorder throughout) -- only where the records live changes, not what is visited."""
    monkeypatch.setenv("PT_BVH_BFS_LEVELS", str(levels))
    name, res = LARGE[0]
    a = oracle.load_scene(scene_path(name), res=res)
    b = ptamd.SceneFile(scene_path(name), res=res)
    r = oracle.Renderer(a, oracle.options(**BIT))
    tr = ptamd.PathTracer(b)
    try:
        for it in range(1, 4):
            r.trace(it)
        tr.trace_frames(1, 3)
        assert _eq(tr.image(), r.image), levels
    finally:
        tr.free()


@pytest.mark.gpu
@pytest.mark.parametrize("bound", [0, 19])
def test_bounded_tree_height_does_not_change_results(bound, oracle, ptamd, monkeypatch):
    """PT_BVH_MAX_HEIGHT: the SAH tree over the reference's leaves with its height bounded (median
    splits where SAH would leave a child no room; 0: unbounded) -- the same leaves are visited, so
    the image is the oracle's."""
    monkeypatch.setenv("PT_BVH_MAX_HEIGHT", str(bound))
    name, res = LARGE[1]
    a = oracle.load_scene(scene_path(name), res=res)
    b = ptamd.SceneFile(scene_path(name), res=res)
    r = oracle.Renderer(a, oracle.options(**BIT))
    tr = ptamd.PathTracer(b)
    try:
        for it in range(1, 4):
            r.trace(it)
        tr.trace_frames(1, 3)
        assert _eq(tr.image(), r.image), bound
    finally:
        tr.free()


@pytest.mark.gpu
@pytest.mark.parametrize("quad", [0, 1])
@pytest.mark.parametrize("name,res,depth,lanes", [("cornell_obj_bnnuy", (96, 96), None, 40),
                                                   ("cornell_obj_khaslana", (64, 64), 12, 56),
                                                   ("cornell_obj_cyrene", (48, 48), None, 8)])
def test_four_wide_records_bitexact(name, res, depth, lanes, quad, oracle, ptamd, monkeypatch):
    """PT_BVH_QUAD: the traversal kernels on 4-wide records (two levels of the hierarchy in one
    128-B line; by default for trees of 65,536 refs or more) or on the pairs, forced either way on
    every mesh scene -- multi-frame passes and API frames bit-exact, live counts included."""
    monkeypatch.setenv("PT_BVH_QUAD", str(quad))
    monkeypatch.setenv("PT_BVH_TAIL_LANES", str(lanes))
    a = oracle.load_scene(scene_path(name), res=res, depth=depth)
    b = ptamd.SceneFile(scene_path(name), res=res, depth=depth)
    r = oracle.Renderer(a, oracle.options(**BIT))
    tr = ptamd.PathTracer(b)
    try:
        segs = 0
        for it in range(1, 5):
            segs += int(np.maximum(r.trace(it), 0).sum())
        tr.trace_frames(1, 4)
        st = tr.stats()
        assert sum(st["queued_total"]) > 0
        assert _eq(tr.image(), r.image), (name, quad)
        assert st["segments_total"] == segs
        for it in (5, 6):
            live = r.trace(it)
            tr.trace(it, copy_image=True)
            assert tr.stats()["live"][:a.trace_depth] == [int(x) if x >= 0 else 0 for x in live][:a.trace_depth]
        assert _eq(tr.image(), r.image), (name, quad)
    finally:
        tr.free()


@pytest.mark.gpu
@pytest.mark.parametrize("lds,quad", [(2, 1), (5, 1), (3, 0), (16, 1)])
@pytest.mark.parametrize("name,res,depth", [("cornell_obj_bnnuy", (96, 96), None),
                                            ("cornell_obj_khaslana", (64, 64), 12),
                                            ("cornell_obj_cyrene", (48, 48), None)])
def test_spilled_stack_bitexact(name, res, depth, lds, quad, oracle, ptamd, monkeypatch):
    """PT_BVH_STACK_LDS: only the first `lds` traversal stack entries in LDS, deeper ones in a spill
    row per queue slot -- through the hand-over too (its saved stack is the LDS part; the spilled
    entries stay in the slot's row) -- bit-exact, with 4-wide records and pairs."""
    monkeypatch.setenv("PT_BVH_STACK_LDS", str(lds))
    monkeypatch.setenv("PT_BVH_QUAD", str(quad))
    a = oracle.load_scene(scene_path(name), res=res, depth=depth)
    b = ptamd.SceneFile(scene_path(name), res=res, depth=depth)
    r = oracle.Renderer(a, oracle.options(**BIT))
    tr = ptamd.PathTracer(b)
    try:
        segs = 0
        for it in range(1, 4):
            segs += int(np.maximum(r.trace(it), 0).sum())
        tr.trace_frames(1, 3)
        assert _eq(tr.image(), r.image), (name, lds, quad)
        assert tr.stats()["segments_total"] == segs
        for it in (4, 5):
            r.trace(it)
            tr.trace(it, copy_image=True)
        assert _eq(tr.image(), r.image), (name, lds, quad)
    finally:
        tr.free()
