"""Survivors ordered by their next pre-test superset (PT_SORT_NEXT=1, SceneDev::sort_next).

In candidate-table scenes (16..64 geoms, e.g. khaslana's 44) the pre-test runs each lane's
superset of geoms in a per-lane loop, so a wave pays for its largest superset.  With sort_next the
fused bounce kernel writes each block's survivors in the order of their next superset's size
(block_append_keyed: key = min(15, superset size), (key, wave, lane) order), so the next bounce's
waves hold rays of like superset size.  Only the order of paths in the wavefront changes; every
path's arithmetic and RNG key are its own, so images and live counts stay bit-identical to the
oracle (the reference's order).
"""
import numpy as np
import pytest

from conftest import scene_path

BIT = dict(trig_mode=1, arg_order=0)
pytestmark = pytest.mark.gpu


def _eq(x, y):
    return np.asarray(x).tobytes() == np.asarray(y).tobytes()


@pytest.mark.parametrize("fused_tail", [0, 1])
@pytest.mark.parametrize("res,frames", [((64, 64), 4), ((160, 96), 2)])
def test_sorted_survivors_bitexact(res, frames, fused_tail, oracle, ptamd, monkeypatch):
    monkeypatch.setenv("PT_SORT_NEXT", "1")
    monkeypatch.setenv("PT_BVH_TAIL_FUSED", str(fused_tail))
    name, depth = "cornell_obj_khaslana", 12
    a = oracle.load_scene(scene_path(name), res=res, depth=depth)
    b = ptamd.SceneFile(scene_path(name), res=res, depth=depth)
    r = oracle.Renderer(a, oracle.options(**BIT))
    tr = ptamd.PathTracer(b)
    try:
        tot = np.zeros(depth, np.int64)
        for it in range(1, frames + 1):
            tot += np.maximum(r.trace(it), 0)[:depth]
        tr.trace_frames(1, frames)
        assert tr.stats()["live_total"][:depth] == tot.tolist()
        assert _eq(tr.image(), r.image)
        for it in (frames + 1, frames + 2):          # single frames (the API's pathtrace())
            live = r.trace(it)
            tr.trace(it, copy_image=True)
            assert tr.stats()["live"][:depth] == [int(x) if x >= 0 else 0 for x in live][:depth]
        assert _eq(tr.image(), r.image)
    finally:
        tr.free()


def test_sorted_survivors_sections(ptamd, monkeypatch):
    """The section-counter build reports the superset sizes: the waves' largest superset per wave
    is at least the mean per lane, with and without the ordering."""
    import os
    out = {}
    for arm in ("0", "1"):
        monkeypatch.setenv("PT_SORT_NEXT", arm)
        b = ptamd.SceneFile(scene_path("cornell_obj_khaslana"), res=(128, 128), depth=12)
        tr = ptamd.PathTracer(b, variant=190)
        try:
            tr.trace_frames(1, 2)
            tr.synchronize()
            tr.section_counters(reset=True)
            tr.trace_frames(3, 2)
            tr.synchronize()
            c = tr.section_counters(reset=True)
        finally:
            tr.free()
        assert c["n_sup"] > 0 and c["n_sup_wmax"] > 0
        out[arm] = c["n_sup_wmax"]
    assert os.environ.get("PT_SORT_NEXT") == "1"
    assert out["1"] <= out["0"], out
