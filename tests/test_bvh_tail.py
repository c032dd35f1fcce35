"""Handed-over traversals (k_bvh_bounce -> k_bvh_tail levels, pt_runtime.hip).

Once no more than PT_BVH_TAIL_LANES lanes of a traversal wave are still traversing, those rays'
traversal state (best hit, next node, stack) is written out and a k_bvh_tail launch resumes them 64
to a wave -- handing on again, up to PT_BVH_TAIL_LEVELS levels, the last one finishing them.  The
result must not depend on where a traversal was cut: every setting below renders the mesh scenes
bit-identical to the oracle (the reference's DFS order), live counts included, through multi-frame
passes and single API frames.  lanes = 32 with 4 levels hands over the most rays and reaches the
third and fourth levels; lanes = 1 only the last lane of a wave.  A level's buffer holds at most
PT_BVH_TAIL_CHUNKS x 256 rays per segment: with 1 chunk most waves find it full and finish their
rays themselves (tail_put's refusal path).
"""
import numpy as np
import pytest

from conftest import scene_path

BIT = dict(trig_mode=1, arg_order=0)
pytestmark = pytest.mark.gpu


def _eq(x, y):
    return np.asarray(x).tobytes() == np.asarray(y).tobytes()


@pytest.mark.parametrize("lanes,levels,chunks", [(0, 1, 128), (1, 1, 128), (16, 1, 128), (16, 2, 128),
                                                 (32, 4, 128), (32, 3, 1)])
@pytest.mark.parametrize("name,res,depth", [("cornell_obj_bnnuy", (96, 96), None),
                                            ("cornell_obj_khaslana", (64, 64), 12)])
def test_handed_over_traversals_bitexact(name, res, depth, lanes, levels, chunks, oracle, ptamd, monkeypatch):
    monkeypatch.setenv("PT_BVH_TAIL_LANES", str(lanes))
    monkeypatch.setenv("PT_BVH_TAIL_CHUNKS", str(chunks))
    monkeypatch.setenv("PT_BVH_TAIL_LEVELS", str(levels))
    a = oracle.load_scene(scene_path(name), res=res, depth=depth)
    b = ptamd.SceneFile(scene_path(name), res=res, depth=depth)
    r = oracle.Renderer(a, oracle.options(**BIT))
    tr = ptamd.PathTracer(b)
    try:
        segs = 0
        for it in range(1, 7):                     # one pass of 6 frames
            live = r.trace(it)
            segs += int(np.maximum(live, 0).sum())
        tr.trace_frames(1, 6)
        assert _eq(tr.image(), r.image), (name, lanes, levels)
        assert tr.stats()["segments_total"] == segs
        for it in (7, 8):                          # single frames (the API's pathtrace())
            live = r.trace(it)
            tr.trace(it, copy_image=True)
            assert tr.stats()["live"][:a.trace_depth] == [int(x) if x >= 0 else 0 for x in live][:a.trace_depth]
        assert _eq(tr.image(), r.image), (name, lanes, levels)
    finally:
        tr.free()
