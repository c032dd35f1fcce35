"""Handed-over traversals (k_bvh_bounce -> k_bvh_tail_trav -> k_bvh_tail_shade, pt_runtime.hip).

Once no more than PT_BVH_TAIL_LANES lanes of a traversal wave are still traversing, those rays'
traversal state (best hit, next node, stack) is written out; k_bvh_tail_trav resumes them in waves
that refill their lanes from the segment's shared counter as rays finish (PT_BVH_TAIL_REFILL idle
lanes at a time), and k_bvh_tail_shade shades them in full waves.  The result must not depend on where a
traversal was cut or which wave finished it: every setting below renders the mesh scenes
bit-identical to the oracle (the reference's DFS order), live counts included, through
multi-frame passes and single API frames.  A tail segment holds at most PT_BVH_TAIL_CHUNKS x 256
rays: with 1 chunk most waves find it full and finish their rays themselves (tail_put's refusal
path).  PT_BVH_TAIL_SHADE_BLOCKS=1: one k_bvh_tail_shade block per segment loops over all of its
chunks (0: a block per chunk of the capacity).
"""
import numpy as np
import pytest

from conftest import scene_path

BIT = dict(trig_mode=1, arg_order=0)
pytestmark = pytest.mark.gpu


def _eq(x, y):
    return np.asarray(x).tobytes() == np.asarray(y).tobytes()


@pytest.mark.parametrize("lanes,chunks,refill,shade", [(0, 0, 16, 512), (1, 0, 16, 512), (32, 0, 16, 512),
                                                       (56, 0, 1, 1), (24, 0, 64, 0), (32, 1, 16, 512),
                                                       (8, 1, 64, 1)])
@pytest.mark.parametrize("name,res,depth", [("cornell_obj_bnnuy", (96, 96), None),
                                            ("cornell_obj_khaslana", (64, 64), 12)])
def test_handed_over_traversals_bitexact(name, res, depth, lanes, chunks, refill, shade, oracle, ptamd, monkeypatch):
    monkeypatch.setenv("PT_BVH_TAIL_REFILL", str(refill))
    monkeypatch.setenv("PT_BVH_TAIL_SHADE_BLOCKS", str(shade))
    monkeypatch.setenv("PT_BVH_TAIL_LANES", str(lanes))
    monkeypatch.setenv("PT_BVH_TAIL_CHUNKS", str(chunks))
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
        assert _eq(tr.image(), r.image), (name, lanes, chunks, refill, shade)
        assert tr.stats()["segments_total"] == segs
        for it in (7, 8):                          # single frames (the API's pathtrace())
            live = r.trace(it)
            tr.trace(it, copy_image=True)
            assert tr.stats()["live"][:a.trace_depth] == [int(x) if x >= 0 else 0 for x in live][:a.trace_depth]
        assert _eq(tr.image(), r.image), (name, lanes, chunks, refill, shade)
    finally:
        tr.free()

