"""Print the traversal hierarchy's shape per mesh scene (PT_BVH_TREE_INFO=1 at pt_init; tools only):
SAH tree height, pair / 4-wide record counts and the stack entries each layout can need (the
traversal kernels hold that many 1-KB LDS rows per 256-thread block).

    python tools/tree_info.py [scene.json ...]
"""
import os
import sys

os.environ["PT_BVH_TREE_INFO"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))
import ptamd  # noqa: E402

scenes = sys.argv[1:] or [os.path.join(REPO, "scenes", n + ".json") for n in
                          ("cornell_obj_bnnuy", "cornell_obj_khaslana", "cornell_obj_cyrene", "cornell_obj_phainon")]
for sc in scenes:
    print("==", os.path.basename(sc), flush=True)
    b = ptamd.SceneFile(sc, res=(64, 64))
    tr = ptamd.PathTracer(b)
    tr.free()
    sys.stderr.flush()
