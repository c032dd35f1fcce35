"""Host vs GPU BVH build time (scene.cpp:445-525 vs csrc/pt_bvh_build.hip) on the mesh stand-ins
and a synthetic 1M-triangle mesh; checks the trees are identical.  Prints one JSON line.  Tools only."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    import ptamd
    import oracle as O
    out = {}
    meshes = {}
    s = ptamd.SceneFile(os.path.join(REPO, "scenes", "cornell_obj_khaslana.json"), viewer_camera=False)
    meshes["khaslana_49760"] = s.triangles
    rng = np.random.default_rng(0)
    n = 1 << 20
    t = np.zeros(n, ptamd.TRIANGLE)
    c = rng.random((n, 3)).astype(np.float32) * 10
    for k, v in enumerate(("v1", "v2", "v3")):
        t[v]["position"] = c + (rng.random((n, 3)).astype(np.float32) * 0.01)
    t["centroid"] = ((t["v1"]["position"] + t["v2"]["position"] + t["v3"]["position"]) / np.float32(3)).astype(np.float32)
    meshes["random_1M"] = t
    ptamd.build_bvh(meshes["khaslana_49760"][:1000])   # warm the device
    for name, tris in meshes.items():
        tris = np.ascontiguousarray(tris, O.TRIANGLE)
        m = len(tris)
        nodes = np.zeros(2 * m, O.BVHNODE)
        idx = np.zeros(m, np.int32)
        t0 = time.perf_counter()
        nn = O.lib().or_build_bvh(tris.ctypes.data, m, nodes.ctypes.data, idx.ctypes.data)
        th = time.perf_counter() - t0
        tg = []
        for _ in range(3):
            t0 = time.perf_counter()
            gn, gi = ptamd.build_bvh(tris)
            tg.append(time.perf_counter() - t0)
        tg = min(tg)
        out[name] = {"host_ms": round(1e3 * th, 1), "gpu_ms": round(1e3 * tg, 1), "nodes": int(nn),
                     "identical": bool(gn.tobytes() == nodes[:nn].tobytes() and gi.tobytes() == idx.tobytes())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
