import os, sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "project3-cuda-path-tracer-2025_amd"); sys.path.insert(0, "oracle")
import ptamd, oracle
from test_gpu_parity import _random_paths
sc = ptamd.SceneFile("scenes/synthetic_textured_bump.json", res=(96, 96))
tr = ptamd.PathTracer(sc, variant=10)
cam = tr.test_camera(3)[:4000]
paths = np.concatenate([_random_paths(3000, 11).astype(oracle.PATH), cam])
g = tr.test_intersect(paths)
print(os.environ.get("PTAMD_LIB"), "hit frac", (g["t"] > 0).mean(), "cam hits", (g["t"][3000:] > 0).mean(),
      "rand hits", (g["t"][:3000] > 0).mean(), "cam dir0", cam["direction"][0], cam["origin"][0])
tr.free()
