"""Renders each scene of tests/golden/ref_renders.json at the image's sample count on the GPU and
compares 16x16 tile means of the saveImage PNG with the reference authors' own render."""
import json, os, sys, tempfile
import numpy as np
from PIL import Image
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))
import ptamd
meta = json.load(open(os.path.join(REPO, "tests/golden/ref_renders.json")))
ref = np.load(os.path.join(REPO, "tests/golden/ref_renders.npz"))
T = meta["tile"]
out = {}
cache = {}
for key, c in meta["cases"].items():
    k = (c["scene"], c["spp"])
    if k not in cache:
        sc = ptamd.SceneFile(os.path.join(REPO, "scenes", c["scene"]))
        tr = ptamd.PathTracer(sc)
        tr.trace_frames(1, c["spp"])
        img = tr.image()
        with tempfile.TemporaryDirectory() as d:
            ptamd.save_png(img, tr.width, tr.height, c["spp"], os.path.join(d, "x"))
            rgb = np.asarray(Image.open(os.path.join(d, "x.png")).convert("RGB"))
        tr.free(); sc.close()
        cache[k] = rgb.reshape(rgb.shape[0] // T, T, rgb.shape[1] // T, T, 3).astype(np.float64).mean(axis=(1, 3))
    ours = cache[k]
    d = np.abs(ours - ref[key])
    out[c["image"]] = {"scene": c["scene"], "spp": c["spp"], "mean_abs": round(float(d.mean()), 3),
                       "p99_abs": round(float(np.percentile(d, 99)), 3), "max_abs": round(float(d.max()), 3),
                       "ours_mean": round(float(ours.mean()), 3), "ref_mean": round(float(ref[key].mean()), 3)}
print(json.dumps(out, indent=1))
