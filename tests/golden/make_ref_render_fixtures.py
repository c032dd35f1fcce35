"""Makes tests/golden/ref_renders.npz: 16x16-pixel tile means of renders the reference's authors
committed (/root/reference/img, saveImage PNGs of 800x800 scenes at N spp).  The PNGs stay in the
reference; only these tile means (data) travel.  Run in the container that has /root/reference:

    python tests/golden/make_ref_render_fixtures.py
"""
import json
import os

import numpy as np
from PIL import Image

REF_IMG = "/root/reference/img"
HERE = os.path.dirname(os.path.abspath(__file__))
TILE = 16
# image -> (scene, samples).  README.md:112 "basic diffuse output" (cornell.json; 5000 spp, the
# scene's ITERATIONS), README.md:267-270 "Transmissive material" (5000samp) and "Glass material"
# (1809samp).  Candidates that match no scene of the checkout are left out (tools/ref_render_compare.py
# measured them): the microfacet images (README.md:300-303; other light and parameters), the
# aperture series (README.md:246; mean |tile difference| ~4.3),
# REFERENCE_cornell.5000samp.png (the course's base-code image: mean 31.8 vs 38.6) and
# cornell.2025-09-25_21-04-50z.5000samp.png (a transmissive bug image, README.md:326).
CASES = {
    "diffuse.png": ("cornell.json", 5000),
    # README.md:133-136: the render of the measurement that gives BASELINE's 42.204 ms/frame
    "diffuse_stream_compaction.png": ("cornell.json", 5000),
    "cornell.2025-09-25_23-38-19z.5000samp.png": ("cornell_transmissive_test.json", 5000),
    "cornell.2025-09-25_23-49-57z.1809samp.png": ("cornell_glass_test.json", 1809),
}


def tile_means(rgb):
    h, w, _ = rgb.shape
    return rgb.reshape(h // TILE, TILE, w // TILE, TILE, 3).astype(np.float64).mean(axis=(1, 3)).astype(np.float32)


def main():
    arrays, meta = {}, {}
    for i, (name, (scene, spp)) in enumerate(CASES.items()):
        rgb = np.asarray(Image.open(os.path.join(REF_IMG, name)).convert("RGB"))
        arrays[f"t{i}"] = tile_means(rgb)
        meta[f"t{i}"] = {"image": name, "scene": scene, "spp": spp}
    np.savez_compressed(os.path.join(HERE, "ref_renders.npz"), **arrays)
    with open(os.path.join(HERE, "ref_renders.json"), "w") as f:
        json.dump({"tile": TILE, "cases": meta}, f, indent=1)


if __name__ == "__main__":
    main()
