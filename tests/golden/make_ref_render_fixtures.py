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
# image -> (scene, samples, camera overrides): the images tools/ref_render_sweep.py finds matched by
# a scene of the checkout (tests/golden/ref_render_sweep.json, every 800x800 image of
# /root/reference/img against every primitive-only scene variant).  README.md:112 "basic diffuse
# output" (cornell.json; 5000 spp, the scene's ITERATIONS), README.md:267-270 "Transmissive
# material" (5000samp) and "Glass material" (1809samp); cornell_multiple_glass -- glass spheres, a
# glass cube and a MIRROR cube (interactions.cu:465-470) -- in README.md:166's material-sort pair and
# a dated render, and with APERTURE 0.4 / 0.8 / 1.2 in README.md:246's depth-of-field series
# (sampleAperture, pathtrace.cu:231-237).  Nothing matches the microfacet images (the sweep's best
# mean |tile difference| is 17-25 of 255 with the camera refitted), so the Cook-Torrance branch has
# no reference-held pin.
CASES = {
    "diffuse.png": ("cornell.json", 5000, {}),
    # README.md:133-136: the render of the measurement that gives BASELINE's 42.204 ms/frame
    "diffuse_stream_compaction.png": ("cornell.json", 5000, {}),
    "cornell.2025-09-25_23-38-19z.5000samp.png": ("cornell_transmissive_test.json", 5000, {}),
    "cornell.2025-09-25_23-49-57z.1809samp.png": ("cornell_glass_test.json", 1809, {}),
    "no_mat_sorting.png": ("cornell_multiple_glass.json", 5000, {}),
    "mat_sort_on.png": ("cornell_multiple_glass.json", 5000, {}),
    "cornell.2025-09-27_20-31-32z.2014samp.png": ("cornell_multiple_glass.json", 2014, {}),
    "cam_aperture_0.4.png": ("cornell_multiple_glass.json", 5000, {"APERTURE": 0.4}),
    "cam_aperture_0.8.png": ("cornell_multiple_glass.json", 5000, {"APERTURE": 0.8}),
    "cam_aperture_1.2.png": ("cornell_multiple_glass.json", 5000, {"APERTURE": 1.2}),
}


def tile_means(rgb):
    h, w, _ = rgb.shape
    return rgb.reshape(h // TILE, TILE, w // TILE, TILE, 3).astype(np.float64).mean(axis=(1, 3)).astype(np.float32)


def main():
    arrays, meta = {}, {}
    for i, (name, (scene, spp, camera)) in enumerate(CASES.items()):
        rgb = np.asarray(Image.open(os.path.join(REF_IMG, name)).convert("RGB"))
        arrays[f"t{i}"] = tile_means(rgb)
        meta[f"t{i}"] = {"image": name, "scene": scene, "spp": spp, "camera": camera}
    np.savez_compressed(os.path.join(HERE, "ref_renders.npz"), **arrays)
    with open(os.path.join(HERE, "ref_renders.json"), "w") as f:
        json.dump({"tile": TILE, "cases": meta}, f, indent=1)


if __name__ == "__main__":
    main()
