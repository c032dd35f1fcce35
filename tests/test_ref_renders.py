"""The BSDFs against the reference's OWN renders (statistical pin).

interactions.cu cannot be built here, so scatterRay / the diffuse, transmissive and
glass BSDFs have no bit-level pin.  The reference's authors committed saveImage PNGs of three
scenes of this checkout (README.md:112, 267-270).  tests/golden/ref_renders.npz holds their 16x16
tile means (tests/golden/make_ref_render_fixtures.py); here the same scenes are traced on the
MI355X at the same sample counts, written with pt_save_png (saveImage's bytes) and compared tile
by tile.  The reference rendered with CUDA's libdevice sin/cos and a different RNG stream order
on an RTX 3060, so agreement is statistical: converged images, not bits.
Measured: mean |tile difference| 0.16-0.22 of 255, max 1.7-2.0, image means within 0.03.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, SCENES

pytestmark = pytest.mark.gpu


def _cases():
    meta = json.load(open(os.path.join(GOLDEN, "ref_renders.json")))
    return sorted(meta["cases"].items())


@pytest.mark.parametrize("key,case", _cases(), ids=[c["image"] for _, c in _cases()])
def test_render_matches_reference_authors_image(key, case, tmp_path, ptamd):
    from PIL import Image
    tile = json.load(open(os.path.join(GOLDEN, "ref_renders.json")))["tile"]
    ref = np.load(os.path.join(GOLDEN, "ref_renders.npz"))[key].astype(np.float64)
    sc = ptamd.SceneFile(os.path.join(SCENES, case["scene"]))
    tr = ptamd.PathTracer(sc)
    tr.trace_frames(1, case["spp"])
    ptamd.save_png(tr.image(), tr.width, tr.height, case["spp"], str(tmp_path / "ours"))
    tr.free()
    rgb = np.asarray(Image.open(tmp_path / "ours.png").convert("RGB"))
    h, w, _ = rgb.shape
    ours = rgb.reshape(h // tile, tile, w // tile, tile, 3).astype(np.float64).mean(axis=(1, 3))
    d = np.abs(ours - ref)
    assert d.mean() < 0.4, (case, d.mean())
    assert d.max() < 3.0, (case, d.max())
    assert abs(ours.mean() - ref.mean()) < 0.15, (case, ours.mean(), ref.mean())
