"""The BSDFs against the reference's OWN renders (statistical pin).

interactions.cu cannot be built here, so scatterRay and its BSDFs have no bit-level
pin.  The reference's authors committed saveImage PNGs of scenes of this checkout; the sweep of
every 800x800 image against every primitive-only scene variant (tools/ref_render_sweep.py,
tests/golden/ref_render_sweep.json) matches ten of them:
  * diffuse (cornell.json: README.md:112, 133-136),
  * transmissive and glass (README.md:267-270),
  * cornell_multiple_glass -- glass spheres, a glass cube and a MIRROR cube -- in README.md:166's
    material-sort pair and a dated render,
  * the same scene with APERTURE 0.4 / 0.8 / 1.2: README.md:246's depth-of-field series.
tests/golden/ref_renders.npz holds their 16x16 tile means (tests/golden/make_ref_render_fixtures.py);
here the same scenes are traced on the MI355X at the same sample counts, written with pt_save_png
(saveImage's bytes) and compared tile by tile.  The reference rendered with CUDA's libdevice
sin/cos on an RTX 3060, so agreement is statistical: converged images, not bits.

Two bars: the whole image (mean |tile difference| < 0.4 of 255, max < 3), and, tighter, the tiles
whose pixels' first hit is a mirror / glass / transmissive surface (found with the production
camera + intersection kernels): mean < 0.6, max < 2, and |signed mean| < 0.35 per channel, so a
biased specular term confined to those few tiles cannot hide in the image-wide average.
Measured (tools/ref_render_sweep.py): whole image 0.16-0.22 mean, max 1.5-2.0; specular tiles
0.36-0.45 mean, max <= 1.40, signed mean within 0.2.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, SCENES

pytestmark = pytest.mark.gpu


def _meta():
    with open(os.path.join(GOLDEN, "ref_renders.json")) as f:
        return json.load(f)


def _cases():
    return sorted(_meta()["cases"].items())


def _specular_tile_mask(tr, sc, tile):
    """Tiles (in saveImage's x-flipped PNG layout) whose pixels' first hit, for iteration 1's camera
    rays, is mostly a reflective or refractive material."""
    paths = tr.test_camera(1)
    hits = tr.test_intersect(paths)
    mats = sc.materials
    spec = (mats["hasReflective"] > 0) | (mats["hasRefractive"] > 0)
    m = (hits["t"] > 0) & spec[np.clip(hits["materialId"], 0, len(mats) - 1)]
    img = m.reshape(tr.height, tr.width)[:, ::-1]
    return img.reshape(tr.height // tile, tile, tr.width // tile, tile).mean(axis=(1, 3)) >= 0.5


@pytest.mark.parametrize("key,case", _cases(), ids=[c["image"] for _, c in _cases()])
def test_render_matches_reference_authors_image(key, case, tmp_path, ptamd):
    from PIL import Image
    tile = _meta()["tile"]
    ref = np.load(os.path.join(GOLDEN, "ref_renders.npz"))[key].astype(np.float64)
    path = os.path.join(SCENES, case["scene"])
    if case.get("camera"):
        with open(path) as f:
            d = json.load(f)
        d["Camera"].update(case["camera"])
        path = str(tmp_path / case["scene"])
        with open(path, "w") as f:
            json.dump(d, f)
    sc = ptamd.SceneFile(path)
    tr = ptamd.PathTracer(sc)
    spec = _specular_tile_mask(tr, sc, tile)
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
    if "glass" in case["scene"] or "transmissive" in case["scene"]:
        assert spec.sum() >= 20, (case, int(spec.sum()))
    if spec.any():
        ds = d.max(axis=2)[spec]
        signed = (ours - ref)[spec].mean(axis=0)
        assert ds.mean() < 0.6, (case, ds.mean())
        assert ds.max() < 2.0, (case, ds.max())
        assert np.all(np.abs(signed) < 0.35), (case, signed)
