"""Sweep of the reference authors' committed renders against every primitive-only scene of the
checkout (VERDICT r02 "Next round" 2): which images does our path tracer reproduce, statistically?

Two steps, because the reference's images never travel to the GPU box:

  render   (GPU box)  python tools/ref_render_sweep.py render --out gpurun_out/ref_sweep.npz
           traces every scene VARIANT below once, up to 5000 spp, and at every sample count any
           800x800 reference image names writes the saveImage PNG (pt_save_png, byte-identical to
           the reference's) and keeps its 16x16-pixel tile means.
  compare  (here)     python tools/ref_render_sweep.py compare --tiles gpurun_out/ref_sweep.npz
           reads /root/reference/img, and for every 800x800 image and every variant at the image's
           sample count (5000 when the name gives none: every scene's ITERATIONS) computes the tile
           distance; writes tests/golden/ref_render_sweep.json (the full table, best match first).

A variant is a scene file plus parameter overrides: the microfacet scene with the metallic /
roughness its three README images name (README.md:300-303), the aperture series' APERTURE values
on cornell.json (README.md:246).
"""
import argparse
import json
import os
import re
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "scenes")
REF_IMG = "/root/reference/img"
TILE = 16
MAX_SPP = 5000

# name -> (scene file, {material: {key: value}}, {camera key: value})
VARIANTS = {
    "cornell": ("cornell.json", {}, {}),
    "cornell_glass_test": ("cornell_glass_test.json", {}, {}),
    "cornell_transmissive_test": ("cornell_transmissive_test.json", {}, {}),
    "cornell_reflective_test": ("cornell_reflective_test.json", {}, {}),
    "cornell_multiple_glass": ("cornell_multiple_glass.json", {}, {}),
    "cornell_microfacet_test": ("cornell_microfacet_test.json", {}, {}),
    "microfacet_m0.5_r0.01": ("cornell_microfacet_test.json", {"microfacet_mat": {"METALLIC": 0.5, "ROUGHNESS": 0.01}}, {}),
    "microfacet_m0.1_r0.9": ("cornell_microfacet_test.json", {"microfacet_mat": {"METALLIC": 0.1, "ROUGHNESS": 0.9}}, {}),
    "microfacet_m0.9_r0.01": ("cornell_microfacet_test.json", {"microfacet_mat": {"METALLIC": 0.9, "ROUGHNESS": 0.01}}, {}),
    "cornell_aperture_0.4": ("cornell.json", {}, {"APERTURE": 0.4}),
    "cornell_aperture_0.8": ("cornell.json", {}, {"APERTURE": 0.8}),
    "cornell_aperture_1.2": ("cornell.json", {}, {"APERTURE": 1.2}),
    # the aperture series is of cornell_multiple_glass (it is the best plain match of cam_aperture_0.4)
    "multiple_glass_aperture_0.4": ("cornell_multiple_glass.json", {}, {"APERTURE": 0.4}),
    "multiple_glass_aperture_0.8": ("cornell_multiple_glass.json", {}, {"APERTURE": 0.8}),
    "multiple_glass_aperture_1.2": ("cornell_multiple_glass.json", {}, {"APERTURE": 1.2}),
    # the README microfacet images' framing: the back wall 1.35x and the sphere 1.6x the size they
    # have from EYE z = 10.5, i.e. the eye at z ~ 6.5 (the light then leaves the frame)
    "microfacet_m0.5_r0.01_eye6.0": ("cornell_microfacet_test.json", {"microfacet_mat": {"METALLIC": 0.5, "ROUGHNESS": 0.01}},
                                     {"EYE": [0.0, 5.0, 6.0]}),
    "microfacet_m0.5_r0.01_eye6.5": ("cornell_microfacet_test.json", {"microfacet_mat": {"METALLIC": 0.5, "ROUGHNESS": 0.01}},
                                     {"EYE": [0.0, 5.0, 6.5]}),
    "microfacet_m0.5_r0.01_eye7.0": ("cornell_microfacet_test.json", {"microfacet_mat": {"METALLIC": 0.5, "ROUGHNESS": 0.01}},
                                     {"EYE": [0.0, 5.0, 7.0]}),
    "microfacet_m0.1_r0.9_eye6.5": ("cornell_microfacet_test.json", {"microfacet_mat": {"METALLIC": 0.1, "ROUGHNESS": 0.9}},
                                    {"EYE": [0.0, 5.0, 6.5]}),
    "microfacet_m0.9_r0.01_eye6.5": ("cornell_microfacet_test.json", {"microfacet_mat": {"METALLIC": 0.9, "ROUGHNESS": 0.01}},
                                     {"EYE": [0.0, 5.0, 6.5]}),
}


def image_spp(name):
    """Samples per pixel a reference image name states (cornell.<time>.<N>samp.png,
    *_<N>_iterations.png); None when it states none."""
    m = re.search(r"\.(\d+)samp\.png$", name) or re.search(r"_(\d+)_iterations?\.png$", name)
    return int(m.group(1)) if m else None


def tile_means(rgb):
    h, w, _ = rgb.shape
    return rgb.reshape(h // TILE, TILE, w // TILE, TILE, 3).astype(np.float64).mean(axis=(1, 3)).astype(np.float32)


def render(args):
    from PIL import Image
    sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))
    import ptamd
    spps = sorted(set(json.load(open(args.spps)) + [MAX_SPP]))
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, (scene, mats, cam) in VARIANTS.items():
            with open(os.path.join(SCENES, scene)) as f:
                d = json.load(f)
            for m, kv in mats.items():
                d["Materials"][m].update(kv)
            d["Camera"].update(cam)
            path = os.path.join(tmp, name + ".json")
            with open(path, "w") as f:
                json.dump(d, f)
            sc = ptamd.SceneFile(path)
            tr = ptamd.PathTracer(sc)
            done = 0
            for n in spps:
                tr.trace_frames(done + 1, n - done)
                done = n
                ptamd.save_png(tr.image(), tr.width, tr.height, n, os.path.join(tmp, "x"))
                out[f"{name}@{n}"] = tile_means(np.asarray(Image.open(os.path.join(tmp, "x.png")).convert("RGB")))
            tr.free()
            sc.close()
            print(f"{name}: {len(spps)} snapshots up to {done} spp", flush=True)
    np.savez_compressed(args.out, **out)


def reference_images():
    from PIL import Image
    imgs = {}
    for f in sorted(os.listdir(REF_IMG)):
        if not f.endswith(".png"):
            continue
        im = Image.open(os.path.join(REF_IMG, f))
        if im.size == (800, 800):
            imgs[f] = np.asarray(im.convert("RGB"))
    return imgs


def compare(args):
    tiles = np.load(args.tiles)
    table = {}
    for name, rgb in reference_images().items():
        ref = tile_means(rgb).astype(np.float64)
        spp = image_spp(name) or MAX_SPP
        rows = []
        for v in VARIANTS:
            ours = tiles[f"{v}@{spp}"].astype(np.float64)
            dd = np.abs(ours - ref)
            rows.append({"variant": v, "mean_abs": round(float(dd.mean()), 3),
                         "p99_abs": round(float(np.percentile(dd, 99)), 3), "max_abs": round(float(dd.max()), 3),
                         "ours_mean": round(float(ours.mean()), 3), "ref_mean": round(float(ref.mean()), 3)})
        rows.sort(key=lambda r: r["mean_abs"])
        table[name] = {"spp": spp, "spp_from_name": image_spp(name) is not None, "best": rows[0]["variant"],
                       "match": rows[0]["mean_abs"] < args.match and rows[0]["max_abs"] < args.match_max,
                       "rows": rows}
    out = {"tile": TILE, "match_rule": f"mean |tile difference| < {args.match} of 255 and max < {args.match_max:g} "
                                 "(tests/test_ref_renders.py's bounds)",
           "variants": {k: {"scene": s, "materials": m, "camera": c} for k, (s, m, c) in VARIANTS.items()},
           "images": table}
    with open(args.table, "w") as f:
        json.dump(out, f, indent=1)
    for name, t in table.items():
        r = t["rows"][0]
        print(f"{'MATCH' if t['match'] else '     '} {name:55s} spp {t['spp']:5d}  best {r['variant']:26s} "
              f"mean {r['mean_abs']:7.3f} max {r['max_abs']:7.2f}")


def spp_list(args):
    spps = sorted({image_spp(n) or MAX_SPP for n in reference_images()})
    with open(args.out, "w") as f:
        json.dump(spps, f)
    print(spps)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("spps")
    p.add_argument("--out", default=os.path.join(REPO, "tools", "ref_sweep_spps.json"))
    p = sub.add_parser("render")
    p.add_argument("--spps", default=os.path.join(REPO, "tools", "ref_sweep_spps.json"))
    p.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "ref_sweep.npz"))
    p = sub.add_parser("compare")
    p.add_argument("--tiles", default=os.path.join(REPO, "gpurun_out", "ref_sweep.npz"))
    p.add_argument("--table", default=os.path.join(REPO, "tests", "golden", "ref_render_sweep.json"))
    p.add_argument("--match", type=float, default=0.4)
    p.add_argument("--match-max", type=float, default=3.0)
    a = ap.parse_args()
    {"spps": spp_list, "render": render, "compare": compare}[a.cmd](a)


if __name__ == "__main__":
    main()
