"""Writes tests/golden/ref_pin.json from the reference's OWN code (TEST INFRASTRUCTURE).

Runs oracle/_ref/ref_harness (built by make_fixtures.sh from /root/reference/src/{intersections.cu,
scene.cpp, utilities.cpp, stb.cpp, image.cpp} with g++ and the image's real CUDA headers) and
records:
  * layout     sizeof / offsetof of every sceneStructs.h field
  * scenes     per scene JSON of scenes/: sha256 of the packed geoms / materials / triangles /
               triIndices / bvhNodes / vertices / camera (scene.cpp only) / texels, plus counts
  * isect      per ISECT_SCENES scene: sha256 of computeIntersections over tests/refpins.rays()
               (box / sphere / bvhMeshIntersectionTest of the reference), of the per-geom
               box / sphere results and of intersectTriangle / aabbIntersectionTest probes
  * png        saveImage + Image::savePNG (stb_image_write) bytes of a synthetic float image
Only digests and tiny samples are committed; the tests regenerate the same inputs.
Usage (this container only): python oracle/ref_pins/make_ref_fixtures.py <harness> <out.json>
"""
import base64
import glob
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tests"))
import refpins as R  # noqa: E402


def run(*args):
    subprocess.run([str(a) for a in args], check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


def main():
    harness, out_path = sys.argv[1], sys.argv[2]
    fx = {"generator": "oracle/ref_pins/make_ref_fixtures.py", "harness": "oracle/ref_pins/ref_harness.cpp"}
    fx["layout"] = json.loads(subprocess.run([harness, "layout"], check=True, capture_output=True, text=True).stdout)
    fx["scenes"] = {}
    fx["isect"] = {}
    with tempfile.TemporaryDirectory() as tmp:
        for path in sorted(glob.glob(os.path.join(REPO, "scenes", "*.json"))):
            name = os.path.basename(path)[:-5]
            d = os.path.join(tmp, name)
            os.makedirs(d)
            try:
                run(harness, "scene", path, d)
            except subprocess.CalledProcessError:
                fx["scenes"][name] = {"load_error": True}
                continue
            meta = json.load(open(os.path.join(d, "meta.json")))
            rd = lambda f, dt: np.fromfile(os.path.join(d, f), dt)  # noqa: E731
            arrs = {"geoms": rd("geoms.bin", R.P_GEOM), "materials": rd("materials.bin", R.P_MATERIAL),
                    "triangles": rd("triangles.bin", R.P_TRIANGLE), "triIndices": rd("triidx.bin", "<i4"),
                    "bvhNodes": rd("bvh.bin", R.P_BVHNODE), "vertices": rd("vertices.bin", R.P_VERTEX),
                    "camera": rd("camera.bin", R.P_CAMERA), "texels": rd("textures.bin", "u1")}
            meta["sha256"] = {k: R.digest(v) for k, v in arrs.items()}
            fx["scenes"][name] = meta
            if name not in R.ISECT_SCENES:
                continue
            targets = R.scene_targets(arrs["geoms"], arrs["triangles"])
            rays = R.rays(R.ISECT_RAYS, seed=len(name), targets=targets)
            rp = os.path.join(d, "rays.bin")
            rays.tofile(rp)
            run(harness, "isect", path, rp, os.path.join(d, "isect.bin"))
            run(harness, "prims", path, rp, os.path.join(d, "prims.bin"))
            run(harness, "tris", path, rp, os.path.join(d, "tris.bin"), R.TRIS_K)
            isect = np.fromfile(os.path.join(d, "isect.bin"), R.P_ISECT)
            prims = np.fromfile(os.path.join(d, "prims.bin"), R.P_PRIM)
            nt = min(R.TRIS_K, len(arrs["triangles"]))
            nn = min(R.TRIS_K, len(arrs["bvhNodes"]))
            raw = np.fromfile(os.path.join(d, "tris.bin"), "<i4").reshape(len(rays), 4 * nt + nn)
            tri = raw[:, :4 * nt].copy().view(R.P_TRI).reshape(len(rays), nt)
            aabb = raw[:, 4 * nt:].copy()
            fx["isect"][name] = {
                "rays": len(rays), "rays_sha256": R.digest(rays),
                "isect_sha256": R.digest(isect), "prims_sha256": R.digest(prims),
                "tri_sha256": R.digest(tri), "aabb_sha256": R.digest(aabb),
                "hits": int((isect["t"] > 0).sum()),
                "tri_hits": int(tri["hit"].sum()), "aabb_hits": int(aabb.sum()),
                "sample": [[float(x["t"]), int(x["materialId"])] for x in isect[:8]],
            }
        w, h, it, img = R.png_input()
        ip = os.path.join(tmp, "img.f32")
        img.tofile(ip)
        run(harness, "png", ip, w, h, it, os.path.join(tmp, "out"))
        png = open(os.path.join(tmp, "out.png"), "rb").read()
        fx["png"] = {"width": w, "height": h, "iteration": it, "input": "tests/refpins.png_input()",
                     "png_base64": base64.b64encode(png).decode()}
        w, h, it, img = R.png_input_large()
        img.tofile(ip)
        run(harness, "png", ip, w, h, it, os.path.join(tmp, "big"))
        png = open(os.path.join(tmp, "big.png"), "rb").read()
        fx["png_large"] = {"width": w, "height": h, "iteration": it, "input": "tests/refpins.png_input_large()",
                           "png_sha256": hashlib.sha256(png).hexdigest(), "png_bytes": len(png)}
    with open(out_path, "w") as f:
        json.dump(fx, f, indent=1, sort_keys=True)
    print("ref fixtures:", out_path, len(fx["scenes"]), "scenes,", len(fx["isect"]), "isect scenes")


if __name__ == "__main__":
    main()
