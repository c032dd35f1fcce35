"""The oracle, the C++ scene loader and the struct layouts checked against the reference's OWN
code (CPU only).

tests/golden/ref_pin.json is written by oracle/ref_pins/make_ref_fixtures.py from
oracle/_ref/ref_harness: /root/reference/src/intersections.cu, scene.cpp, utilities.cpp, stb.cpp
and image.cpp compiled in place with g++ against the CUDA runtime headers shipped in the image.
What it pins, bit-exactly (floats compared with NaNs canonicalised):
  * layout: sizeof / offsetof of every sceneStructs.h field == include/pt/scene_structs.h;
  * ingest: geoms, materials, triangles (tinyobj + tangents), triIndices and bvhNodes
    (buildBVHRecursive), the scene.cpp camera and the texels of every scene the reference loads;
  * intersections: computeIntersections (restated loop over the reference's box / sphere /
    bvhMeshIntersectionTest) on 4096 probe rays per scene, the per-geom box / sphere results and
    intersectTriangle / aabbIntersectionTest probes — against the oracle here, and against the
    HIP kernels in test_gpu_parity.py::test_intersections_match_reference;
  * saveImage + Image::savePNG: the 8-bit pixels (and bytes) of the PNG the reference writes.
"""
import base64
import ctypes
import json
import os
import subprocess
import zlib

import numpy as np
import pytest

import refpins as R
from conftest import GOLDEN, REPO, scene_path


@pytest.fixture(scope="module")
def pin():
    with open(os.path.join(GOLDEN, "ref_pin.json")) as f:
        return json.load(f)


with open(os.path.join(GOLDEN, "ref_pin.json")) as _f:
    PIN = json.load(_f)
LOADED = sorted(k for k, v in PIN["scenes"].items() if not v.get("load_error"))
FAILED = sorted(k for k, v in PIN["scenes"].items() if v.get("load_error"))
ISECT = sorted(PIN["isect"])

# ---------------------------------------------------------------------------------------------
# layout
# ---------------------------------------------------------------------------------------------
_STRUCTS = {"Ray": "pt_ray", "Geom": "pt_geom", "Material": "pt_material", "Texture": "pt_texture",
            "Vertex": "pt_vertex", "Triangle": "pt_triangle", "AABB": "pt_aabb", "BVHNode": "pt_bvh_node",
            "Camera": "pt_camera", "PathSegment": "pt_path_segment", "ShadeableIntersection": "pt_shadeable_isect"}


def test_struct_layout_matches_reference(pin, tmp_path):
    """offsetof / sizeof of include/pt/scene_structs.h (compiled here) == sceneStructs.h's."""
    lay = pin["layout"]
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "pt/scene_structs.h"', "int main(void) {"]
    for ref, ours in _STRUCTS.items():
        src.append(f'printf("S {ref} %zu\\n", sizeof({ours}));')
    for key in lay["fields"]:
        s, f = key.split(".", 1)
        src.append(f'printf("F {key} %zu %zu\\n", offsetof({_STRUCTS[s]}, {f}), sizeof((({_STRUCTS[s]}*)0)->{f}));')
    src.append("return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(c), "-o", str(exe)], check=True)
    got_s, got_f = {}, {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        p = line.split()
        if p[0] == "S":
            got_s[p[1]] = int(p[2])
        else:
            got_f[p[1]] = [int(p[2]), int(p[3])]
    assert got_s == lay["sizeof"]
    assert got_f == lay["fields"]


def test_numpy_layouts_match_reference(pin, oracle, ptamd):
    """the Python mirrors (oracle.py, ptamd) use the reference's sizes and field offsets"""
    lay = pin["layout"]
    for mod in (oracle, ptamd):
        for ref, dt in (("Geom", mod.GEOM), ("Material", mod.MATERIAL), ("Vertex", mod.VERTEX),
                        ("Triangle", mod.TRIANGLE), ("BVHNode", mod.BVHNODE), ("Camera", mod.CAMERA),
                        ("PathSegment", mod.PATH), ("ShadeableIntersection", mod.ISECT)):
            assert dt.itemsize == lay["sizeof"][ref], (mod.__name__, ref)
            for key, (off, size) in lay["fields"].items():
                s, f = key.split(".", 1)
                if s != ref:
                    continue
                name = {"specular.exponent": "spec_exponent", "specular.color": "spec_color"}.get(f, f)
                if ref == "BVHNode" and f == "aabb":
                    name = "min"
                if ref == "PathSegment" and f == "ray":
                    name = "origin"
                assert dt.fields[name][1] == off, (mod.__name__, key)


def test_value_initialised_defaults(pin):
    d = pin["layout"]["defaults"]
    assert d["Material.roughness"] == -1 and d["Material.metallic"] == -1
    assert d["Material.textureID"] == -1 and d["Material.bumpID"] == -1 and d["Material.bumpScale"] == 0.5


# ---------------------------------------------------------------------------------------------
# scene ingest
# ---------------------------------------------------------------------------------------------
def _digests_ptamd(ptamd, name):
    s = ptamd.SceneFile(scene_path(name), viewer_camera=False)
    tex = np.concatenate([t.reshape(-1) for t in s.textures]) if s.textures else np.zeros(0, np.uint8)
    d = {"geoms": R.digest(R.pack(s.geoms, R.P_GEOM)),
         "materials": R.digest(R.pack(s.materials, R.P_MATERIAL)),
         "triangles": R.digest(R.pack(s.triangles, R.P_TRIANGLE)),
         "triIndices": R.digest(s.tri_indices.astype("<i4")),
         "bvhNodes": R.digest(R.pack(s.bvh_nodes, R.P_BVHNODE)),
         "camera": R.digest(R.pack(s.camera, R.P_CAMERA)),
         "texels": R.digest(tex)}
    info = {"iterations": s.iterations, "traceDepth": s.trace_depth, "imageName": s.image_name,
            "textures": [[t.shape[1], t.shape[0], 4] for t in s.textures]}
    s.close()
    return d, info


@pytest.mark.parametrize("name", LOADED)
def test_scene_loader_matches_reference(name, pin, ptamd):
    """host/scene.cpp (the C++ Scene the drop-in hands over) == the reference's Scene(json)"""
    ref = pin["scenes"][name]
    got, info = _digests_ptamd(ptamd, name)
    for k, v in got.items():
        assert v == ref["sha256"][k], (name, k)
    assert info["iterations"] == ref["iterations"] and info["traceDepth"] == ref["traceDepth"]
    assert info["imageName"] == ref["imageName"]
    assert info["textures"] == ref["textures"]


@pytest.mark.parametrize("name", [n for n in LOADED if n != "synthetic_textured_bump"])
def test_oracle_loader_matches_reference(name, pin, oracle):
    """oracle.load_scene's geoms / materials / triangles / BVH (the checker's own ingest)"""
    ref = pin["scenes"][name]["sha256"]
    s = oracle.load_scene(scene_path(name))
    assert R.digest(R.pack(s.geoms, R.P_GEOM)) == ref["geoms"]
    assert R.digest(R.pack(s.materials, R.P_MATERIAL)) == ref["materials"]
    assert R.digest(R.pack(s.triangles, R.P_TRIANGLE)) == ref["triangles"]
    assert R.digest(s.tri_indices.astype("<i4")) == ref["triIndices"]
    assert R.digest(R.pack(s.bvh_nodes, R.P_BVHNODE)) == ref["bvhNodes"]


@pytest.mark.parametrize("name", FAILED)
def test_loader_refuses_what_the_reference_refuses(name, ptamd):
    """the reference aborts on these (missing OBJ: runtime_error, scene.cpp:245-247; missing
    Camera.APERTURE: json assertion, scene.cpp:198); the loader reports an error instead"""
    with pytest.raises(ptamd.PtError):
        ptamd.SceneFile(scene_path(name))


# ---------------------------------------------------------------------------------------------
# intersections
# ---------------------------------------------------------------------------------------------
def probe_rays(ptamd, name):
    s = ptamd.SceneFile(scene_path(name), viewer_camera=False)
    rays = R.rays(R.ISECT_RAYS, seed=len(name), targets=R.scene_targets(s.geoms, s.triangles))
    return s, rays


@pytest.mark.parametrize("name", ISECT)
def test_oracle_intersections_match_reference(name, pin, oracle, ptamd):
    ref = pin["isect"][name]
    s, rays = probe_rays(ptamd, name)
    assert R.digest(rays) == ref["rays_sha256"]
    rays = np.ascontiguousarray(rays, oracle.PATH)
    sc = oracle.load_scene(scene_path(name))
    L = oracle.lib()
    cs = sc.c_struct()
    out = np.zeros(len(rays), oracle.ISECT)
    L.or_compute_intersections(ctypes.byref(cs), ctypes.byref(oracle.options()), rays.ctypes.data, len(rays),
                               out.ctypes.data)
    assert R.digest(R.pack(out, R.P_ISECT)) == ref["isect_sha256"]
    assert int((out["t"] > 0).sum()) == ref["hits"]
    # per-geom box / sphere results
    ng = len(sc.geoms)
    prim = np.zeros(len(rays) * ng, R.P_PRIM)
    L.or_prim_probe(sc.geoms.ctypes.data, ng, rays.ctypes.data, len(rays), prim.ctypes.data)
    assert R.digest(prim) == ref["prims_sha256"]
    # intersectTriangle / aabbIntersectionTest probes
    nt, nn = min(R.TRIS_K, len(sc.triangles)), min(R.TRIS_K, len(sc.bvh_nodes))
    raw = np.zeros((len(rays), 4 * nt + nn), np.int32)
    L.or_tri_probe(sc.triangles.ctypes.data if nt else None, nt, sc.bvh_nodes.ctypes.data if nn else None, nn,
                   rays.ctypes.data, len(rays), raw.ctypes.data)
    tri = raw[:, :4 * nt].copy().view(R.P_TRI).reshape(len(rays), nt)
    assert R.digest(tri) == ref["tri_sha256"]
    assert R.digest(raw[:, 4 * nt:].copy()) == ref["aabb_sha256"]
    s.close()


# ---------------------------------------------------------------------------------------------
# saveImage + Image::savePNG
# ---------------------------------------------------------------------------------------------
def _png_pixels(data: bytes):
    """decode an 8-bit RGB PNG (any filter) -> (h, w, 3) uint8, with zlib + the PNG unfilter"""
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n = int.from_bytes(data[pos:pos + 4], "big")
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        if typ == b"IHDR":
            w, h = int.from_bytes(body[:4], "big"), int.from_bytes(body[4:8], "big")
            assert body[8] == 8 and body[9] == 2
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    stride = 3 * w
    out = np.zeros((h, stride), np.int32)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f = raw[y * (stride + 1)]
        line = np.frombuffer(raw[y * (stride + 1) + 1:(y + 1) * (stride + 1)], np.uint8).astype(np.int32)
        cur = np.zeros(stride, np.int32)
        for i in range(stride):
            a = cur[i - 3] if i >= 3 else 0
            b = prev[i]
            c = prev[i - 3] if i >= 3 else 0
            if f == 0:
                p = 0
            elif f == 1:
                p = a
            elif f == 2:
                p = b
            elif f == 3:
                p = (a + b) >> 1
            else:
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                p = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
            cur[i] = (line[i] + p) & 255
        out[y] = cur
        prev = cur
    return out.reshape(h, w, 3).astype(np.uint8)


def test_save_png_matches_reference(pin, ptamd, tmp_path):
    """pt_save_png (main.cpp:395-419 saveImage + image.cpp:23-43 savePNG): the flip, 1/spp,
    clamp and truncation give the reference's 8-bit pixels, and the file is byte-identical to
    stb_image_write's (its zlib and filter choice restated in host/image_io.cpp)."""
    p = pin["png"]
    w, h, it, img = R.png_input()
    ref = base64.b64decode(p["png_base64"])
    out = tmp_path / "ours"
    ptamd.save_png(img, w, h, it, str(out))
    ours = (tmp_path / "ours.png").read_bytes()
    assert np.array_equal(_png_pixels(ours), _png_pixels(ref))
    assert ours == ref


def test_save_png_large_matches_reference(pin, ptamd, tmp_path):
    """a 320x200 image: long matches, the 32 KiB window and hash-chain trimming of stb's deflate"""
    import hashlib
    p = pin["png_large"]
    w, h, it, img = R.png_input_large()
    ptamd.save_png(img, w, h, it, str(tmp_path / "big"))
    ours = (tmp_path / "big.png").read_bytes()
    assert len(ours) == p["png_bytes"]
    assert hashlib.sha256(ours).hexdigest() == p["png_sha256"]
