"""ctypes front end of the CPU oracle (oracle/pt_oracle.c) plus an independent scene loader.

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker; the product path (ptamd) never imports this module.

The scene loader restates /root/reference/src/scene.cpp:47-224 (JSON), :226-363 (OBJ) and the
camera set-up of main.cpp:359-380 / :423-444 in Python, delegating every float operation to the
C oracle so each result is rounded exactly as the reference's float code rounds it.
"""
from __future__ import annotations

import ctypes
import json
import os
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

# ---------------------------------------------------------------------------------------------
# numpy record layouts == include/pt/scene_structs.h == reference sceneStructs.h
# ---------------------------------------------------------------------------------------------
GEOM = np.dtype([("type", "<i4"), ("materialid", "<i4"), ("translation", "<f4", (3,)),
                 ("rotation", "<f4", (3,)), ("scale", "<f4", (3,)), ("transform", "<f4", (4, 4)),
                 ("inverseTransform", "<f4", (4, 4)), ("invTranspose", "<f4", (4, 4))])
MATERIAL = np.dtype([("color", "<f4", (3,)), ("spec_exponent", "<f4"), ("spec_color", "<f4", (3,)),
                     ("hasReflective", "<f4"), ("hasRefractive", "<f4"), ("roughness", "<f4"),
                     ("metallic", "<f4"), ("indexOfRefraction", "<f4"), ("emittance", "<f4"),
                     ("hasTexture", "u1"), ("_pad0", "u1", (3,)), ("textureID", "<i4"),
                     ("hasBumpMap", "u1"), ("_pad1", "u1", (3,)), ("bumpID", "<i4"),
                     ("bumpScale", "<f4")])
VERTEX = np.dtype([("materialID", "<i4"), ("position", "<f4", (3,)), ("normal", "<f4", (3,)),
                   ("uv", "<f4", (2,))])
TRIANGLE = np.dtype([("v1", VERTEX), ("v2", VERTEX), ("v3", VERTEX), ("centroid", "<f4", (3,)),
                     ("materialID", "<i4"), ("dpdu", "<f4", (3,)), ("dpdv", "<f4", (3,))])
BVHNODE = np.dtype([("min", "<f4", (3,)), ("max", "<f4", (3,)), ("left", "<i4"), ("right", "<i4"),
                    ("start", "<i4"), ("triCount", "<i4")])
CAMERA = np.dtype([("resolution", "<i4", (2,)), ("position", "<f4", (3,)), ("lookAt", "<f4", (3,)),
                   ("view", "<f4", (3,)), ("up", "<f4", (3,)), ("right", "<f4", (3,)),
                   ("fov", "<f4", (2,)), ("pixelLength", "<f4", (2,)), ("aperture", "<f4"),
                   ("focalDist", "<f4")])
PATH = np.dtype([("origin", "<f4", (3,)), ("direction", "<f4", (3,)), ("color", "<f4", (3,)),
                 ("pixelIndex", "<i4"), ("remainingBounces", "<i4")])
ISECT = np.dtype([("t", "<f4"), ("surfaceNormal", "<f4", (3,)), ("materialId", "<i4"),
                  ("uv", "<f4", (2,)), ("dpdu", "<f4", (3,)), ("dpdv", "<f4", (3,))])
for _dt, _n in ((GEOM, 236), (MATERIAL, 72), (VERTEX, 36), (TRIANGLE, 148), (BVHNODE, 40),
                (CAMERA, 92), (PATH, 44), (ISECT, 52)):
    assert _dt.itemsize == _n, (_dt, _n)

PT_SPHERE, PT_CUBE = 0, 1


class Vec3(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float)]


class CameraC(ctypes.Structure):
    _fields_ = [("raw", ctypes.c_uint8 * 92)]


class OrScene(ctypes.Structure):
    _fields_ = [("geoms", ctypes.c_void_p), ("num_geoms", ctypes.c_int32),
                ("materials", ctypes.c_void_p), ("num_materials", ctypes.c_int32),
                ("triangles", ctypes.c_void_p), ("num_triangles", ctypes.c_int32),
                ("tri_indices", ctypes.c_void_p), ("num_tri_indices", ctypes.c_int32),
                ("bvh_nodes", ctypes.c_void_p), ("num_bvh_nodes", ctypes.c_int32),
                ("camera", CameraC), ("trace_depth", ctypes.c_int32), ("num_textures", ctypes.c_int32),
                ("textures", ctypes.c_void_p)]


class TextureC(ctypes.Structure):
    """pt_texture (include/pt/scene_structs.h) == the reference's Texture (sceneStructs.h:60-66)"""
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("_pad", ctypes.c_int32), ("data", ctypes.c_void_p)]


class OrOptions(ctypes.Structure):
    _fields_ = [("stream_compaction", ctypes.c_int32), ("material_sort", ctypes.c_int32),
                ("bvh", ctypes.c_int32), ("trig_mode", ctypes.c_int32), ("arg_order", ctypes.c_int32),
                ("num_threads", ctypes.c_int32)]


def options(stream_compaction=1, material_sort=0, bvh=1, trig_mode=0, arg_order=0, num_threads=0):
    return OrOptions(stream_compaction, material_sort, bvh, trig_mode, arg_order, num_threads)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle library missing: {LIB_PATH} (run `make -C oracle`)")
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float
        sig = {
            "or_utilhash": (ctypes.c_uint32, [ctypes.c_uint32]),
            "or_rng_draws": (None, [i32, i32, i32, i32, vp]),
            "or_box_test": (f32, [vp, vp, vp, vp, vp]),
            "or_sphere_test": (f32, [vp, vp, vp, vp, vp]),
            "or_triangle_test": (i32, [vp, vp, vp, vp, vp, vp, vp]),
            "or_aabb_test": (i32, [vp, vp]),
            "or_compute_intersection": (None, [vp, vp, vp, vp]),
            "or_compute_intersections": (None, [vp, vp, vp, i32, vp]),
            "or_prim_probe": (None, [vp, i32, vp, i32, vp]),
            "or_tri_probe": (None, [vp, i32, vp, i32, vp, i32, vp]),
            "or_shade": (None, [vp, vp, i32, vp, vp]),
            "or_scatter": (None, [vp, vp, Vec3, Vec3, vp, i32]),
            "or_generate_ray": (None, [vp, i32, i32, i32, i32, vp, vp]),
            "or_pathtrace": (i32, [vp, vp, i32, vp, vp]),
            "or_pathtrace_dump": (i32, [vp, vp, i32, vp, vp, vp]),
            "or_image_to_pbo": (None, [vp, i32, i32, vp]),
            "or_cpu_scan": (None, [i32, vp, vp]),
            "or_cpu_compact_without_scan": (i32, [i32, vp, vp]),
            "or_cpu_compact_with_scan": (i32, [i32, vp, vp]),
            "or_build_transform": (None, [Vec3, Vec3, Vec3, vp]),
            "or_mat4_inverse": (None, [vp, vp]),
            "or_mat4_inverse_transpose": (None, [vp, vp]),
            "or_make_geom": (None, [i32, i32, Vec3, Vec3, Vec3, vp]),
            "or_camera_setup": (None, [i32, i32, f32, Vec3, Vec3, Vec3, f32, vp]),
            "or_triangle_tangents": (None, [vp]),
            "or_build_bvh": (i32, [vp, i32, vp, vp]),
            "or_obj_to_triangles": (i32, [vp, vp, vp, vp, i32, i32, vp, vp, vp]),
            "or_mat4_mul_v4": (None, [vp, vp, vp]),
            "or_glm_normalize": (None, [vp, vp]),
            "or_glm_reflect": (None, [vp, vp, vp]),
            "or_glm_refract": (None, [vp, vp, f32, vp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data if a is not None and a.size else None


def v3(x) -> Vec3:
    return Vec3(float(x[0]), float(x[1]), float(x[2]))


# ---------------------------------------------------------------------------------------------
# scene ingest (restates scene.cpp:47-224)
# ---------------------------------------------------------------------------------------------
@dataclass
class Scene:
    geoms: np.ndarray
    materials: np.ndarray
    triangles: np.ndarray
    tri_indices: np.ndarray
    bvh_nodes: np.ndarray
    camera: np.ndarray           # CAMERA record, shape (1,)
    trace_depth: int
    iterations: int
    image_name: str
    material_names: list = field(default_factory=list)
    textures: list = field(default_factory=list)     # (h, w, 4) uint8 RGBA arrays

    @property
    def width(self):
        return int(self.camera["resolution"][0][0])

    @property
    def height(self):
        return int(self.camera["resolution"][0][1])

    @property
    def pixelcount(self):
        return self.width * self.height

    def c_struct(self) -> OrScene:
        s = OrScene()
        s.geoms, s.num_geoms = _p(self.geoms), len(self.geoms)
        s.materials, s.num_materials = _p(self.materials), len(self.materials)
        s.triangles, s.num_triangles = _p(self.triangles), len(self.triangles)
        s.tri_indices, s.num_tri_indices = _p(self.tri_indices), len(self.tri_indices)
        s.bvh_nodes, s.num_bvh_nodes = _p(self.bvh_nodes), len(self.bvh_nodes)
        ctypes.memmove(ctypes.addressof(s.camera), self.camera.ctypes.data, 92)
        s.trace_depth = self.trace_depth
        tex = (TextureC * max(1, len(self.textures)))()
        for i, t in enumerate(self.textures):
            tex[i].width, tex[i].height, tex[i].channels = t.shape[1], t.shape[0], 4
            tex[i].data = t.ctypes.data
        s.num_textures, s.textures = len(self.textures), ctypes.addressof(tex)
        self._keep = (s, tex)
        return s


def _load_texture(path: str, textures: list) -> int:
    """Scene::loadTexture (scene.cpp:366-392): stbi_load(..., STBI_rgb_alpha) -> RGBA8; -1 on
    failure.  Decoded here with Pillow, independently of the framework's own PNG decoder."""
    try:
        from PIL import Image
        with Image.open(path) as im:
            rgba = np.ascontiguousarray(np.asarray(im.convert("RGBA"), np.uint8))
    except Exception:
        return -1
    textures.append(rgba)
    return len(textures) - 1


def _material(p: dict, json_path: str = "", textures: list | None = None) -> np.void:
    """`Material newMaterial{}` then the TYPE switch of scene.cpp:53-133."""
    m = np.zeros(1, MATERIAL)[0]
    m["roughness"] = -1.0
    m["metallic"] = -1.0
    m["textureID"] = -1
    m["bumpID"] = -1
    m["bumpScale"] = 0.5
    t = p.get("TYPE")
    rgb = p.get("RGB")
    if t == "Diffuse":
        m["color"] = rgb
    elif t == "Emitting":
        m["color"] = rgb
        m["emittance"] = p["EMITTANCE"]
    elif t == "Glass":
        m["hasReflective"] = 1
        m["hasRefractive"] = 1
        m["indexOfRefraction"] = p["IOR"]
        m["color"] = rgb
    elif t == "Reflective":
        m["hasReflective"] = 1
        m["hasRefractive"] = 0
        m["color"] = rgb
    elif t == "Transmissive":
        m["hasReflective"] = 0
        m["hasRefractive"] = 1
        m["indexOfRefraction"] = p["IOR"]
        m["color"] = rgb
    elif t == "Microfacet":
        m["roughness"] = p["ROUGHNESS"]
        m["metallic"] = p["METALLIC"]
        m["indexOfRefraction"] = p["IOR"]
        m["color"] = rgb
    # TEXTURE / BUMP_MAP (scene.cpp:102-133): path relative to the JSON's directory
    # (basePath + "/" + name); a failed load leaves id -1 with hasTexture / hasBumpMap set.
    k = json_path.rfind("/")
    base = (json_path[:k] if k >= 0 else json_path)
    if base and not base.endswith("/"):
        base += "/"
    if "TEXTURE" in p:
        m["textureID"] = _load_texture(base + p["TEXTURE"], textures) if textures is not None else -1
        m["hasTexture"] = 1
    if "BUMP_MAP" in p:
        m["bumpID"] = _load_texture(base + p["BUMP_MAP"], textures) if textures is not None else -1
        m["hasBumpMap"] = 1
        m["bumpScale"] = p["BUMP_SCALE"]
    return m


def parse_obj(path: str):
    """Minimal restatement of tinyobj::LoadObj(triangulate=true) for v/vt/vn/f records:
    triangles kept, quads split on the shorter diagonal (tiny_obj_loader.h:1520-1628),
    larger polygons fanned.  Returns positions, normals, texcoords, faces[(v,vt,vn)*3]."""
    pos, nrm, tex, faces = [], [], [], []
    with open(path) as f:
        for line in f:
            tok = line.split()
            if not tok:
                continue
            if tok[0] == "v":
                pos.append([float(tok[1]), float(tok[2]), float(tok[3])])
            elif tok[0] == "vn":
                nrm.append([float(tok[1]), float(tok[2]), float(tok[3])])
            elif tok[0] == "vt":
                tex.append([float(tok[1]), float(tok[2]) if len(tok) > 2 else 0.0])
            elif tok[0] == "f":
                poly = []
                for t in tok[1:]:
                    parts = t.split("/")
                    def idx(k, n):
                        if k >= len(parts) or parts[k] == "":
                            return -1
                        i = int(parts[k])
                        return i - 1 if i > 0 else n + i
                    poly.append((idx(0, len(pos)), idx(1, len(tex)), idx(2, len(nrm))))
                if len(poly) < 3:
                    continue
                if len(poly) == 3:
                    faces.append(poly)
                elif len(poly) == 4:
                    p32 = np.asarray(pos, np.float32)
                    v = [p32[q[0]] for q in poly]
                    e02 = v[2] - v[0]
                    e13 = v[3] - v[1]
                    sqr02 = np.float32(e02[0] * e02[0] + e02[1] * e02[1] + e02[2] * e02[2])
                    sqr13 = np.float32(e13[0] * e13[0] + e13[1] * e13[1] + e13[2] * e13[2])
                    if sqr02 < sqr13:
                        faces += [[poly[0], poly[1], poly[2]], [poly[0], poly[2], poly[3]]]
                    else:
                        faces += [[poly[0], poly[1], poly[3]], [poly[1], poly[2], poly[3]]]
                else:
                    for i in range(1, len(poly) - 1):
                        faces.append([poly[0], poly[i], poly[i + 1]])
    return (np.asarray(pos, np.float32).reshape(-1, 3), np.asarray(nrm, np.float32).reshape(-1, 3),
            np.asarray(tex, np.float32).reshape(-1, 2), np.asarray(faces, np.int32).reshape(-1, 3, 3))


def load_scene(path: str, res=None, depth=None, obj_dir: str | None = None) -> Scene:
    """scene.cpp:47-224.  `res`/`depth` override RES/DEPTH before the camera is derived,
    exactly as editing the JSON would (pixelLength is recomputed).  `obj_dir` replaces the
    directory OBJ paths are resolved against (the reference uses the scene file's folder)."""
    L = lib()
    with open(path) as f:
        data = json.load(f)
    mats = data["Materials"]
    names = sorted(mats.keys())                     # nlohmann::json objects are std::map
    materials = np.zeros(len(names), MATERIAL)
    textures = []
    for i, n in enumerate(names):
        materials[i] = _material(mats[n], path, textures)
    ids = {n: i for i, n in enumerate(names)}
    geoms, tris = [], []
    base = os.path.dirname(path) if obj_dir is None else obj_dir
    for p in data["Objects"]:
        mat = ids.get(p["MATERIAL"], 0)             # unordered_map::operator[] inserts 0
        if p["TYPE"] == "obj":
            T = np.zeros((4, 4), np.float32)
            IT = np.zeros((4, 4), np.float32)
            L.or_build_transform(v3(p["TRANS"]), v3(p["ROTAT"]), v3(p["SCALE"]), T.ctypes.data)
            L.or_mat4_inverse_transpose(T.ctypes.data, IT.ctypes.data)
            objpath = base + p["PATH"]               # basePath has no trailing slash (scene.cpp:141-143)
            P, N, UV, F = parse_obj(objpath)
            out = np.zeros(len(F), TRIANGLE)
            n = L.or_obj_to_triangles(_p(P), _p(N), _p(UV), _p(np.ascontiguousarray(F)), len(F), mat,
                                      T.ctypes.data, IT.ctypes.data, _p(out))
            tris.append(out[:n])
        else:
            g = np.zeros(1, GEOM)
            gtype = PT_CUBE if p["TYPE"] == "cube" else PT_SPHERE
            L.or_make_geom(gtype, mat, v3(p["TRANS"]), v3(p["ROTAT"]), v3(p["SCALE"]), g.ctypes.data)
            geoms.append(g)
    cam = data["Camera"]
    rx, ry = (cam["RES"] if res is None else res)
    tdepth = cam["DEPTH"] if depth is None else depth
    camera = np.zeros(1, CAMERA)
    L.or_camera_setup(int(rx), int(ry), float(cam["FOVY"]), v3(cam["EYE"]), v3(cam["LOOKAT"]), v3(cam["UP"]),
                      float(cam["APERTURE"]), camera.ctypes.data)
    triangles = np.concatenate(tris) if tris else np.zeros(0, TRIANGLE)
    if len(triangles):
        nodes = np.zeros(max(1, 2 * len(triangles)), BVHNODE)
        idx = np.zeros(len(triangles), np.int32)
        nn = L.or_build_bvh(_p(triangles), len(triangles), _p(nodes), _p(idx))
        nodes = nodes[:nn].copy()
    else:
        nodes = np.zeros(0, BVHNODE)
        idx = np.zeros(0, np.int32)
    return Scene(geoms=np.concatenate(geoms) if geoms else np.zeros(0, GEOM), materials=materials,
                 triangles=triangles, tri_indices=idx, bvh_nodes=nodes, camera=camera,
                 trace_depth=int(tdepth), iterations=int(cam["ITERATIONS"]), image_name=str(cam["FILE"]),
                 material_names=names, textures=textures)


# ---------------------------------------------------------------------------------------------
# rendering
# ---------------------------------------------------------------------------------------------
class Renderer:
    """pathtraceInit / pathtrace on the oracle: keeps the accumulated image across iterations."""

    def __init__(self, scene: Scene, opts: OrOptions | None = None):
        self.scene = scene
        self.opts = opts or options()
        self.cs = scene.c_struct()
        self.image = np.zeros((scene.pixelcount, 3), np.float32)
        self.iteration = 0

    def trace(self, iteration: int | None = None, dump: bool = False):
        """One pathtrace(pbo, 0, iteration) call.  Returns live counts (and the per-bounce
        PathSegment dumps if asked)."""
        L = lib()
        self.iteration = self.iteration + 1 if iteration is None else iteration
        live = np.full(self.scene.trace_depth, -1, np.int32)
        if dump:
            d = np.zeros((self.scene.trace_depth, self.scene.pixelcount), PATH)
            L.or_pathtrace_dump(ctypes.byref(self.cs), ctypes.byref(self.opts), self.iteration,
                                self.image.ctypes.data, live.ctypes.data, d.ctypes.data)
            return live, d
        L.or_pathtrace(ctypes.byref(self.cs), ctypes.byref(self.opts), self.iteration, self.image.ctypes.data,
                       live.ctypes.data)
        return live

    def pbo(self) -> np.ndarray:
        out = np.zeros((self.scene.pixelcount, 4), np.uint8)
        lib().or_image_to_pbo(self.image.ctypes.data, self.scene.pixelcount, self.iteration, out.ctypes.data)
        return out


def rng_draws(iteration: int, index: int, depth: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.float32)
    lib().or_rng_draws(iteration, index, depth, n, out.ctypes.data)
    return out
