"""ptamd — Python binding of the MI355X wavefront path tracer (build/libptamd.so, C-ABI in
include/pt/pathtrace_abi.h).

It mirrors the reference's boundary (src/pathtrace.h:6-9):

    Scene(path)                       -> SceneFile(path)            (scene.cpp:22-37, C++ loader)
    pathtraceInit(scene)              -> PathTracer(scene, **opts)
    pathtrace(pbo, frame, iteration)  -> PathTracer.trace(iteration, pbo=None)
    pathtraceFree()                   -> PathTracer.free()

The native library is mandatory: importing this module raises if it is missing, and every
call goes to HIP kernels — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("PTAMD_LIB", os.path.join(PKG_ROOT, "build", "libptamd.so"))

# ---- numpy record layouts == include/pt/scene_structs.h (== reference sceneStructs.h) ----
GEOM = np.dtype([("type", "<i4"), ("materialid", "<i4"), ("translation", "<f4", (3,)),
                 ("rotation", "<f4", (3,)), ("scale", "<f4", (3,)), ("transform", "<f4", (4, 4)),
                 ("inverseTransform", "<f4", (4, 4)), ("invTranspose", "<f4", (4, 4))])
MATERIAL = np.dtype([("color", "<f4", (3,)), ("spec_exponent", "<f4"), ("spec_color", "<f4", (3,)),
                     ("hasReflective", "<f4"), ("hasRefractive", "<f4"), ("roughness", "<f4"),
                     ("metallic", "<f4"), ("indexOfRefraction", "<f4"), ("emittance", "<f4"),
                     ("hasTexture", "u1"), ("_pad0", "u1", (3,)), ("textureID", "<i4"),
                     ("hasBumpMap", "u1"), ("_pad1", "u1", (3,)), ("bumpID", "<i4"), ("bumpScale", "<f4")])
VERTEX = np.dtype([("materialID", "<i4"), ("position", "<f4", (3,)), ("normal", "<f4", (3,)), ("uv", "<f4", (2,))])
TRIANGLE = np.dtype([("v1", VERTEX), ("v2", VERTEX), ("v3", VERTEX), ("centroid", "<f4", (3,)),
                     ("materialID", "<i4"), ("dpdu", "<f4", (3,)), ("dpdv", "<f4", (3,))])
BVHNODE = np.dtype([("min", "<f4", (3,)), ("max", "<f4", (3,)), ("left", "<i4"), ("right", "<i4"),
                    ("start", "<i4"), ("triCount", "<i4")])
CAMERA = np.dtype([("resolution", "<i4", (2,)), ("position", "<f4", (3,)), ("lookAt", "<f4", (3,)),
                   ("view", "<f4", (3,)), ("up", "<f4", (3,)), ("right", "<f4", (3,)), ("fov", "<f4", (2,)),
                   ("pixelLength", "<f4", (2,)), ("aperture", "<f4"), ("focalDist", "<f4")])
PATH = np.dtype([("origin", "<f4", (3,)), ("direction", "<f4", (3,)), ("color", "<f4", (3,)),
                 ("pixelIndex", "<i4"), ("remainingBounces", "<i4")])
ISECT = np.dtype([("t", "<f4"), ("surfaceNormal", "<f4", (3,)), ("materialId", "<i4"), ("uv", "<f4", (2,)),
                  ("dpdu", "<f4", (3,)), ("dpdv", "<f4", (3,))])

PT_OK = 0
PIPELINE_FUSED, PIPELINE_STAGED = 0, 1
SHARD_NONE, SHARD_PIXELS, SHARD_SAMPLES = 0, 1, 2
COMBINE_PEER, COMBINE_RCCL = 0, 1
MAX_DEVICES = 16


class PtError(RuntimeError):
    pass


class _Options(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "stream_compaction", "material_sort", "bvh", "arg_order", "pipeline", "use_graph", "device",
        "shard_mode", "shard_rank", "shard_count", "shard_rows", "block_size", "variant", "frames_per_pass",
        "num_devices")] + [("device_ids", ctypes.c_int32 * MAX_DEVICES), ("combine", ctypes.c_int32)]


class _SceneView(ctypes.Structure):
    _fields_ = [("geoms", ctypes.c_void_p), ("num_geoms", ctypes.c_int32),
                ("materials", ctypes.c_void_p), ("num_materials", ctypes.c_int32),
                ("textures", ctypes.c_void_p), ("num_textures", ctypes.c_int32),
                ("triangles", ctypes.c_void_p), ("num_triangles", ctypes.c_int32),
                ("tri_indices", ctypes.c_void_p), ("num_tri_indices", ctypes.c_int32),
                ("bvh_nodes", ctypes.c_void_p), ("num_bvh_nodes", ctypes.c_int32),
                ("camera", ctypes.c_uint8 * 92), ("trace_depth", ctypes.c_int32)]


class _FrameStats(ctypes.Structure):
    _fields_ = [("iteration", ctypes.c_int32), ("bounces", ctypes.c_int32), ("live", ctypes.c_int64 * 64),
                ("segments", ctypes.c_int64), ("pixels", ctypes.c_int64), ("frames_total", ctypes.c_int64),
                ("live_total", ctypes.c_int64 * 65), ("segments_total", ctypes.c_int64),
                ("frames_per_pass", ctypes.c_int32), ("last_pass_frames", ctypes.c_int32),
                ("queued_total", ctypes.c_int64 * 65), ("handed_total", ctypes.c_int64 * 65),
                ("handed_stack_total", ctypes.c_int64 * 65)]


class _KernelTimes(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_int32), ("frame_ms", ctypes.c_float), ("bounce_ms", ctypes.c_float * 64),
                ("compact_ms", ctypes.c_float), ("intersect_ms", ctypes.c_float), ("shade_ms", ctypes.c_float),
                ("camera_ms", ctypes.c_float), ("sort_ms", ctypes.c_float), ("compact_bytes", ctypes.c_int64),
                ("frame_bytes", ctypes.c_int64), ("compact_scan_ms", ctypes.c_float), ("passes", ctypes.c_int32),
                ("combine_ms", ctypes.c_float), ("bvh_ms", ctypes.c_float * 64), ("tail_ms", ctypes.c_float),
                ("tail_from", ctypes.c_int32)]


# every symbol the C-ABI header declares (tests check the library exports all of them)
ABI_SYMBOLS = [
    "pt_abi_version", "pt_last_error", "pt_default_options", "pt_init_data_container", "pt_init", "pt_free",
    "pt_trace", "pt_trace_frames", "pt_synchronize", "pt_get_image", "pt_get_image_device", "pt_set_image",
    "pt_get_frame_stats", "pt_reset_stats", "pt_set_camera", "pt_scene_load", "pt_scene_get_view", "pt_scene_get_info",
    "pt_scene_material_name", "pt_scene_free", "pt_scene_last_error", "pt_test_camera", "pt_test_intersect",
    "pt_debug_section_counters", "pt_texture_load",
    "pt_save_png", "pt_scene_load_ex", "pt_bvh_build", "pt_bvh_build_last_error", "pt_test_shade", "pt_test_compact", "pt_test_sort", "pt_test_rng", "pt_test_pbo", "pt_profile_frames", "pt_prepare_frames",
    "pt_device_alloc", "pt_device_free", "pt_device_read", "pt_set_trace_depth", "pt_set_speculation",
    "pt_debug_spec_counts",
]
# include/pt/pt_viewer.h (the headless interactive viewer)
VIEWER_SYMBOLS = [
    "pt_viewer_create", "pt_viewer_destroy", "pt_viewer_mouse_button", "pt_viewer_cursor_pos", "pt_viewer_key",
    "pt_viewer_update_camera", "pt_viewer_run_frame", "pt_viewer_display", "pt_viewer_title", "pt_viewer_get_state",
    "pt_viewer_save_image", "pt_viewer_last_error",
]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"ptamd: native library not built: {LIB_PATH} (run `make -C {PKG_ROOT}`); "
                          "there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    sig = {
        "pt_abi_version": (i32, []), "pt_last_error": (ctypes.c_char_p, []),
        "pt_default_options": (None, [vp]), "pt_init_data_container": (i32, [vp]),
        "pt_init": (i32, [vp, vp]), "pt_free": (i32, []), "pt_trace": (i32, [vp, i32, i32, vp]),
        "pt_trace_frames": (i32, [i32, i32]), "pt_synchronize": (i32, []), "pt_get_image": (i32, [vp, i64]),
        "pt_get_image_device": (i32, [vp, vp]), "pt_set_image": (i32, [vp, i64]),
        "pt_get_frame_stats": (i32, [vp]), "pt_reset_stats": (i32, []), "pt_set_camera": (i32, [vp]),
        "pt_scene_load": (i32, [ctypes.c_char_p, i32, i32, i32, i32, vp]), "pt_scene_get_view": (i32, [vp, vp]),
        "pt_scene_get_info": (i32, [vp, vp, vp, ctypes.c_char_p, i32]),
        "pt_scene_material_name": (i32, [vp, i32, ctypes.c_char_p, i32]), "pt_scene_free": (None, [vp]),
        "pt_scene_last_error": (ctypes.c_char_p, []),
        "pt_test_camera": (i32, [i32, vp, i64]), "pt_test_intersect": (i32, [vp, i64, vp]),
        "pt_test_shade": (i32, [i32, vp, vp, i64]), "pt_test_compact": (i32, [vp, i64, vp, vp]),
        "pt_test_sort": (i32, [vp, i64, vp]), "pt_test_rng": (i32, [vp, i64, i32, vp]),
        "pt_test_pbo": (i32, [vp, i64, i32, vp]), "pt_profile_frames": (i32, [i32, i32, vp]), "pt_prepare_frames": (i32, [i32]),
        "pt_debug_section_counters": (i32, [vp, i32, i32]),
        "pt_texture_load": (i32, [ctypes.c_char_p, vp, vp, vp, i64]),
        "pt_save_png": (i32, [vp, i32, i32, i32, ctypes.c_char_p]),
        "pt_scene_load_ex": (i32, [ctypes.c_char_p, i32, i32, i32, i32, vp]),
        "pt_bvh_build": (i32, [vp, i32, vp, i32, vp, vp]),
        "pt_bvh_build_last_error": (ctypes.c_char_p, []),
        "pt_set_trace_depth": (i32, [i32]), "pt_set_speculation": (i32, [i32]), "pt_debug_spec_counts": (i32, [vp, vp]),
        "pt_device_alloc": (i32, [i64, vp]), "pt_device_free": (i32, [vp]), "pt_device_read": (i32, [vp, vp, i64]),
        "pt_viewer_create": (i32, [vp, vp, ctypes.c_char_p, ctypes.c_char_p, vp]), "pt_viewer_destroy": (None, [vp]),
        "pt_viewer_mouse_button": (i32, [vp, i32, i32, i32]),
        "pt_viewer_cursor_pos": (i32, [vp, ctypes.c_double, ctypes.c_double]),
        "pt_viewer_key": (i32, [vp, i32, i32, i32, i32]), "pt_viewer_update_camera": (i32, [vp, vp]),
        "pt_viewer_run_frame": (i32, [vp, vp]), "pt_viewer_display": (i32, [vp, vp, i64]),
        "pt_viewer_title": (i32, [vp, ctypes.c_char_p, i32]), "pt_viewer_get_state": (i32, [vp, vp]),
        "pt_viewer_save_image": (i32, [vp, ctypes.c_char_p, i32]), "pt_viewer_last_error": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


lib = _load()


def _check(rc: int, what: str = ""):
    if rc != PT_OK:
        raise PtError(f"{what}: {lib.pt_last_error().decode(errors='replace')} (code {rc})")


def _ptr(a):
    return a.ctypes.data if a is not None and a.size else None


def default_options(**kw) -> _Options:
    """pt_options with overrides.  `devices=[0, 0, 1]` traces every frame as one pixel shard per
    entry on those GPUs (pt_options.num_devices / device_ids); `combine="peer"|"rccl"`."""
    o = _Options()
    lib.pt_default_options(ctypes.byref(o))
    devices = kw.pop("devices", None)
    if devices is not None:
        devices = list(devices)
        if len(devices) > MAX_DEVICES:
            raise ValueError(f"at most {MAX_DEVICES} devices")
        o.num_devices = len(devices)
        for i, d in enumerate(devices):
            o.device_ids[i] = int(d)
    if isinstance(kw.get("combine"), str):
        kw["combine"] = {"peer": COMBINE_PEER, "rccl": COMBINE_RCCL}[kw["combine"]]
    for k, v in kw.items():
        if not hasattr(o, k) or k == "device_ids":
            raise TypeError(f"unknown option {k}")
        setattr(o, k, int(v))
    return o


def load_texture(path: str) -> np.ndarray:
    """PNG -> (h, w, 4) uint8 RGBA with the scene loader's decoder (stbi STBI_rgb_alpha rules)."""
    w, h = ctypes.c_int32(), ctypes.c_int32()
    rc = lib.pt_texture_load(path.encode(), ctypes.byref(w), ctypes.byref(h), None, 0)
    if rc != PT_OK:
        raise PtError(f"pt_texture_load: {lib.pt_scene_last_error().decode(errors='replace')}")
    out = np.empty((h.value, w.value, 4), np.uint8)
    _check(lib.pt_texture_load(path.encode(), ctypes.byref(w), ctypes.byref(h), out.ctypes.data, out.size),
           "pt_texture_load")
    return out


class _TextureC(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("_pad", ctypes.c_int32), ("data", ctypes.c_void_p)]


class SceneFile:
    """The reference's Scene (scene.h:6-28) loaded by the framework's C++ loader."""

    def __init__(self, path: str, res=None, depth=None, viewer_camera: bool = True, gpu_bvh: bool = False):
        h = ctypes.c_void_p()
        rx, ry = (res if res is not None else (0, 0))
        flags = (1 if viewer_camera else 0) | (2 if gpu_bvh else 0)
        rc = lib.pt_scene_load_ex(path.encode(), int(rx), int(ry), -1 if depth is None else int(depth), flags,
                                  ctypes.byref(h))
        if rc != PT_OK:
            raise PtError(f"pt_scene_load({path}): {lib.pt_scene_last_error().decode(errors='replace')}")
        self._h = h
        self._view = _SceneView()
        _check(lib.pt_scene_get_view(self._h, ctypes.byref(self._view)), "pt_scene_get_view")
        it, td = ctypes.c_int32(), ctypes.c_int32()
        name = ctypes.create_string_buffer(256)
        _check(lib.pt_scene_get_info(self._h, ctypes.byref(it), ctypes.byref(td), name, 256), "pt_scene_get_info")
        self.iterations, self.trace_depth, self.image_name = it.value, td.value, name.value.decode()
        v = self._view
        self.geoms = self._arr(v.geoms, v.num_geoms, GEOM)
        self.materials = self._arr(v.materials, v.num_materials, MATERIAL)
        self.triangles = self._arr(v.triangles, v.num_triangles, TRIANGLE)
        self.tri_indices = self._arr(v.tri_indices, v.num_tri_indices, np.dtype("<i4"))
        self.bvh_nodes = self._arr(v.bvh_nodes, v.num_bvh_nodes, BVHNODE)
        self.camera = np.frombuffer(bytes(v.camera), CAMERA).copy()
        self.textures = []                       # (h, w, 4) uint8 RGBA, Scene::textures order
        for i in range(v.num_textures):
            t = _TextureC.from_address(v.textures + i * ctypes.sizeof(_TextureC))
            px = np.frombuffer((ctypes.c_uint8 * (t.width * t.height * 4)).from_address(t.data), np.uint8)
            self.textures.append(px.reshape(t.height, t.width, 4).copy())
        self.material_names = []
        buf = ctypes.create_string_buffer(256)
        for i in range(v.num_materials):
            _check(lib.pt_scene_material_name(self._h, i, buf, 256), "material name")
            self.material_names.append(buf.value.decode())

    @staticmethod
    def _arr(ptr, n, dt):
        if not n:
            return np.zeros(0, dt)
        return np.frombuffer((ctypes.c_char * (n * dt.itemsize)).from_address(ptr), dt).copy()

    @property
    def width(self):
        return int(self.camera["resolution"][0][0])

    @property
    def height(self):
        return int(self.camera["resolution"][0][1])

    def view(self) -> _SceneView:
        return self._view

    def close(self):
        if getattr(self, "_h", None):
            lib.pt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def scene_view_from_arrays(geoms, materials, camera, trace_depth, triangles=None, tri_indices=None, bvh_nodes=None):
    """A pt_scene_view over caller-owned numpy arrays (reference layouts)."""
    v = _SceneView()
    keep = []

    def put(arr, dt):
        if arr is None or len(arr) == 0:
            return None, 0
        a = np.ascontiguousarray(arr, dtype=dt)
        keep.append(a)
        return a.ctypes.data, len(a)

    v.geoms, v.num_geoms = put(geoms, GEOM)
    v.materials, v.num_materials = put(materials, MATERIAL)
    v.triangles, v.num_triangles = put(triangles, TRIANGLE)
    v.tri_indices, v.num_tri_indices = put(tri_indices, np.dtype("<i4"))
    v.bvh_nodes, v.num_bvh_nodes = put(bvh_nodes, BVHNODE)
    cam = np.ascontiguousarray(camera, CAMERA).reshape(1)
    ctypes.memmove(ctypes.addressof(v.camera), cam.ctypes.data, 92)
    v.trace_depth = int(trace_depth)
    v._keep = keep
    return v


class PathTracer:
    """pathtraceInit / pathtrace / pathtraceFree (pathtrace.cu:134-787) on one GPU."""

    _live = None

    def __init__(self, scene, **options):
        if PathTracer._live is not None:
            PathTracer._live.free()       # the library state is process-global, like the reference's
        self.opts = default_options(**options)
        view = scene.view() if hasattr(scene, "view") else scene
        self.scene = scene
        cam = np.frombuffer(bytes(view.camera), CAMERA)
        self.width, self.height = int(cam["resolution"][0][0]), int(cam["resolution"][0][1])
        self.trace_depth = int(view.trace_depth)
        _check(lib.pt_init(ctypes.byref(view), ctypes.byref(self.opts)), "pt_init")
        PathTracer._live = self
        self.iteration = 0
        self._host_image = None

    @property
    def pixels(self):
        return self.width * self.height

    def trace(self, iteration: int | None = None, pbo_device_ptr: int | None = None, copy_image: bool = False):
        """One pathtrace(pbo, 0, iteration) call.  With copy_image, returns the accumulated image
        copied into this tracer's host buffer (the reference's scene->state.image): a view that
        the next trace(copy_image=True) overwrites."""
        self.iteration = self.iteration + 1 if iteration is None else int(iteration)
        img = None
        if copy_image:
            # one host buffer per tracer, like the reference's scene->state.image
            if self._host_image is None:
                self._host_image = np.empty((self.pixels, 3), np.float32)
            img = self._host_image
        _check(lib.pt_trace(pbo_device_ptr, 0, self.iteration, _ptr(img)), "pt_trace")
        return img

    def set_trace_depth(self, depth: int):
        """RenderState::traceDepth for the next frames (re-read per pathtrace call, pathtrace.cu:641)."""
        _check(lib.pt_set_trace_depth(int(depth)), "pt_set_trace_depth")
        self.trace_depth = int(depth)

    def set_speculation(self, enabled: bool):
        """Next-frame speculation of single-frame calls that copy the image out (default on)."""
        _check(lib.pt_set_speculation(int(bool(enabled))), "pt_set_speculation")

    def spec_counts(self):
        """(frames speculated, frames taken over) since init, over every shard."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        _check(lib.pt_debug_spec_counts(ctypes.byref(a), ctypes.byref(b)), "pt_debug_spec_counts")
        return a.value, b.value

    def trace_frames(self, first_iteration: int, count: int):
        _check(lib.pt_trace_frames(int(first_iteration), int(count)), "pt_trace_frames")
        self.iteration = first_iteration + count - 1

    def prepare_frames(self, count: int):
        """Capture the pass graphs trace_frames(., count) replays (keeps capture out of timing)."""
        _check(lib.pt_prepare_frames(int(count)), "pt_prepare_frames")

    def synchronize(self):
        _check(lib.pt_synchronize(), "pt_synchronize")

    def image(self) -> np.ndarray:
        out = np.empty((self.pixels, 3), np.float32)
        _check(lib.pt_get_image(out.ctypes.data, out.size), "pt_get_image")
        return out

    def set_image(self, img: np.ndarray):
        img = np.ascontiguousarray(img, np.float32)
        _check(lib.pt_set_image(img.ctypes.data, img.size), "pt_set_image")

    def image_device_ptr(self):
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        _check(lib.pt_get_image_device(ctypes.byref(p), ctypes.byref(n)), "pt_get_image_device")
        return p.value, n.value

    def stats(self) -> dict:
        s = _FrameStats()
        _check(lib.pt_get_frame_stats(ctypes.byref(s)), "pt_get_frame_stats")
        return {"iteration": s.iteration, "live": [s.live[i] for i in range(s.bounces)],
                "segments": s.segments, "pixels": s.pixels, "frames_total": s.frames_total,
                "live_total": [s.live_total[i] for i in range(s.bounces + 1)],
                "segments_total": s.segments_total, "frames_per_pass": s.frames_per_pass,
                "last_pass_frames": s.last_pass_frames,
                "queued_total": [s.queued_total[i] for i in range(s.bounces + 1)],
                "handed_total": [s.handed_total[i] for i in range(s.bounces + 1)],
                "handed_stack_total": [s.handed_stack_total[i] for i in range(s.bounces + 1)]}

    def reset_stats(self):
        _check(lib.pt_reset_stats(), "pt_reset_stats")

    def profile(self, first_iteration: int, count: int) -> dict:
        t = _KernelTimes()
        _check(lib.pt_profile_frames(int(first_iteration), int(count), ctypes.byref(t)), "pt_profile_frames")
        self.iteration = first_iteration + count - 1
        return {"frames": t.frames, "passes": t.passes, "frame_ms": t.frame_ms, "combine_ms": t.combine_ms,
                "bounce_ms": [t.bounce_ms[i] for i in range(max(1, self.trace_depth))],
                "bvh_ms": [t.bvh_ms[i] for i in range(max(1, self.trace_depth))],
                "compact_ms": t.compact_ms, "intersect_ms": t.intersect_ms, "shade_ms": t.shade_ms,
                "camera_ms": t.camera_ms, "sort_ms": t.sort_ms, "compact_scan_ms": t.compact_scan_ms,
                "tail_ms": t.tail_ms, "tail_from": t.tail_from}

    SECTIONS = ["load", "cull", "exact", "finish", "shade", "store", "n_exact", "n_cand", "n_iters", "n_waves",
                "n_lanes", "n_nodes", "n_tris", "n_bvh_rays", "n_aabb_mismatch", "n_bvh_witers", "n_leaves",
                "n_bvh_hits", "n_miss_nodes", "n_root_culled"]

    def section_counters(self, reset: bool = True) -> dict:
        """Fused-kernel section counters (variant bit 4); see pathtrace_abi.h."""
        buf = (ctypes.c_uint64 * 76)()
        _check(lib.pt_debug_section_counters(buf, 76, int(reset)), "pt_debug_section_counters")
        out = {k: int(buf[i]) for i, k in enumerate(self.SECTIONS)}
        out["bvh_lanes_hist"] = [int(buf[len(self.SECTIONS) + i]) for i in range(16)]
        out["tail_lanes_hist"] = [int(buf[len(self.SECTIONS) + 16 + i]) for i in range(16)]
        out["tail_by_sp"] = [int(buf[len(self.SECTIONS) + 32 + i]) for i in range(16)]
        out["tail_by_hit"] = [int(buf[len(self.SECTIONS) + 48 + i]) for i in range(4)]
        # candidate-table scenes: superset sizes summed over live lanes, and the waves' maxima
        out["n_sup"] = int(buf[len(self.SECTIONS) + 52])
        out["n_sup_wmax"] = int(buf[len(self.SECTIONS) + 53])
        out["n_sup_wunion"] = int(buf[len(self.SECTIONS) + 54])
        return out

    # ---- single-kernel entry points (tests) ----
    def test_camera(self, iteration: int) -> np.ndarray:
        out = np.zeros(self.pixels, PATH)
        _check(lib.pt_test_camera(int(iteration), out.ctypes.data, out.size), "pt_test_camera")
        return out

    def test_intersect(self, paths: np.ndarray) -> np.ndarray:
        paths = np.ascontiguousarray(paths, PATH)
        out = np.zeros(len(paths), ISECT)
        _check(lib.pt_test_intersect(_ptr(paths), len(paths), _ptr(out)), "pt_test_intersect")
        return out

    def test_shade(self, iteration: int, isects: np.ndarray, paths: np.ndarray) -> np.ndarray:
        isects = np.ascontiguousarray(isects, ISECT)
        paths = np.array(paths, PATH)
        _check(lib.pt_test_shade(int(iteration), _ptr(isects), _ptr(paths), len(paths)), "pt_test_shade")
        return paths

    def test_compact(self, paths: np.ndarray):
        paths = np.ascontiguousarray(paths, PATH)
        out = np.zeros(len(paths), PATH)
        alive = ctypes.c_int64()
        _check(lib.pt_test_compact(_ptr(paths), len(paths), _ptr(out), ctypes.byref(alive)), "pt_test_compact")
        return out[:alive.value]

    def test_sort(self, isects: np.ndarray) -> np.ndarray:
        isects = np.ascontiguousarray(isects, ISECT)
        perm = np.zeros(len(isects), np.int32)
        _check(lib.pt_test_sort(_ptr(isects), len(isects), _ptr(perm)), "pt_test_sort")
        return perm

    def free(self):
        lib.pt_free()
        self._host_image = None
        if PathTracer._live is self:
            PathTracer._live = None


class _ViewerState(ctypes.Structure):
    _fields_ = [("zoom", ctypes.c_float), ("theta", ctypes.c_float), ("phi", ctypes.c_float),
                ("iteration", ctypes.c_int32), ("camchanged", ctypes.c_int32), ("left", ctypes.c_int32),
                ("right", ctypes.c_int32), ("middle", ctypes.c_int32), ("last_x", ctypes.c_double),
                ("last_y", ctypes.c_double), ("should_close", ctypes.c_int32), ("exited", ctypes.c_int32),
                ("traced_depth", ctypes.c_int32), ("saved_images", ctypes.c_int32),
                ("og_look_at", ctypes.c_float * 3), ("camera", ctypes.c_uint8 * 92)]


class Viewer:
    """The reference's interactive viewer (main.cpp) without a window (include/pt/pt_viewer.h):
    GLFW-style events in, runCuda() per display frame, the displayed pixels and saveImage out.
    `scene` must be loaded with viewer_camera=False (the viewer applies main.cpp's recompute)."""

    PRESS, RELEASE = 1, 0
    LEFT, RIGHT, MIDDLE = 0, 1, 2
    KEY_SPACE, KEY_S, KEY_ESCAPE = 32, 83, 256

    def __init__(self, scene: SceneFile, image_dir: str = "../img", time_tag: str | None = None, **options):
        self.scene = scene
        self._opts = default_options(**options)
        h = ctypes.c_void_p()
        rc = lib.pt_viewer_create(scene._h, ctypes.byref(self._opts), image_dir.encode(),
                                  None if time_tag is None else time_tag.encode(), ctypes.byref(h))
        if rc != PT_OK:
            raise PtError(f"pt_viewer_create: {lib.pt_viewer_last_error().decode(errors='replace')}")
        self._h = h

    def _c(self, rc, what):
        if rc != PT_OK:
            raise PtError(f"{what}: {lib.pt_viewer_last_error().decode(errors='replace')} (code {rc})")

    def mouse_button(self, button: int, action: int, mods: int = 0):
        self._c(lib.pt_viewer_mouse_button(self._h, button, action, mods), "mouse_button")

    def cursor_pos(self, x: float, y: float):
        self._c(lib.pt_viewer_cursor_pos(self._h, float(x), float(y)), "cursor_pos")

    def key(self, key: int, action: int = 1):
        self._c(lib.pt_viewer_key(self._h, key, 0, action, 0), "key")

    def update_camera(self) -> bool:
        r = ctypes.c_int32()
        self._c(lib.pt_viewer_update_camera(self._h, ctypes.byref(r)), "update_camera")
        return bool(r.value)

    def run_frame(self) -> bool:
        """One runCuda(); True when ITERATIONS were reached (image saved, tracer freed)."""
        e = ctypes.c_int32()
        self._c(lib.pt_viewer_run_frame(self._h, ctypes.byref(e)), "run_frame")
        return bool(e.value)

    def state(self) -> dict:
        st = _ViewerState()
        self._c(lib.pt_viewer_get_state(self._h, ctypes.byref(st)), "get_state")
        d = {k: getattr(st, k) for k, _ in _ViewerState._fields_ if k not in ("og_look_at", "camera")}
        d["og_look_at"] = np.array(st.og_look_at, np.float32)
        d["camera"] = np.frombuffer(bytes(st.camera), CAMERA).copy()
        return d

    def title(self) -> str:
        buf = ctypes.create_string_buffer(128)
        self._c(lib.pt_viewer_title(self._h, buf, 128), "title")
        return buf.value.decode()

    def display(self) -> np.ndarray:
        cam = self.state()["camera"]
        w, h = int(cam["resolution"][0][0]), int(cam["resolution"][0][1])
        out = np.empty((h, w, 3), np.uint8)
        self._c(lib.pt_viewer_display(self._h, out.ctypes.data, out.size), "display")
        return out

    def save_image(self) -> str:
        buf = ctypes.create_string_buffer(4096)
        self._c(lib.pt_viewer_save_image(self._h, buf, 4096), "save_image")
        return buf.value.decode()

    def image(self) -> np.ndarray:
        """The accumulated (not averaged) image of the frames since the last restart (the copy
        pathtrace wrote into renderState->image), read from the tracer the viewer drives."""
        cam = self.state()["camera"]
        n = int(cam["resolution"][0][0]) * int(cam["resolution"][0][1])
        out = np.empty((n, 3), np.float32)
        _check(lib.pt_get_image(out.ctypes.data, out.size), "pt_get_image")
        return out

    def close(self):
        if getattr(self, "_h", None):
            lib.pt_viewer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rng_draws(seeds: np.ndarray, n: int) -> np.ndarray:
    """u01 draws of makeSeededRandomEngine(iter, index, depth) on the GPU; seeds: (m, 3) int32."""
    seeds = np.ascontiguousarray(seeds, np.int32).reshape(-1, 3)
    out = np.zeros((len(seeds), n), np.float32)
    _check(lib.pt_test_rng(_ptr(seeds), len(seeds), int(n), _ptr(out)), "pt_test_rng")
    return out


def build_bvh(triangles: np.ndarray):
    """scene.cpp:445-525 on the GPU (pt_bvh_build): (bvh_nodes, tri_indices), bit-identical to the
    host build."""
    tris = np.ascontiguousarray(triangles, TRIANGLE)
    n = len(tris)
    nodes = np.zeros(max(1, 2 * n - 1), BVHNODE)
    idx = np.zeros(max(1, n), np.int32)
    cnt = ctypes.c_int32()
    rc = lib.pt_bvh_build(_ptr(tris), n, nodes.ctypes.data, len(nodes), ctypes.byref(cnt), idx.ctypes.data)
    if rc != PT_OK:
        raise PtError(f"pt_bvh_build: {lib.pt_bvh_build_last_error().decode(errors='replace')} (code {rc})")
    return nodes[:cnt.value].copy(), idx[:n].copy()


def save_png(image: np.ndarray, width: int, height: int, iteration: int, base_path: str):
    """saveImage + Image::savePNG (main.cpp:395-419, image.cpp:23-43) -> base_path + ".png"."""
    image = np.ascontiguousarray(image, np.float32).reshape(-1, 3)
    if len(image) != width * height:
        raise ValueError("image size != width * height")
    rc = lib.pt_save_png(image.ctypes.data, int(width), int(height), int(iteration), base_path.encode())
    if rc != PT_OK:
        raise PtError(f"pt_save_png: {lib.pt_scene_last_error().decode(errors='replace')}")


def image_to_pbo(image: np.ndarray, iteration: int) -> np.ndarray:
    image = np.ascontiguousarray(image, np.float32).reshape(-1, 3)
    out = np.zeros((len(image), 4), np.uint8)
    _check(lib.pt_test_pbo(_ptr(image), len(image), int(iteration), _ptr(out)), "pt_test_pbo")
    return out
