"""pathtrace()'s next-frame speculation (pt_runtime.hip spec_*).

main.cpp calls pathtrace(pbo, frame, ++iteration) once per frame and the reference copies the
accumulated image to host memory every call (pathtrace.cu:783).  After tracing frame N the library
traces frame N + 1 on a second stream -- into a plane and a FrameCtl of its own -- while frame N's
image is copied out, and forms image + plane at its end; the call for N + 1 copies that sum out at
once while it becomes the image and the frame's counters are taken over.
These tests drive every way a caller can break the sequence (another iteration, a repeated one, a
depth change, a camera change, set_image, stats resets, multi-frame passes in between, a PBO) and
require the image, the PBO, the per-bounce live counts and TracedDepth to equal the oracle's
sequential frames bit for bit, and equal the library with speculation off (PT_SPECULATE=0).
"""
import ctypes

import numpy as np
import pytest

from conftest import scene_path

BIT = dict(trig_mode=1, arg_order=0)
pytestmark = pytest.mark.gpu


def _eq(x, y):
    return np.asarray(x).tobytes() == np.asarray(y).tobytes()


def _pair(oracle, ptamd, name, res, depth=None):
    return (oracle.load_scene(scene_path(name), res=res, depth=depth),
            ptamd.SceneFile(scene_path(name), res=res, depth=depth))


def _check_frame(tr, r, a, it, td):
    live = r.trace(it)
    img = tr.trace(it, copy_image=True)
    assert _eq(img, r.image), (it, int(np.sum(img.view(np.uint32) != r.image.view(np.uint32))))
    st = tr.stats()
    assert st["live"][:a.trace_depth] == [int(x) if x >= 0 else 0 for x in live][:a.trace_depth], it
    ran = next((k for k in range(1, a.trace_depth) if live[k] <= 0), max(1, a.trace_depth))
    assert td.value == ran, (it, td.value, ran)


@pytest.mark.parametrize("name,res,opts", [
    ("cornell", (64, 64), {}),
    ("cornell_glass_test", (64, 48), {"material_sort": 1}),
    ("cornell_obj_bnnuy", (64, 64), {}),
    # several device contexts (shards sharing GPU 0 on the test box): every shard speculates its
    # own pixels, the call for N + 1 takes each over and combines them (peer pull / RCCL group)
    ("cornell", (64, 64), {"devices": [0, 0]}),
    ("cornell_glass_test", (64, 48), {"material_sort": 1, "devices": [0, 0, 0], "combine": "rccl"}),
    ("cornell_obj_bnnuy", (64, 64), {"devices": [0, 0, 0], "combine": "rccl"}),
    ("cornell_obj_bnnuy", (64, 64), {"devices": [0, 0, 0, 0]}),
    ("cornell_glass_test", (64, 61), {"devices": [0, 0, 0], "band_copy": "1"}),   # host copy by row bands
])
def test_speculated_api_frames_bitexact(name, res, opts, oracle, ptamd, monkeypatch):
    monkeypatch.delenv("PT_SPECULATE", raising=False)
    opts = dict(opts)
    monkeypatch.setenv("PT_BAND_COPY", opts.pop("band_copy", "-1"))
    a, b = _pair(oracle, ptamd, name, res)
    td = ctypes.c_int32(-7)
    ptamd.lib.pt_init_data_container(ctypes.byref(td))
    tr = ptamd.PathTracer(b, **opts)
    r = oracle.Renderer(a, oracle.options(material_sort=opts.get("material_sort", 0), **BIT))
    try:
        for it in (1, 2, 3, 4):                      # consecutive: frames 2..4 were speculated
            _check_frame(tr, r, a, it, td)
        launched, adopted = tr.spec_counts()
        assert adopted == 3 * len(opts.get("devices", [0])) and launched >= adopted, (launched, adopted)
        for it in (6, 7, 7, 8):                      # a skipped and a repeated iteration
            _check_frame(tr, r, a, it, td)
        tr.set_trace_depth(3)                        # depth change: the speculated frame is dropped
        a.trace_depth = r.cs.trace_depth = 3
        for it in (9, 10):
            _check_frame(tr, r, a, it, td)
        tr.set_trace_depth(a.trace_depth)            # unchanged depth keeps the speculation
        _check_frame(tr, r, a, 11, td)
        img = np.full((a.pixelcount, 3), 0.25, np.float32)   # set_image between frames
        tr.set_image(img)
        r.image[:] = img
        for it in (12, 13):
            _check_frame(tr, r, a, it, td)
        tr.reset_stats()                             # counters reset between frames
        _check_frame(tr, r, a, 14, td)
        assert tr.stats()["frames_total"] == 1
        for it in range(15, 19):                     # multi-frame passes in between
            r.trace(it)
        tr.trace_frames(15, 4)
        assert _eq(tr.image(), r.image)
        for it in (19, 20):
            _check_frame(tr, r, a, it, td)
    finally:
        tr.free()
        ptamd.lib.pt_init_data_container(None)


@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_speculation_on_off_identical_with_pbo(devices, oracle, ptamd, monkeypatch):
    """the same call sequence with PT_SPECULATE=0 and with speculation: images and PBOs equal;
    a call without the host copy in the middle takes over the frame the previous one started"""
    a, b = _pair(oracle, ptamd, "cornell_glass_test", (48, 48))
    pbo = ctypes.c_void_p()
    assert ptamd.lib.pt_device_alloc(4 * a.pixelcount, ctypes.byref(pbo)) == 0
    out = {}
    try:
        for mode in ("0", "1"):
            monkeypatch.setenv("PT_SPECULATE", mode)
            tr = ptamd.PathTracer(b, **({} if devices is None else {"devices": devices}))
            imgs, pbos = [], []
            for it in (1, 2, 3, 5, 6, 7, 8):
                tr.trace(it, pbo_device_ptr=pbo.value, copy_image=it != 6)
                imgs.append(tr.image())
                h = np.zeros((a.pixelcount, 4), np.uint8)
                assert ptamd.lib.pt_device_read(h.ctypes.data, pbo, h.nbytes) == 0
                pbos.append(h)
            tr.free()
            out[mode] = (imgs, pbos)
    finally:
        ptamd.lib.pt_device_free(pbo)
    for x, y in zip(out["0"][0] + out["0"][1], out["1"][0] + out["1"][1]):
        assert _eq(x, y)


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_camera_change_drops_the_speculated_frame(devices, oracle, ptamd, monkeypatch):
    """pt_set_camera with a different camera between frames: the frame traced after it uses the
    new camera (equal to a fresh tracer on the moved camera); setting the SAME camera keeps it.
    (Speculation starts only in calls that copy the image out, as main.cpp's do.)"""
    monkeypatch.delenv("PT_SPECULATE", raising=False)
    a, b = _pair(oracle, ptamd, "cornell", (48, 48))
    b2 = ptamd.SceneFile(scene_path("cornell"), res=(48, 48))
    cam = b2.camera.copy()
    cam["position"][0][1] += 0.25                 # eye moved up
    dev = {} if devices is None else {"devices": devices}
    tr = ptamd.PathTracer(b, **dev)
    tr.trace(1, copy_image=True)
    tr.trace(2, copy_image=True)
    assert ptamd.lib.pt_set_camera(b.camera.ctypes.data) == 0      # unchanged
    base = tr.trace(3, copy_image=True).copy()
    assert ptamd.lib.pt_set_camera(cam.ctypes.data) == 0           # moved: frame 4 on the new camera
    got = tr.trace(4, copy_image=True).copy()
    assert _eq(tr.image(), got)
    tr.free()
    # reference: frames 1..3 on the old camera, then frame 4 on the moved one, no speculation
    monkeypatch.setenv("PT_SPECULATE", "0")
    t2 = ptamd.PathTracer(b, **dev)
    for it in (1, 2, 3):
        t2.trace(it)
    assert _eq(t2.image(), base)
    assert ptamd.lib.pt_set_camera(cam.ctypes.data) == 0
    t2.trace(4)
    assert _eq(t2.image(), got)
    t2.free()


def test_speculated_frames_deep_trace(oracle, ptamd, monkeypatch):
    """trace depth 40: 41 counter rows x 8 segments -- more counters than k_adopt_frame's block has
    threads; every row's live count taken over from the speculated frame"""
    monkeypatch.delenv("PT_SPECULATE", raising=False)
    a, b = _pair(oracle, ptamd, "cornell_glass_test", (32, 32), depth=40)
    td = ctypes.c_int32(-7)
    ptamd.lib.pt_init_data_container(ctypes.byref(td))
    tr = ptamd.PathTracer(b)
    r = oracle.Renderer(a, oracle.options(**BIT))
    try:
        for it in (1, 2, 3, 4, 5):
            _check_frame(tr, r, a, it, td)
        st = tr.stats()
        assert st["frames_total"] == 5
        assert st["segments_total"] > 0
    finally:
        tr.free()
        ptamd.lib.pt_init_data_container(None)
