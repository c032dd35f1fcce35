"""Several GPUs behind one pathtrace() (pt_options.num_devices / device_ids / combine).

SURVEY §8b puts the multi-GPU split inside the boundary: the reference's caller
(main.cpp:463, one pathtrace() per frame) must not change.  Every frame is split into
interleaved row bands, one shard context per entry of device_ids, and after every call the first
device's image receives each shard's pixels (xGMI peer reads, or one RCCL send / recv group).
The image is bit-identical to one device's: pixels are independent (the RNG is keyed by pixel,
iteration and depth) and the combine only copies.

The GPU box has one MI355X, so the shards share device 0 (each on its own stream; the RCCL case
is a one-rank communicator whose sends and receives go to itself).  The CPU tests cover the
option plumbing (PT_DEVICES / PT_COMBINE environment defaults, validation).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG, REPO, scene_path

BIT = dict(trig_mode=1, arg_order=0)


def _eq(x, y):
    return np.asarray(x).tobytes() == np.asarray(y).tobytes()


def _pair(oracle, ptamd, name, res, depth=None):
    a = oracle.load_scene(scene_path(name), res=res, depth=depth)
    b = ptamd.SceneFile(scene_path(name), res=res, depth=depth)
    return a, b


# ---------------------------------------------------------------------------------------------
# CPU: options
# ---------------------------------------------------------------------------------------------
def _defaults_in_child(env):
    code = ("import sys; sys.path.insert(0, %r); import ptamd; o = ptamd.default_options(); "
            "print(o.num_devices, list(o.device_ids)[:4], o.combine)" % PKG)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, **env), check=True).stdout.split("\n")[-2]
    return out


def test_default_options_single_device(ptamd):
    o = ptamd.default_options()
    if "PT_DEVICES" not in os.environ:
        assert o.num_devices == 0
    assert list(o.device_ids) == list(range(ptamd.MAX_DEVICES)) and o.combine == ptamd.COMBINE_PEER
    o = ptamd.default_options(devices=[0, 0, 1], combine="rccl")
    assert o.num_devices == 3 and list(o.device_ids)[:3] == [0, 0, 1] and o.combine == ptamd.COMBINE_RCCL


@pytest.mark.parametrize("env,want", [({"PT_DEVICES": "4"}, "4 [0, 1, 2, 3] 0"),
                                      ({"PT_DEVICES": "0,0,1", "PT_COMBINE": "rccl"}, "3 [0, 0, 1, 3] 1"),
                                      ({"PT_DEVICES": "2,5"}, "2 [2, 5, 2, 3] 0")])
def test_environment_reaches_the_dropin_defaults(env, want):
    """the drop-in (dropin/pathtrace.cpp) has no options channel but the environment"""
    assert _defaults_in_child(env) == want


def test_multi_device_option_validation(ptamd):
    sc = ptamd.SceneFile(scene_path("cornell"), res=(16, 16))
    with pytest.raises(ptamd.PtError, match="num_devices"):
        ptamd.PathTracer(sc, num_devices=17)
    with pytest.raises(ptamd.PtError, match="shard_mode"):
        ptamd.PathTracer(sc, devices=[0, 0], shard_mode=1, shard_count=2)
    with pytest.raises(ptamd.PtError, match="row bands"):      # 16 rows / 8 = 2 bands < 3 shards
        ptamd.PathTracer(sc, devices=[0, 0, 0])


# ---------------------------------------------------------------------------------------------
# GPU: bit-exact frames through the C-ABI
# ---------------------------------------------------------------------------------------------
MULTI_CASES = [
    ("cornell", (64, 64), [0, 0], "peer", {}),
    ("cornell", (64, 64), [0, 0, 0], "rccl", {}),
    ("cornell_glass_test", (64, 48), [0, 0, 0, 0], "peer", {"material_sort": 1}),
    ("cornell_obj_bnnuy", (64, 64), [0, 0, 0], "peer", {}),
    ("cornell_obj_bnnuy", (64, 64), [0, 0], "rccl", {}),
    ("cornell_obj_khaslana", (48, 48), [0, 0, 0], "peer", {}),
    ("cornell", (64, 64), [0, 0, 0], "peer", {"pipeline": 1}),
    # host copy split over the shards' row bands: a shorter last band owned by a middle shard
    # (61 rows = 7 bands of 8 + one of 5, band 7 -> shard 1), more shards than some get bands of
    ("cornell", (64, 61), [0, 0, 0], "peer", {}),
    ("cornell_glass_test", (40, 37), [0, 0, 0, 0, 0], "rccl", {"shard_rows": 2}),
    ("cornell", (48, 20), [0, 0, 0], "peer", {"shard_rows": 8, "pipeline": 1}),
]


@pytest.mark.gpu
@pytest.mark.parametrize("band_copy", ["-1", "1"])
@pytest.mark.parametrize("name,res,devices,combine,opts", MULTI_CASES)
def test_multi_device_api_frames_bitexact(name, res, devices, combine, opts, band_copy, oracle, ptamd, monkeypatch):
    """pathtrace() as main.cpp calls it (one frame per call, host image copied every call, a PBO),
    split over shard contexts: image, PBO, live counts and TracedDepth equal the oracle's.
    PT_BAND_COPY=1: the host copy split over the shards' row bands (by default only when every
    shard has a GPU of its own, which the one-GPU box never has)."""
    monkeypatch.setenv("PT_BAND_COPY", band_copy)
    a, b = _pair(oracle, ptamd, name, res, 12 if "khaslana" in name else None)
    td = ctypes.c_int32(-7)
    ptamd.lib.pt_init_data_container(ctypes.byref(td))
    tr = ptamd.PathTracer(b, devices=devices, combine=combine, **opts)
    r = oracle.Renderer(a, oracle.options(material_sort=opts.get("material_sort", 0), **BIT))
    pbo = ctypes.c_void_p()
    assert ptamd.lib.pt_device_alloc(4 * a.pixelcount, ctypes.byref(pbo)) == 0
    try:
        for it in (1, 2, 3):
            live = r.trace(it)
            img = tr.trace(it, pbo_device_ptr=pbo.value, copy_image=True)
            assert _eq(img, r.image), (it, int(np.sum(img.view(np.uint32) != r.image.view(np.uint32))))
            st = tr.stats()
            assert st["pixels"] == a.pixelcount
            assert st["live"] == [int(x) if x >= 0 else 0 for x in live], (st["live"], live.tolist())
            ran = next((k for k in range(1, a.trace_depth) if live[k] <= 0), a.trace_depth)
            assert td.value == ran
        host_pbo = np.zeros((a.pixelcount, 4), np.uint8)
        assert ptamd.lib.pt_device_read(host_pbo.ctypes.data, pbo, host_pbo.nbytes) == 0
        assert _eq(host_pbo, r.pbo())
        assert _eq(tr.image(), r.image)
    finally:
        ptamd.lib.pt_device_free(pbo)
        tr.free()
        ptamd.lib.pt_init_data_container(None)


@pytest.mark.gpu
@pytest.mark.parametrize("name,res,devices,combine,fpp", [
    ("cornell", (96, 96), [0, 0, 0, 0], "peer", 0),
    ("cornell", (96, 96), [0, 0, 0], "rccl", 2),
    ("cornell_obj_bnnuy", (64, 64), [0, 0], "peer", 3),
    ("cornell_multiple_glass", (64, 64), [0, 0, 0], "rccl", 0),
])
def test_multi_device_passes_bitexact(name, res, devices, combine, fpp, oracle, ptamd):
    """pt_trace_frames over shard contexts (each shard's passes queued before the combine):
    the image after 5 + 2 frames equals the oracle's sequential frames, segment totals included."""
    a, b = _pair(oracle, ptamd, name, res)
    tr = ptamd.PathTracer(b, devices=devices, combine=combine, frames_per_pass=fpp)
    r = oracle.Renderer(a, oracle.options(**BIT))
    segs = 0
    for it in range(1, 8):
        segs += int(np.maximum(r.trace(it), 0).sum())
    tr.prepare_frames(5)
    tr.trace_frames(1, 5)
    tr.trace_frames(6, 2)
    st = tr.stats()
    assert st["frames_total"] == 7 and st["segments_total"] == segs
    assert _eq(tr.image(), r.image)
    # pt_set_image reaches every shard: reset to zero and trace again
    tr.set_image(np.zeros((a.pixelcount, 3), np.float32))
    r.image[:] = 0
    r.trace(8)
    tr.trace_frames(8, 1)
    assert _eq(tr.image(), r.image)
    tr.free()


@pytest.mark.gpu
@pytest.mark.parametrize("name,res,devices,opts", [
    ("cornell", (64, 64), [0, 0], {}),
    ("cornell_glass_test", (64, 48), [0, 0, 0, 0], {"material_sort": 1}),
    ("cornell_obj_bnnuy", (64, 56), [0, 0, 0], {"shard_rows": 4}),
])
def test_multi_device_staged_peer_combine_bitexact(name, res, devices, opts, oracle, ptamd, monkeypatch):
    """the PEER combine's branch for a shard the first device cannot read in place
    (no peer access): k_pack_tile on the shard's stream -> hipMemcpyPeerAsync -> the one
    k_gather_shards launch reading the packed tiles.  PT_COMBINE_FORCE_STAGED=1 takes it although
    the shards share device 0; API frames (TracedDepth, host copy) and multi-frame passes."""
    monkeypatch.setenv("PT_COMBINE_FORCE_STAGED", "1")
    a, b = _pair(oracle, ptamd, name, res)
    td = ctypes.c_int32(-7)
    ptamd.lib.pt_init_data_container(ctypes.byref(td))
    tr = ptamd.PathTracer(b, devices=devices, combine="peer", **opts)
    r = oracle.Renderer(a, oracle.options(material_sort=opts.get("material_sort", 0), **BIT))
    try:
        for it in (1, 2):
            live = r.trace(it)
            img = tr.trace(it, copy_image=True)
            assert _eq(img, r.image), it
            assert td.value == next((k for k in range(1, a.trace_depth) if live[k] <= 0), a.trace_depth)
        for it in range(3, 8):
            r.trace(it)
        tr.trace_frames(3, 5)
        assert _eq(tr.image(), r.image)
    finally:
        tr.free()
        ptamd.lib.pt_init_data_container(None)


@pytest.mark.gpu
def test_multi_device_equals_single_device_full_resolution(ptamd):
    """BASELINE configs[1] (cornell 800x800 d8): 8 shard contexts == one context, bit for bit."""
    b = ptamd.SceneFile(scene_path("cornell"))
    one = ptamd.PathTracer(b)
    one.trace_frames(1, 4)
    want = one.image()
    one.free()
    tr = ptamd.PathTracer(b, devices=[0] * 8, frames_per_pass=4)
    tr.trace_frames(1, 4)
    assert _eq(tr.image(), want)
    tr.free()


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_set_trace_depth_between_frames(devices, oracle, ptamd):
    """RenderState::traceDepth is re-read every pathtrace() (pathtrace.cu:641)"""
    a, b = _pair(oracle, ptamd, "cornell_glass_test", (48, 48))
    kw = {} if devices is None else {"devices": devices}
    tr = ptamd.PathTracer(b, **kw)
    r = oracle.Renderer(a, oracle.options(**BIT))
    for it, d in ((1, 8), (2, 3), (3, 3), (4, 0), (5, 5)):
        a.trace_depth = r.cs.trace_depth = d
        tr.set_trace_depth(d)
        r.trace(it)
        tr.trace(it)
        assert _eq(tr.image(), r.image), (it, d)
    tr.prepare_frames(3)
    a.trace_depth = r.cs.trace_depth = 6
    tr.set_trace_depth(6)
    for it in (6, 7, 8):
        r.trace(it)
    tr.trace_frames(6, 3)
    assert _eq(tr.image(), r.image)
    with pytest.raises(ptamd.PtError):
        tr.set_trace_depth(65)
    tr.free()


@pytest.mark.gpu
def test_multi_device_test_entry_points_refused(ptamd):
    b = ptamd.SceneFile(scene_path("cornell"), res=(32, 32))
    tr = ptamd.PathTracer(b, devices=[0, 0])
    with pytest.raises(ptamd.PtError, match="one device context"):
        tr.test_camera(1)
    with pytest.raises(ptamd.PtError, match="one device context"):
        tr.profile(1, 2)
    tr.free()


@pytest.mark.gpu
def test_trace_frames_then_grow_without_sync(oracle, ptamd):
    """a pass still running when a larger pass re-sizes the buffers (pt_trace_frames
    does not wait) -- the stream is drained before its graph and buffers are released."""
    a, b = _pair(oracle, ptamd, "cornell", (64, 64))
    tr = ptamd.PathTracer(b, frames_per_pass=16)
    r = oracle.Renderer(a, oracle.options(**BIT))
    for it in range(1, 18):
        r.trace(it)
    tr.trace_frames(1, 1)
    tr.trace_frames(2, 16)
    assert _eq(tr.image(), r.image)
    tr.free()


@pytest.mark.gpu
def test_pt_render_devices_flag(tmp_path, oracle, ptamd):
    """the framework's own main.cpp (build/pt_render) reaches the split with --devices"""
    exe = os.path.join(PKG, "build", "pt_render")
    out = str(tmp_path / "cornell")
    p = subprocess.run([exe, scene_path("cornell"), "--spp", "3", "--res", "64x64", "--devices", "0,0,0",
                        "--combine", "rccl", "--out", out], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    with open(out + ".pfm", "rb") as f:
        head = [f.readline() for _ in range(3)]
        got = np.frombuffer(f.read(), np.float32).reshape(64, 64, 3)[::-1].reshape(-1, 3)
    assert head[0].strip() == b"PF"
    a = oracle.load_scene(scene_path("cornell"), res=(64, 64))
    r = oracle.Renderer(a, oracle.options(**BIT))
    for it in (1, 2, 3):
        r.trace(it)
    assert _eq(got, r.image)
