"""The drop-in behind the reference's own caller.

oracle/_ref/dropin_main is built (oracle/ref_pins/make_fixtures.sh) from a main.cpp-shaped
driver, the reference's OWN headers (src/pathtrace.h, scene.h, sceneStructs.h with glm) and host
sources (src/scene.cpp, utilities.cpp, stb.cpp), and the drop-in source
project3-cuda-path-tracer-2025_amd/dropin/pathtrace.cpp, linked against libptamd.so.  So these
tests check that the four entry points of src/pathtrace.h:6-9 link with the caller's types, and
(GPU) that frames traced through them equal the oracle's bit for bit.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, scene_path

EXE = os.path.join(REPO, "oracle", "_ref", "dropin_main")
needs_exe = pytest.mark.skipif(not os.path.exists(EXE), reason="oracle/_ref/dropin_main not built "
                               "(needs /root/reference and the CUDA runtime headers: make_fixtures.sh)")


@needs_exe
def test_dropin_exports_the_reference_signatures():
    """the caller's own mangled names: uchar4 / Scene / GuiDataContainer as main.cpp sees them"""
    out = subprocess.run(["nm", EXE], check=True, capture_output=True, text=True).stdout
    defined = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for sym in ("_Z17InitDataContainerP16GuiDataContainer", "_Z13pathtraceInitP5Scene", "_Z13pathtraceFreev",
                "_Z9pathtraceP6uchar4ii"):
        assert sym in defined, sym
    undefined = {l.split()[-1] for l in out.splitlines() if " U " in l}
    assert {"pt_init", "pt_trace", "pt_free", "pt_set_camera", "pt_init_data_container", "pt_set_trace_depth"} <= undefined


@needs_exe
@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK | os.W_OK),
                    reason="a GPU is visible: covered by test_dropin_frames_bitexact")
def test_dropin_fails_loudly_without_a_device(tmp_path):
    """pathtraceInit without a device: message + exit(EXIT_FAILURE), like checkCUDAErrorFn"""
    p = subprocess.run([EXE, scene_path("cornell"), "1", str(tmp_path / "x.f32")], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 1
    assert "HIP error" in p.stderr and "pathtraceInit" in p.stderr


def _small_scene(tmp_path, name, res):
    with open(scene_path(name)) as f:
        d = json.load(f)
    d["Camera"]["RES"] = list(res)
    os.symlink(os.path.join(REPO, "scenes", "obj"), tmp_path / "obj")
    p = tmp_path / f"{name}.json"
    p.write_text(json.dumps(d))
    return str(p)


@needs_exe
@pytest.mark.gpu
@pytest.mark.parametrize("name,res,frames", [("cornell", (64, 64), 3), ("cornell_glass_test", (48, 40), 2),
                                              ("cornell_obj_bnnuy", (48, 48), 2)])
def test_dropin_frames_bitexact(name, res, frames, tmp_path, oracle):
    """main.cpp's call sequence through the drop-in on the reference's own Scene: the
    accumulated state.image equals the oracle's frames (portable trig) bit for bit, and
    TracedDepth is the depth the last frame ran."""
    path = _small_scene(tmp_path, name, res)
    out = tmp_path / "img.f32"
    p = subprocess.run([EXE, path, str(frames), str(out)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    got = np.fromfile(out, np.float32).reshape(-1, 3)
    sc = oracle.load_scene(path)
    r = oracle.Renderer(sc, oracle.options(trig_mode=1, arg_order=0))
    for it in range(1, frames + 1):
        live = r.trace(it)
    assert got.tobytes() == r.image.tobytes(), int(np.sum(got.view(np.uint32) != r.image.view(np.uint32)))
    ran = next((k for k in range(1, sc.trace_depth) if live[k] <= 0), sc.trace_depth)
    assert f"traced_depth {ran}" in p.stdout


@needs_exe
@pytest.mark.gpu
def test_dropin_rereads_trace_depth_every_frame(tmp_path, oracle):
    """pathtrace.cu:641 reads state.traceDepth at every call: a caller that lowers it before frame 2
    gets frames 2.. at the new depth (oracle traced the same way), bit for bit."""
    path = _small_scene(tmp_path, "cornell", (48, 48))
    out = tmp_path / "img.f32"
    p = subprocess.run([EXE, path, "3", str(out), "2:3"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    got = np.fromfile(out, np.float32).reshape(-1, 3)
    sc = oracle.load_scene(path)
    r = oracle.Renderer(sc, oracle.options(trig_mode=1, arg_order=0))
    r.trace(1)
    sc.trace_depth = r.cs.trace_depth = 3
    for it in (2, 3):
        live = r.trace(it)
    assert got.tobytes() == r.image.tobytes(), int(np.sum(got.view(np.uint32) != r.image.view(np.uint32)))
    ran = next((k for k in range(1, 3) if live[k] <= 0), 3)
    assert f"traced_depth {ran}" in p.stdout


@needs_exe
@pytest.mark.gpu
@pytest.mark.parametrize("devices,combine", [("0,0", "peer"), ("0,0,0", "rccl")])
def test_dropin_several_device_shards(devices, combine, tmp_path, oracle):
    """the reference's caller reaches the multi-device frame split through the environment
    (PT_DEVICES / PT_COMBINE, read by pt_default_options): same image, same TracedDepth."""
    path = _small_scene(tmp_path, "cornell_obj_bnnuy", (48, 48))
    out = tmp_path / "img.f32"
    env = dict(os.environ, PT_DEVICES=devices, PT_COMBINE=combine)
    p = subprocess.run([EXE, path, "2", str(out)], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    got = np.fromfile(out, np.float32).reshape(-1, 3)
    sc = oracle.load_scene(path)
    r = oracle.Renderer(sc, oracle.options(trig_mode=1, arg_order=0))
    for it in (1, 2):
        live = r.trace(it)
    assert got.tobytes() == r.image.tobytes(), int(np.sum(got.view(np.uint32) != r.image.view(np.uint32)))
    ran = next((k for k in range(1, sc.trace_depth) if live[k] <= 0), sc.trace_depth)
    assert f"traced_depth {ran}" in p.stdout
