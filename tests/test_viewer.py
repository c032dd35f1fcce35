"""The headless interactive viewer (include/pt/pt_viewer.h, host/viewer.cpp): main.cpp's GLFW
camera controls, runCuda's camera recompute / restart, the window title, the displayed PBO and
saveImage, without a window.

CPU tests replay tests/golden/viewer_events.txt and compare, after every `frame` event, the
camera and phi / theta / zoom BITS with tests/golden/viewer_pin.json, which
oracle/ref_pins/viewer_pin.cpp produced from the same events on the reference's own Scene
(src/scene.cpp) and glm (main.cpp's callback bodies restated on those types: main.cpp needs
GLFW / OpenGL / ImGui and cannot be built here).  The GPU tests render a recorded session and
check the accumulated image and the displayed pixels bit-exactly against the oracle traced with
the viewer's camera.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, REPO, scene_path

EVENTS = os.path.join(GOLDEN, "viewer_events.txt")
VIEWER_SCENE = os.path.join(GOLDEN, "viewer_scene.json")
BIT = dict(trig_mode=1, arg_order=0)


def _events(path=EVENTS):
    out = []
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].split()
            if line:
                out.append((line[0], line[1:]))
    return out


def _bits(x):
    return np.asarray(x, np.float32).view(np.uint32).tolist()


def _play(v, events, on_frame):
    for cmd, args in events:
        if cmd == "button":
            v.mouse_button(int(args[0]), int(args[1]))
        elif cmd == "cursor":
            v.cursor_pos(float(args[0]), float(args[1]))
        elif cmd == "key":
            v.key(int(args[0]))
        elif cmd == "frame":
            on_frame(int(args[0]) if args else 1)


def _gpu_visible():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except ImportError:
        return False


def test_viewer_exports_every_declared_symbol(ptamd):
    import re
    with open(os.path.join(REPO, "include", "pt", "pt_viewer.h")) as f:
        names = sorted(set(re.findall(r"^\s*(?:int32_t|void|const char\*)\s+(pt_\w+)\s*\(", f.read(), re.M)))
    assert names == sorted(ptamd.VIEWER_SYMBOLS)
    for n in names:
        assert hasattr(ptamd.lib, n), n


@pytest.mark.parametrize("scene", ["cornell.json", "viewer_scene.json"])
def test_camera_controls_match_reference_pin(scene, tmp_path, ptamd):
    pin = json.load(open(os.path.join(GOLDEN, "viewer_pin.json")))["scenes"][scene]["frames"]
    path = scene_path("cornell") if scene == "cornell.json" else VIEWER_SCENE
    sc = ptamd.SceneFile(path, viewer_camera=False)
    v = ptamd.Viewer(sc, image_dir=str(tmp_path), time_tag="T")
    got = []

    def frame(n):
        reset = v.update_camera()
        st = v.state()
        cam = st["camera"][0]
        got.append({"reset": int(reset), "phi": _bits(st["phi"]), "theta": _bits(st["theta"]),
                    "zoom": _bits(st["zoom"]), "position": _bits(cam["position"]), "lookAt": _bits(cam["lookAt"]),
                    "view": _bits(cam["view"]), "up": _bits(cam["up"]), "right": _bits(cam["right"]),
                    "focalDist": _bits(cam["focalDist"])})
    _play(v, _events(), frame)
    assert len(got) == len(pin)
    for k, (g, p) in enumerate(zip(got, pin)):
        assert g == p, (scene, k, g, p)
    # the first recompute is exactly what the library's one-shot viewer camera applies
    sc2 = ptamd.SceneFile(path, viewer_camera=True)
    first = pin[0]
    c2 = sc2.camera[0]
    assert _bits(c2["position"]) == first["position"] and _bits(c2["view"]) == first["view"]
    # S saved one image (the camera was unchanged by it), named like main.cpp:411-414
    st = v.state()
    assert st["saved_images"] == 1 and st["theta"] == np.float32(st["theta"])
    v.close()


def test_mouse_and_key_state_machine(tmp_path, ptamd):
    sc = ptamd.SceneFile(VIEWER_SCENE, viewer_camera=False)
    v = ptamd.Viewer(sc, image_dir=str(tmp_path), time_tag="2026-01-01_00-00-00z")
    st = v.state()
    assert st["camchanged"] == 1 and st["iteration"] == 0 and (st["last_x"], st["last_y"]) == (0.0, 0.0)
    assert v.title() == "CIS565 Path Tracer | 0 Iterations"
    v.mouse_button(v.LEFT, v.PRESS)
    assert v.state()["left"] == 1
    v.mouse_button(v.RIGHT, v.PRESS)                 # a new press clears the other buttons
    st = v.state()
    assert (st["left"], st["right"], st["middle"]) == (0, 1, 0)
    v.mouse_button(v.RIGHT, v.RELEASE)
    assert v.state()["right"] == 0
    v.cursor_pos(5.0, 7.0)
    v.cursor_pos(5.0, 9.0)                           # equal x: ignored, lastY stays
    st = v.state()
    assert (st["last_x"], st["last_y"]) == (5.0, 7.0)
    v.update_camera()
    assert v.update_camera() is False                # camchanged cleared by the recompute
    v.key(v.KEY_S, v.RELEASE)                        # releases do nothing
    assert v.state()["saved_images"] == 0
    v.key(v.KEY_S)
    name = "viewer_test.2026-01-01_00-00-00z.0samp"  # imageName . startTime . samples "samp"
    assert os.path.exists(tmp_path / (name + ".png"))
    v.key(v.KEY_ESCAPE)
    st = v.state()
    assert st["should_close"] == 1 and st["saved_images"] == 2
    # saveImage writes the same bytes as pt_save_png for the accumulated image (zeros, 0 spp)
    img = np.zeros((96 * 64, 3), np.float32)
    ptamd.save_png(img, 96, 64, 0, str(tmp_path / "ref"))
    assert (tmp_path / "ref.png").read_bytes() == (tmp_path / (name + ".png")).read_bytes()
    v.close()


def test_run_frame_without_device_fails_loudly(tmp_path, ptamd):
    if _gpu_visible():
        pytest.skip("a GPU is visible: covered by the gpu tests")
    sc = ptamd.SceneFile(VIEWER_SCENE, viewer_camera=False)
    v = ptamd.Viewer(sc, image_dir=str(tmp_path), time_tag="T")
    with pytest.raises(ptamd.PtError):
        v.run_frame()
    with pytest.raises(ptamd.PtError):
        v.display()                                  # nothing traced
    v.close()


@pytest.mark.gpu
def test_viewer_session_renders_like_oracle(tmp_path, oracle, ptamd):
    """A recorded session on the GPU: orbit, 2 frames, pan, 3 frames; the accumulated image and
    the window's pixels equal the oracle traced with the viewer's camera for iterations 1..3
    (the pan restarted accumulation), then runCuda saves and exits after ITERATIONS."""
    sc = ptamd.SceneFile(VIEWER_SCENE, viewer_camera=False)
    v = ptamd.Viewer(sc, image_dir=str(tmp_path), time_tag="T")
    v.mouse_button(v.LEFT, v.PRESS)
    v.cursor_pos(10.0, 10.0)
    v.cursor_pos(16.0, 7.0)
    v.mouse_button(v.LEFT, v.RELEASE)
    for _ in range(2):
        assert v.run_frame() is False
    assert v.title() == "CIS565 Path Tracer | 2 Iterations"
    v.mouse_button(v.MIDDLE, v.PRESS)
    v.cursor_pos(30.0, 20.0)
    v.cursor_pos(25.0, 28.0)
    v.mouse_button(v.MIDDLE, v.RELEASE)
    for _ in range(3):
        assert v.run_frame() is False
    st = v.state()
    assert st["iteration"] == 3 and st["traced_depth"] >= 1

    a = oracle.load_scene(VIEWER_SCENE)
    a.camera = st["camera"].copy()
    r = oracle.Renderer(a, oracle.options(**BIT))
    for it in (1, 2, 3):
        r.trace(it)
    img = v.image()
    assert img.tobytes() == r.image.tobytes()
    pbo = r.pbo().reshape(64, 96, 4)[:, ::-1, :3]     # the window mirrors x (main.cpp:99-104)
    assert np.array_equal(v.display(), pbo)

    for _ in range(3):                                # iterations 4..6
        assert v.run_frame() is False
    assert v.run_frame() is True                      # ITERATIONS reached: saveImage + exit
    saved = tmp_path / "viewer_test.T.6samp.png"
    assert saved.exists()
    for it in (4, 5, 6):
        r.trace(it)
    ptamd.save_png(r.image, 96, 64, 6, str(tmp_path / "want"))
    assert saved.read_bytes() == (tmp_path / "want.png").read_bytes()
    with pytest.raises(ptamd.PtError):
        v.run_frame()
    v.close()


@pytest.mark.gpu
def test_pt_render_events_session(tmp_path):
    """pt_render --events replays a session file end to end (the headless main loop)."""
    import subprocess
    exe = os.path.join(REPO, "project3-cuda-path-tracer-2025_amd", "build", "pt_render")
    ev = tmp_path / "session.txt"
    ev.write_text("frame 2\nbutton 0 1\ncursor 10 10\ncursor 14 12\nbutton 0 0\nframe 3\n"
                  f"display {tmp_path / 'window.png'}\nkey 83\nframe 10\n")
    out = subprocess.run([exe, VIEWER_SCENE, "--events", str(ev), "--img-dir", str(tmp_path), "--time-tag", "T"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "reached ITERATIONS" in out.stdout and "6 Iterations" in out.stdout
    assert (tmp_path / "window.png").exists()
    assert (tmp_path / "viewer_test.T.3samp.png").exists()      # S after 3 frames
    assert (tmp_path / "viewer_test.T.6samp.png").exists()      # runCuda's save at ITERATIONS
