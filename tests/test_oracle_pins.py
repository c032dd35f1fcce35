"""The oracle checked against everything that pins it (CPU only).

* rocThrust fixtures (oracle/ref_pins/rng_pin.cpp): the reference's RNG dependency.
* glm / json / utilities.cpp fixtures (oracle/ref_pins/ingest_pin.cpp): the reference's own
  src/utilities.cpp and its vendored glm 0.9.6 + nlohmann json 3.11.3, built from source.
* SURVEY.md §8a known answers measured on the reference itself: per-bounce live-path counts of
  cornell 800x800 depth 8 (iterations 1-2 average), Σn of the glass scene, the first NaN pixel.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, scene_path


def _f(bits):
    return np.array(bits, dtype=np.uint32).view(np.float32)


@pytest.fixture(scope="module")
def rng_pin():
    with open(os.path.join(GOLDEN, "rng_pin.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def ingest_pin():
    with open(os.path.join(GOLDEN, "ingest_pin.json")) as f:
        return json.load(f)


def test_rng_matches_rocthrust(oracle, rng_pin):
    assert rng_pin["thrust_version"] == 200805
    for it, index, depth, h, draws in rng_pin["cases"]:
        # makeSeededRandomEngine's hash (pathtrace.cu:54)
        key = (0x80000000 | (depth << 22) | it) & 0xFFFFFFFF
        assert (oracle.lib().or_utilhash(key) ^ oracle.lib().or_utilhash(index & 0xFFFFFFFF)) == h
        got = oracle.rng_draws(it, index, depth, len(draws))
        assert got.view(np.uint32).tolist() == draws, (it, index, depth)


def test_rng_u01_can_be_one(oracle):
    # u01 = float(x-1) / 2^31 rounds up to exactly 1.0f for x close to 2^31-1
    x = np.uint32(2147483646)
    assert np.float32(np.float32(x - 1) / np.float32(2 ** 31)) == np.float32(1.0)


def test_materials_alphabetical(oracle, ingest_pin):
    for name, d in ingest_pin["scenes"].items():
        sc = oracle.load_scene(scene_path(name)) if _loadable(name) else None
        if sc is None:
            continue
        assert sc.material_names == d["materials"], name


def _loadable(name):
    # scenes whose OBJ meshes have stand-ins (or none are needed)
    with open(scene_path(name)) as f:
        data = json.load(f)
    for o in data["Objects"]:
        if o["TYPE"] == "obj" and not os.path.exists(os.path.join(os.path.dirname(scene_path(name)), o["PATH"].lstrip("/"))):
            return False
    return "APERTURE" in data["Camera"]


def test_geom_matrices_match_glm(oracle, ingest_pin):
    checked = 0
    for name, d in ingest_pin["scenes"].items():
        with open(scene_path(name)) as f:
            objs = json.load(f)["Objects"]
        for o, ref in zip(objs, d["objects"]):
            T = np.zeros((4, 4), np.float32)
            I = np.zeros((4, 4), np.float32)
            IT = np.zeros((4, 4), np.float32)
            L = oracle.lib()
            L.or_build_transform(oracle.v3(o["TRANS"]), oracle.v3(o["ROTAT"]), oracle.v3(o["SCALE"]), T.ctypes.data)
            L.or_mat4_inverse(T.ctypes.data, I.ctypes.data)
            L.or_mat4_inverse_transpose(T.ctypes.data, IT.ctypes.data)
            assert T.reshape(-1).view(np.uint32).tolist() == ref["transform"], (name, o)
            assert I.reshape(-1).view(np.uint32).tolist() == ref["inverse"], (name, o)
            assert IT.reshape(-1).view(np.uint32).tolist() == ref["invTranspose"], (name, o)
            checked += 1
    assert checked > 300


def test_camera_matches_glm(oracle, ingest_pin):
    for name, d in ingest_pin["scenes"].items():
        with open(scene_path(name)) as f:
            cam = json.load(f)["Camera"]
        c = np.zeros(1, oracle.CAMERA)
        oracle.lib().or_camera_setup(cam["RES"][0], cam["RES"][1], float(cam["FOVY"]), oracle.v3(cam["EYE"]),
                                     oracle.v3(cam["LOOKAT"]), oracle.v3(cam["UP"]), float(cam.get("APERTURE", 0.0)),
                                     c.ctypes.data)
        ref = d["camera"]
        for k in ("view", "up", "right", "position"):
            assert c[k][0].view(np.uint32).tolist() == ref[k], (name, k)
        assert c["focalDist"].view(np.uint32)[0] == ref["focalDist"], name
        assert c["pixelLength"][0].view(np.uint32).tolist() == ref["pixelLength"], name


def test_glm_vector_semantics(oracle, ingest_pin):
    L = oracle.lib()
    for case in ingest_pin["glm"]:
        I = _f(case["I"]).copy()
        N = _f(case["N"]).copy()
        eta = _f([case["eta"]])[0]
        n = np.zeros(3, np.float32)
        L.or_glm_normalize(N.ctypes.data, n.ctypes.data)
        assert n.view(np.uint32).tolist() == case["normalize"]
        r = np.zeros(3, np.float32)
        L.or_glm_reflect(I.ctypes.data, n.ctypes.data, r.ctypes.data)
        assert r.view(np.uint32).tolist() == case["reflect"]
        In = np.zeros(3, np.float32)
        L.or_glm_normalize(I.ctypes.data, In.ctypes.data)
        t = np.zeros(3, np.float32)
        L.or_glm_refract(In.ctypes.data, n.ctypes.data, float(eta), t.ctypes.data)
        got, want = t.view(np.uint32).tolist(), case["refract"]
        # NaN payloads may differ; NaN-ness (glm 0.9.6 TIR -> NaN) must not
        assert [np.isnan(x) for x in t] == [np.isnan(x) for x in _f(want)]
        assert [g for g, x in zip(got, t) if not np.isnan(x)] == [w for w, x in zip(want, t) if not np.isnan(x)]


# ------------------------- SURVEY.md §8a known answers (reference run) -------------------------
SURVEY_CORNELL_LIVE = [640000, 522838, 360056, 277476, 221092, 179000, 146086, 119486]


def test_known_answer_cornell_live_counts(oracle):
    sc = oracle.load_scene(scene_path("cornell"))
    r = oracle.Renderer(sc, oracle.options(trig_mode=0, arg_order=0))
    l1, l2 = r.trace(1), r.trace(2)
    avg = [int(round((a + b) / 2)) for a, b in zip(l1, l2)]   # SURVEY rounds half to even
    assert avg == SURVEY_CORNELL_LIVE
    assert (int(l1.sum()) + int(l2.sum())) // 2 == 2466034


def test_known_answer_glass_segments(oracle):
    sc = oracle.load_scene(scene_path("cornell_glass_test"))
    r = oracle.Renderer(sc, oracle.options(trig_mode=0, arg_order=0))
    s1, s2 = int(r.trace(1).sum()), int(r.trace(2).sum())
    assert (s1 + s2) / 2 == 2519347


def test_known_answer_first_nan_pixel(oracle):
    sc = oracle.load_scene(scene_path("cornell"))
    r = oracle.Renderer(sc, oracle.options(trig_mode=0, arg_order=0))
    for it in range(1, 8):
        r.trace(it)
        assert np.isfinite(r.image).all(), it
    r.trace(8)
    bad = np.where(~np.isfinite(r.image).all(axis=1))[0]
    assert bad.tolist() == [406300]


def test_known_answer_config1_live_counts(oracle):
    """SURVEY §8a config 1 (cornell 400x400 depth 4): 160000, 130706, 90064, 69475, Σ 450,244.
    These are the per-bounce MEANS over iterations 1-4 (130705.5 rounds to 130706; the sum of the
    unrounded means is 450244.5), i.e. the counts of SURVEY's 4-spp timing run — not one
    iteration's.  Exhaustive search over windows of iterations 1..200, both vec2 argument orders
    and depths 4 / 5 / 8 finds only this window (round-1 VERDICT "What's weak" 1)."""
    sc = oracle.load_scene(scene_path("cornell"), res=(400, 400), depth=4)
    r = oracle.Renderer(sc, oracle.options(trig_mode=0, arg_order=0))
    rows = np.array([r.trace(it) for it in range(1, 5)], np.float64)
    m = rows.mean(axis=0)
    assert m.tolist() == [160000.0, 130705.5, 90064.0, 69475.0]
    assert int(m.sum()) == 450244
