"""The host ingest behind the C-ABI under AddressSanitizer + UndefinedBehaviorSanitizer.

The library parses files a caller hands it: scene JSON (host/json_lite.h), OBJ meshes (host/scene.cpp)
and PNG textures (host/png_decode.cpp, a from-scratch inflate).  `make asan` builds those sources with
-fsanitize=address,undefined,float-cast-overflow into a standalone driver
(host/ingest_check.cpp -> build/asan/ingest_check; no device code, no ctypes), and this test runs it
over every scene and texture of the repository and over the committed corpus of truncated and
corrupt files (tests/golden/corrupt/, made by tests/golden/make_corrupt_corpus.py).

Bar: zero sanitizer reports (any report aborts the driver), and the reference's failure semantics:
a scene it cannot read fails (scene.cpp:245-247 throws; here PT_E_INVALID = -1 with a message), a
texture it cannot decode gets id -1 and the scene still loads (scene.cpp:372-375).
"""
import glob
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN, PKG, REPO

EXE = os.path.join(PKG, "build", "asan", "ingest_check")
CORPUS = os.path.join(GOLDEN, "corrupt")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0:allocator_may_return_null=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="no g++ for the sanitizer build")


@pytest.fixture(scope="module")
def driver():
    subprocess.run(["make", "-C", PKG, "asan"], check=True, capture_output=True, timeout=600)
    return EXE


def _run(driver, mode, files):
    p = subprocess.run([driver, mode] + files, capture_output=True, text=True, timeout=600, env=ENV)
    out = p.stdout + p.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out and "LeakSanitizer" not in out, out[-4000:]
    assert p.returncode == 0, out[-4000:]
    res = {}
    for line in p.stdout.splitlines():
        if ": " in line and (" rc=" in line):
            name, rest = line.split(": ", 1)
            res[os.path.basename(name)] = rest
    assert len(res) == len(files), (len(res), len(files))
    return res


def _expect(res):
    for name, rest in res.items():
        if name.startswith("bad_"):
            assert "rc=-1 err=" in rest, (name, rest)
        elif name.startswith("badtex_"):
            assert rest.startswith("scene rc=0") and "bad_tex=1" in rest, (name, rest)
        else:
            assert " rc=0" in " " + rest, (name, rest)


def test_corrupt_scenes_and_meshes(driver):
    files = sorted(glob.glob(os.path.join(CORPUS, "*.json")))
    assert len(files) > 80
    _expect(_run(driver, "scene", files))


def test_corrupt_pngs(driver):
    files = sorted(glob.glob(os.path.join(CORPUS, "*.png")))
    assert len(files) > 25
    _expect(_run(driver, "png", files))


def test_every_repository_scene_and_texture(driver):
    scenes = sorted(glob.glob(os.path.join(REPO, "scenes", "*.json")))
    res = _run(driver, "scene", scenes)
    loaded = [n for n, r in res.items() if r.startswith("scene rc=0")]
    assert "cornell.json" in loaded and "cornell_obj_bnnuy.json" in loaded and "cornell_obj_khaslana.json" in loaded
    for n, r in res.items():   # the refusals are the reference's: absent OBJs, sphere.json's APERTURE
        if r.startswith("scene rc=-1"):
            assert "Failed to load" in r or "APERTURE" in r, (n, r)
    # the SAH traversal tree is the same tree under every pair numbering (PT_BVH_BFS_LEVELS)
    for n in ("cornell_obj_bnnuy.json", "cornell_obj_khaslana.json"):
        assert "sah_orders_equal=1" in res[n], (n, res[n])
        # the height bound at its tightest, 1 + ceil(log2 leaves), still holds every leaf once
        kv = dict(x.split("=") for x in res[n].split() if "=" in x)
        leaves = int(kv["leaves"])
        assert int(kv["sah_tight"]) == 1 + (leaves - 1).bit_length(), (n, res[n])
        assert int(kv["tight_leaves"]) == leaves, (n, res[n])
        # the 4-wide records hold every leaf once and every record but the root is one child
        assert kv["quad_ok"] == "1" and 0 < int(kv["quads"]) < leaves, (n, res[n])
    pngs = sorted(glob.glob(os.path.join(REPO, "scenes", "textures", "*.png")) +
                  glob.glob(os.path.join(GOLDEN, "*.png")))
    if pngs:
        for n, r in _run(driver, "png", pngs).items():
            assert r.startswith("png rc=0"), (n, r)


def test_save_png_special_values(driver, tmp_path):
    p = subprocess.run([driver, "savepng", str(tmp_path / "x"), "37", "23"], capture_output=True, text=True,
                       timeout=120, env=ENV)
    assert p.returncode == 0 and "savepng rc=0" in p.stdout, p.stdout + p.stderr
    assert (tmp_path / "x.png").stat().st_size > 0
