"""Scene ingest of the product (C++ loader in libptamd.so, host/scene.cpp) against the oracle's
independent loader and against the reference's own glm / utilities.cpp fixtures.  CPU only:
the loader is host code, so these run without a GPU."""
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, SCENES, scene_path
from test_oracle_pins import _loadable

SCENE_NAMES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(SCENES, "*.json")))
LOADABLE = [n for n in SCENE_NAMES if _loadable(n)]


def test_enough_scenes_loadable():
    assert {"cornell.json", "cornell_glass_test.json", "cornell_obj_bnnuy.json",
            "cornell_obj_khaslana.json"} <= set(LOADABLE)


@pytest.mark.parametrize("name", LOADABLE)
def test_loader_bit_identical_to_oracle(name, oracle, ptamd):
    a = oracle.load_scene(scene_path(name))
    b = ptamd.SceneFile(scene_path(name))
    assert a.material_names == b.material_names
    for field in ("geoms", "materials", "triangles", "tri_indices", "bvh_nodes", "camera"):
        x, y = getattr(a, field), getattr(b, field)
        assert x.tobytes() == y.tobytes(), (name, field)
    assert (a.trace_depth, a.iterations, a.image_name) == (b.trace_depth, b.iterations, b.image_name)
    # textures: the framework's PNG decoder vs the oracle's (Pillow), same ids / order
    assert len(a.textures) == len(b.textures), name
    for ta, tb in zip(a.textures, b.textures):
        assert ta.shape == tb.shape and ta.tobytes() == tb.tobytes(), name


def test_textured_scenes_load_textures(ptamd):
    """Ids as scene.cpp:102-133 assigns them: materials in (alphabetical) load order, each
    TEXTURE before its BUMP_MAP; -1 (with hasTexture kept) on failure, which takes no id."""
    b = ptamd.SceneFile(scene_path("synthetic_textured_bump"))
    m = dict(zip(b.material_names, b.materials))
    assert len(b.textures) == 3 and all(t.shape == (512, 512, 4) for t in b.textures)
    assert (m["textured_box"]["hasTexture"], m["textured_box"]["textureID"]) == (1, 0)
    assert (m["textured_bump"]["hasTexture"], m["textured_bump"]["textureID"]) == (1, 1)
    assert (m["textured_bump"]["hasBumpMap"], m["textured_bump"]["bumpID"]) == (1, 2)
    assert abs(float(m["textured_bump"]["bumpScale"]) - 0.3) < 1e-7
    assert (m["textured_missing"]["hasTexture"], m["textured_missing"]["textureID"]) == (1, -1)
    t = ptamd.SceneFile(scene_path("cornell_obj_phatphuck_texture_test"))
    tm = dict(zip(t.material_names, t.materials))["wood_textured_phat_phuck"]
    assert (tm["textureID"], tm["hasBumpMap"], tm["bumpID"]) == (0, 1, -1)   # wood_normal.png is absent


@pytest.mark.parametrize("res,depth", [((64, 64), 8), ((400, 400), 4), ((100, 37), 3)])
def test_overrides_recompute_camera(res, depth, oracle, ptamd):
    a = oracle.load_scene(scene_path("cornell"), res=res, depth=depth)
    b = ptamd.SceneFile(scene_path("cornell"), res=res, depth=depth)
    assert a.camera.tobytes() == b.camera.tobytes()
    assert b.width == res[0] and b.height == res[1] and b.trace_depth == depth


def test_loader_matches_reference_glm(ptamd):
    with open(os.path.join(GOLDEN, "ingest_pin.json")) as f:
        pin = json.load(f)
    n = 0
    for name in LOADABLE:
        if name not in pin["scenes"]:          # our own synthetic scenes have no reference pin
            continue
        ref = pin["scenes"][name]
        b = ptamd.SceneFile(scene_path(name))
        with open(scene_path(name)) as f:
            objs = json.load(f)["Objects"]
        prims = [r for o, r in zip(objs, ref["objects"]) if o["TYPE"] != "obj"]
        assert len(prims) == len(b.geoms)
        for g, r in zip(b.geoms, prims):
            assert g["transform"].reshape(-1).view(np.uint32).tolist() == r["transform"]
            assert g["inverseTransform"].reshape(-1).view(np.uint32).tolist() == r["inverse"]
            assert g["invTranspose"].reshape(-1).view(np.uint32).tolist() == r["invTranspose"]
            n += 1
        assert b.material_names == ref["materials"]
        for k in ("view", "up", "right", "position"):
            assert b.camera[k][0].view(np.uint32).tolist() == ref["camera"][k], (name, k)
    assert n >= 100


def test_unknown_material_name_maps_to_zero(ptamd):
    # khaslana's wings name "specular_red_glass " (trailing space): unordered_map::operator[]
    # default-inserts 0
    b = ptamd.SceneFile(scene_path("cornell_obj_khaslana"))
    with open(scene_path("cornell_obj_khaslana")) as f:
        objs = json.load(f)["Objects"]
    wings = [o for o in objs if o.get("PATH") == "/obj/khaslana_wings.obj"]
    assert wings and wings[0]["MATERIAL"] not in b.material_names
    assert b.material_names[0] == "brighter_golden_light"
    mats = set(b.triangles["materialID"].tolist())
    assert 0 in mats


def test_bvh_structure(ptamd):
    b = ptamd.SceneFile(scene_path("cornell_obj_bnnuy"))
    nodes, idx, tris = b.bvh_nodes, b.tri_indices, b.triangles
    assert sorted(idx.tolist()) == list(range(len(tris)))
    seen = np.zeros(len(tris), np.int32)
    for nd in nodes:
        if nd["triCount"] > 0 and nd["start"] >= 0:
            assert nd["triCount"] <= 4
            for k in range(nd["start"], nd["start"] + nd["triCount"]):
                seen[idx[k]] += 1
                t = tris[idx[k]]
                for v in ("v1", "v2", "v3"):
                    p = t[v]["position"]
                    assert (p >= nd["min"]).all() and (p <= nd["max"]).all()
        else:
            assert nd["left"] > 0 and nd["right"] > 0
    assert (seen == 1).all()


def test_missing_file_raises(ptamd):
    with pytest.raises(ptamd.PtError):
        ptamd.SceneFile(os.path.join(SCENES, "does_not_exist.json"))
    with pytest.raises(ptamd.PtError):
        ptamd.SceneFile(os.path.join(SCENES, "cornell.txt"))
