"""The drop-in C-ABI surface, checked without a GPU: the library loads, exports every function
include/pt/pathtrace_abi.h declares, and fails loudly (error codes, no crash, no CPU fallback)
when no device is present or calls come out of order."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO, scene_path


def _declared(header):
    with open(os.path.join(REPO, "include", "pt", header)) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|void|const char\*)\s+(pt_\w+)\s*\(", text, re.M)))


def test_exports_every_declared_symbol(ptamd):
    names = _declared("pathtrace_abi.h")
    assert len(names) >= 25
    for n in names:
        assert hasattr(ptamd.lib, n), n
    assert sorted(ptamd.ABI_SYMBOLS) == names


def test_version_and_defaults(ptamd):
    assert ptamd.lib.pt_abi_version() == 3
    o = ptamd.default_options()
    # the reference's compile-time defaults, pathtrace.cu:20-24
    assert (o.stream_compaction, o.material_sort, o.bvh) == (1, 0, 1)
    assert o.block_size == 256 and o.use_graph == 1 and o.pipeline == 0 and o.variant == 186


def test_call_order_errors(ptamd):
    ptamd.lib.pt_free()
    assert ptamd.lib.pt_trace(None, 0, 1, None) == -2            # PT_E_STATE
    assert ptamd.lib.pt_get_image(None, 0) == -2
    assert b"pt_init" in ptamd.lib.pt_last_error()
    assert ptamd.lib.pt_free() == 0                              # idempotent


def test_no_device_fails_loudly(ptamd):
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("a GPU is visible: covered by the gpu suite")
    except ImportError:
        pass
    sc = ptamd.SceneFile(scene_path("cornell"), res=(16, 16))
    with pytest.raises(ptamd.PtError):
        ptamd.PathTracer(sc)
    p = ctypes.c_void_p(1)
    assert ptamd.lib.pt_device_alloc(1024, ctypes.byref(p)) == -4 and not p.value   # PT_E_NODEVICE
    assert ptamd.lib.pt_device_alloc(0, ctypes.byref(p)) == -1                        # PT_E_INVALID
    assert ptamd.lib.pt_device_free(None) == 0


def test_scene_view_round_trip(ptamd):
    sc = ptamd.SceneFile(scene_path("cornell_obj_bnnuy"), res=(32, 32), depth=5)
    v = sc.view()
    assert v.num_geoms == len(sc.geoms) == 6 and v.trace_depth == 5
    assert v.num_triangles == 5040 and v.num_tri_indices == 5040 and v.num_bvh_nodes == len(sc.bvh_nodes)
    v2 = ptamd.scene_view_from_arrays(sc.geoms, sc.materials, sc.camera, 5, sc.triangles, sc.tri_indices, sc.bvh_nodes)
    assert bytes(v2.camera) == bytes(v.camera) and v2.num_bvh_nodes == v.num_bvh_nodes
