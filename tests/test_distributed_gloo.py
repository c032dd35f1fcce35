"""Multi-process (world_size 2, gloo, CPU) coverage of the multi-GPU frame logic in
ptamd/dist.py: the PIXELS shard mapping, the SAMPLES iteration schedule and the framebuffer
combine.  Each rank's per-pixel results come from the CPU oracle (pixels are independent, so
which rank traces a pixel cannot change its value); the combine is the same TileGather /
ImageReduce code bench.py runs over RCCL, here with gloo on host tensors."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import ORACLE, PKG, scene_path

RES = (24, 20)
SPP = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_pixel_shard_mapping_partitions_the_frame():
    sys.path.insert(0, PKG)
    from ptamd import dist as D
    for (w, h, rows, world) in [(24, 20, 8, 2), (800, 800, 8, 8), (37, 13, 3, 4), (5, 7, 8, 3)]:
        seen = np.zeros(w * h, np.int32)
        for r in range(world):
            nrows = len(D.owned_rows(h, rows, world, r))
            pix = D.local_to_pixel(np.arange(nrows * w), w, rows, world, r)
            if nrows == 0:
                continue
            assert pix.min() >= 0 and pix.max() < w * h
            assert set((pix // w).tolist()) == set(D.owned_rows(h, rows, world, r).tolist())
            seen[pix] += 1
        assert (seen == 1).all()


def test_sample_schedule_covers_each_iteration_once():
    sys.path.insert(0, PKG)
    from ptamd import dist as D
    for world in (1, 2, 3, 8):
        its = sorted(i for r in range(world) for i in D.sample_iterations(5, world, r))
        assert its == list(range(1, 5 * world + 1))


class _HostTracer:
    """The slice of ptamd.PathTracer the combiners use, over an oracle-rendered host image."""

    def __init__(self, img, w, h):
        self.img, self.width, self.height = img, w, h

    def image(self):
        return self.img.copy()

    def set_image(self, img):
        self.img = np.asarray(img, np.float32).reshape(-1, 3).copy()


def _worker(rank, world, port, mode, rows, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, PKG)
    sys.path.insert(0, ORACLE)
    import torch.distributed as dist
    import oracle as O
    from ptamd import dist as D
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = O.load_scene(scene_path("cornell"), res=RES)
    r = O.Renderer(sc, O.options(num_threads=1))
    w, h = RES
    if mode == "pixels":
        for it in range(1, SPP + 1):
            r.trace(it)
        img = r.image.copy()
        mask = np.zeros(h, bool)
        mask[D.owned_rows(h, rows, world, rank)] = True
        img[~np.repeat(mask, w)] = 0.0
        tr = _HostTracer(img, w, h)
        D.TileGather(tr, rows, world, rank, backend="gloo").run()    # the gather bench.py times
    else:
        for it in D.sample_iterations(-(-SPP // world), world, rank):
            if it <= SPP:
                r.trace(it)
        tr = _HostTracer(r.image.copy(), w, h)
        D.ImageReduce(tr, rank, backend="gloo").run()
    if rank == 0:
        np.save(os.path.join(out_dir, f"{mode}.npy"), tr.image())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,world,rows", [("pixels", 2, 8), ("pixels", 3, 1), ("pixels", 2, 4), ("samples", 2, 8)])
def test_multi_rank_frame_combine(mode, world, rows, tmp_path, oracle):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), mode, rows, str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / f"{mode}.npy")
    sc = oracle.load_scene(scene_path("cornell"), res=RES)
    r = oracle.Renderer(sc, oracle.options(num_threads=1))
    for it in range(1, SPP + 1):
        r.trace(it)
    if mode == "pixels":
        assert got.tobytes() == r.image.tobytes()          # x + 0 == x: bit-identical to one GPU
    else:
        fin = np.isfinite(r.image)
        np.testing.assert_allclose(got[fin], r.image[fin], rtol=2e-6, atol=1e-6)
        assert (np.isnan(got) == np.isnan(r.image)).all()


def test_bench_shard_rows_split_evenly():
    sys.path.insert(0, os.path.dirname(PKG))
    import bench
    for h, world in [(800, 1), (800, 2), (800, 8), (1600, 8), (800, 3), (20, 2)]:
        rows = bench.shard_rows(h, world)
        assert rows in (8, 4, 2, 1)
        if h % world == 0:
            assert h % (rows * world) == 0


def test_bench_refuses_world_size_mismatch():
    """--gpus must match the launcher's WORLD_SIZE (checked before any GPU work)"""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(os.path.dirname(PKG), "bench.py"), "--gpus", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr


def test_bench_refuses_more_rccl_ranks_than_gpus():
    """RCCL ranks are one per GPU: a world larger than the visible devices is refused before any
    GPU work (gloo rehearsals, PT_BENCH_BACKEND=gloo, may share a GPU)"""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", HIP_VISIBLE_DEVICES="")
    env.pop("PT_BENCH_BACKEND", None)
    p = subprocess.run([sys.executable, os.path.join(os.path.dirname(PKG), "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "RCCL ranks" in p.stderr, p.stderr[-400:]


def test_bench_sub_records_have_traffic_digests():
    """Every bench `configs` sub-record names a committed PMC digest (profiles/rNN_traffic_<tag>.json)
    with HBM bytes per frame for the kernels its roofline covers, so no record's `traffic` is null."""
    sys.path.insert(0, os.path.dirname(PKG))
    import bench
    for cfg in bench.SUB_CONFIGS:
        tag = bench.traffic_tag(cfg)
        assert tag, cfg[0]
        d = bench._pmc_digest(tag)
        assert d, (cfg[0], tag)
        k = "k_compact_scatter" if cfg[5] == "staged" else "k_bounce"
        assert d.get(k, {}).get("hbm_bytes_per_frame", 0) > 0, (cfg[0], tag)
