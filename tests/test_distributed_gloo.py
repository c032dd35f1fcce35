"""Multi-process (world_size 2, gloo, CPU) coverage of the multi-GPU frame logic in
ptamd/dist.py: the PIXELS shard mapping, the SAMPLES iteration schedule and the framebuffer
combine.  Each rank's per-pixel results come from the CPU oracle (pixels are independent, so
which rank traces a pixel cannot change its value); the combine is the same
torch.distributed.reduce the GPU path issues over RCCL."""
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


def _worker(rank, world, port, mode, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, PKG)
    sys.path.insert(0, ORACLE)
    import torch
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
        mask[D.owned_rows(h, 8, world, rank)] = True
        img[~np.repeat(mask, w)] = 0.0
    else:
        for it in D.sample_iterations(-(-SPP // world), world, rank):
            if it <= SPP:
                r.trace(it)
        img = r.image.copy()
    t = torch.from_numpy(img.reshape(-1).copy())
    D.combine(t)
    if rank == 0:
        np.save(os.path.join(out_dir, f"{mode}.npy"), t.numpy().reshape(-1, 3))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["pixels", "samples"])
def test_two_rank_frame_combine(mode, tmp_path, oracle):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), mode, str(tmp_path)), nprocs=2, join=True)
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
