"""Child process of test_gpu_parity.py::test_rccl_framebuffer_combine_device_branches (needs a GPU).

Initialises a world-size-1 `nccl` (RCCL) process group on cuda:0 and runs the framebuffer
combines of ptamd/dist.py through their DEVICE branches -- what an N-GPU bench.py run executes:

1. TileGather.run(): index_select of the owned rows from a zero-copy view of the library's HBM
   image, dist.gather over RCCL, (rank 0) index_copy_ back -- on an unsharded frame;
2. the N-rank scatter: N pixel shards traced one after another on this GPU, each shard's packed
   device tile made by TileGather.pack(); rank 0's tile goes through an RCCL gather, and
   TileGather.unpack() writes the other shards' tiles into rank 0's framebuffer with index_copy_;
3. ImageReduce.run(): dist.reduce(SUM) over RCCL of the library's HBM image.

The host-copy entry points of the tracer are disabled while the combines run.  Prints one JSON
line; the test compares its images with the unsharded frame bit for bit.
"""
import json
import os
import socket
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _NoHostCopy:
    """Replaces a tracer's host-memory image methods while a device combine runs."""

    def __init__(self, tr):
        self.tr = tr

    def __enter__(self):
        def boom(*a, **k):
            raise AssertionError("host copy of the framebuffer inside a device combine")
        self.saved = (self.tr.image, self.tr.set_image)
        self.tr.image = self.tr.set_image = boom

    def __exit__(self, *exc):
        self.tr.image, self.tr.set_image = self.saved


def main():
    scene_path, n_shards, frames = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
    import torch
    import torch.distributed as dist
    import ptamd
    from ptamd import dist as D

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    out = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    sc = ptamd.SceneFile(scene_path, res=(64, 48))
    rows = 8

    # the unsharded frame
    tr = ptamd.PathTracer(sc)
    tr.trace_frames(1, frames)
    full = tr.image()
    # 1. TileGather.run() at world size 1 on the library's HBM image: the image must not change
    tg = D.TileGather(tr, rows, 1, 0, "nccl", 0)
    tr.synchronize()
    with _NoHostCopy(tr):
        tg.run()
        assert tg.tile.is_cuda and all(b.is_cuda for b in tg.bufs)
    out["tilegather_run_identity"] = tr.image().tobytes() == full.tobytes()
    # 3. ImageReduce.run() at world size 1: reduce(SUM) of one rank = the image itself
    ir = D.ImageReduce(tr, 0, "nccl", 0)
    with _NoHostCopy(tr):
        ir.run()
    out["imagereduce_run_identity"] = tr.image().tobytes() == full.tobytes()
    tr.free()

    # 2. N pixel shards traced one after another; their device tiles scattered into rank 0's image
    tiles = {}
    for r in range(1, n_shards):
        t = ptamd.PathTracer(sc, shard_mode=ptamd.SHARD_PIXELS, shard_rank=r, shard_count=n_shards, shard_rows=rows)
        t.trace_frames(1, frames)
        t.synchronize()
        g = D.TileGather(t, rows, n_shards, r, "nccl", 0)
        with _NoHostCopy(t):
            tiles[r] = g.pack().clone()
        torch.cuda.synchronize()
        t.free()
    t0 = ptamd.PathTracer(sc, shard_mode=ptamd.SHARD_PIXELS, shard_rank=0, shard_count=n_shards, shard_rows=rows)
    t0.trace_frames(1, frames)
    t0.synchronize()
    g0 = D.TileGather(t0, rows, n_shards, 0, "nccl", 0)
    with _NoHostCopy(t0):
        g0.pack()
        got0 = [torch.empty_like(g0.tile)]
        dist.gather(g0.tile, got0, dst=0)                       # RCCL
        g0.unpack([got0[0]] + [tiles[r] for r in range(1, n_shards)])
        torch.cuda.current_stream().synchronize()
    img = t0.image()
    out["shards_scatter_equal"] = img.tobytes() == full.tobytes()
    out["mismatch"] = int(np.sum(img.view(np.uint32) != full.view(np.uint32)))
    out["image_sum"] = float(np.nansum(full))
    t0.free()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
