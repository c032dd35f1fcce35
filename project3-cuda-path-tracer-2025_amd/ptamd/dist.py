"""Multi-GPU frames: one process per GPU (torch.distributed, RCCL over xGMI on MI355X, gloo on
CPU for tests).  The reference is single-GPU (main.cpp:174); pixels are independent (the RNG
is keyed by pixel index, pathtrace.cu:54), so a frame shards without any data-path exchange:

* SAMPLES (weak scaling): rank r traces a contiguous block of iterations of the whole frame
  (contiguous so pt_trace_frames groups them into multi-frame passes); the accumulated images
  are summed once per reported frame.  Sum order differs from one GPU, so the
  combined image equals the single-GPU one to float rounding of the final sum (not bit-wise).
* PIXELS (strong scaling): rank r traces every iteration for its interleaved row bands
  ((y // rows) % W == r), zeros elsewhere; the sum is exact (x + 0 == x), bit-identical to
  one GPU.

The only collective is that framebuffer combine: one reduce of width*height*3 floats to rank 0
(30.7 MB at 1600x1600) per reported frame, never per sample.
"""
from __future__ import annotations

import numpy as np


def owned_rows(height: int, rows: int, world: int, rank: int) -> np.ndarray:
    """Rows of the image a PIXELS-mode rank traces (mirror of shard_pixel in pt_kernels.h)."""
    y = np.arange(height)
    return y[(y // rows) % world == rank]


def local_to_pixel(local: np.ndarray, width: int, rows: int, world: int, rank: int) -> np.ndarray:
    """Local path id -> global pixel index, exactly as the kernels map it."""
    lr, x = np.divmod(local, width)
    band, within = np.divmod(lr, rows)
    y = (band * world + rank) * rows + within
    return x + y * width


def sample_iterations(steps: int, world: int, rank: int, first: int = 1) -> list:
    """Iterations traced by `rank` for `steps` local frames in SAMPLES mode (a contiguous block)."""
    return [first + rank * steps + k for k in range(steps)]


def combine(image, dst: int = 0, group=None):
    """Sum the ranks' accumulated framebuffers into `dst` (in place; torch tensor)."""
    import torch.distributed as dist
    dist.reduce(image, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return image


def render(scene_path: str, spp: int, mode: str = "pixels", res=None, depth=None, rows: int = 8, device=None,
           **options):
    """Distributed pathtrace of `spp` samples per pixel.  Call on every rank after
    torch.distributed.init_process_group; returns the combined (accumulated) image on rank 0
    as a numpy array (None elsewhere)."""
    import torch
    import torch.distributed as dist
    import ptamd

    world, rank = dist.get_world_size(), dist.get_rank()
    dev = torch.cuda.current_device() if device is None else device
    sc = ptamd.SceneFile(scene_path, res=res, depth=depth)
    if mode == "pixels":
        tr = ptamd.PathTracer(sc, device=dev, shard_mode=ptamd.SHARD_PIXELS, shard_rank=rank, shard_count=world,
                              shard_rows=rows, **options)
        tr.trace_frames(1, spp)
    elif mode == "samples":
        tr = ptamd.PathTracer(sc, device=dev, **options)
        its = [it for it in sample_iterations(-(-spp // world), world, rank) if it <= spp]
        if its:
            tr.trace_frames(its[0], len(its))
    else:
        raise ValueError(mode)
    tr.synchronize()
    img = torch.from_numpy(tr.image().reshape(-1)).to(f"cuda:{dev}")
    tr.free()
    combine(img)
    return img.cpu().numpy().reshape(-1, 3) if rank == 0 else None
