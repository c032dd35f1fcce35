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

The only exchange is that framebuffer combine, once per reported frame, never per sample:
PIXELS gathers the ranks' disjoint tiles into rank 0 (each rank sends 1/world of the image:
3.8 MB of 30.7 MB at 1600x1600, 8 ranks); SAMPLES reduces the whole framebuffer.
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


def device_image(tr, device):
    """Zero-copy torch view (float32, width*height*3) of the library's HBM framebuffer."""
    import torch
    ptr, n = tr.image_device_ptr()

    class _Cai:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 2}
    return torch.as_tensor(_Cai(), device=f"cuda:{device}")


class TileGather:
    """PIXELS combine: every rank owns the interleaved row bands (y // rows) % world == rank; one
    gather of the packed tiles (1/world of the image each) into rank 0, which writes them into its
    own framebuffer in place.  The rows a rank does not own are zero on that rank, so rank 0's image
    is then bit-identical to one GPU's.  With RCCL the tiles never leave HBM (zero-copy views of the
    library buffer); with gloo (CPU tests) they go through host memory."""

    def __init__(self, tr, rows: int, world: int, rank: int, backend: str = "nccl", device: int = 0):
        import torch
        self.tr, self.world, self.rank, self.backend = tr, world, rank, backend
        H, W = tr.height, tr.width
        self.shape = (H, W, 3)
        owned = [owned_rows(H, rows, world, r) for r in range(world)]
        self.nmax = max(len(o) for o in owned)
        dev = f"cuda:{device}" if backend == "nccl" else "cpu"
        self.idx = [torch.as_tensor(o, dtype=torch.int64, device=dev) for o in owned]
        self.tile = torch.zeros((self.nmax, W, 3), dtype=torch.float32, device=dev)
        self.bufs = [torch.empty_like(self.tile) for _ in range(world)] if rank == 0 else None
        self.device = device

    def _image(self):
        import torch
        if self.backend == "nccl":
            return device_image(self.tr, self.device).view(self.shape)
        return torch.from_numpy(self.tr.image()).view(self.shape)

    def pack(self):
        """This rank's rows of the framebuffer into the packed tile (on the device with RCCL)."""
        self._img = self._image()
        own = self.idx[self.rank]
        self.tile[:len(own)] = self._img.index_select(0, own)
        return self.tile

    def unpack(self, tiles):
        """Rank 0: write every other rank's packed tile into the framebuffer's rows, in place."""
        for r in range(1, self.world):
            self._img.index_copy_(0, self.idx[r], tiles[r][:len(self.idx[r])])
        if self.backend != "nccl":
            self.tr.set_image(self._img.numpy().reshape(-1, 3))

    def run(self):
        import torch
        import torch.distributed as dist
        self.pack()
        dist.gather(self.tile, self.bufs, dst=0)
        if self.rank == 0:
            self.unpack(self.bufs)
        if self.backend == "nccl":
            # the library's own stream reads the framebuffer next: finish torch's writes first
            torch.cuda.current_stream().synchronize()


class ImageReduce:
    """SAMPLES combine: one reduce(SUM) of the full framebuffers into rank 0 (in place)."""

    def __init__(self, tr, rank: int, backend: str = "nccl", device: int = 0):
        self.tr, self.rank, self.backend, self.device = tr, rank, backend, device

    def run(self):
        import torch
        if self.backend == "nccl":
            combine(device_image(self.tr, self.device))
            torch.cuda.current_stream().synchronize()
        else:
            img = torch.from_numpy(self.tr.image().reshape(-1))
            combine(img)
            if self.rank == 0:
                self.tr.set_image(img.numpy().reshape(-1, 3))


def render(scene_path: str, spp: int, mode: str = "pixels", res=None, depth=None, rows: int = 8, device=None,
           backend: str | None = None, **options):
    """Distributed pathtrace of `spp` samples per pixel.  Call on every rank after
    torch.distributed.init_process_group; returns the combined (accumulated) image on rank 0
    as a numpy array (None elsewhere).  The combine runs on the library's HBM buffer (RCCL) or,
    for the gloo backend, through host memory."""
    import torch
    import torch.distributed as dist
    import ptamd

    world, rank = dist.get_world_size(), dist.get_rank()
    backend = backend or dist.get_backend()
    dev = torch.cuda.current_device() if device is None else device
    sc = ptamd.SceneFile(scene_path, res=res, depth=depth)
    if mode == "pixels":
        tr = ptamd.PathTracer(sc, device=dev, shard_mode=ptamd.SHARD_PIXELS, shard_rank=rank, shard_count=world,
                              shard_rows=rows, **options)
        tr.trace_frames(1, spp)
        comb = TileGather(tr, rows, world, rank, backend, dev)
    elif mode == "samples":
        tr = ptamd.PathTracer(sc, device=dev, **options)
        its = [it for it in sample_iterations(-(-spp // world), world, rank) if it <= spp]
        if its:
            tr.trace_frames(its[0], len(its))
        comb = ImageReduce(tr, rank, backend, dev)
    else:
        raise ValueError(mode)
    tr.synchronize()
    comb.run()
    if backend == "nccl":
        torch.cuda.synchronize()
    out = tr.image() if rank == 0 else None
    tr.free()
    return out
