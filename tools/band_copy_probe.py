"""What one shard's host copy costs on its own PCIe link (tools only; one GPU).

pathtrace() copies the 800x800 float3 image (7.68 MB) to pageable host memory every call.  With
N devices each shard copies only its own interleaved row bands (pt_runtime.hip band_prepare: one
hipMemcpy2DAsync of bands of 8 rows, N bands apart).  On an N-GPU node each shard has a link of
its own, so a call's copy costs what ONE shard's band copy costs alone; this box has one GPU and
one link, so that is what is timed here: the whole image as one copy, then shard 0's bands for
N = 2, 4, 8 (each alone, one thread), then all N shards' band copies at once from N threads
(what the one-GPU box does with PT_BAND_COPY=1: every shard on the same link).  Medians of 20.

    python tools/band_copy_probe.py
"""
import ctypes
import json
import statistics
import threading
import time

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
D2H = 2
W, H, ROWS, ROW_BYTES = 800, 800, 8, 800 * 12


def chk(e, what):
    if e != 0:
        raise RuntimeError(f"{what}: hip error {e}")


def main():
    nbytes = W * H * 12
    dev = ctypes.c_void_p()
    chk(hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(nbytes)), "hipMalloc")
    chk(hip.hipMemset(dev, 0, ctypes.c_size_t(nbytes)), "hipMemset")
    host = np.empty(nbytes, np.uint8)
    hptr = host.ctypes.data

    def full():
        chk(hip.hipMemcpy(ctypes.c_void_p(hptr), dev, ctypes.c_size_t(nbytes), D2H), "hipMemcpy")

    def bands(n, k):
        band = ROWS * ROW_BYTES
        nb = (H + ROWS - 1) // ROWS
        mine = (nb - 1 - k) // n + 1
        off = k * band
        chk(hip.hipMemcpy2D(ctypes.c_void_p(hptr + off), ctypes.c_size_t(n * band), ctypes.c_void_p(dev.value + off),
                            ctypes.c_size_t(n * band), ctypes.c_size_t(band), ctypes.c_size_t(mine), D2H), "hipMemcpy2D")

    def timed(fn, reps=20, warm=3):
        ts = []
        for r in range(warm + reps):
            t0 = time.perf_counter()
            fn()
            if r >= warm:
                ts.append(1e6 * (time.perf_counter() - t0))
        return round(statistics.median(ts), 1)

    out = {"image_bytes": nbytes, "unit": "us per copy (median of 20)", "full_image_one_copy": timed(full)}
    out["one_shard_alone"] = {f"N={n}": timed(lambda n=n: bands(n, 0)) for n in (1, 2, 4, 8)}

    def all_shards(n):
        th = [threading.Thread(target=bands, args=(n, k)) for k in range(n)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    out["all_shards_one_link_threads"] = {f"N={n}": timed(lambda n=n: all_shards(n)) for n in (2, 4, 8)}
    hip.hipFree(dev)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
