"""One rank's share of an N-GPU pixel-tile bench step, on this one GPU (tools only): the time
rank 0 of N needs for N x K frames over its 1/N of the pixels, next to one GPU's K full frames.
The ranks of a real N-GPU run are independent until the tile gather, so this is each rank's
compute part of the scaling line.  Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))
sys.path.insert(0, REPO)


def run(ptamd, sc, frames, warm, **opts):
    tr = ptamd.PathTracer(sc, **opts)
    tr.trace_frames(1, warm)
    tr.prepare_frames(frames)
    tr.synchronize()
    best = 1e9
    for r in range(3):
        t0 = time.perf_counter()
        tr.trace_frames(1 + warm + r * frames, frames)
        tr.synchronize()
        best = min(best, time.perf_counter() - t0)
    st = tr.stats()
    tr.free()
    return round(1e3 * best, 3), st["frames_per_pass"]


def main():
    import ptamd
    import bench
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    sc = ptamd.SceneFile(os.path.join(REPO, "scenes", "cornell.json"))
    out = {"steps": steps}
    out["n1"] = run(ptamd, sc, steps, 5)
    for n in (2, 4, 8):
        rows = bench.shard_rows(sc.height, n)
        out[f"n{n}_rank0"] = run(ptamd, sc, n * steps, n * 5, shard_mode=ptamd.SHARD_PIXELS, shard_rank=0,
                                  shard_count=n, shard_rows=rows)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
