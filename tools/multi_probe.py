"""Cost of the C-ABI multi-device split (pt_options.num_devices) on ONE GPU (tools only): the same
cornell 800^2 d8 work traced by one context and by N shard contexts that all live on device 0
(each its own stream; the combine pulls their pixels into the first context's image).  On one GPU
the shards share the CUs, so the difference is the split's own overhead: per-shard launches, the
combine kernels and the event hand-offs.  Multi-frame passes (K frames per call) and the API call
(one frame per pathtrace(), host copy off).  Prints one JSON line.

    python tools/multi_probe.py [K]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))


def passes(ptamd, sc, k, **opts):
    tr = ptamd.PathTracer(sc, **opts)
    tr.trace_frames(1, 4)
    tr.prepare_frames(k)
    tr.synchronize()
    best = 1e9
    for r in range(3):
        t0 = time.perf_counter()
        tr.trace_frames(5 + r * k, k)
        tr.synchronize()
        best = min(best, time.perf_counter() - t0)
    tr.free()
    return round(1e3 * best / k, 4)


def api(ptamd, sc, frames=40, copy=False, speculate=True, **opts):
    """ms per pathtrace() call; copy: the image copied to host memory every call (main.cpp's call,
    which is what starts the next-frame speculation; speculate=False turns it off)"""
    tr = ptamd.PathTracer(sc, **opts)
    tr.set_speculation(speculate)
    for it in range(1, 6):
        tr.trace(it, copy_image=copy)
    tr.synchronize()
    t0 = time.perf_counter()
    for it in range(6, 6 + frames):
        tr.trace(it, copy_image=copy)
    tr.synchronize()
    dt = (time.perf_counter() - t0) / frames
    tr.free()
    return round(1e3 * dt, 4)


def enqueue(ptamd, sc, f, calls=20, **opts):
    """host microseconds per shard for pt_trace_frames(., f) to RETURN (the passes' launches or
    graph replays and the combine's enqueue, no wait): the serial host walk over the shards"""
    tr = ptamd.PathTracer(sc, **opts)
    n = len(opts.get("devices") or [0])
    tr.trace_frames(1, 2 * f)
    tr.prepare_frames(f)
    tr.synchronize()
    ts = []
    for c in range(calls):
        tr.synchronize()
        t0 = time.perf_counter()
        tr.trace_frames(1 + (2 + c) * f, f)
        ts.append(time.perf_counter() - t0)
    tr.synchronize()
    tr.free()
    ts.sort()
    return round(1e6 * ts[len(ts) // 2] / n, 1)


def main():
    import ptamd
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    sc = ptamd.SceneFile(os.path.join(REPO, "scenes", "cornell.json"))
    out = {"scene": "cornell.json 800x800 depth 8", "frames_per_call": k, "unit": "ms per frame"}
    out["passes"] = {"1 context": passes(ptamd, sc, k)}
    out["api"] = {"1 context": api(ptamd, sc)}
    # with the host copy (main.cpp's call): next-frame speculation on / off
    out["api_copy"] = {"1 context": api(ptamd, sc, copy=True)}
    out["api_copy_no_speculation"] = {"1 context": api(ptamd, sc, copy=True, speculate=False)}
    for n, comb in ((2, "peer"), (4, "peer"), (8, "peer"), (2, "rccl"), (8, "rccl")):
        key = f"{n} shards on device 0, {comb}"
        out["passes"][key] = passes(ptamd, sc, k, devices=[0] * n, combine=comb)
        out["api"][key] = api(ptamd, sc, devices=[0] * n, combine=comb)
        out["api_copy"][key] = api(ptamd, sc, copy=True, devices=[0] * n, combine=comb)
        out["api_copy_no_speculation"][key] = api(ptamd, sc, copy=True, speculate=False, devices=[0] * n, combine=comb)
    out["enqueue_us_per_shard"] = {}
    if os.environ.get("PT_MULTI_F1_DIRECT"):
        out["note"] = "PT_MULTI_F1_DIRECT=1: single-frame passes of shards launched directly (no graph)"
    for n in (1, 2, 8):
        for f in (1, 20):
            kw = {} if n == 1 else {"devices": [0] * n}
            out["enqueue_us_per_shard"][f"{n} shard(s), F={f}"] = enqueue(ptamd, sc, f, **kw)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
