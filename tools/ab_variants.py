"""In-process A/B of fused-kernel variants (cdna guide rule 24: interleaved rounds, one
process).  Every variant renders the same iterations; images must be bit-identical.

    python tools/ab_variants.py [--variants 0,1,2,3] [--rounds 5] [--frames 40] [--scene cornell]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--res", default="")
    ap.add_argument("--pipeline", type=int, default=0)
    ap.add_argument("--fpp", default="0", help="frames_per_pass values to A/B (0 = auto)")
    args = ap.parse_args()
    import ptamd
    res = tuple(int(x) for x in args.res.split("x")) if args.res else None
    sc = ptamd.SceneFile(os.path.join(REPO, "scenes", args.scene + ".json"), res=res)
    variants = [(int(v), int(f)) for v in args.variants.split(",") for f in args.fpp.split(",")]
    times = {v: [] for v in variants}
    kern = {v: [] for v in variants}
    ref = None
    for r in range(args.rounds):
        for v in variants:
            tr = ptamd.PathTracer(sc, variant=v[0], frames_per_pass=v[1], pipeline=args.pipeline)
            tr.trace_frames(1, 3)
            tr.synchronize()
            t0 = time.perf_counter()
            tr.trace_frames(4, args.frames)
            tr.synchronize()
            times[v].append((time.perf_counter() - t0) / args.frames * 1e3)
            p = tr.profile(4 + args.frames, 16)
            kern[v].append(p["bounce_ms"] + [p["frame_ms"], p["combine_ms"]])
            img = tr.image()
            if ref is None:
                ref = img
            assert img.tobytes() == ref.tobytes(), f"variant {v} image differs"
            tr.free()
    out = {}
    for v in variants:
        out[f"var{v[0]}_fpp{v[1]}"] = {"ms_per_frame_median": float(np.median(times[v])), "ms_per_frame_min": float(np.min(times[v])),
                  "per_launch_bounce_ms_then_frame_ms_combine_ms": [round(float(x), 4) for x in np.median(np.array(kern[v]), axis=0)]}
    print(json.dumps({"scene": args.scene, "frames": args.frames, "rounds": args.rounds, "results": out}, indent=1))


if __name__ == "__main__":
    main()
