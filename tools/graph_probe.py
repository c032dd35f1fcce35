"""Graph replay vs direct launches for the driver-shaped timed region (tools only): cornell
800^2 d8, 5 warm-up frames, then K frames as one pass timed host-side (launch + synchronise),
interleaved rounds in one process, pt_options.use_graph 1 vs 0.  Prints one JSON line.

    python tools/graph_probe.py [K] [rounds]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))


def main():
    import ptamd
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    sc = ptamd.SceneFile(os.path.join(REPO, "scenes", "cornell.json"))
    res = {1: [], 0: []}
    for r in range(rounds):
        for g in (1, 0):
            tr = ptamd.PathTracer(sc, use_graph=g)
            tr.prepare_frames(k)
            tr.trace_frames(1, 5)
            tr.synchronize()
            t0 = time.perf_counter()
            tr.trace_frames(6, k)
            tr.synchronize()
            res[g].append((time.perf_counter() - t0) / k * 1e3)
            tr.free()
    med = {f"use_graph={g}": round(sorted(v)[len(v) // 2], 5) for g, v in res.items()}
    print(json.dumps({"frames": k, "rounds": rounds, "ms_per_frame_median": med,
                      "all": {f"use_graph={g}": [round(x, 5) for x in v] for g, v in res.items()}}))


if __name__ == "__main__":
    main()
