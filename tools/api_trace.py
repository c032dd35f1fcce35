"""The API-faithful frame (pathtrace(pbo, 0, iter) as main.cpp:463 calls it: one frame per call)
under a kernel trace, and the anatomy of its wall time.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/api -o run -- python tools/api_trace.py run [eager]
    python tools/api_trace.py analyse gpurun_out/api/run_kernel_trace.csv [--out profiles/r04_api_f1.json]

`run` traces 40 warm-up + 60 timed single-frame calls of cornell 800^2 d8 (no host copy, no PBO:
the bench's `api.ms_per_frame_no_copy`) and prints the median wall time per call.  `analyse` splits
each timed call into kernel time (sum of its kernels' durations), idle gaps between its kernels
(graph node to graph node) and the gap before its first kernel (host: Python + memset + graph
launch).
"""
import csv
import json
import os
import statistics as st
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(use_graph=1, copy=False):
    sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))
    import ptamd
    sc = ptamd.SceneFile(os.path.join(REPO, "scenes", "cornell.json"))
    tr = ptamd.PathTracer(sc, use_graph=use_graph)
    ts = []
    for k in range(100):
        t0 = time.perf_counter()
        tr.trace(k + 1, copy_image=copy)
        if not copy:
            tr.synchronize()
        if k >= 40:
            ts.append(1e3 * (time.perf_counter() - t0))
    print(json.dumps({"wall_ms_per_call_median": round(st.median(ts), 4), "calls": len(ts), "use_graph": use_graph,
                      "host_copy": copy}))
    tr.free()


def overlap(kernel_csv, copy_csv, out=None):
    """`run copy` (main.cpp's call: image copied to the host every call) with --memory-copy-trace:
    per device-to-host image copy, its duration and the share of it during which a kernel of the
    next (speculated) frame was running -- the overlap pt_trace's speculation buys."""
    kern = []
    with open(kernel_csv) as f:
        for r in csv.DictReader(f):
            kern.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    kern.sort()
    copies = []
    with open(copy_csv) as f:
        for r in csv.DictReader(f):
            if "DEVICE_TO_HOST" in r.get("Direction", "") or "D2H" in r.get("Direction", ""):
                copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    copies.sort()
    copies = copies[-60:]
    durs, shares = [], []
    for s, e in copies:
        busy = 0
        for ks, ke in kern:
            if ke <= s or ks >= e:
                continue
            busy += min(e, ke) - max(s, ks)
        durs.append((e - s) / 1e3)
        shares.append(min(1.0, busy / max(1, e - s)))
    res = {"copies": len(copies), "copy_us_median": round(st.median(durs), 2) if durs else None,
           "kernel_busy_share_during_copy_median": round(st.median(shares), 3) if shares else None}
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


def analyse(path, out=None):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    frames, cur = [], None
    for s, e, n in rows:
        if "k_frame_begin" in n or (cur is None):
            cur = []
            frames.append(cur)
        cur.append((s, e, n))
    frames = [f for f in frames if any("k_bounce" in n for _, _, n in f)][-60:]
    kern, gaps, lead, per_kernel = [], [], [], {}
    for i, f in enumerate(frames):
        kern.append(sum(e - s for s, e, _ in f) / 1e3)
        gaps.append(sum(max(0, f[j + 1][0] - f[j][1]) for j in range(len(f) - 1)) / 1e3)
        if i > 0:
            lead.append((f[0][0] - frames[i - 1][-1][1]) / 1e3)
        for s, e, n in f:
            k = n.split("(")[0].replace("void ", "")
            per_kernel.setdefault(k, []).append((e - s) / 1e3)
    res = {"frames": len(frames), "kernels_per_frame": round(st.mean(len(f) for f in frames), 2),
           "kernel_us_per_frame": round(st.median(kern), 2), "gaps_between_kernels_us": round(st.median(gaps), 2),
           "span_us_per_frame": round(st.median((f[-1][1] - f[0][0]) / 1e3 for f in frames), 2),
           "gap_before_frame_us": round(st.median(lead), 2) if lead else None,
           "per_kernel_us": {k: round(st.median(v), 2) for k, v in per_kernel.items()}}
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(0 if "eager" in sys.argv[2:] else 1, "copy" in sys.argv[2:])
    elif sys.argv[1] == "overlap":
        overlap(sys.argv[2], sys.argv[3], sys.argv[5] if len(sys.argv) > 5 and sys.argv[4] == "--out" else None)
    else:
        analyse(sys.argv[2], sys.argv[4] if len(sys.argv) > 4 and sys.argv[3] == "--out" else None)
