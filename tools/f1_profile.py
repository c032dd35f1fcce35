"""F = 1 frame anatomy (the API path): per-launch kernel durations of single-frame passes vs the
wall time per frame of graph replays."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "project3-cuda-path-tracer-2025_amd"))
import ptamd
sc = ptamd.SceneFile(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scenes", "cornell.json"))
tr = ptamd.PathTracer(sc, frames_per_pass=1)
tr.trace_frames(1, 20); tr.synchronize()
tr.prepare_frames(50); tr.synchronize()
t0 = time.perf_counter(); tr.trace_frames(21, 50); tr.synchronize(); wall = (time.perf_counter() - t0) / 50 * 1e3
p = tr.profile(71, 50)
print(json.dumps({"wall_ms_per_frame": round(wall, 4), "frame_ms_stream": p.get("frame_ms"),
                  "bounce_ms": [round(x, 4) for x in p["bounce_ms"][:8]], "kernel_sum_ms": round(sum(p["bounce_ms"][:8]), 4)}))
tr.free()
