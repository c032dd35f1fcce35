import json, os, sys
sys.path.insert(0, "project3-cuda-path-tracer-2025_amd")
import ptamd
sc = ptamd.SceneFile("scenes/cornell.json")
tr = ptamd.PathTracer(sc, variant=30, frames_per_pass=8)
tr.trace_frames(1, 8); tr.synchronize(); tr.section_counters(reset=True)
tr.trace_frames(9, 8); tr.synchronize()
c = tr.section_counters(reset=True)
w = max(1, c["n_bvh_rays"])
print(json.dumps({"redist_waves": w, "pairs_per_wave": c["n_exact"] / w, "rounds_per_wave": c["n_iters"] / w,
                  "sphere_pairs_frac": c["n_cand"] / max(1, c["n_exact"])}))
