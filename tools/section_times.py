"""Where the fused bounce kernel spends its cycles: runs the section-timing variant
(pt_options.variant bit 4, wave-level s_memtime deltas) and prints per-section shares and work
counters per live lane.

    python tools/section_times.py [--scene cornell] [--frames 16] [--variant 6]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "project3-cuda-path-tracer-2025_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--variant", type=int, default=6)
    ap.add_argument("--res", default="")
    ap.add_argument("--depth", type=int, default=-1)
    ap.add_argument("--out", default="", help="also write the JSON here")
    args = ap.parse_args()
    import ptamd
    res = tuple(int(x) for x in args.res.split("x")) if args.res else None
    sc = ptamd.SceneFile(os.path.join(REPO, "scenes", args.scene + ".json"), res=res,
                         depth=args.depth if args.depth >= 0 else None)
    tr = ptamd.PathTracer(sc, variant=args.variant)
    tr.trace_frames(1, 8)
    tr.synchronize()
    tr.section_counters(reset=True)
    tr.trace_frames(9, args.frames)
    tr.synchronize()
    c = tr.section_counters(reset=True)
    secs = ["load", "cull", "exact", "finish", "shade", "store"]
    tot = sum(c[k] for k in secs)
    lanes = max(1, c["n_lanes"])
    out = {"scene": args.scene, "frames": args.frames,
           "cycle_share": {k: round(c[k] / tot, 4) for k in secs},
           "wave_cycles_per_wave": {k: round(c[k] / max(1, c["n_waves"]), 1) for k in secs},
           "exact_tests_per_live_lane": round(c["n_exact"] / lanes, 3),
           "candidates_per_live_lane": round(c["n_cand"] / lanes, 3),
           "loop_iters_per_wave": round(c["n_iters"] / max(1, c["n_waves"]), 3),
           "live_lanes_per_wave": round(lanes / max(1, c["n_waves"]), 2),
           "bvh_nodes_per_ray": round(c["n_nodes"] / max(1, c["n_bvh_rays"]), 2),
           "bvh_inner_per_ray": round((c["n_nodes"] - c["n_leaves"]) / max(1, c["n_bvh_rays"]), 2),
           "bvh_leaves_per_ray": round(c["n_leaves"] / max(1, c["n_bvh_rays"]), 2),
           "bvh_tris_per_leaf": round(c["n_tris"] / max(1, c["n_leaves"]), 3),
           "bvh_rays_winning_mesh": round(c["n_bvh_hits"] / max(1, c["n_bvh_rays"]), 4),
           "bvh_nodes_per_losing_ray": round(c["n_miss_nodes"] / max(1, c["n_bvh_rays"] - c["n_bvh_hits"]), 2),
           "bvh_nodes_per_winning_ray": round((c["n_nodes"] - c["n_miss_nodes"]) / max(1, c["n_bvh_hits"]), 2),
           "bvh_rays_root_culled": round(c["n_root_culled"] / max(1, c["n_bvh_rays"]), 4),
           "bvh_tris_per_ray": round(c["n_tris"] / max(1, c["n_bvh_rays"]), 2),
           "bvh_wave_iters_per_wave": round(c["n_bvh_witers"] / max(1, c["n_waves"]), 2),
           "bvh_simt_efficiency": round(c["n_nodes"] / max(1, 64 * c["n_bvh_witers"]), 3),
           "aabb_decision_mismatches": c["n_aabb_mismatch"],
           "superset_per_live_lane": round(c["n_sup"] / lanes, 3),
           "superset_wave_max_per_wave": round(c["n_sup_wmax"] / max(1, c["n_waves"]), 3),
           "superset_wave_union_per_wave": round(c["n_sup_wunion"] / max(1, c["n_waves"]), 3), "raw": c}
    # k_bvh_bounce wave steps by active lanes (bins of 4): the steps a wave takes below a given
    # occupancy, and the lane-steps they do (bin centres)
    for key, name in (("bvh_lanes_hist", "bvh_steps_by_active_lanes"), ("tail_lanes_hist", "tail_steps_by_active_lanes")):
        h = c[key]
        wt = max(1, sum(h))
        lane_steps = sum(h[i] * (4 * i + 2.5) for i in range(16))
        out[name] = {
            "bins_of_4": h,
            "wave_steps": sum(h),
            "simt_efficiency_est": round(lane_steps / (64 * wt), 3),
            "share_of_wave_steps_below": {str(4 * k): round(sum(h[:k]) / wt, 4) for k in (2, 4, 8)},
            "share_of_lane_steps_below": {str(4 * k): round(sum(h[i] * (4 * i + 2.5) for i in range(k)) /
                                                            max(1, lane_steps), 4) for k in (2, 4, 8)}}
    # handed-over rays: how many, and the nodes they still visit, by stack depth and by whether a
    # hit was found before the hand-over
    bs, bh = c["tail_by_sp"], c["tail_by_hit"]
    out["tail_rays_by_stack_depth"] = {lab: {"rays": bs[2 * k], "nodes_per_ray": round(bs[2 * k + 1] / max(1, bs[2 * k]), 2)}
                                       for k, lab in enumerate(["0", "1", "2", "3", "4-5", "6-7", "8-11", "12+"])}
    out["tail_rays_by_hit_before"] = {"no": {"rays": bh[0], "nodes_per_ray": round(bh[1] / max(1, bh[0]), 2)},
                                      "yes": {"rays": bh[2], "nodes_per_ray": round(bh[3] / max(1, bh[2]), 2)}}
    out["skip_camera"] = os.environ.get("PT_SECTIONS_SKIP_CAMERA") is not None
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    tr.free()


if __name__ == "__main__":
    main()
