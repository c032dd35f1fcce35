"""Summarise tools/valu_attrib.sh: VALU instructions of k_bounce (bounces >= 1 and the camera
bounce) per path segment, by section = (duplicated build - product build).

    python tools/valu_attrib.py [--dir gpurun_out/valu] [--out profiles/r03_valu_sections.json]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

SECTIONS = {"dup1": "candidate pre-test (cull_candidates)", "dup2": "exchanged exact tests (geom_test)",
            "dup3": "shading (shade_path: BSDF sample, RNG, throughput)", "dup4": "winner's hit record (finish_hit)"}


def load(d):
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(int)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                if "k_bounce" not in k:
                    continue
                fam = "camera" if "k_bounce<true" in k else "later"
                acc[fam][row["Counter_Name"]] += float(row["Counter_Value"])
                if row["Counter_Name"] == "SQ_WAVES":
                    n[fam] += 1
    return acc, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="gpurun_out/valu")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    base, nb = load(os.path.join(args.dir, "new"))
    # segments: bench's 45 profiled frames (warm-up 5 + timed 20 + eager replay 20) of cornell 800^2
    # d8: 640,000 camera segments and 1,826,297 later segments per frame (bench config line)
    frames = 45
    seg = {"camera": 640000 * frames, "later": 1826297.2 * frames}
    out = {"scene": "cornell.json 800x800 depth 8 (bench --steps 20 --warmup 5, 45 frames traced)",
           "unit": "VALU lane-instructions per path segment (wave64 instructions x 64 / segments)",
           "total": {f: round(base[f]["SQ_INSTS_VALU"] * 64 / seg[f], 1) for f in base},
           "salu_per_segment": {f: round(base[f]["SQ_INSTS_SALU"] * 64 / seg[f], 1) for f in base},
           "lds_per_segment": {f: round(base[f]["SQ_INSTS_LDS"] * 64 / seg[f], 1) for f in base},
           "sections": {}}
    for tag, name in SECTIONS.items():
        d = os.path.join(args.dir, tag)
        if not os.path.isdir(d):
            continue
        acc, _ = load(d)
        out["sections"][name] = {f: round((acc[f]["SQ_INSTS_VALU"] - base[f]["SQ_INSTS_VALU"]) * 64 / seg[f], 1)
                                 for f in base}
    later = out["total"].get("later", 0)
    out["later_rest"] = round(later - sum(v.get("later", 0) for v in out["sections"].values()), 1)
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
