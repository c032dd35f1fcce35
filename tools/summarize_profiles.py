"""Summarise rocprofv3 output (gpurun_out/) into the committed profiles/ directory.

    python tools/summarize_profiles.py --round r01 [--stats-dir gpurun_out/prof --tag fused]...
        [--pmc-dir gpurun_out/pmc --pmc-tag fused_]

* kernel stats: copies run_kernel_stats.csv to profiles/<round>_kernel_stats_<tag>.csv and writes
  a JSON digest (per kernel: calls, average / total ns).
* PMC passes (tools/pmc.sh): per kernel family, the mean of every counter per dispatch, and the
  HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md "HBM [CDNA4]": on
  gfx950 FETCH_SIZE reports half the bytes of wide streaming reads; WRITE_SIZE is exact for
  16-B-per-lane stores; both in KB) -> profiles/<round>_traffic.json, which bench.py reads for
  roofline.traffic.
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def family(name: str) -> str:
    """Kernel family used by bench.py's roofline keys: template arguments and signature dropped."""
    n = re.sub(r"^void ", "", name)
    n = n.split("(")[0]
    return n.split("<")[0]


def kernel_stats(path):
    out = []
    with open(path) as f:
        for row in csv.DictReader(f):
            out.append({"name": row["Name"], "calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                        "total_ns": float(row["TotalDurationNs"]), "pct": float(row["Percentage"])})
    return out


def pmc(pmc_dir, prefix, frames=0):
    """mean counter value per dispatch, per kernel family, over every pass <prefix>p*/.  With
    `frames` (frames each profiled run traced: warmup + timed + bench's profiling replay), also the
    HBM bytes per FRAME: the sum over the run's dispatches / frames, independent of how the run's
    frames were grouped into passes (bench.py scales it to its own launches)."""
    acc = defaultdict(lambda: defaultdict(list))
    for d in sorted(glob.glob(os.path.join(pmc_dir, prefix + "p*"))):
        if not os.path.isdir(d):
            continue
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    fam = family(row["Kernel_Name"])
                    acc[fam][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for fam, cs in acc.items():
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        e["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes_per_launch"] = int((2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024)
            if frames:
                tot = (2 * sum(cs["FETCH_SIZE"]) + sum(cs["WRITE_SIZE"])) * 1024
                e["hbm_bytes_per_frame"] = int(tot / frames)
                e["frames_per_run"] = frames
        res[fam] = e
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r01")
    ap.add_argument("--stats", nargs=2, action="append", metavar=("DIR", "TAG"), default=[])
    ap.add_argument("--pmc", nargs=2, action="append", metavar=("DIR", "PREFIX"), default=[])
    ap.add_argument("--pmc-frames", type=int, default=72,
                    help="frames per profiled run (tools/pmc.sh: warmup 8 + steps 32 + bench's replay 32)")
    ap.add_argument("--traffic-name", default=None,
                    help="output file name under profiles/ (default <round>_traffic.json)")
    args = ap.parse_args()
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    digest = {}
    for d, tag in args.stats:
        src = os.path.join(d, "run_kernel_stats.csv")
        shutil.copy(src, os.path.join(prof, f"{args.round}_kernel_stats_{tag}.csv"))
        digest[tag] = kernel_stats(src)
    if digest:
        with open(os.path.join(prof, f"{args.round}_kernel_stats.json"), "w") as f:
            json.dump(digest, f, indent=1)
    traffic = {}
    for d, prefix in args.pmc:
        for fam, e in pmc(d, prefix, args.pmc_frames).items():
            traffic.setdefault(fam, {}).update(e)
            traffic[fam]["source"] = f"{prefix or 'default'} passes"
    if traffic:
        with open(os.path.join(prof, args.traffic_name or f"{args.round}_traffic.json"), "w") as f:
            json.dump(traffic, f, indent=1, sort_keys=True)
    print(json.dumps({k: [(x["name"][:60], x["calls"], round(x["avg_ns"])) for x in v[:8]] for k, v in digest.items()},
                     indent=1))
    for fam, e in traffic.items():
        print(fam, {k: (round(v, 1) if isinstance(v, float) else v) for k, v in e.items()})


if __name__ == "__main__":
    main()
