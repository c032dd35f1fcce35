#!/usr/bin/env bash
# BVH-scene GPU parity tests + the two mesh configs (c4 bunny, c5 khaslana) -> gpurun_out/bvh.jsonl
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "bnnuy or khaslana or phatphuck or textured" > gpurun_out/t_bvh.log 2>&1 || { tail -30 gpurun_out/t_bvh.log; exit 1; }
tail -1 gpurun_out/t_bvh.log
: > gpurun_out/bvh.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 --warmup 8 --scene scenes/cornell_obj_bnnuy.json \
    | tail -1 >> gpurun_out/bvh.jsonl || exit 2
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 16 --warmup 4 --scene scenes/cornell_obj_khaslana.json \
    --res 1600x1600 --depth 12 | tail -1 >> gpurun_out/bvh.jsonl || exit 3
python3 - <<'PY'
import json
for l in open("gpurun_out/bvh.jsonl"):
    d = json.loads(l)
    k = d.get("kernels", {})
    print(d["config"]["workload"][:40], d["ms_per_step"], [round(a - b, 3) for a, b in zip(k["per_launch_bounce_ms"], k["per_launch_bvh_ms"])], k["per_launch_bvh_ms"])
PY
