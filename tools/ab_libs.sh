#!/usr/bin/env bash
# A/B two builds of libptamd.so in interleaved processes (same box, same scene):
#   AB_LIBS="project3-cuda-path-tracer-2025_amd/build/ab/base.so project3-cuda-path-tracer-2025_amd/build/libptamd.so" AB_ARGS="--scene scenes/cornell.json" bash tools/ab_libs.sh
# prints ms_per_step per (round, lib) and the per-lib medians; images are not compared here
# (the GPU parity tests do that for the product build).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
LIBS=${AB_LIBS:-"project3-cuda-path-tracer-2025_amd/build/ab/base.so project3-cuda-path-tracer-2025_amd/build/libptamd.so"}
ROUNDS=${AB_ROUNDS:-3}
OUT=gpurun_out/ab_libs_${AB_TAG:-x}.jsonl
: > "$OUT"
for r in $(seq "$ROUNDS"); do
  for lib in $LIBS; do
    line=$(PTAMD_LIB=$PWD/$lib timeout -k 10 240 python bench.py --no-cpu-baseline --no-configs --no-api --no-spread \
           ${AB_ARGS:-} | tail -1) || { echo "bench failed for $lib"; exit 2; }
    echo "{\"round\": $r, \"lib\": \"$lib\", \"line\": $line}" >> "$OUT"
  done
done
python3 - "$OUT" <<'PY'
import json, sys, statistics as st
rows = [json.loads(l) for l in open(sys.argv[1])]
libs = {}
for r in rows:
    libs.setdefault(r["lib"], []).append(r["line"]["ms_per_step"])
for k, v in libs.items():
    print(k, "median ms/frame", round(st.median(v), 5), v)
PY
