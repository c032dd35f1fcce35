#!/usr/bin/env bash
# A/B settings of one build in interleaved processes (same box, same scene): each arm is one or
# more environment assignments joined by commas (or "-" for none) applied to a bench run
#   AB_ENVS="PT_BVH_TAIL_LANES=0 PT_BVH_TAIL_LANES=8" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" bash tools/ab_env.sh
# prints ms_per_step per (round, arm) and the per-arm medians
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ROUNDS=${AB_ROUNDS:-3}
OUT=gpurun_out/ab_env_${AB_TAG:-x}.jsonl
: > "$OUT"
for r in $(seq "$ROUNDS"); do
  for arm in $AB_ENVS; do
    if [ "$arm" = "-" ]; then set --; else set -- $(echo "$arm" | tr ',' ' '); fi
    line=$(env "$@" timeout -k 10 240 python bench.py --no-cpu-baseline --no-configs --no-api --no-spread \
           ${AB_ARGS:-} | tail -1) || { echo "bench failed for $arm"; exit 2; }
    echo "{\"round\": $r, \"arm\": \"$arm\", \"line\": $line}" >> "$OUT"
  done
done
python3 - "$OUT" <<'PY'
import json, sys, statistics as st
rows = [json.loads(l) for l in open(sys.argv[1])]
arms = {}
for r in rows:
    arms.setdefault(r["arm"], []).append(r["line"]["ms_per_step"])
for k, v in arms.items():
    print(k, "median ms/frame", round(st.median(v), 5), v)
PY
