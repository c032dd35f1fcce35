#!/usr/bin/env bash
# A/B of environment knobs in interleaved bench processes (same box, same library):
#   AB_ENVS="PT_BVH_TREE=ref;PT_BVH_TREE=sah" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" bash tools/ab_env.sh
# prints ms_per_step per (round, setting) and the per-setting medians
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
IFS=';' read -ra ENVS <<< "${AB_ENVS:-X=0;X=1}"
ROUNDS=${AB_ROUNDS:-3}
OUT=gpurun_out/ab_env_${AB_TAG:-x}.jsonl
: > "$OUT"
for r in $(seq "$ROUNDS"); do
  for e in "${ENVS[@]}"; do
    line=$(env $e timeout -k 10 240 python bench.py --no-cpu-baseline --no-configs --no-api --no-spread \
           ${AB_ARGS:-} | tail -1) || { echo "bench failed for $e"; exit 2; }
    echo "{\"round\": $r, \"env\": \"$e\", \"line\": $line}" >> "$OUT"
  done
done
python3 - "$OUT" <<'PY'
import json, sys, statistics as st
rows = [json.loads(l) for l in open(sys.argv[1])]
d = {}
for r in rows:
    d.setdefault(r["env"], []).append(r["line"]["ms_per_step"])
for k, v in d.items():
    print(k, "median ms/frame", round(st.median(v), 5), v)
PY
