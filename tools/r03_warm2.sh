#!/usr/bin/env bash
# What makes the first pass after a short warm-up slow?  Interleaved bench processes:
# warm-up length, allocation size (PT_ALLOC_FRAMES_MIN) and graph reuse (W = K: the warm-up pass
# replays the same pass graph the timed region does).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/r03_warm2.jsonl
: > "$OUT"
B="python bench.py --no-cpu-baseline --no-configs --no-api"
CASES=("X=0|--steps 20 --warmup 5" "PT_ALLOC_FRAMES_MIN=128|--steps 20 --warmup 5" "X=0|--steps 20 --warmup 20"
       "X=0|--steps 20 --warmup 40" "X=0|--steps 100 --warmup 10" "PT_ALLOC_FRAMES_MIN=128|--steps 100 --warmup 10"
       "X=0|--steps 100 --warmup 100")
for r in 1 2 3; do
  for c in "${CASES[@]}"; do
    e=${c%%|*}; a=${c#*|}
    line=$(env $e timeout -k 10 240 $B $a | tail -1) || { echo "bench failed: $c"; exit 2; }
    echo "{\"round\": $r, \"env\": \"$e\", \"args\": \"$a\", \"line\": $line}" >> "$OUT"
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], d['kernels']['frame_ms'], d['kernels']['ms_per_frame_spread']['median'])" "$line" "$c"
  done
done
echo warm2 done
