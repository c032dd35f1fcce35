#!/usr/bin/env bash
# Why is the driver's K = 20 headline faster per frame than the 100-step line, and both slower
# than the per-pass spread measured later in the same process?  Same bench, different warm-up
# lengths and pass shapes, interleaved; plus the GPU clock before / after (rocm-smi, read-only).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/r03_warm.jsonl
: > "$OUT"
B="python bench.py --no-cpu-baseline --no-configs --no-api"
for r in ${WARM_ROUNDS:-1 2}; do
  for args in "--steps 20 --warmup 5" "--steps 100 --warmup 10" "--steps 20 --warmup 500" "--steps 100 --warmup 500" "--steps 20 --warmup 2000"; do
    line=$(timeout -k 10 240 $B $args | tail -1) || { echo "bench failed: $args"; exit 2; }
    echo "{\"round\": $r, \"args\": \"$args\", \"line\": $line}" >> "$OUT"
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], d['kernels']['frame_ms'], d['kernels']['ms_per_frame_spread']['median'])" "$line" "$args"
  done
done
timeout -k 10 30 rocm-smi --showclocks > gpurun_out/r03_clocks.txt 2>&1 || true
echo warm done
