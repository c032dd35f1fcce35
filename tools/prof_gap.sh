#!/usr/bin/env bash
# eager profiled replay right after the timed region vs after an idle gap: avg k_bounce launch
set -u
cd "$(dirname "$0")/.."
B="python bench.py --no-cpu-baseline --no-configs --no-api --no-spread --steps ${STEPS:-20} --warmup 5"
for r in 1 2 3; do
  for gap in 0 0.3; do
    echo "gap $gap $(PT_BENCH_PROF_GAP=$gap timeout -k 10 120 $B 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
  done
done
