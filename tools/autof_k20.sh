#!/usr/bin/env bash
# headline at the driver's K = 20: auto target 21M vs 84M paths (buffer sizes), alternating
set -u
cd "$(dirname "$0")/.."
B="python bench.py --no-cpu-baseline --no-configs --no-api --no-spread --steps 20 --warmup 5"
for r in 1 2 3 4; do
  for t in 21000000 84000000; do
    echo "$t $(PT_AUTO_PATHS=$t timeout -k 10 120 $B 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])')"
  done
done
