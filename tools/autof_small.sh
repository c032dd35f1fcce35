#!/usr/bin/env bash
# cornell 800^2 d8 headline at 100 steps: auto target -> F = 20 / 40 / 100 (one pass), alternating
set -u
cd "$(dirname "$0")/.."
B="python bench.py --no-cpu-baseline --no-configs --no-api --no-spread --steps ${STEPS:-100} --warmup 10 ${EXTRA:-}"
for r in 1 2 3; do
  for t in ${TARGETS:-12800000 25600000 84000000}; do
    echo "$t $(PT_AUTO_PATHS=$t timeout -k 10 120 $B 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])')"
  done
done
