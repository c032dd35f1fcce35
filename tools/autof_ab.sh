#!/usr/bin/env bash
# paths-in-flight target of the auto frames-per-pass rule (PT_AUTO_PATHS), alternating processes
set -u
cd "$(dirname "$0")/.."
B="python bench.py --no-cpu-baseline --no-configs --no-api --no-spread"
ms() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["config"]["frames_per_pass"])'; }
for r in 1 2; do
  for t in 21000000 42000000 84000000; do
    echo "kh  $t $(PT_AUTO_PATHS=$t timeout -k 10 200 $B --steps 32 --warmup 4 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 2>/dev/null | ms)"
    echo "bun $t $(PT_AUTO_PATHS=$t timeout -k 10 200 $B --steps 64 --warmup 4 --scene scenes/cornell_obj_bnnuy.json 2>/dev/null | ms)"
    echo "cor $t $(PT_AUTO_PATHS=$t timeout -k 10 200 $B --steps 128 --warmup 8 2>/dev/null | ms)"
  done
done
