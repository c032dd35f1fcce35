#!/usr/bin/env bash
# k_tail on multi-frame passes (PT_TAIL_BATCH=1, start bounce PT_TAIL_FROM) vs off, headline bench
set -u
cd "$(dirname "$0")/.."
B="python bench.py --no-cpu-baseline --no-configs --no-api --no-spread"
for r in 1 2 3; do
  echo "off   $(timeout -k 10 120 $B --steps ${STEPS:-20} --warmup 5 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])')"
  for f in 5 6 7; do
    echo "from$f $(PT_TAIL_BATCH=1 PT_TAIL_FROM=$f timeout -k 10 120 $B --steps ${STEPS:-20} --warmup 5 2>/dev/null | python3 -c 'import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])["ms_per_step"])')"
  done
done
