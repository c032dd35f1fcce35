#!/usr/bin/env bash
# single-frame (API) path with and without the k_tail launch (PT_TAIL=0), alternating processes
set -u
cd "$(dirname "$0")/.."
for r in 1 2 3; do
  for t in 1 0; do
    echo "PT_TAIL=$t $(PT_TAIL=$t timeout -k 10 120 python tools/f1_profile.py 2>/dev/null)"
  done
done
