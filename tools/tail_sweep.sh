#!/usr/bin/env bash
# k_tail start bounce sweep on the single-frame path (PT_TAIL_FROM), alternating processes
set -u
cd "$(dirname "$0")/.."
for r in 1 2; do
  for f in ${FROMS:-1 2 3 4 5}; do
    echo "FROM=$f $(PT_TAIL_FROM=$f timeout -k 10 120 python tools/f1_profile.py 2>/dev/null)"
  done
done
