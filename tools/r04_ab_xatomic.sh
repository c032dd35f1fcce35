#!/usr/bin/env bash
# Price of block_append's returning atomic: the product build against a tool build that waits for
# a second one (PT_EXTRA_ATOMIC), headline and glass + grouping
set -u
cd "$(dirname "$0")/.."
B=project3-cuda-path-tracer-2025_amd/build
L="$B/ab/committed.so $B/ab/xatomic.so"
AB_TAG=xatomic_cornell AB_ROUNDS=4 AB_LIBS="$L" AB_ARGS="--steps 20 --warmup 5" bash tools/ab_libs.sh && \
AB_TAG=xatomic_glass AB_ROUNDS=3 AB_LIBS="$L" AB_ARGS="--scene scenes/cornell_glass_test.json --sort --steps 20 --warmup 5" bash tools/ab_libs.sh
