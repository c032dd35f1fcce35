#!/usr/bin/env bash
# Price of k_bounce's per-block LDS geom staging: the product build against builds that stage the
# table 2x / 3x per block (tools/pt_tool_hooks.h PT_STAGE_REPS), khaslana 1600^2 d12 and cornell
set -u
cd "$(dirname "$0")/.."
L="project3-cuda-path-tracer-2025_amd/build/libptamd.so project3-cuda-path-tracer-2025_amd/build/ab/stage2.so project3-cuda-path-tracer-2025_amd/build/ab/stage3.so"
AB_TAG=stage_khaslana AB_ROUNDS=3 AB_LIBS="$L" AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 20 --warmup 5" bash tools/ab_libs.sh && \
AB_TAG=stage_cornell AB_ROUNDS=3 AB_LIBS="$L" AB_ARGS="--steps 20 --warmup 5" bash tools/ab_libs.sh
