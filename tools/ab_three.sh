#!/usr/bin/env bash
# A/B of project3-cuda-path-tracer-2025_amd/build/ab/base.so vs the current build on the headline and both mesh configs
set -u
cd "$(dirname "$0")/.."
AB_LIBS=${AB_LIBS3:-"project3-cuda-path-tracer-2025_amd/build/ab/base.so project3-cuda-path-tracer-2025_amd/build/libptamd.so"} AB_TAG=cornell AB_ARGS="--steps 100 --warmup 10" bash tools/ab_libs.sh || exit 2
AB_LIBS=${AB_LIBS3:-"project3-cuda-path-tracer-2025_amd/build/ab/base.so project3-cuda-path-tracer-2025_amd/build/libptamd.so"} AB_TAG=bunny AB_ARGS="--steps 48 --warmup 8 --scene scenes/cornell_obj_bnnuy.json" bash tools/ab_libs.sh || exit 3
AB_LIBS=${AB_LIBS3:-"project3-cuda-path-tracer-2025_amd/build/ab/base.so project3-cuda-path-tracer-2025_amd/build/libptamd.so"} AB_TAG=kh AB_ROUNDS=2 AB_ARGS="--steps 16 --warmup 4 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12" bash tools/ab_libs.sh || exit 4
