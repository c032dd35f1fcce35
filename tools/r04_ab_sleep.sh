#!/usr/bin/env bash
# Why does staging k_bounce's geom table twice speed khaslana up?  Product vs 2x staging vs a pure
# delay of all waves vs a delay of waves 2-3 (stagger), khaslana 1600^2 d12
set -u
cd "$(dirname "$0")/.."
B=project3-cuda-path-tracer-2025_amd/build
AB_TAG=sleep_khaslana AB_ROUNDS=3 AB_LIBS="$B/libptamd.so $B/ab/stage2.so $B/ab/sleepall.so $B/ab/sleephi.so" \
  AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 20 --warmup 5" bash tools/ab_libs.sh
