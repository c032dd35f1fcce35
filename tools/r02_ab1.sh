#!/usr/bin/env bash
# round-2 session A/B: parity subset on the product build and on project3-cuda-path-tracer-2025_amd/build/ab/ww.so, then timing
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
K="frames_bitexact or benched or intersect or khaslana or skewed"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/t_main.log 2>&1; tail -n 2 gpurun_out/t_main.log
PTAMD_LIB=$PWD/project3-cuda-path-tracer-2025_amd/build/ab/ww.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/t_ww.log 2>&1; tail -n 2 gpurun_out/t_ww.log
M=project3-cuda-path-tracer-2025_amd/build/libptamd.so
AB_LIBS="project3-cuda-path-tracer-2025_amd/build/ab/base.so project3-cuda-path-tracer-2025_amd/build/ab/cull.so" AB_TAG=cornell AB_ARGS="--steps 100 --warmup 10" bash tools/ab_libs.sh || exit 2
AB_LIBS="project3-cuda-path-tracer-2025_amd/build/ab/base.so project3-cuda-path-tracer-2025_amd/build/ab/cull.so $M project3-cuda-path-tracer-2025_amd/build/ab/ww.so" AB_TAG=bunny AB_ARGS="--steps 48 --warmup 8 --scene scenes/cornell_obj_bnnuy.json" bash tools/ab_libs.sh || exit 3
AB_LIBS="project3-cuda-path-tracer-2025_amd/build/ab/base.so project3-cuda-path-tracer-2025_amd/build/ab/cull.so $M project3-cuda-path-tracer-2025_amd/build/ab/ww.so" AB_TAG=kh AB_ROUNDS=2 AB_ARGS="--steps 16 --warmup 4 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12" bash tools/ab_libs.sh || exit 4
