#!/usr/bin/env bash
# parity subset on the product build, then a mesh-config A/B: AB_LIBS2 (default project3-cuda-path-tracer-2025_amd/build/ab/fast.so vs build)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
K=${AB_K:-"frames_bitexact or benched or intersect or khaslana or skewed or bnnuy or phatphuck"}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/t_main.log 2>&1 || { tail -n 30 gpurun_out/t_main.log; exit 1; }
tail -n 1 gpurun_out/t_main.log
M=project3-cuda-path-tracer-2025_amd/build/libptamd.so
L=${AB_LIBS2:-"project3-cuda-path-tracer-2025_amd/build/ab/fast.so $M"}
AB_LIBS="$L" AB_TAG=bunny AB_ARGS="--steps 48 --warmup 8 --scene scenes/cornell_obj_bnnuy.json" bash tools/ab_libs.sh || exit 3
AB_LIBS="$L" AB_TAG=kh AB_ROUNDS=2 AB_ARGS="--steps 16 --warmup 4 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12" bash tools/ab_libs.sh || exit 4
[ -n "${AB_CORNELL:-}" ] && { AB_LIBS="$L" AB_TAG=cornell AB_ARGS="--steps 100 --warmup 10" bash tools/ab_libs.sh || exit 2; }
exit 0
