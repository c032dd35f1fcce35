#!/usr/bin/env bash
# A/B of a k_bvh_bounce change: mesh parity of the product build, then build/ab/committed.so
# against it on bunny 800^2 d8 and khaslana 1600^2 d12
set -u
cd "$(dirname "$0")/.."
B=project3-cuda-path-tracer-2025_amd/build
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_device.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mesh_tests.log 2>&1 || { tail -30 gpurun_out/mesh_tests.log; exit 3; }
tail -n 1 gpurun_out/mesh_tests.log
L="$B/ab/committed.so $B/libptamd.so"
AB_TAG=mesh_bunny AB_ROUNDS=4 AB_LIBS="$L" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json --steps 20 --warmup 5" bash tools/ab_libs.sh && \
AB_TAG=mesh_khaslana AB_ROUNDS=3 AB_LIBS="$L" AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 20 --warmup 5" bash tools/ab_libs.sh
