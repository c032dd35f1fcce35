#!/usr/bin/env bash
# k_bvh_bounce with the SAH hierarchy's top pairs read from LDS (PT_BVH_TOPK): parity at 31, then
# bunny and khaslana 1600^2 d12 over TOPK 0 / 7 / 31 / 63, and the build without the code path
set -u
cd "$(dirname "$0")/.."
B=project3-cuda-path-tracer-2025_amd/build
PT_BVH_TOPK=31 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "bvh or mesh or bnnuy or khaslana" > gpurun_out/topk_tests.log 2>&1 || { tail -30 gpurun_out/topk_tests.log; exit 3; }
tail -n 1 gpurun_out/topk_tests.log
E="PT_BVH_TOPK=0;PT_BVH_TOPK=7;PT_BVH_TOPK=31;PT_BVH_TOPK=63"
AB_TAG=topk_bunny AB_ROUNDS=3 AB_ENVS="$E" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json --steps 20 --warmup 5" bash tools/ab_env.sh && \
AB_TAG=topk_khaslana AB_ROUNDS=2 AB_ENVS="$E" AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 20 --warmup 5" bash tools/ab_env.sh && \
AB_TAG=topk_base AB_ROUNDS=3 AB_LIBS="$B/ab/base.so $B/libptamd.so" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json --steps 20 --warmup 5" bash tools/ab_libs.sh
