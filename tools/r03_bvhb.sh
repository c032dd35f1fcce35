#!/usr/bin/env bash
# GPU BVH build: parity tests, then host vs GPU build times (PT_BVH_TIMING per-level split on stderr)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    -k "gpu_bvh or skewed_gpu" > gpurun_out/r03_bvhb_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r03_bvhb_tests.log; [ $rc -eq 0 ] || exit $rc
PT_BVH_TIMING=1 timeout -k 10 300 python -u tools/bvh_build_time.py > gpurun_out/r03_bvhb_time.log 2>&1; rc=$?; tail -20 gpurun_out/r03_bvhb_time.log; exit $rc
