#!/usr/bin/env bash
# The pre-test's away drop for one cube per lane (the origin's) instead of every kept cube:
# parity of the fused path, then the headline (cornell), glass + grouping, bunny
set -u
cd "$(dirname "$0")/.."
B=project3-cuda-path-tracer-2025_amd/build
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_device.py -x -q --timeout 300 --timeout-method thread > gpurun_out/away_tests.log 2>&1 || { tail -30 gpurun_out/away_tests.log; exit 3; }
tail -n 2 gpurun_out/away_tests.log
L="$B/ab/base_prod.so $B/libptamd.so"
AB_TAG=away_cornell AB_ROUNDS=4 AB_LIBS="$L" AB_ARGS="--steps 20 --warmup 5" bash tools/ab_libs.sh && \
AB_TAG=away_glass AB_ROUNDS=3 AB_LIBS="$L" AB_ARGS="--scene scenes/cornell_glass_test.json --sort --steps 20 --warmup 5" bash tools/ab_libs.sh && \
AB_TAG=away_bunny AB_ROUNDS=3 AB_LIBS="$L" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json --steps 20 --warmup 5" bash tools/ab_libs.sh
