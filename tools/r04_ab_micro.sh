#!/usr/bin/env bash
# A/B of k_bounce micro-changes: fused-path parity of the product build and of every variant in
# $AB_VARIANTS (build/ab/NAME.so), then build/ab/$AB_BASE.so, the product build and the variants
# on the headline (cornell), glass + grouping and bunny
set -u
cd "$(dirname "$0")/.."
B=project3-cuda-path-tracer-2025_amd/build
PT="python -u -m pytest tests/test_gpu_parity.py tests/test_multi_device.py -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT > gpurun_out/micro_tests.log 2>&1 || { tail -30 gpurun_out/micro_tests.log; exit 3; }
tail -n 1 gpurun_out/micro_tests.log
L="$B/ab/${AB_BASE:-away}.so $B/libptamd.so"
for v in ${AB_VARIANTS:-}; do
    PTAMD_LIB=$PWD/$B/ab/$v.so timeout -k 10 600 $PT > gpurun_out/micro_tests_$v.log 2>&1 || { tail -30 gpurun_out/micro_tests_$v.log; exit 3; }
    echo "$v: $(tail -n 1 gpurun_out/micro_tests_$v.log)"
    L="$L $B/ab/$v.so"
done
AB_TAG=micro_cornell AB_ROUNDS=4 AB_LIBS="$L" AB_ARGS="--steps 20 --warmup 5" bash tools/ab_libs.sh && \
AB_TAG=micro_glass AB_ROUNDS=3 AB_LIBS="$L" AB_ARGS="--scene scenes/cornell_glass_test.json --sort --steps 20 --warmup 5" bash tools/ab_libs.sh && \
AB_TAG=micro_bunny AB_ROUNDS=3 AB_LIBS="$L" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json --steps 20 --warmup 5" bash tools/ab_libs.sh
[ -n "${AB_KHASLANA:-}" ] && AB_TAG=micro_khaslana AB_ROUNDS=2 AB_LIBS="$L" \
  AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 20 --warmup 5" bash tools/ab_libs.sh
exit 0
