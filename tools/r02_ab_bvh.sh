#!/usr/bin/env bash
# mesh parity subset on the current build, then bunny / khaslana A/B over AB_LIBS
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    -k "bnnuy or khaslana or intersections or skewed or phatphuck or bump or benched or config5 or intersect" > gpurun_out/par.log 2>&1
rc=$?; tail -3 gpurun_out/par.log; [ $rc -eq 0 ] || exit 1
AB_TAG=bunny AB_ARGS="--steps 48 --warmup 8 --scene scenes/cornell_obj_bnnuy.json" bash tools/ab_libs.sh || exit 3
[ -n "${AB_NO_KH:-}" ] || AB_TAG=kh AB_ROUNDS=2 AB_ARGS="--steps 16 --warmup 4 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12" bash tools/ab_libs.sh || exit 4
