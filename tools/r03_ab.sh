#!/usr/bin/env bash
# A/B of project3-cuda-path-tracer-2025_amd/build/ab/*.so builds on cornell (headline shape), glass, bunny and khaslana (interleaved
# processes, tools/ab_libs.sh).  Usage: AB_LIBS="project3-cuda-path-tracer-2025_amd/build/ab/a.so project3-cuda-path-tracer-2025_amd/build/ab/b.so" bash tools/r03_ab.sh [scenes]
set -u
cd "$(dirname "$0")/.."
SC=${1:-"cornell bunny khaslana"}
for s in $SC; do
  case $s in
    cornell) A="--steps 20 --warmup 5";;
    glass) A="--steps 48 --warmup 4 --scene scenes/cornell_glass_test.json";;
    bunny) A="--steps 48 --warmup 4 --scene scenes/cornell_obj_bnnuy.json";;
    khaslana) A="--steps 32 --warmup 2 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12";;
  esac
  AB_TAG=$s AB_ROUNDS=${AB_ROUNDS:-3} AB_ARGS="$A" timeout -k 10 600 bash tools/ab_libs.sh || exit 5
done
echo "ab done"
