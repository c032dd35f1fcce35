#!/usr/bin/env bash
# Round-3 probes on one GPU box: the reference-render sweep (tools/ref_render_sweep.py render) and the
# section counters of the headline / mesh kernels (tools/section_times.py).  Each GPU step has its own
# time limit; a failing step ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {   # run NAME TIMEOUT CMD...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = sweep ]; then
    run ref_sweep 600 python -u tools/ref_render_sweep.py render --out gpurun_out/ref_sweep.npz
fi
if [ "$MODE" = all ] || [ "$MODE" = sections ]; then
    PT_SECTIONS_SKIP_CAMERA=1 run sec_cornell 300 python -u tools/section_times.py --scene cornell --variant 158 --frames 16 --out gpurun_out/sec_cornell.json
    run sec_bunny 300 python -u tools/section_times.py --scene cornell_obj_bnnuy --variant 190 --frames 16 --out gpurun_out/sec_bunny.json
    run sec_khaslana 300 python -u tools/section_times.py --scene cornell_obj_khaslana --res 1600x1600 --depth 12 --variant 190 --frames 8 --out gpurun_out/sec_khaslana.json
fi

if [ "$MODE" = probe_ab ]; then
    AB_TAG=probe_bunny AB_ROUNDS=3 AB_LIBS="project3-cuda-path-tracer-2025_amd/build/ab/base.so project3-cuda-path-tracer-2025_amd/build/ab/probe_load.so project3-cuda-path-tracer-2025_amd/build/ab/probe_valu20.so" \
        AB_ARGS="--steps 48 --warmup 4 --scene scenes/cornell_obj_bnnuy.json" timeout -k 10 600 bash tools/ab_libs.sh || exit 5
    AB_TAG=probe_khaslana AB_ROUNDS=3 AB_LIBS="project3-cuda-path-tracer-2025_amd/build/ab/base.so project3-cuda-path-tracer-2025_amd/build/ab/probe_load.so project3-cuda-path-tracer-2025_amd/build/ab/probe_valu20.so" \
        AB_ARGS="--steps 32 --warmup 2 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12" timeout -k 10 600 bash tools/ab_libs.sh || exit 6
fi
echo "probe done"
