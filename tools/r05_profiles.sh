#!/usr/bin/env bash
# Round-5 profiles: rocprofv3 kernel stats (headline at the driver's K = 20, bunny, khaslana
# 1600^2 d12), PMC passes (headline; bunny and khaslana traffic + instruction mix + texture
# addresser), and the section counters of k_bounce / k_bvh_bounce (tools/section_times.py).
# Counters only with --kernel-trace, one pass per process (tools/pmc.sh).  Summarised by
# tools/summarize_profiles.py into profiles/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-configs --no-api --no-spread"
MODE=${1:-all}
st() {   # st TAG ARGS...
    local tag=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- $B "$@" \
        > gpurun_out/prof_$tag.log 2>&1 || { echo "stats $tag failed"; tail -5 gpurun_out/prof_$tag.log; exit 3; }
    echo "stats $tag ok"
}
run() {   # run NAME TIMEOUT CMD...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
IM="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_SMEM,SQ_INSTS_VMEM,SQ_WAVE_CYCLES;SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_ANY,GRBM_GUI_ACTIVE,TA_BUSY_avr,TA_TA_BUSY_sum"
KH="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12"
if [ "$MODE" = all ] || [ "$MODE" = stats ]; then
    # the API frame (pathtrace() per frame, F = 1): kernel trace + stats, anatomy by tools/api_trace.py
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_api_f1 -o run --output-format csv -- \
        python tools/api_trace.py run > gpurun_out/prof_api_f1.log 2>&1 || { echo "api trace failed"; exit 3; }
    python tools/api_trace.py analyse gpurun_out/prof_api_f1/run_kernel_trace.csv --out gpurun_out/api_f1.json
    st fused_k20 --steps 20 --warmup 5
    st c4_bunny --steps 48 --warmup 4 --scene scenes/cornell_obj_bnnuy.json
    st c5_khaslana --steps 32 --warmup 2 $KH
    st staged_c2 --steps 48 --warmup 4 --scene scenes/cornell_glass_test.json --sort --pipeline staged
    # main.cpp's call (image copied out every call): the copy against the next frame's kernels
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_api_copy -o run --output-format csv -- \
        python tools/api_trace.py run copy > gpurun_out/prof_api_copy.log 2>&1 || { echo "api copy trace failed"; exit 3; }
    python tools/api_trace.py overlap gpurun_out/prof_api_copy/run_kernel_trace.csv gpurun_out/prof_api_copy/run_memory_copy_trace.csv --out gpurun_out/api_copy_overlap.json
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
    PMC_TAG=fused_ bash tools/pmc.sh || exit 4
    PMC_TAG=stg_ PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES,SQ_INSTS_VALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,GRBM_GUI_ACTIVE" bash tools/pmc.sh --scene scenes/cornell_glass_test.json --sort --pipeline staged || exit 9
    PMC_TAG=bvh2_ bash tools/pmc.sh --scene scenes/cornell_obj_bnnuy.json || exit 5
    PMC_TAG=imta_ PMC_SETS="$IM" bash tools/pmc.sh --scene scenes/cornell_obj_bnnuy.json || exit 6
    PMC_TAG=khtr_ PMC_STEPS=8 PMC_WARMUP=2 bash tools/pmc.sh $KH || exit 7
    PMC_TAG=khim_ PMC_STEPS=8 PMC_WARMUP=2 PMC_SETS="$IM" bash tools/pmc.sh $KH || exit 8
fi
if [ "$MODE" = all ] || [ "$MODE" = sections ]; then
    PT_SECTIONS_SKIP_CAMERA=1 run sec_cornell 300 python -u tools/section_times.py --scene cornell --variant 158 --frames 16 --out gpurun_out/sec_cornell.json
    run sec_bunny 300 python -u tools/section_times.py --scene cornell_obj_bnnuy --variant 190 --frames 16 --out gpurun_out/sec_bunny.json
    run sec_khaslana 300 python -u tools/section_times.py --scene cornell_obj_khaslana --res 1600x1600 --depth 12 --variant 190 --frames 8 --out gpurun_out/sec_khaslana.json
fi
echo "profiles done"
