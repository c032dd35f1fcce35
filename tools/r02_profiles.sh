#!/usr/bin/env bash
# Round-2 profile refresh: rocprofv3 kernel stats (headline, bunny, khaslana 1600^2 d12) and PMC
# passes (headline traffic; bunny traffic + instruction mix + texture-addresser busy).  Counters
# only with --kernel-trace, one pass per process (tools/pmc.sh).  Summarised by
# tools/summarize_profiles.py into profiles/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-configs --no-api --no-spread"
st() {   # st TAG ARGS...
    local tag=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- $B "$@" \
        > gpurun_out/prof_$tag.log 2>&1 || { echo "stats $tag failed"; tail -5 gpurun_out/prof_$tag.log; exit 3; }
    echo "stats $tag ok"
}
st fused --steps 100 --warmup 10
st c4_bunny --steps 48 --warmup 8 --scene scenes/cornell_obj_bnnuy.json
st c5_khaslana --steps 32 --warmup 4 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12
PMC_TAG=fused_ bash tools/pmc.sh || exit 4
PMC_TAG=bvh2_ bash tools/pmc.sh --scene scenes/cornell_obj_bnnuy.json || exit 5
PMC_TAG=imta_ PMC_SETS="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_SMEM,SQ_INSTS_VMEM,SQ_WAVE_CYCLES;SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_ANY,GRBM_GUI_ACTIVE,TA_BUSY_avr,TA_TA_BUSY_sum" \
    bash tools/pmc.sh --scene scenes/cornell_obj_bnnuy.json || exit 6
echo "profiles done"
