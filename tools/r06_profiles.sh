#!/usr/bin/env bash
# Round-6 profiles: rocprofv3 kernel stats (headline at the driver's K = 20, bunny, khaslana
# 1600^2 d12, the 262k-triangle stand-in), PMC traffic passes (headline, bunny, khaslana, 262k),
# and the section counters of the mesh kernels.  Counters only with --kernel-trace, one pass per
# process (tools/pmc.sh).  Summarised by tools/summarize_profiles.py into profiles/.
#   bash tools/r06_profiles.sh [all|stats|pmc|sections]
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
KH="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12"
CY="--scene scenes/cornell_obj_cyrene.json"
if [ "$MODE" = all ] || [ "$MODE" = stats ]; then
    st fused_k20 --steps 20 --warmup 5
    st c4_bunny --steps 48 --warmup 4 --scene scenes/cornell_obj_bnnuy.json
    st c5_khaslana --steps 32 --warmup 2 $KH
    st m262k_cyrene --steps 24 --warmup 2 $CY
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
    T="FETCH_SIZE;WRITE_SIZE"
    PMC_TAG=fused_ bash tools/pmc.sh || exit 4
    PMC_TAG=bvh2_ PMC_SETS="$T" bash tools/pmc.sh --scene scenes/cornell_obj_bnnuy.json || exit 5
    PMC_TAG=khtr_ PMC_STEPS=8 PMC_WARMUP=2 PMC_SETS="$T" bash tools/pmc.sh $KH || exit 7
    PMC_TAG=cyr_ PMC_STEPS=16 PMC_WARMUP=2 PMC_SETS="$T" bash tools/pmc.sh $CY || exit 8
fi
if [ "$MODE" = all ] || [ "$MODE" = sections ]; then
    run sec_bunny 300 python -u tools/section_times.py --scene cornell_obj_bnnuy --variant 190 --frames 16 --out gpurun_out/sec_bunny.json
    PT_SECTIONS_SKIP_CAMERA=1 run sec_khaslana 300 python -u tools/section_times.py --scene cornell_obj_khaslana --res 1600x1600 --depth 12 --variant 190 --frames 8 --out gpurun_out/sec_khaslana.json
    run sec_cyrene 300 python -u tools/section_times.py --scene cornell_obj_cyrene --variant 190 --frames 16 --out gpurun_out/sec_cyrene.json
fi
echo "profiles done"
