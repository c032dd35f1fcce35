#!/usr/bin/env bash
# rocprofv3 PMC passes (counters only with --kernel-trace/--stats, never with sys/runtime traces)
# over a short bench run (warmup 8 + 32 timed frames + bench's 32-frame profiling replay = 72 frames,
# no sub-configs / api / spread runs); each pass in its own process.  Usage: tools/pmc.sh [extra bench args]
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p "$OUT"
i=0
SETS=${PMC_SETS:-"SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS;SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY;SQ_ACTIVE_INST_VALU,SQ_INSTS_VMEM,SQ_WAIT_INST_ANY,GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum,TCC_MISS_sum"}
IFS=';' read -ra SETARR <<< "$SETS"
for set in "${SETARR[@]}"; do
    set=${set//,/ }
    i=$((i+1))
    echo "== pass $i: $set"
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d "$OUT/${PMC_TAG:-}p$i" -o run --output-format csv -- \
        python bench.py --steps ${PMC_STEPS:-32} --warmup ${PMC_WARMUP:-8} --no-cpu-baseline --no-configs --no-api --no-spread "$@" > "$OUT/${PMC_TAG:-}p$i.log" 2>&1
    rc=$?
    echo "rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/${PMC_TAG:-}p$i.log"; exit $rc; fi
done
echo "pmc done"
