#!/usr/bin/env bash
# Where k_bounce's VALU instructions go (headline scene): rocprofv3 PMC SQ_INSTS_VALU over the
# driver-shaped bench run for the product library and for builds that execute one section twice
# (PT_DUP=1 pre-test, 2 exchanged exact tests, 3 shading, 4 winner's hit record; the duplicate's
# result is discarded).  The difference is that section's VALU count.  tools/valu_attrib.py reads it.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/valu
mkdir -p "$OUT"
for lib in ${VA_LIBS:-project3-cuda-path-tracer-2025_amd/build/ab/new.so project3-cuda-path-tracer-2025_amd/build/ab/dup1.so project3-cuda-path-tracer-2025_amd/build/ab/dup2.so project3-cuda-path-tracer-2025_amd/build/ab/dup3.so project3-cuda-path-tracer-2025_amd/build/ab/dup4.so}; do
    tag=$(basename "$lib" .so)
    PTAMD_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS \
        -d "$OUT/$tag" -o run --output-format csv -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs --no-api --no-spread > "$OUT/$tag.log" 2>&1
    rc=$?
    echo "$tag rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$tag.log"; exit $rc; fi
done
echo "valu done"
