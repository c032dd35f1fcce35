#!/usr/bin/env bash
# Round-4 closing GPU session, part 1: the GPU suite, smoke(), the driver-shaped bench and the
# default bench, then the VALU attribution builds (tools/valu_attrib.sh)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
B=project3-cuda-path-tracer-2025_amd/build/ab
bash tools/r04_session.sh gpu bench bench100 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -n 2 gpurun_out/smoke.log
VA_LIBS="$B/new.so $B/dup1.so $B/dup2.so $B/dup3.so $B/dup4.so" bash tools/valu_attrib.sh
