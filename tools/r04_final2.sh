#!/usr/bin/env bash
# Round-4 closing session on the final build: GPU suite, smoke(), driver-shaped bench, the
# profiles (tools/r04_profiles.sh) and the VALU total of the product build (tools/valu_attrib.sh)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r04_session.sh gpu bench || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -n 1 gpurun_out/smoke.log
bash tools/r04_profiles.sh all > gpurun_out/r04_profiles.log 2>&1 || { tail -20 gpurun_out/r04_profiles.log; exit 5; }
tail -n 1 gpurun_out/r04_profiles.log
rm -rf gpurun_out/valu
VA_LIBS=project3-cuda-path-tracer-2025_amd/build/libptamd.so bash tools/valu_attrib.sh
