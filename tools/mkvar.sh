#!/bin/bash
# mkvar.sh NAME "EXTRA FLAGS" : build a variant libptamd.so into project3-cuda-path-tracer-2025_amd/build/ab/NAME.so
# (travels to the GPU box with the build; delete build/ab after the A/B)
set -e
cd /root/repo/project3-cuda-path-tracer-2025_amd
N=$1; shift
D=/tmp/var_$N; mkdir -p $D
HF="--offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fPIC -std=c++17 -Wall -I../include -Icsrc -Ihost -I../tools -DPT_TOOLS $*"
hipcc $HF -c csrc/pt_runtime.hip -o $D/pt_runtime.o
mkdir -p build/ab && hipcc --offload-arch=gfx950 -shared -fPIC -o build/ab/$N.so $D/pt_runtime.o build/pt_bvh_build.o build/scene.o build/scene_abi.o build/pathtrace_cpp.o build/image_io.o build/png_decode.o build/viewer.o build/trav_tree.o
echo built build/ab/$N.so
