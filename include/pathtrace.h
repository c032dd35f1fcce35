// pathtrace.h — C++ mirror of the reference's hot-path boundary, src/pathtrace.h:6-9, with the
// reference's exact signatures.  Implemented (host/pathtrace_cpp.cpp) on top of the C-ABI in
// pt/pathtrace_abi.h; like the reference it keeps a non-owning Scene* and, on any device
// error, prints the error and exits (pathtrace.cu:27-49).
#pragma once

#include "pt/pathtrace_abi.h"
#include "scene.h"

void InitDataContainer(GuiDataContainer* guiData);
void pathtraceInit(Scene* scene);
void pathtraceFree();
void pathtrace(uchar4* pbo, int frame, int iteration);

// Framework addition: run-time replacement of the reference's compile-time switches
// (ERRORCHECK / STREAM_COMPACTION / MATERIAL_SORTING / BVH_ACCELERATION, pathtrace.cu:20-24).
// Takes effect at the next pathtraceInit.
void pathtraceSetOptions(const pt_options& opts);
