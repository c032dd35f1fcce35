// scene_file.h — the C-ABI scene handle (pt_scene_file, include/pt/pathtrace_abi.h): the
// framework's C++ Scene behind an opaque pointer (shared by scene_abi.cpp and viewer.cpp).
#pragma once

#include "scene.h"

struct pt_scene_file {
    Scene* scene;
};
