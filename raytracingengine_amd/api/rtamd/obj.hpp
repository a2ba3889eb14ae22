// rtamd/obj.hpp — Wavefront OBJ import into a Model, the reference application's LoadObject
// (RaytracingEngine.cpp:15-65) without tinyobjloader.
//
// Same result as LoadObject through tinyobjloader v1.0.x with triangulation on: every `v`
// position is read into a float (tinyobj's real_t) and widened to double; every `f` face
// (`i`, `i/t`, `i//n`, `i/t/n` corners, 1-based or negative = relative indices) is fanned from
// its first corner into triangles, faces in file order; all other statements are ignored.
// Throws std::runtime_error("Failed to load/parse .obj.") when the file cannot be read, like
// LoadObject.  Defined in namespace rtamd so an application keeping its own LoadObject still
// links; define RTAMD_GLOBAL_LOADOBJECT before including this header to get ::LoadObject.
#pragma once

#include <string>

#include "rtamd/shapes.hpp"

namespace rtamd {
Model LoadObject(const std::string& modelName, const Transform& transform = Transform(),
                 const Material& material = Material());
}  // namespace rtamd

#ifdef RTAMD_GLOBAL_LOADOBJECT
using rtamd::LoadObject;
#endif
