// rtamd/image.hpp — PPM output (Image.h:7) and the device tonemap entry points.
//
// writePPM keeps the reference's signature and behaviour (Image.cpp:11-31): binary P6,
// std::runtime_error on open/write failure, "Image written to <file>" on stdout.
//
// The reference defines tonemap()/tonemapAll() in its application file
// (RaytracingEngine.cpp:165-214).  The device versions live in namespace rtamd so they do not
// collide with an application that still defines its own; define RTAMD_GLOBAL_TONEMAP before
// including this header to get them as the global ::tonemap / ::tonemapAll instead.
#pragma once

#include <string>
#include <vector>

#include "rtamd/math.hpp"

void writePPM(const std::string& filename, const std::vector<Color>& pixels, size_t width,
              size_t height);

namespace rtamd {
// One operator (rt_tonemap_op) followed by toColor(), evaluated on the GPU.
// tonemap() and tonemapAll() run on rtamd::current_device() (scene.hpp).
std::vector<Color> tonemapOp(const std::vector<Vec3>& pixels, int op, int device = 0);
// tonemap(): ACES (RaytracingEngine.cpp:165-174).
std::vector<Color> tonemap(const std::vector<Vec3>& pixels);
// tonemapAll(): simple, reinhardSimple, reinhardExtended, reinhardExtendedLuminance,
// reinhardJodie, uncharted2, aces — one device pass (RaytracingEngine.cpp:176-214).
std::vector<std::vector<Color>> tonemapAll(const std::vector<Vec3> pixels);
}  // namespace rtamd

#ifdef RTAMD_GLOBAL_TONEMAP
using rtamd::tonemap;
using rtamd::tonemapAll;
#endif
