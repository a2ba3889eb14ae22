// rtamd/image.cpp — writePPM (host I/O boundary) and the device tonemap wrappers.
#include "rtamd/image.hpp"

#include <cstdio>
#include <iostream>
#include <stdexcept>

#include "rt_capi.h"
#include "rtamd/scene.hpp"

void writePPM(const std::string& filename, const std::vector<Color>& pixels, size_t width,
              size_t height) {
    std::FILE* f = std::fopen(filename.c_str(), "wb");
    if (!f) throw std::runtime_error("Could not open file for writing");
    const std::string header = "P6\n" + std::to_string(width) + " " + std::to_string(height) +
                               "\n255\n";
    bool ok = std::fwrite(header.data(), 1, header.size(), f) == header.size();
    // Color is three packed bytes (static_assert in math.hpp): the payload is the vector.
    if (ok && !pixels.empty())
        ok = std::fwrite(pixels.data(), sizeof(Color), pixels.size(), f) == pixels.size();
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) throw std::runtime_error("Error occurred while writing to file");
    std::cout << "Image written to " << filename << "\n";
}

namespace rtamd {

std::vector<Color> tonemapOp(const std::vector<Vec3>& pixels, int op, int device) {
    std::vector<Color> out(pixels.size());
    check(rt_tonemap(thread_context(device), reinterpret_cast<const double*>(pixels.data()),
                     pixels.size(), op, reinterpret_cast<uint8_t*>(out.data())),
          "rt_tonemap");
    return out;
}

std::vector<Color> tonemap(const std::vector<Vec3>& pixels) {
    return tonemapOp(pixels, RT_TONEMAP_ACES, current_device());
}

std::vector<std::vector<Color>> tonemapAll(const std::vector<Vec3> pixels) {
    std::vector<Color> planes(pixels.size() * RT_TONEMAP_COUNT);
    check(rt_tonemap(thread_context(current_device()),
                     reinterpret_cast<const double*>(pixels.data()), pixels.size(), RT_TONEMAP_COUNT, reinterpret_cast<uint8_t*>(planes.data())),
          "rt_tonemap");
    std::vector<std::vector<Color>> all(RT_TONEMAP_COUNT);
    for (int k = 0; k < RT_TONEMAP_COUNT; ++k)
        all[k].assign(planes.begin() + static_cast<long>(k * pixels.size()),
                      planes.begin() + static_cast<long>((k + 1) * pixels.size()));
    return all;
}

}  // namespace rtamd
