// rtamd/light.hpp — point light (/root/reference/RaytracingEngine/Light.h:6-59).
// The renderer reads position, color and intensity; the helper members are kept for API
// compatibility (the reference's shading does not call them either).
#pragma once

#include "rtamd/math.hpp"

// (build with -ffp-contract=off: no multiply-add fusion, as the reference's SSE2 build)

struct Light {
    Vec3 position;
    Vec3 color;
    double intensity;

    Light(const Vec3& position_, const Vec3& color_, const double& intensity_)
        : position(position_), color(color_), intensity(intensity_) {}
    Light() : position(Vec3(0, 0, 0)), color(Vec3(1, 1, 1)), intensity(1.0) {}

    Vec3 toLightDirection(const Vec3& point) const { return position - point; }
    double distanceTo(const Vec3& point) const { return toLightDirection(point).length(); }
    Vec3 dirTo(const Vec3& point) const {
        const Vec3 v = position - point;
        const double sq = v.x * v.x + v.y * v.y + v.z * v.z;
        if (sq <= 1e-12 * 1e-12) return Vec3{0, 0, 0};
        return (1.0 / std::sqrt(sq)) * v;
    }
    Rayon shadowRayFrom(const Vec3& hitPoint, double bias) const {
        const Vec3 l = dirTo(hitPoint);
        return Rayon{hitPoint + l * bias, l};
    }
    Vec3 emitted() const { return color * intensity; }
    Vec3 contributionFrom(double dist, double NdotL) const {
        if (dist <= 1e-12 || NdotL <= 0.0) return Vec3{0, 0, 0};
        return emitted() * (1.0 / (dist * dist) * NdotL);
    }
};
