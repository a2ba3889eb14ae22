// rtamd/math.hpp — host value types of the drop-in API: Vec3, Color, Rayon, Camera.
//
// Same names, members, constructors and semantics as the reference's Math.h
// (/root/reference/RaytracingEngine/Math.h:9-122) so scene-building code compiles unchanged.
// Arithmetic is IEEE double in the reference's operation order (build with
// -ffp-contract=off); the GPU renderer never calls these — they are the host-side value API.
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <stdexcept>

// (build with -ffp-contract=off: no multiply-add fusion, as the reference's SSE2 build)

struct Vec3 {
    double x, y, z;

    explicit Vec3(double x_ = 0.0, double y_ = 0.0, double z_ = 0.0) : x(x_), y(y_), z(z_) {}
    explicit Vec3(double v) : x(v), y(v), z(v) {}  // Math.h:12 (never selected: ambiguous with the default-argument form, as in the reference)

    // component-wise operators (Math.h:14-25); division is a true division per component
    Vec3 operator+(const Vec3& o) const noexcept { return Vec3{x + o.x, y + o.y, z + o.z}; }
    Vec3 operator+(double s) const noexcept { return Vec3{x + s, y + s, z + s}; }
    Vec3 operator-(const Vec3& o) const noexcept { return Vec3{x - o.x, y - o.y, z - o.z}; }
    Vec3 operator-(double s) const noexcept { return Vec3{x - s, y - s, z - s}; }
    Vec3 operator*(double s) const noexcept { return Vec3{x * s, y * s, z * s}; }
    Vec3 operator*(const Vec3& o) const noexcept { return Vec3{x * o.x, y * o.y, z * o.z}; }
    Vec3 operator/(const Vec3& o) const noexcept { return Vec3{x / o.x, y / o.y, z / o.z}; }
    Vec3 operator/(double s) const noexcept { return Vec3{x / s, y / s, z / s}; }
    Vec3 operator-() const noexcept { return Vec3{-x, -y, -z}; }
    Vec3& operator+=(const Vec3& o) noexcept {
        x += o.x;
        y += o.y;
        z += o.z;
        return *this;
    }
    Vec3& operator/=(double s) noexcept {
        x /= s;
        y /= s;
        z /= s;
        return *this;
    }
    Vec3& operator*=(double s) noexcept {
        x *= s;
        y *= s;
        z *= s;
        return *this;
    }

    double dot(const Vec3& o) const noexcept { return x * o.x + y * o.y + z * o.z; }
    Vec3 cross(const Vec3& o) const noexcept {
        return Vec3{y * o.z - z * o.y, z * o.x - x * o.z, x * o.y - y * o.x};
    }
    double length() const noexcept { return std::sqrt(dot(*this)); }
    // zero vector when the length is <= 1e-12 (Math.h:31-37)
    Vec3 normalize() const noexcept {
        const double len = length();
        return len <= 1e-12 ? Vec3{0.0, 0.0, 0.0} : (*this) / len;
    }
    Vec3 reflect(const Vec3& n) const noexcept { return (*this) - n * 2.0 * dot(n); }
    Vec3 refract(const Vec3& normal, double eta) const {
        const Vec3 I = normalize();
        const Vec3 N = normal.normalize();
        double cosi = I.dot(N);
        cosi = cosi < -1.0 ? -1.0 : (1.0 < cosi ? 1.0 : cosi);
        const double k = 1.0 - eta * eta * (1.0 - cosi * cosi);
        if (k < 0.0) return Vec3{0.0, 0.0, 0.0};
        return I * eta - N * (eta * cosi + std::sqrt(k));
    }
    double unsafeIndex(int index) const {
        if (index == 0) return x;
        if (index == 1) return y;
        if (index == 2) return z;
        throw std::out_of_range("Vec3 index out of range");
    }
    Vec3& lerp(const Vec3& target, double t) noexcept {
        x = x + (target.x - x) * t;
        y = y + (target.y - y) * t;
        z = z + (target.z - z) * t;
        return *this;
    }
    friend Vec3 operator*(double s, const Vec3& v) noexcept { return v * s; }
};

static_assert(sizeof(Vec3) == 3 * sizeof(double), "Vec3 must be three packed doubles");

// 8-bit RGB pixel (Math.h:73-76) — the PPM payload.
struct Color {
    uint8_t r, g, b;
    Color(uint8_t r_ = 0, uint8_t g_ = 0, uint8_t b_ = 0) : r(r_), g(g_), b(b_) {}
};

static_assert(sizeof(Color) == 3, "Color must be three packed bytes");

// Ray (Math.h:78-83).
struct Rayon {
    Vec3 origin;
    Vec3 direction;
    Rayon(const Vec3& o, const Vec3& d) : origin(o), direction(d) {}
    Vec3 pointAtDistance(double t) const noexcept { return origin + direction * t; }
};

namespace rtamd {
// Build-defined U[0,1) draw shared with the device kernels (the reference's jitter comes from
// a random_device-seeded mt19937 and cannot be reproduced).
inline double jitter_u01(uint64_t seed, uint64_t pixel, uint32_t stream, uint32_t index) {
    auto mix = [](uint64_t z) {
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    };
    auto hash32 = [](uint32_t x) {
        x ^= x >> 16;
        x *= 0x7feb352dU;
        x ^= x >> 15;
        x *= 0x846ca68bU;
        x ^= x >> 16;
        return x;
    };
    const uint64_t k = mix(seed ^ (0x9E3779B97F4A7C15ULL * (pixel + 1ULL)));
    const uint32_t key = static_cast<uint32_t>(k ^ (k >> 32));
    const uint32_t skey = hash32(key ^ (stream * 0x9E3779B9U));
    return static_cast<double>(hash32(skey + index * 0x85EBCA6BU)) * 0x1.0p-32;
}
}  // namespace rtamd

// Pinhole camera (Math.h:85-122).  `forward` is stored but unused, near/far are stored and
// not read by the trace — exactly as in the reference.
struct Camera {
    Vec3 position;
    Vec3 forward;
    std::size_t width;
    std::size_t height;
    double focal;
    double farPlaneDistance;
    double nearPlaneDistance;

    int antiAliasingAmount = 32;  // reference default (Math.h:94)
    uint64_t jitterSeed = 0x5EED;  // build-defined: key of the AA jitter RNG

    Camera(const Vec3& position_, double focal_ = 1.0, std::size_t width_ = 800,
           std::size_t height_ = 600, double nearPlaneDistance_ = 1.0,
           double farPlaneDistance_ = 1000.0)
        : position(position_), forward{0, 0, 1}, width(width_), height(height_), focal(focal_),
          farPlaneDistance(farPlaneDistance_), nearPlaneDistance(nearPlaneDistance_) {}

    // Pixel-corner ray; with `aa` the jitter is U[0,1)² (1.0/double(bool) == 1, Math.h:106).
    // Host utility: Scene::RenderImage generates its rays on the device.
    Rayon getRay(std::size_t pixelX, std::size_t pixelY, bool aa, uint32_t sample = 1) const {
        double sx = static_cast<double>(pixelX) - static_cast<double>(width) / 2.0;
        double sy = static_cast<double>(height) / 2.0 - static_cast<double>(pixelY);
        double jx = 0.0, jy = 0.0;
        if (aa) {
            const uint64_t pix = static_cast<uint64_t>(pixelY) * width + pixelX;
            jx = rtamd::jitter_u01(jitterSeed, pix, sample, 0u);
            jy = rtamd::jitter_u01(jitterSeed, pix, sample, 1u);
        }
        sx += jx;
        sy += jy;
        const Vec3 screen(sx, sy, position.z + focal);
        return Rayon{position, (screen - position).normalize()};
    }
};
