// rtamd/shapes.hpp — Transform, Material, HitType, HitInfo, Sphere, Plane, Triangle, Model.
//
// Public names, constructors, getters and setters of the reference's Shape.h
// (/root/reference/RaytracingEngine/Shape.h:7-307).  The per-shape Intersect/GetHitInfoAt
// members stay available as host utilities with the reference's semantics; the renderer
// itself flattens the shapes into the C-ABI records (rt_capi.h) and intersects on the GPU.
#pragma once

#include <optional>
#include <utility>
#include <vector>

#include "rtamd/math.hpp"

// (build with -ffp-contract=off: no multiply-add fusion, as the reference's SSE2 build)

struct Transform {
    Vec3 position;
    Vec3 rotation;
    Vec3 scale;
};

struct Material {
    Vec3 color;
    double shininess = 128.0;
    double specular = 0.0;
    double transparency = 0.0;
    double refractiveIndex = 1.0;
};

enum class HitType : unsigned char { NONE, SPHERE, PLANE, TRIANGLE };

struct HitInfo {
    HitType type;
    double distance;
    size_t index;
    Material material;
    Vec3 normal;
    Vec3 hitPoint;

    bool isCloserThan(const HitInfo& other) const { return distance < other.distance; }
    double normalizedDistance(const Camera& camera) const {
        return (distance - camera.nearPlaneDistance) /
               (camera.farPlaneDistance - camera.nearPlaneDistance);
    }
    static HitInfo getClosestIntersection(const std::vector<HitInfo>& hits) {
        HitInfo best = hits[0];
        for (const HitInfo& h : hits)
            if (h.isCloserThan(best)) best = h;
        return best;
    }
};

class Sphere {
    double radius;
    Transform transform;
    Material material;

public:
    explicit Sphere(double r = 1.0, const Vec3& pos = Vec3(0, 0, 0), const Material& mat = Material())
        : radius(r), transform{pos, Vec3(0, 0, 0), Vec3(1, 1, 1)}, material(mat) {}

    // quadratic root selection of Shape.h:72-98 (near root, else far root, eps 1e-6)
    std::optional<double> Intersect(const Rayon& ray) const {
        const Vec3 oc = ray.origin - transform.position;
        const double a = ray.direction.dot(ray.direction);
        const double b = 2.0 * oc.dot(ray.direction);
        const double c = oc.dot(oc) - radius * radius;
        const double disc = b * b - 4.0 * a * c;
        if (disc < 0.0) return std::nullopt;
        const double root = std::sqrt(disc);
        double t0 = (-b - root) / (2.0 * a);
        double t1 = (-b + root) / (2.0 * a);
        if (t0 > t1) std::swap(t0, t1);
        double t = t0;  // a NaN root is returned as a hit, as in the reference
        if (t < 1e-6) {
            t = t1;
            if (t < 1e-6) return std::nullopt;
        }
        return t;
    }
    std::optional<Vec3> GetNormalAt(const Vec3& point) const {
        return (point - transform.position).normalize();
    }
    std::optional<HitInfo> GetHitInfoAt(const Rayon& ray, size_t index) const {
        const auto t = Intersect(ray);
        if (!t) return std::nullopt;
        const Vec3 p = ray.pointAtDistance(*t);
        return HitInfo{HitType::SPHERE, *t, index, material, *GetNormalAt(p), p};
    }
    double getRadius() const { return radius; }
    void setRadius(double r) { radius = r; }
    Material getMaterial() const { return material; }
    Transform getTransform() const { return transform; }
    static Sphere getHitObject(const HitInfo& hit, const std::vector<Sphere>& spheres) {
        return spheres[hit.index];
    }
};

class Plane {
    Vec3 normal;
    Transform transform;
    Material material;

public:
    // the constructor stores the normalized normal (Shape.h:141-142)
    Plane(const Vec3& pos = Vec3(0, 1, 0), const Vec3& norm = Vec3(0, 1, 0),
          const Material& mat = Material())
        : normal(norm.normalize()), transform{pos, Vec3(0, 0, 0), Vec3(1, 1, 1)}, material(mat) {}

    std::optional<double> Intersect(const Rayon& ray) const {
        const double denom = normal.dot(ray.direction);
        if (!(std::abs(denom) > 1e-6)) return std::nullopt;
        const double t = (transform.position - ray.origin).dot(normal) / denom;
        if (t >= 0.0) return t;
        return std::nullopt;
    }
    Vec3 GetNormalAt() const { return normal; }
    std::optional<HitInfo> GetHitInfoAt(const Rayon& ray, size_t index) const {
        const auto t = Intersect(ray);
        if (!t) return std::nullopt;
        return HitInfo{HitType::PLANE, *t, index, material, normal, ray.pointAtDistance(*t)};
    }
    Vec3 GetNormal() const { return normal; }
    void SetNormal(const Vec3& n) { normal = n.normalize(); }
    Material GetMaterial() const { return material; }
    Transform GetTransform() const { return transform; }
};

class Triangle {
    Vec3 v0, v1, v2;
    Transform transform;
    Material material;

public:
    Triangle(const Vec3& a, const Vec3& b, const Vec3& c, const Material& mat = Material(),
             const Transform& t = Transform())
        : v0(a), v1(b), v2(c), transform(t), material(mat) {}

    // translated vertices (Shape.h:198-200)
    Vec3 tv0() const { return v0 + transform.position; }
    Vec3 tv1() const { return v1 + transform.position; }
    Vec3 tv2() const { return v2 + transform.position; }

    // Möller–Trumbore, Shape.h:202-220
    std::optional<double> Intersect(const Rayon& ray) const {
        const Vec3 a0 = tv0();
        const Vec3 e1 = tv1() - a0;
        const Vec3 e2 = tv2() - a0;
        const Vec3 h = ray.direction.cross(e2);
        const double det = e1.dot(h);
        if (det > -1e-6 && det < 1e-6) return std::nullopt;
        const double f = 1.0 / det;
        const Vec3 s = ray.origin - a0;
        const double u = f * s.dot(h);
        if (u < 0.0 || u > 1.0) return std::nullopt;
        const Vec3 q = s.cross(e1);
        const double v = f * ray.direction.dot(q);
        if (v < 0.0 || u + v > 1.0) return std::nullopt;
        const double t = f * e2.dot(q);
        if (t > 1e-6) return t;
        return std::nullopt;
    }
    // normal of the untranslated triangle (Shape.h:222-227)
    std::optional<Vec3> GetNormalAt() const { return (v1 - v0).cross(v2 - v0).normalize(); }
    std::optional<HitInfo> GetHitInfoAt(const Rayon& ray, size_t index) const {
        const auto t = Intersect(ray);
        if (!t) return std::nullopt;
        return HitInfo{HitType::TRIANGLE, *t, index, material, *GetNormalAt(),
                       ray.pointAtDistance(*t)};
    }
    Material GetMaterial() const { return material; }

    // access for the flattening into rt_triangle records
    const Vec3& vertex(int i) const { return i == 0 ? v0 : (i == 1 ? v1 : v2); }
    const Transform& transformRef() const { return transform; }
};

class Model {
    std::vector<int> vertices;
    std::vector<Vec3> vertexPositions;
    Transform transform;
    Material material;

public:
    Model(const std::vector<int>& vertices_, const Transform& transform_ = Transform(),
          const Material& material_ = Material(),
          const std::vector<Vec3>& vertexPositions_ = std::vector<Vec3>())
        : vertices(vertices_), vertexPositions(vertexPositions_), transform(transform_),
          material(material_) {}

    std::vector<Triangle> GetTrianglesFromModel(const Material& overrideMaterial) const {
        std::vector<Triangle> out;
        out.reserve(vertices.size() / 3);
        for (size_t i = 0; i + 2 < vertices.size(); i += 3)
            out.emplace_back(vertexPositions[vertices[i]], vertexPositions[vertices[i + 1]],
                             vertexPositions[vertices[i + 2]], overrideMaterial, transform);
        return out;
    }
    // every triangle carries the model's material and transform (Shape.h:269-283)
    std::optional<HitInfo> GetHitInfoAt(const Rayon& ray, size_t index) const {
        std::optional<HitInfo> best;
        for (const Triangle& t : GetTrianglesFromModel(material)) {
            auto h = t.GetHitInfoAt(ray, index);
            if (h && (!best || h->isCloserThan(*best))) best = h;
        }
        return best;
    }
    std::optional<double> Intersect(const Rayon& ray) const {
        std::optional<double> best;
        for (const Triangle& t : GetTrianglesFromModel(material)) {
            auto d = t.Intersect(ray);
            if (d && (!best || *d < *best)) best = d;
        }
        return best;
    }
    Transform GetTransform() const { return transform; }
    Material GetMaterial() const { return material; }
    void SetTransform(const Transform& t) { transform = t; }
    void SetMaterial(const Material& m) { material = m; }
};
