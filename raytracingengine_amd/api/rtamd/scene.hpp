// rtamd/scene.hpp — the drop-in Scene (/root/reference/RaytracingEngine/Scene.h:14-329).
//
// Same constructor, Add* methods and public query/render methods.  Every method that the
// reference evaluates per pixel runs on the MI355X through the C-ABI (include/rt_capi.h):
//   RenderImage()            → rt_render                (Scene.h:311-328)
//   GeneratePixelAt(x, y)    → rt_render of row y        (Scene.h:283-304)
//   GenerateAntiAliasing(..) → rt_trace_rays             (Scene.h:306-309)
//   IntersectClosest(ray)    → rt_intersect_rays         (Scene.h:218-257)
//   CalculatePixelDepth(..)  → rt_intersect_rays         (Scene.h:278-281)
// IntersectAnyBefore (Scene.h:259-276, unused by the reference) is a host utility over the
// shapes' Intersect members.  Failures throw std::runtime_error(rt_last_error()).
//
// The Add* methods take `const T&` — a compatible superset of the reference's `T&`.
#pragma once

#include <cstdint>
#include <memory>
#include <optional>
#include <vector>

#include "rtamd/light.hpp"
#include "rtamd/math.hpp"
#include "rt_capi.h"
#include "rtamd/shapes.hpp"

namespace rtamd {
struct SceneDevice;  // uploaded copy of a Scene on one device (scene.cpp)

// The calling thread's context for `device` (created on first use, one per thread+device).
rt_context* thread_context(int device);
// The device of this thread's last single-GPU Scene call (Scene::SetDevice; 0 before any):
// tonemap() / tonemapAll() run there, next to the frame they usually follow.
int current_device();
// Throws std::runtime_error carrying rt_last_error() when st != RT_OK.
void check(rt_status st, const char* what);
}  // namespace rtamd

class Scene {
    std::vector<Sphere> spheres;
    std::vector<Plane> planes;
    std::vector<Triangle> triangles;
    std::vector<Model> models;
    std::vector<Light> lights;

    Camera camera;
    int maxRecursion = 10;  // Scene.h:24

    // GPU side (RenderImage is const, so the upload cache is mutable)
    int device_ = 0;
    uint64_t version_ = 1;
    std::optional<rt_area_light> areaLight_;
    mutable std::shared_ptr<rtamd::SceneDevice> dev_;
    mutable rt_stats lastStats_{};
    bool countRays_ = false;

    std::vector<int> devices_;  // > 1 entries: RenderImage over these GPUs (rt_render_multi)
    mutable std::vector<std::shared_ptr<rtamd::SceneDevice>> multi_;

    rt_scene* upload() const;
    std::shared_ptr<rtamd::SceneDevice> uploadTo(int device) const;
    bool renderMulti(const rt_render_opts& o, double* h64, float* h32, uint8_t* h8) const;
    rt_camera cameraDesc() const;
    rt_render_opts optsDesc(int tonemap) const;
    void touch() { ++version_; }

public:
    explicit Scene(const Camera& camera_);

    void AddSphere(const Sphere& sphere) { spheres.emplace_back(sphere); touch(); }
    void AddPlane(const Plane& plane) { planes.emplace_back(plane); touch(); }
    void AddLight(const Light& light) { lights.emplace_back(light); touch(); }
    void AddTriangle(const Triangle& triangle) { triangles.emplace_back(triangle); touch(); }
    void AddModel(const Model& model) { models.emplace_back(model); touch(); }

    size_t GetPixelIndex(size_t x, size_t y) const { return y * camera.width + x; }

    std::optional<HitInfo> IntersectClosest(const Rayon& ray) const;
    bool IntersectAnyBefore(const Rayon& ray, double maxDist) const;
    std::optional<HitInfo> CalculatePixelDepth(size_t x, size_t y, bool aa) const;
    Vec3 GeneratePixelAt(int x, int y) const;
    std::optional<Vec3> GenerateAntiAliasing(size_t x, size_t y, bool isActive, double bias) const;
    std::vector<Vec3> RenderImage() const;

    // ---- extensions (not in the reference) -------------------------------------------
    // Render and tonemap in one launch (fused on the device; `op` is an rt_tonemap_op).
    std::vector<Color> RenderImageTonemapped(int op = RT_TONEMAP_ACES) const;
    // float32 HDR framebuffer (12 B/px) instead of the reference's FP64 Vec3 (24 B/px).
    std::vector<float> RenderImageF32() const;
    void SetDevice(int device) { device_ = device; dev_.reset(); devices_.clear(); }
    // RenderImage / RenderImageTonemapped / RenderImageF32 over several GPUs of the node from
    // this process: one scene copy per GPU, block-cyclic rows, assembled on the host (distinct
    // device ids: one context per device and thread)
    void SetDevices(const std::vector<int>& devices) { devices_ = devices; multi_.clear(); }
    void SetMaxRecursion(int depth) { maxRecursion = depth; }
    // build-defined area light (BASELINE config 5); nullopt removes it
    void SetAreaLight(const std::optional<rt_area_light>& light) { areaLight_ = light; touch(); }
    const Camera& GetCamera() const { return camera; }
    // ray counting (a second, counting launch per render; off by default)
    void SetCountRays(bool on) { countRays_ = on; }
    // ray counts of the last RenderImage* call with counting on (TraceRay reaching
    // IntersectClosest, computeTransmittance calls)
    rt_stats LastStats() const { return lastStats_; }
};
