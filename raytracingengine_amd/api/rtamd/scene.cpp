// rtamd/scene.cpp — Scene methods over the C-ABI (see scene.hpp for the mapping).
#include "rtamd/scene.hpp"

#include <cstring>
#include <map>
#include <stdexcept>
#include <string>

namespace rtamd {

void check(rt_status st, const char* what) {
    if (st != RT_OK) throw std::runtime_error(std::string(what) + ": " + rt_last_error());
}

namespace {
struct ThreadContexts {
    std::map<int, rt_context*> by_device;
    ~ThreadContexts() {
        for (auto& kv : by_device) rt_context_destroy(kv.second);
    }
};
thread_local ThreadContexts t_contexts;
thread_local int t_device = 0;  // the device this thread's last Scene render ran on

void put3(double* d, const Vec3& v) {
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
}
rt_material material_desc(const Material& m) {
    rt_material o;
    put3(o.color, m.color);
    o.shininess = m.shininess;
    o.specular = m.specular;
    o.transparency = m.transparency;
    o.refractive_index = m.refractiveIndex;
    return o;
}
}  // namespace

int current_device() { return t_device; }

rt_context* thread_context(int device) {
    auto it = t_contexts.by_device.find(device);
    if (it != t_contexts.by_device.end()) return it->second;
    rt_context* ctx = nullptr;
    check(rt_context_create(device, &ctx), "rt_context_create");
    t_contexts.by_device[device] = ctx;
    return ctx;
}

// A Scene's upload on one device; remembers which Scene version it holds.
struct SceneDevice {
    int device = -1;
    rt_context* ctx = nullptr;
    rt_scene* scene = nullptr;
    uint64_t version = 0;
    std::vector<long> triangle_owner;  // flat triangle -> -1 (standalone) or model index
    std::vector<size_t> triangle_local;  // flat triangle -> index within its owner list
    ~SceneDevice() {
        if (scene) rt_scene_destroy(scene);
    }
};

}  // namespace rtamd

Scene::Scene(const Camera& camera_) : camera(camera_) {}

rt_camera Scene::cameraDesc() const {
    rt_camera c;
    std::memset(&c, 0, sizeof c);
    c.position[0] = camera.position.x;
    c.position[1] = camera.position.y;
    c.position[2] = camera.position.z;
    c.focal = camera.focal;
    c.width = static_cast<uint32_t>(camera.width);
    c.height = static_cast<uint32_t>(camera.height);
    c.aa_samples = camera.antiAliasingAmount;
    c.near_plane = camera.nearPlaneDistance;
    c.far_plane = camera.farPlaneDistance;
    return c;
}

rt_render_opts Scene::optsDesc(int tonemap) const {
    rt_render_opts o;
    rt_render_opts_default(&o);
    o.max_recursion = maxRecursion;
    o.tonemap = tonemap;
    o.seed = camera.jitterSeed;
    return o;
}

rt_scene* Scene::upload() const {
    rtamd::t_device = device_;
    if (dev_ && dev_->version == version_ && dev_->device == device_) return dev_->scene;
    dev_ = uploadTo(device_);
    return dev_->scene;
}

std::shared_ptr<rtamd::SceneDevice> Scene::uploadTo(int device) const {
    using namespace rtamd;
    auto sd = std::make_shared<SceneDevice>();
    sd->device = device;
    sd->ctx = thread_context(device);

    std::vector<rt_sphere> sp(spheres.size());
    for (size_t i = 0; i < spheres.size(); ++i) {
        put3(sp[i].center, spheres[i].getTransform().position);
        sp[i].radius = spheres[i].getRadius();
        sp[i].material = material_desc(spheres[i].getMaterial());
    }
    std::vector<rt_plane> pl(planes.size());
    for (size_t i = 0; i < planes.size(); ++i) {
        put3(pl[i].point, planes[i].GetTransform().position);
        put3(pl[i].normal, planes[i].GetNormal());
        pl[i].material = material_desc(planes[i].GetMaterial());
    }
    // standalone triangles first, then each model's triangles (IntersectClosest order)
    std::vector<rt_triangle> tr;
    auto push_tri = [&](const Triangle& t, long owner, size_t local) {
        rt_triangle r;
        put3(r.v0, t.vertex(0));
        put3(r.v1, t.vertex(1));
        put3(r.v2, t.vertex(2));
        put3(r.translation, t.transformRef().position);
        r.material = material_desc(t.GetMaterial());
        tr.push_back(r);
        sd->triangle_owner.push_back(owner);
        sd->triangle_local.push_back(local);
    };
    for (size_t i = 0; i < triangles.size(); ++i) push_tri(triangles[i], -1, i);
    for (size_t m = 0; m < models.size(); ++m) {
        const auto tris = models[m].GetTrianglesFromModel(models[m].GetMaterial());
        for (size_t k = 0; k < tris.size(); ++k) push_tri(tris[k], static_cast<long>(m), k);
    }
    std::vector<rt_light> lt(lights.size());
    for (size_t i = 0; i < lights.size(); ++i) {
        put3(lt[i].position, lights[i].position);
        put3(lt[i].color, lights[i].color);
        lt[i].intensity = lights[i].intensity;
    }
    rt_scene_desc d;
    d.spheres = sp.data();
    d.n_spheres = static_cast<int32_t>(sp.size());
    d.planes = pl.data();
    d.n_planes = static_cast<int32_t>(pl.size());
    d.triangles = tr.data();
    d.n_triangles = static_cast<int32_t>(tr.size());
    d.lights = lt.data();
    d.n_lights = static_cast<int32_t>(lt.size());
    check(rt_scene_create(sd->ctx, &d, &sd->scene), "rt_scene_create");
    if (areaLight_) check(rt_scene_set_area_light(sd->scene, &*areaLight_), "rt_scene_set_area_light");
    sd->version = version_;
    return sd;
}

bool Scene::renderMulti(const rt_render_opts& o, double* h64, float* h32, uint8_t* h8) const {
    if (devices_.size() < 2) return false;
    if (multi_.size() != devices_.size()) multi_.assign(devices_.size(), nullptr);
    std::vector<rt_context*> ctxs;
    std::vector<rt_scene*> scs;
    for (size_t i = 0; i < devices_.size(); ++i) {
        if (!multi_[i] || multi_[i]->version != version_ || multi_[i]->device != devices_[i])
            multi_[i] = uploadTo(devices_[i]);
        ctxs.push_back(multi_[i]->ctx);
        scs.push_back(multi_[i]->scene);
    }
    const rt_camera cam = cameraDesc();
    rtamd::check(rt_render_multi(ctxs.data(), scs.data(), static_cast<int>(ctxs.size()), &cam,
                                 &o, h64, h32, h8, countRays_ ? &lastStats_ : nullptr),
                 "rt_render_multi");
    return true;
}

std::vector<Vec3> Scene::RenderImage() const {
    const rt_render_opts o = optsDesc(RT_TONEMAP_NONE);
    std::vector<Vec3> img(camera.width * camera.height, Vec3(0, 0, 0));
    if (renderMulti(o, reinterpret_cast<double*>(img.data()), nullptr, nullptr)) return img;
    rt_scene* sc = upload();
    const rt_camera cam = cameraDesc();
    // Vec3 is three packed doubles: the device writes the reference's vector<Vec3> layout.
    rtamd::check(rt_render(dev_->ctx, sc, &cam, &o, reinterpret_cast<double*>(img.data()), nullptr,
                           nullptr, countRays_ ? &lastStats_ : nullptr),
                 "rt_render");
    return img;
}

std::vector<Color> Scene::RenderImageTonemapped(int op) const {
    const rt_render_opts o = optsDesc(op);
    std::vector<Color> img(camera.width * camera.height);
    if (renderMulti(o, nullptr, nullptr, reinterpret_cast<uint8_t*>(img.data()))) return img;
    rt_scene* sc = upload();
    const rt_camera cam = cameraDesc();
    rtamd::check(rt_render(dev_->ctx, sc, &cam, &o, nullptr, nullptr,
                           reinterpret_cast<uint8_t*>(img.data()), countRays_ ? &lastStats_ : nullptr),
                 "rt_render");
    return img;
}

std::vector<float> Scene::RenderImageF32() const {
    const rt_render_opts o = optsDesc(RT_TONEMAP_NONE);
    std::vector<float> img(camera.width * camera.height * 3);
    if (renderMulti(o, nullptr, img.data(), nullptr)) return img;
    rt_scene* sc = upload();
    const rt_camera cam = cameraDesc();
    rtamd::check(rt_render(dev_->ctx, sc, &cam, &o, nullptr, img.data(), nullptr, countRays_ ? &lastStats_ : nullptr),
                 "rt_render");
    return img;
}

Vec3 Scene::GeneratePixelAt(int x, int y) const {
    if (x < 0 || y < 0 || static_cast<size_t>(x) >= camera.width ||
        static_cast<size_t>(y) >= camera.height)
        throw std::out_of_range("GeneratePixelAt: pixel outside the image");
    rt_scene* sc = upload();
    const rt_camera cam = cameraDesc();
    rt_render_opts o = optsDesc(RT_TONEMAP_NONE);
    o.row_begin = static_cast<uint32_t>(y);
    o.row_end = static_cast<uint32_t>(y) + 1;
    std::vector<Vec3> row(camera.width, Vec3(0, 0, 0));
    rtamd::check(rt_render(dev_->ctx, sc, &cam, &o, reinterpret_cast<double*>(row.data()),
                           nullptr, nullptr, nullptr),
                 "rt_render");
    return row[static_cast<size_t>(x)];
}

std::optional<Vec3> Scene::GenerateAntiAliasing(size_t x, size_t y, bool isActive,
                                                double bias) const {
    rt_scene* sc = upload();
    const Rayon ray = camera.getRay(x, y, isActive);
    const double r[6] = {ray.origin.x, ray.origin.y, ray.origin.z,
                         ray.direction.x, ray.direction.y, ray.direction.z};
    rt_render_opts o = optsDesc(RT_TONEMAP_NONE);
    o.bias = bias;
    double rgb[3];
    rtamd::check(rt_trace_rays(dev_->ctx, sc, &o, r, 1, rgb, nullptr), "rt_trace_rays");
    return Vec3(rgb[0], rgb[1], rgb[2]);
}

std::optional<HitInfo> Scene::IntersectClosest(const Rayon& ray) const {
    rt_scene* sc = upload();
    const double r[6] = {ray.origin.x, ray.origin.y, ray.origin.z,
                         ray.direction.x, ray.direction.y, ray.direction.z};
    double h[9];
    rtamd::check(rt_intersect_rays(dev_->ctx, sc, r, 1, h), "rt_intersect_rays");
    const int type = static_cast<int>(h[0]);
    if (type == 0) return std::nullopt;
    const size_t idx = static_cast<size_t>(h[1]);
    const Material none;
    HitInfo hit{HitType::NONE, h[2], idx, none, Vec3(h[3], h[4], h[5]), Vec3(h[6], h[7], h[8])};
    if (type == 1) {
        hit.type = HitType::SPHERE;
        hit.material = spheres[idx].getMaterial();
    } else if (type == 2) {
        hit.type = HitType::PLANE;
        hit.material = planes[idx].GetMaterial();
    } else {
        hit.type = HitType::TRIANGLE;
        const long owner = dev_->triangle_owner[idx];
        if (owner < 0) {
            hit.index = dev_->triangle_local[idx];
            hit.material = triangles[hit.index].GetMaterial();
        } else {  // the reference reports the model's index for model hits (Scene.h:251-253)
            hit.index = static_cast<size_t>(owner);
            hit.material = models[hit.index].GetMaterial();
        }
    }
    return hit;
}

bool Scene::IntersectAnyBefore(const Rayon& ray, double maxDist) const {
    auto within = [&](const std::optional<double>& d) { return d && *d > 0.0 && *d < maxDist; };
    for (const auto& s : spheres)
        if (within(s.Intersect(ray))) return true;
    for (const auto& p : planes)
        if (within(p.Intersect(ray))) return true;
    for (const auto& t : triangles)
        if (within(t.Intersect(ray))) return true;
    for (const auto& m : models)
        if (within(m.Intersect(ray))) return true;
    return false;
}

std::optional<HitInfo> Scene::CalculatePixelDepth(size_t x, size_t y, bool aa) const {
    return IntersectClosest(camera.getRay(x, y, aa));
}
