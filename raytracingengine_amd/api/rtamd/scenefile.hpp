// rtamd/scenefile.hpp — load the line-oriented scene format written by
// raytracingengine_amd/scene.py (SceneData.to_text) into a drop-in Scene.
//
//   camera px py pz focal width height near far aa
//   sphere cx cy cz radius  r g b shininess specular transparency ior
//   plane  px py pz nx ny nz  <material>
//   triangle v0(3) v1(3) v2(3) translation(3) <material>
//   model  ntri tx ty tz <material>   followed by ntri lines "v x0 y0 z0 x1 y1 z1 x2 y2 z2"
//   light  px py pz r g b intensity
// Doubles are parsed with strtod, so repr()-formatted values round-trip exactly.
#pragma once

#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "rtamd/scene.hpp"

namespace rtamd {

struct LoadedScene {
    Camera camera{Vec3(0, 0, 0)};
    std::vector<Sphere> spheres;
    std::vector<Plane> planes;
    std::vector<Triangle> triangles;
    std::vector<Model> models;
    std::vector<Light> lights;

    Scene build() const {
        Scene s(camera);
        for (const auto& x : spheres) s.AddSphere(x);
        for (const auto& x : planes) s.AddPlane(x);
        for (const auto& x : triangles) s.AddTriangle(x);
        for (const auto& x : models) s.AddModel(x);
        for (const auto& x : lights) s.AddLight(x);
        return s;
    }
};

inline LoadedScene load_scene_file(const std::string& path) {
    std::ifstream in(path);
    if (!in) throw std::runtime_error("cannot open scene file " + path);
    auto num = [](std::istringstream& s) {
        std::string tok;
        if (!(s >> tok)) throw std::runtime_error("scene file: missing number");
        return std::stod(tok);
    };
    auto vec = [&](std::istringstream& s) {
        const double x = num(s), y = num(s), z = num(s);
        return Vec3(x, y, z);
    };
    auto mat = [&](std::istringstream& s) {
        Material m;
        m.color = vec(s);
        m.shininess = num(s);
        m.specular = num(s);
        m.transparency = num(s);
        m.refractiveIndex = num(s);
        return m;
    };
    LoadedScene L;
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream s(line);
        std::string tag;
        s >> tag;
        if (tag == "camera") {
            const Vec3 p = vec(s);
            const double focal = num(s);
            const auto w = static_cast<size_t>(num(s)), h = static_cast<size_t>(num(s));
            const double nearp = num(s), farp = num(s);
            L.camera = Camera(p, focal, w, h, nearp, farp);
            L.camera.antiAliasingAmount = static_cast<int>(num(s));
        } else if (tag == "sphere") {
            const Vec3 c = vec(s);
            const double r = num(s);
            L.spheres.emplace_back(r, c, mat(s));
        } else if (tag == "plane") {
            const Vec3 p = vec(s), n = vec(s);
            L.planes.emplace_back(p, n, mat(s));
        } else if (tag == "triangle") {
            const Vec3 a = vec(s), b = vec(s), c = vec(s), t = vec(s);
            const Material m = mat(s);
            L.triangles.emplace_back(a, b, c, m, Transform{t, Vec3(0, 0, 0), Vec3(1, 1, 1)});
        } else if (tag == "model") {
            const auto n = static_cast<size_t>(num(s));
            const Vec3 t = vec(s);
            const Material m = mat(s);
            std::vector<Vec3> pos;
            std::vector<int> idx;
            for (size_t i = 0; i < n; ++i) {
                if (!std::getline(in, line)) throw std::runtime_error("scene file: short model");
                std::istringstream v(line);
                std::string vt;
                v >> vt;
                for (int k = 0; k < 3; ++k) {
                    pos.push_back(vec(v));
                    idx.push_back(static_cast<int>(pos.size()) - 1);
                }
            }
            L.models.emplace_back(idx, Transform{t, Vec3(0, 0, 0), Vec3(1, 1, 1)}, m, pos);
        } else if (tag == "light") {
            const Vec3 p = vec(s), c = vec(s);
            const double i = num(s);
            L.lights.emplace_back(p, c, i);
        }
    }
    return L;
}

}  // namespace rtamd
