// examples/render_scenefile.cpp — exercises every GPU-backed entry of the drop-in C++ API on a
// scene file (raytracingengine_amd/scene.py format) and dumps the results for the parity tests
// (tests/test_gpu_cpp_api.py):
//   hdr.f64      Scene::RenderImage()
//   fused1.u8    Scene::RenderImageTonemapped(RT_TONEMAP_REINHARD)
//   tmall.u8     rtamd::tonemapAll(hdr)     (7 planes)     tmaces.u8  rtamd::tonemap(hdr)
//   probe.f64    per probe pixel: GeneratePixelAt (3), GenerateAntiAliasing (3),
//                CalculatePixelDepth/IntersectClosest (9: type, index, distance, n, p)
//   image.ppm    writePPM of the fused image
//   stats.txt    "<trace rays> <shadow rays>"
//   closest.f64  with a third argument <rays.f64>: Scene::IntersectClosest per ray (n*9)
#include <cstdio>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "Image.h"
#include "Scene.h"
#include "rtamd/scenefile.hpp"

template <class T>
static void dump(const std::string& path, const T* p, size_t n) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), static_cast<std::streamsize>(n * sizeof(T)));
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::cerr << "usage: render_scenefile <scene.txt> <outdir>\n";
        return 2;
    }
    const std::string out = argv[2];
    try {
        const rtamd::LoadedScene L = rtamd::load_scene_file(argv[1]);
        Scene scene = L.build();
        scene.SetCountRays(true);
        const size_t W = L.camera.width, H = L.camera.height;

        const std::vector<Vec3> hdr = scene.RenderImage();
        dump(out + "/hdr.f64", reinterpret_cast<const double*>(hdr.data()), hdr.size() * 3);
        const rt_stats st = scene.LastStats();
        std::ofstream(out + "/stats.txt") << st.trace_rays << " " << st.shadow_rays << "\n";

        const std::vector<Color> fused = scene.RenderImageTonemapped(RT_TONEMAP_REINHARD);
        dump(out + "/fused1.u8", reinterpret_cast<const uint8_t*>(fused.data()), fused.size() * 3);
        writePPM(out + "/image.ppm", fused, W, H);

        const auto all = rtamd::tonemapAll(hdr);
        std::vector<uint8_t> planes;
        for (const auto& img : all)
            planes.insert(planes.end(), reinterpret_cast<const uint8_t*>(img.data()),
                          reinterpret_cast<const uint8_t*>(img.data()) + img.size() * 3);
        dump(out + "/tmall.u8", planes.data(), planes.size());
        const auto aces = rtamd::tonemap(hdr);
        dump(out + "/tmaces.u8", reinterpret_cast<const uint8_t*>(aces.data()), aces.size() * 3);

        const size_t probes[][2] = {{0, 0}, {W - 1, 0}, {W / 2, H / 2}, {W / 3, 2 * H / 3}, {W - 1, H - 1}};
        std::vector<double> pr;
        for (const auto& q : probes) {
            const Vec3 px = scene.GeneratePixelAt(static_cast<int>(q[0]), static_cast<int>(q[1]));
            const Vec3 one = *scene.GenerateAntiAliasing(q[0], q[1], false, 1e-3);
            const auto hit = scene.CalculatePixelDepth(q[0], q[1], false);
            pr.insert(pr.end(), {px.x, px.y, px.z, one.x, one.y, one.z});
            if (hit)
                pr.insert(pr.end(), {double(static_cast<int>(hit->type)), double(hit->index),
                                     hit->distance, hit->normal.x, hit->normal.y, hit->normal.z,
                                     hit->hitPoint.x, hit->hitPoint.y, hit->hitPoint.z});
            else
                pr.insert(pr.end(), {0.0, -1.0, 0, 0, 0, 0, 0, 0, 0});
        }
        dump(out + "/probe.f64", pr.data(), pr.size());

        if (argc > 3) {
            std::ifstream rf(argv[3], std::ios::binary | std::ios::ate);
            const size_t n = static_cast<size_t>(rf.tellg()) / (6 * sizeof(double));
            rf.seekg(0);
            std::vector<double> rays(6 * n), hits;
            rf.read(reinterpret_cast<char*>(rays.data()), static_cast<std::streamsize>(rays.size() * 8));
            for (size_t i = 0; i < n; ++i) {
                const double* r = &rays[6 * i];
                const auto h = scene.IntersectClosest(Rayon(Vec3(r[0], r[1], r[2]), Vec3(r[3], r[4], r[5])));
                if (h)
                    hits.insert(hits.end(), {double(static_cast<int>(h->type)), double(h->index),
                                             h->distance, h->normal.x, h->normal.y, h->normal.z,
                                             h->hitPoint.x, h->hitPoint.y, h->hitPoint.z});
                else
                    hits.insert(hits.end(), {0.0, -1.0, 0, 0, 0, 0, 0, 0, 0});
            }
            dump(out + "/closest.f64", hits.data(), hits.size());
        }
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << "\n";
        return 1;
    }
    return 0;
}
