// tests/sanitize/san_main.cpp — host-code driver for the AddressSanitizer / UBSan build
// (tests/test_sanitizers.py).  Exercises the host code on the path that runs outside the GPU:
//   bvh <tri.bin> <n>          rtamd::build_triangle_bvh (csrc/rt_bvh.cpp) + structure checks
//   chunks <sph.bin> <n>       rtamd::build_sphere_chunks (csrc/rt_bvh.cpp) + containment checks
//   obj <file.obj>             rtamd::LoadObject (api/rtamd/obj.cpp)
//   scene <file.txt>           rtamd::load_scene_file (api/rtamd/scenefile.hpp)
//   oracle <dir> <rows>        oracle_render / tonemap / KAT entry points (oracle/rt_oracle.c)
// Exit 0 = every check held; sanitizer reports abort the process (halt_on_error).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_internal.hpp"
#include "rt_oracle.h"
#include "rtamd/obj.hpp"
#include "rtamd/scenefile.hpp"

namespace {

std::vector<char> slurp(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return {};
    return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

int fail(const char* what) {
    std::fprintf(stderr, "CHECK FAILED: %s\n", what);
    return 1;
}

int run_bvh(const std::string& path, int nt) {
    std::vector<char> raw = slurp(path);
    if (raw.size() != size_t(nt) * rtamd::kTriStride * sizeof(double)) return fail("tri size");
    std::vector<double> tri(raw.size() / sizeof(double));
    std::memcpy(tri.data(), raw.data(), raw.size());
    std::vector<double> nodes;
    std::vector<int32_t> order;
    rtamd::build_triangle_bvh(tri.data(), nt, nodes, order);
    if (nt == 0) return nodes.empty() && order.empty() ? 0 : fail("empty build");
    if (order.size() != size_t(nt)) return fail("order size");
    std::vector<int> seen(static_cast<size_t>(nt), 0);
    for (int32_t t : order) {
        if (t < 0 || t >= nt) return fail("order index");
        seen[static_cast<size_t>(t)]++;
    }
    for (int s : seen)
        if (s != 1) return fail("triangle not exactly once");
    const size_t nn = nodes.size() / rtamd::kBvhNodeStride;
    size_t leaf_tris = 0;
    for (size_t i = 0; i < nn; ++i) {
        const double* n = &nodes[i * rtamd::kBvhNodeStride];
        int32_t fc[2];
        std::memcpy(fc, &n[6], sizeof fc);
        for (int k = 0; k < 3; ++k)
            if (!(n[k] <= n[3 + k])) return fail("box lo > hi");
        if (fc[1] == 0) {
            if (fc[0] < 1 || size_t(fc[0]) + 1 >= nn + 1) return fail("child index");
            for (int c = 0; c < 2; ++c) {
                const double* ch = &nodes[size_t(fc[0] + c) * rtamd::kBvhNodeStride];
                for (int k = 0; k < 3; ++k)
                    if (ch[k] < n[k] || ch[3 + k] > n[3 + k]) return fail("child outside parent");
            }
        } else {
            if (fc[0] < 0 || fc[1] < 0 || size_t(fc[0]) + size_t(fc[1]) > order.size())
                return fail("leaf range");
            leaf_tris += size_t(fc[1]);
            for (int32_t j = fc[0]; j < fc[0] + fc[1]; ++j) {  // leaf box holds its triangles
                const double* t = &tri[size_t(order[size_t(j)]) * rtamd::kTriStride];
                for (int k = 0; k < 3; ++k) {
                    const double v[3] = {t[k], t[k] + t[3 + k], t[k] + t[6 + k]};
                    for (double x : v)
                        if (std::isfinite(x) && (x < n[k] || x > n[3 + k])) return fail("leaf box");
                }
            }
        }
    }
    if (leaf_tris != size_t(nt)) return fail("leaf triangle count");
    std::printf("bvh %d triangles, %zu nodes\n", nt, nn);
    return 0;
}

int run_obj(const std::string& path) {
    try {
        const Model m = rtamd::LoadObject(path);
        const auto tris = m.GetTrianglesFromModel(Material());
        std::printf("obj %zu triangles\n", tris.size());
    } catch (const std::runtime_error& e) {
        std::printf("obj error: %s\n", e.what());  // the reference's own failure mode
    }
    return 0;
}

int run_scene(const std::string& path) {
    try {
        const rtamd::LoadedScene L = rtamd::load_scene_file(path);
        std::printf("scene %zu spheres %zu planes %zu triangles %zu models %zu lights\n",
                    L.spheres.size(), L.planes.size(), L.triangles.size(), L.models.size(),
                    L.lights.size());
    } catch (const std::exception& e) {
        std::printf("scene error: %s\n", e.what());
    }
    return 0;
}

template <typename T>
std::vector<T> records(const std::string& dir, const char* name) {
    std::vector<char> raw = slurp(dir + "/" + name);
    std::vector<T> v(raw.size() / sizeof(T));
    if (!v.empty()) std::memcpy(v.data(), raw.data(), v.size() * sizeof(T));
    return v;
}

int run_oracle(const std::string& dir, uint32_t rows) {
    const auto sp = records<o_sphere>(dir, "spheres.bin");
    const auto pl = records<o_plane>(dir, "planes.bin");
    const auto tr = records<o_triangle>(dir, "triangles.bin");
    const auto lt = records<o_light>(dir, "lights.bin");
    const auto cams = records<o_camera>(dir, "camera.bin");
    const auto area = records<o_area_light>(dir, "area.bin");
    if (cams.size() != 1) return fail("camera");
    o_scene sc{sp.data(), int32_t(sp.size()), pl.data(), int32_t(pl.size()),
               tr.data(), int32_t(tr.size()), lt.data(), int32_t(lt.size())};
    const o_camera cam = cams[0];
    rows = std::min(rows, cam.height);
    o_opts opt{10, 1, 1e-3, 0x5EED, 0, rows, area.empty() ? nullptr : area.data()};
    std::vector<double> img(size_t(rows) * cam.width * 3);
    uint64_t nt = 0, ns = 0;
    if (oracle_render(&sc, &cam, &opt, img.data(), &nt, &ns) != 0) return fail("oracle_render");
    std::vector<uint8_t> ldr(img.size());
    for (int op = 0; op < 7; ++op)
        if (oracle_tonemap(img.data(), img.size() / 3, op, ldr.data()) != 0) return fail("tonemap");
    // per-function entry points on rays through the rendered rows
    double acc = 0;
    for (uint32_t y = 0; y < rows; y += 3)
        for (uint32_t x = 0; x < cam.width; x += 7) {
            double ray[6], hit[7];
            oracle_get_ray(&cam, x, y, 1, 7, 1, ray);
            int32_t idx = -1;
            const int type = oracle_closest(&sc, ray, hit, &idx);
            if (type != 0) acc += hit[0];
            acc += oracle_transmittance(&sc, ray, 50.0, 1e-3);
            double t;
            if (!sp.empty() && oracle_sphere_intersect(ray, &sp[x % sp.size()], &t)) acc += t;
            if (!pl.empty() && oracle_plane_intersect(ray, &pl[x % pl.size()], &t)) acc += t;
            if (!tr.empty() && oracle_triangle_intersect(ray, &tr[x % tr.size()], &t)) acc += t;
        }
    std::printf("oracle %u rows, %llu + %llu rays, checksum %.6g\n", rows,
                static_cast<unsigned long long>(nt), static_cast<unsigned long long>(ns), acc);
    std::FILE* f = std::fopen((dir + "/out.f64").c_str(), "wb");
    if (!f) return fail("open out.f64");
    const size_t w = std::fwrite(img.data(), sizeof(double), img.size(), f);
    std::fclose(f);
    return w == img.size() ? 0 : fail("write out.f64");
}

// The spatial sphere chunks of the packet kernel: a permutation, every sphere once, and each
// 64-sphere chunk's bounding sphere containing every member sphere (or infinite).
int run_chunks(const std::string& path, int ns) {
    std::vector<char> raw = slurp(path);
    if (raw.size() != size_t(ns) * rtamd::kSphStride * sizeof(double)) return fail("sph size");
    std::vector<double> sph(raw.size() / sizeof(double));
    std::memcpy(sph.data(), raw.data(), raw.size());
    std::vector<int32_t> perm;
    std::vector<double> bnd;
    rtamd::build_sphere_chunks(sph.data(), ns, perm, bnd);
    if (perm.size() != size_t(ns)) return fail("perm size");
    const size_t nb = (size_t(ns) + 63) / 64;
    if (bnd.size() != nb * 4) return fail("bounds size");
    std::vector<int> seen(static_cast<size_t>(ns), 0);
    for (int32_t i : perm) {
        if (i < 0 || i >= ns) return fail("perm index");
        seen[static_cast<size_t>(i)]++;
    }
    for (int s : seen)
        if (s != 1) return fail("sphere not exactly once");
    for (size_t c = 0; c < nb; ++c) {
        const double* b = &bnd[c * 4];
        for (size_t j = c * 64; j < std::min(size_t(ns), c * 64 + 64); ++j) {
            const double* s = &sph[size_t(perm[j]) * rtamd::kSphStride];
            const double r = std::sqrt(s[3]);
            if (std::isinf(b[3]) && b[3] > 0) continue;
            const double dx = s[0] - b[0], dy = s[1] - b[1], dz = s[2] - b[2];
            if (!(std::sqrt(dx * dx + dy * dy + dz * dz) + r <= b[3])) return fail("sphere outside its chunk bound");
        }
    }
    std::printf("chunks %d spheres %zu chunks\n", ns, nb);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: san_main bvh|obj|scene|oracle ...\n");
        return 2;
    }
    const std::string mode = argv[1];
    if (mode == "bvh" && argc == 4) return run_bvh(argv[2], std::atoi(argv[3]));
    if (mode == "chunks" && argc == 4) return run_chunks(argv[2], std::atoi(argv[3]));
    if (mode == "obj") return run_obj(argv[2]);
    if (mode == "scene") return run_scene(argv[2]);
    if (mode == "oracle" && argc == 4)
        return run_oracle(argv[2], static_cast<uint32_t>(std::atoi(argv[3])));
    std::fprintf(stderr, "bad arguments\n");
    return 2;
}
