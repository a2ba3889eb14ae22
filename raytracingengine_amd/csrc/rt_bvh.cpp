// rt_bvh.cpp — host build of the triangle BVH used by every trace kernel for scenes with many
// triangles (Model::Intersect of the reference, Shape.h:263-307, tests every triangle of every
// model for every ray; this changes how many are tested, not which hit wins — see
// rt_trace_common.hpp bvh_closest for the ordering argument).
//
// Binned SAH over triangle centroids, leaves of <= 4 triangles, depth <= 48.  Node layout (8
// doubles, 64 B): lo xyz, hi xyz, then {int32 first, int32 count} in the bits of slot 6; count
// == 0 marks an internal node whose children are nodes first and first + 1 (the child of the
// lower centroids first), and slot 7 holds its split axis (int32 0..2; the wave-coherent
// traversal of the packet kernel visits the child nearer along it first).  Boxes are widened
// by 1e-9 of their extent and coordinates plus 1e-300 so that every hit the FP64
// Möller-Trumbore test accepts lies strictly inside its leaf's box.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "rt_internal.hpp"

namespace rtamd {

namespace {

struct Box {
    double lo[3] = {INFINITY, INFINITY, INFINITY};
    double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void add(const double* p) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    void add(const Box& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    double area() const {
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (!(dx >= 0.0)) return 0.0;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct Prim {
    Box box;
    double c[3];
    int32_t idx;
};

struct Builder {
    std::vector<Prim>& prims;
    std::vector<double>& nodes;
    int32_t alloc() {
        nodes.resize(nodes.size() + kBvhNodeStride, 0.0);
        return static_cast<int32_t>(nodes.size() / kBvhNodeStride - 1);
    }
    void write(int32_t n, const Box& b, int32_t first, int32_t count, int32_t axis = 0) {
        double* o = &nodes[size_t(n) * kBvhNodeStride];
        for (int k = 0; k < 3; ++k) {
            const double m = 1e-9 * ((b.hi[k] - b.lo[k]) + std::max(std::fabs(b.lo[k]),
                                                                    std::fabs(b.hi[k]))) +
                             1e-300;
            o[k] = b.lo[k] - m;
            o[3 + k] = b.hi[k] + m;
        }
        int32_t fc[2] = {first, count};
        std::memcpy(&o[6], fc, sizeof fc);
        const int32_t ax[2] = {axis, 0};
        std::memcpy(&o[7], ax, sizeof ax);
    }
    // builds prims[b, e) into node n
    void build(int32_t n, size_t b, size_t e, int depth) {
        Box box, cbox;
        for (size_t i = b; i < e; ++i) {
            box.add(prims[i].box);
            cbox.add(prims[i].c);
        }
        const size_t count = e - b;
        if (count <= 4 || depth >= 48) {
            write(n, box, static_cast<int32_t>(b), static_cast<int32_t>(count));
            return;
        }
        // binned SAH
        constexpr int kBins = 16;
        int best_axis = -1, best_split = 0;
        double best_cost = box.area() * static_cast<double>(count);  // cost of a leaf
        for (int k = 0; k < 3; ++k) {
            const double lo = cbox.lo[k], hi = cbox.hi[k];
            if (!(hi > lo)) continue;
            Box bb[kBins];
            size_t bn[kBins] = {};
            const double scale = kBins / (hi - lo);
            for (size_t i = b; i < e; ++i) {
                int bi = static_cast<int>((prims[i].c[k] - lo) * scale);
                bi = std::min(std::max(bi, 0), kBins - 1);
                bb[bi].add(prims[i].box);
                ++bn[bi];
            }
            double right_area[kBins];
            size_t right_n[kBins];
            Box acc;
            size_t an = 0;
            for (int i = kBins - 1; i > 0; --i) {
                acc.add(bb[i]);
                an += bn[i];
                right_area[i] = acc.area();
                right_n[i] = an;
            }
            Box lacc;
            size_t ln = 0;
            for (int i = 0; i < kBins - 1; ++i) {
                lacc.add(bb[i]);
                ln += bn[i];
                if (ln == 0 || right_n[i + 1] == 0) continue;
                const double cost = 0.125 * box.area() + lacc.area() * static_cast<double>(ln) +
                                    right_area[i + 1] * static_cast<double>(right_n[i + 1]);
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = k;
                    best_split = i + 1;
                }
            }
        }
        size_t mid;
        int32_t split_axis = best_axis;
        if (best_axis < 0) {
            // no useful SAH split: median on the longest centroid axis (or a leaf of equal
            // centroids when it cannot be split)
            int k = 0;
            for (int a = 1; a < 3; ++a)
                if (cbox.hi[a] - cbox.lo[a] > cbox.hi[k] - cbox.lo[k]) k = a;
            split_axis = k;
            if (!(cbox.hi[k] > cbox.lo[k])) {
                if (count <= 16) {
                    write(n, box, static_cast<int32_t>(b), static_cast<int32_t>(count));
                    return;
                }
                mid = b + count / 2;  // identical centroids: split the list
            } else {
                mid = b + count / 2;
                std::nth_element(prims.begin() + b, prims.begin() + mid, prims.begin() + e,
                                 [k](const Prim& x, const Prim& y) { return x.c[k] < y.c[k]; });
            }
        } else {
            const double lo = cbox.lo[best_axis], hi = cbox.hi[best_axis];
            const double scale = kBins / (hi - lo);
            auto it = std::partition(prims.begin() + b, prims.begin() + e, [&](const Prim& p) {
                int bi = static_cast<int>((p.c[best_axis] - lo) * scale);
                bi = std::min(std::max(bi, 0), kBins - 1);
                return bi < best_split;
            });
            mid = static_cast<size_t>(it - prims.begin());
            if (mid == b || mid == e) mid = b + count / 2;
        }
        const int32_t left = alloc();
        alloc();  // right = left + 1
        write(n, box, left, 0, split_axis);
        build(left, b, mid, depth + 1);
        build(left + 1, mid, e, depth + 1);
    }
};

}  // namespace

void build_triangle_bvh(const double* tri, int nt, std::vector<double>& nodes,
                        std::vector<int32_t>& order) {
    nodes.clear();
    order.clear();
    if (nt <= 0) return;
    std::vector<Prim> prims(static_cast<size_t>(nt));
    for (int i = 0; i < nt; ++i) {
        const double* q = tri + size_t(kTriStride) * i;
        // the vertices the device test sees: a0, a0 + edge1, a0 + edge2
        const double v0[3] = {q[0], q[1], q[2]};
        const double v1[3] = {q[0] + q[3], q[1] + q[4], q[2] + q[5]};
        const double v2[3] = {q[0] + q[6], q[1] + q[7], q[2] + q[8]};
        Prim& p = prims[size_t(i)];
        p.box.add(v0);
        p.box.add(v1);
        p.box.add(v2);
        for (int k = 0; k < 3; ++k) p.c[k] = 0.5 * (p.box.lo[k] + p.box.hi[k]);
        p.idx = i;
    }
    Builder B{prims, nodes};
    const int32_t root = B.alloc();
    B.build(root, 0, prims.size(), 0);
    order.resize(prims.size());
    for (size_t i = 0; i < prims.size(); ++i) order[i] = prims[i].idx;
}

}  // namespace rtamd

namespace rtamd {

// Spatial chunks of spheres for the packet kernel's culls (rt_packet.hip): a permutation that
// puts spheres close together into the same 64-sphere chunk (recursive splits of the centre
// bounds along their longest axis, left parts a multiple of 64), and a bounding sphere per chunk
// that contains every sphere of the chunk.  A cull whose bound excludes a chunk's bounding
// sphere excludes every sphere in it, so the chunk's lane-parallel pass is skipped.
void build_sphere_chunks(const double* sph, int ns, std::vector<int32_t>& perm,
                         std::vector<double>& bounds) {
    perm.resize(static_cast<size_t>(ns));
    for (int i = 0; i < ns; ++i) perm[static_cast<size_t>(i)] = i;
    auto c = [&](int i, int k) { return sph[static_cast<size_t>(kSphStride) * i + k]; };
    std::vector<std::pair<int, int>> todo{{0, ns}};
    while (!todo.empty()) {
        const auto [lo, hi] = todo.back();
        todo.pop_back();
        const int n = hi - lo;
        if (n <= 64) continue;
        Box b;
        for (int j = lo; j < hi; ++j) {
            const double p[3] = {c(perm[j], 0), c(perm[j], 1), c(perm[j], 2)};
            if (std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2])) b.add(p);
        }
        int axis = 0;
        for (int k = 1; k < 3; ++k)
            if (b.hi[k] - b.lo[k] > b.hi[axis] - b.lo[axis]) axis = k;
        const int chunks = (n + 63) / 64;
        const int left = 64 * ((chunks + 1) / 2);
        // non-finite centres sort last; ties by index (deterministic order)
        auto key = [&](int i) { const double v = c(i, axis); return std::isfinite(v) ? v : INFINITY; };
        std::nth_element(perm.begin() + lo, perm.begin() + lo + left, perm.begin() + hi,
                         [&](int a, int b2) {
                             const double ka = key(a), kb = key(b2);
                             return ka < kb || (ka == kb && a < b2);
                         });
        todo.push_back({lo, lo + left});
        todo.push_back({lo + left, hi});
    }
    const int nb = (ns + 63) / 64;
    bounds.assign(static_cast<size_t>(nb) * 4, 0.0);
    for (int ch = 0; ch < nb; ++ch) {
        const int lo = 64 * ch, hi = std::min(ns, lo + 64);
        Box b;
        bool finite = true;
        for (int j = lo; j < hi; ++j) {
            const int i = perm[static_cast<size_t>(j)];
            const double r = std::sqrt(c(i, 3));
            const double p[3] = {c(i, 0), c(i, 1), c(i, 2)};
            if (!(std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]) &&
                  std::isfinite(r))) {
                finite = false;
                break;
            }
            const double l[3] = {p[0] - r, p[1] - r, p[2] - r}, h[3] = {p[0] + r, p[1] + r, p[2] + r};
            b.add(l);
            b.add(h);
        }
        double* o = &bounds[static_cast<size_t>(ch) * 4];
        if (!finite) {  // a chunk with a non-finite sphere is never culled
            o[0] = o[1] = o[2] = 0.0;
            o[3] = INFINITY;
            continue;
        }
        double cen[3], R = 0.0;
        for (int k = 0; k < 3; ++k) cen[k] = 0.5 * (b.lo[k] + b.hi[k]);
        for (int j = lo; j < hi; ++j) {
            const int i = perm[static_cast<size_t>(j)];
            const double dx = c(i, 0) - cen[0], dy = c(i, 1) - cen[1], dz = c(i, 2) - cen[2];
            R = std::max(R, std::sqrt(dx * dx + dy * dy + dz * dz) + std::sqrt(c(i, 3)));
        }
        // host rounding: far below 1e-9 of the magnitudes
        const double mag = std::fabs(cen[0]) + std::fabs(cen[1]) + std::fabs(cen[2]) + R;
        o[0] = cen[0];
        o[1] = cen[1];
        o[2] = cen[2];
        o[3] = R * (1.0 + 1e-9) + 1e-9 * mag;
    }
}

}  // namespace rtamd
