/*
 * oracle/rt_oracle.h — TEST INFRASTRUCTURE ONLY.  Never linked into the product library.
 *
 * Plain-C (C11) restatement of the reference CPU hot path of Sorax5/RaytracingEngine
 * (/root/reference/RaytracingEngine/{Math.h,Shape.h,Light.h,Scene.h,RaytracingEngine.cpp}),
 * used as the parity checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg ("port").  Its equality with the compiled reference (oracle/_ref, built by
 * oracle/Makefile from the reference sources where they lie) is pinned by the golden vectors
 * under tests/golden/ (tests/test_oracle_golden.py).
 *
 * The scene structs below have the byte layout of include/rt_capi.h's rt_* structs (the same
 * host buffers are handed to both), but the oracle does not include that header: it stays
 * an independent restatement.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct o_material { double color[3], shininess, specular, transparency, ior; } o_material;
typedef struct o_sphere { double center[3], radius; o_material m; } o_sphere;
typedef struct o_plane { double point[3], normal[3]; o_material m; } o_plane;
typedef struct o_triangle { double v0[3], v1[3], v2[3], t[3]; o_material m; } o_triangle;
typedef struct o_light { double position[3], color[3], intensity; } o_light;
typedef struct o_area_light {
    double corner[3], edge_u[3], edge_v[3], color[3], intensity;
    int32_t samples, _pad0;
} o_area_light;

typedef struct o_scene {
    const o_sphere* spheres; int32_t n_spheres;
    const o_plane* planes; int32_t n_planes;
    const o_triangle* triangles; int32_t n_triangles;
    const o_light* lights; int32_t n_lights;
} o_scene;

typedef struct o_camera {
    double position[3], focal;
    uint32_t width, height;
    int32_t aa_samples, _pad0;
    double near_plane, far_plane;
} o_camera;

typedef struct o_opts {
    int32_t max_recursion;   /* 10 in the reference */
    int32_t nthreads;        /* OpenMP threads for oracle_render (<=0: all)        */
    double bias;             /* 1e-3 in the reference */
    uint64_t seed;           /* AA jitter / area-light RNG key (build-defined)     */
    uint32_t row_begin, row_end;
    const o_area_light* area_light; /* NULL: none (reference semantics)           */
} o_opts;

/* Counter-based U[0,1) draw (build-defined replacement for the reference's
 * thread_local mt19937 of Math.h:109-112, which is seeded from std::random_device and
 * therefore irreproducible). */
double oracle_u01(uint64_t seed, uint64_t pixel, uint32_t stream, uint32_t index);

/* Scene::RenderImage (Scene.h:311-328) over rows [row_begin,row_end): out is rows*W*3
 * doubles.  Ray counts (TraceRay reaching IntersectClosest; computeTransmittance calls)
 * are added to *trace_rays / *shadow_rays when non-NULL. */
int oracle_render(const o_scene* sc, const o_camera* cam, const o_opts* opt, double* out,
                  uint64_t* trace_rays, uint64_t* shadow_rays);

/* Tonemap operator `op` (0..6, tonemapAll order) + toColor() for n pixels → n*3 bytes. */
int oracle_tonemap(const double* hdr, size_t n, int op, uint8_t* out);

/* Known-answer helpers (one call per query). ray = {ox,oy,oz,dx,dy,dz}.
 * *_intersect return 1 and set *t on a hit, 0 on a miss. */
int oracle_sphere_intersect(const double* ray, const o_sphere* s, double* t);
int oracle_plane_intersect(const double* ray, const o_plane* p, double* t);
int oracle_triangle_intersect(const double* ray, const o_triangle* tr, double* t);
/* Camera::getRay (Math.h:99-121) with the build-defined jitter for sample > 0 when aa. */
void oracle_get_ray(const o_camera* cam, uint32_t x, uint32_t y, int aa, uint64_t seed,
                    uint32_t sample, double* ray_out);
/* Scene::IntersectClosest (Scene.h:218-257): returns prim type (0 none, 1 sphere, 2 plane,
 * 3 triangle) and fills out = {t, nx, ny, nz, px, py, pz} and *index. */
int oracle_closest(const o_scene* sc, const double* ray, double* out, int32_t* index);
/* Scene::computeTransmittance (Scene.h:35-77). */
double oracle_transmittance(const o_scene* sc, const double* ray, double max_dist,
                            double bias);

#ifdef __cplusplus
}
#endif

#endif
