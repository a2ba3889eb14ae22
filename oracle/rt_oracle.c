/*
 * oracle/rt_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker; never shipped).
 *
 * A C11 restatement of the reference CPU renderer.  Every routine cites the reference
 * function it follows (paths relative to /root/reference/RaytracingEngine).  Arithmetic is
 * IEEE binary64 in the reference's evaluation order; build with -ffp-contract=off and no
 * -ffast-math (see oracle/Makefile) so no FMA or reassociation changes a rounding.
 *
 * Pinning: tests/test_oracle_golden.py checks this file against vectors produced by the
 * compiled reference itself (oracle/_ref/ref_harness, see tests/golden/make_golden.py).
 *
 * Build-defined parts (the reference has no reproducible semantics for them):
 *   - AA jitter for samples 1..N-1: oracle_u01() instead of a random_device-seeded
 *     thread_local mt19937 (Math.h:105-113).
 *   - area lights (BASELINE config 5; README "Extensions suggérées" only).
 */
#include "rt_oracle.h"

#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { double x, y, z; } V;

static inline V mk(double x, double y, double z) { V r; r.x = x; r.y = y; r.z = z; return r; }
static inline V ld3(const double* p) { return mk(p[0], p[1], p[2]); }
/* Vec3 operators, Math.h:14-25 */
static inline V add(V a, V b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V sub(V a, V b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V scale(V a, double s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline V addsc(V a, double s) { return mk(a.x + s, a.y + s, a.z + s); }
static inline V subsc(V a, double s) { return mk(a.x - s, a.y - s, a.z - s); }
static inline V had(V a, V b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V hdiv(V a, V b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline V divs(V a, double s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline V neg(V a) { return mk(-a.x, -a.y, -a.z); }
/* dot / cross / length / normalize, Math.h:27-37 */
static inline double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V cross(V a, V b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double len(V a) { return sqrt(dot(a, a)); }
static inline V unit(V a) {
    double l = len(a);
    if (l <= 1e-12) return mk(0.0, 0.0, 0.0);
    return divs(a, l);
}
/* std::max / std::min / std::clamp as libstdc++ evaluates them (argument order decides NaN). */
static inline double smax(double a, double b) { return (a < b) ? b : a; }
static inline double smin(double a, double b) { return (b < a) ? b : a; }
static inline double sclamp(double v, double lo, double hi) {
    return (v < lo) ? lo : (hi < v) ? hi : v;
}
/* Vec3::reflect, Math.h:39-41: this - (n*2)*dot */
static inline V reflect(V i, V n) { return sub(i, scale(scale(n, 2.0), dot(i, n))); }
/* Vec3::refract, Math.h:43-52 */
static inline V refract(V v, V n, double eta) {
    V I = unit(v), N = unit(n);
    double cosi = sclamp(dot(I, N), -1.0, 1.0);
    double k = 1.0 - eta * eta * (1.0 - cosi * cosi);
    if (k < 0.0) return mk(0.0, 0.0, 0.0);
    return sub(scale(I, eta), scale(N, eta * cosi + sqrt(k)));
}

/* ---------------------------------------------------------------- build-defined RNG */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* Per pixel a 64-bit splitmix64 finalizer folded to a 32-bit key, per (key, stream) and per draw
 * a 32-bit lowbias32 finalizer (the device's u01, rt_device.hpp).  h * 2^-32 in [0, 1). */
static inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

double oracle_u01(uint64_t seed, uint64_t pixel, uint32_t stream, uint32_t index) {
    const uint64_t k = mix64(seed ^ (0x9E3779B97F4A7C15ULL * (pixel + 1ULL)));
    const uint32_t key = (uint32_t)(k ^ (k >> 32));
    const uint32_t skey = hash32(key ^ (stream * 0x9E3779B9U));
    return (double)hash32(skey + index * 0x85EBCA6BU) * 0x1.0p-32;
}

/* ---------------------------------------------------------------- intersections */
/* Sphere::Intersect, Shape.h:72-98 */
static int sphere_hit(V o, V d, const o_sphere* s, double* tout) {
    V oc = sub(o, ld3(s->center));
    double a = dot(d, d);
    double b = 2.0 * dot(oc, d);
    double c = dot(oc, oc) - s->radius * s->radius;
    double disc = b * b - 4.0 * a * c;
    if (disc < 0.0) return 0;
    double sq = sqrt(disc);
    double t0 = (-b - sq) / (2.0 * a);
    double t1 = (-b + sq) / (2.0 * a);
    if (t0 > t1) { double tmp = t0; t0 = t1; t1 = tmp; }
    double t = t0;
    if (t < 1e-6) {
        t = t1;
        if (t < 1e-6) return 0;
    }
    *tout = t;
    return 1;
}

/* Plane::Intersect, Shape.h:149-159 */
static int plane_hit(V o, V d, const o_plane* p, double* tout) {
    V n = ld3(p->normal);
    double denom = dot(n, d);
    if (fabs(denom) > 1e-6) {
        V p0l0 = sub(ld3(p->point), o);
        double t = dot(p0l0, n) / denom;
        if (t >= 0.0) { *tout = t; return 1; }
    }
    return 0;
}

/* Triangle::Intersect (Möller–Trumbore), Shape.h:202-220; tv0..tv2 Shape.h:198-200 */
static int tri_hit(V o, V d, const o_triangle* tr, double* tout) {
    V T = ld3(tr->t);
    V a0 = add(ld3(tr->v0), T);
    V e1 = sub(add(ld3(tr->v1), T), a0);
    V e2 = sub(add(ld3(tr->v2), T), a0);
    V h = cross(d, e2);
    double a = dot(e1, h);
    if (a > -1e-6 && a < 1e-6) return 0;
    double f = 1.0 / a;
    V s = sub(o, a0);
    double u = f * dot(s, h);
    if (u < 0.0 || u > 1.0) return 0;
    V q = cross(s, e1);
    double v = f * dot(d, q);
    if (v < 0.0 || u + v > 1.0) return 0;
    double t = f * dot(e2, q);
    if (t > 1e-6) { *tout = t; return 1; }
    return 0;
}

typedef struct {
    int type;          /* 1 sphere, 2 plane, 3 triangle */
    int32_t index;
    double t;
    V n, p;
    const o_material* m;
} Hit;

/* Scene::IntersectClosest, Scene.h:218-257: spheres, planes, triangles (+model triangles),
 * replacing only on strict '<' (HitInfo::isCloserThan, Shape.h:36).  The hit point and
 * normal depend only on (ray, primitive, t), so they are formed for the winner only. */
static int closest(const o_scene* sc, V o, V d, Hit* h) {
    int found = 0;
    double t;
    for (int32_t i = 0; i < sc->n_spheres; ++i)
        if (sphere_hit(o, d, &sc->spheres[i], &t) && (!found || t < h->t)) {
            found = 1; h->type = 1; h->index = i; h->t = t; h->m = &sc->spheres[i].m;
        }
    for (int32_t i = 0; i < sc->n_planes; ++i)
        if (plane_hit(o, d, &sc->planes[i], &t) && (!found || t < h->t)) {
            found = 1; h->type = 2; h->index = i; h->t = t; h->m = &sc->planes[i].m;
        }
    for (int32_t i = 0; i < sc->n_triangles; ++i)
        if (tri_hit(o, d, &sc->triangles[i], &t) && (!found || t < h->t)) {
            found = 1; h->type = 3; h->index = i; h->t = t; h->m = &sc->triangles[i].m;
        }
    if (!found) return 0;
    h->p = add(o, scale(d, h->t)); /* Rayon::pointAtDistance, Math.h:82 */
    if (h->type == 1) {
        h->n = unit(sub(h->p, ld3(sc->spheres[h->index].center))); /* Shape.h:100-102 */
    } else if (h->type == 2) {
        h->n = ld3(sc->planes[h->index].normal);                    /* Shape.h:161-163 */
    } else {
        const o_triangle* tr = &sc->triangles[h->index];            /* Shape.h:222-227 */
        h->n = unit(cross(sub(ld3(tr->v1), ld3(tr->v0)), sub(ld3(tr->v2), ld3(tr->v0))));
    }
    return 1;
}

/* Scene::backgroundColor, Scene.h:30-33 */
static V sky(V d) {
    double t = 0.5 * (unit(d).y + 1.0);
    return add(scale(mk(1.0, 1.0, 1.0), 1.0 - t), scale(mk(0.5, 0.7, 1.0), t));
}

/* Scene::computeTransmittance, Scene.h:35-77 */
static double transmittance(const o_scene* sc, V o, V d, double max_dist, double bias) {
    double T = 1.0, traveled = 0.0;
    int safety = 64;
    while (safety-- > 0 && T > 1e-4 && traveled < max_dist) {
        Hit h;
        if (!closest(sc, o, d, &h)) break;
        double t = h.t;
        if (t <= 0.0) {
            o = add(o, scale(d, bias));
            traveled += bias;
            continue;
        }
        if (t <= bias) {
            o = add(add(o, scale(d, t)), scale(d, bias));
            traveled += t + bias;
            continue;
        }
        if (traveled + t >= max_dist) break;
        T *= sclamp(h.m->transparency, 0.0, 1.0);
        o = add(add(o, scale(d, t)), scale(d, bias));
        traveled += t + bias;
    }
    return sclamp(T, 0.0, 1.0);
}

typedef struct {
    const o_scene* sc;
    const o_opts* opt;
    uint64_t pixel;
    uint32_t sample;
    uint64_t ntrace, nshadow;
} Ctx;

/* One light's term of Scene::directLightning's loop body, Scene.h:86-124. */
static void light_term(Ctx* c, V P, V n, V view, const o_material* m, V lpos, V lcol,
                       double lint, double bias, V* diff, V* spec) {
    V v = sub(lpos, P);
    double dist = len(v);
    if (dist <= 0.0) return;
    V L = divs(v, dist);
    double ndl = smax(0.0, dot(n, L));
    if (ndl <= 0.0) return;
    if (dist <= bias) return;
    V so = add(P, scale(n, bias));
    c->nshadow++;
    double T = transmittance(c->sc, so, L, dist - bias, bias);
    if (T <= bias) return;
    V E = scale(lcol, lint);
    V contrib = scale(scale(E, 1.0 / (dist * dist)), ndl);
    *diff = add(*diff, scale(contrib, T));
    if (m->transparency <= 0.0 && m->specular > 0.0) {
        V H = unit(add(L, view));
        double ndh = smax(0.0, dot(n, H));
        if (ndh > 0.0) {
            double sf = pow(ndh, m->shininess);
            *spec = add(*spec, scale(scale(scale(E, 1.0 / (dist * dist)), sf), T));
        }
    }
}

/* Scene::directLightning, Scene.h:79-129 (+ build-defined area-light samples appended
 * after the point lights). */
static V direct(Ctx* c, const Hit* h, V view, V normal_in, double bias, int depth) {
    const o_material* m = h->m;
    V n = unit(normal_in);
    V diff = mk(0.0, 0.0, 0.0), spec = mk(0.0, 0.0, 0.0);
    for (int32_t i = 0; i < c->sc->n_lights; ++i) {
        const o_light* l = &c->sc->lights[i];
        light_term(c, h->p, n, view, m, ld3(l->position), ld3(l->color), l->intensity, bias,
                   &diff, &spec);
    }
    const o_area_light* al = c->opt->area_light;
    if (al && al->samples > 0) {
        int k = (int)lround(sqrt((double)al->samples));
        double li = al->intensity / (double)al->samples;
        uint32_t stream = 0x10000u + (c->sample << 6) + (uint32_t)depth;
        for (int s = 0; s < al->samples; ++s) {
            double r1 = oracle_u01(c->opt->seed, c->pixel, stream, 2u * (uint32_t)s);
            double r2 = oracle_u01(c->opt->seed, c->pixel, stream, 2u * (uint32_t)s + 1u);
            double fu = ((double)(s % k) + r1) / (double)k;
            double fv = ((double)(s / k) + r2) / (double)k;
            V lp = add(add(ld3(al->corner), scale(ld3(al->edge_u), fu)), scale(ld3(al->edge_v), fv));
            light_term(c, h->p, n, view, m, lp, ld3(al->color), li, bias, &diff, &spec);
        }
    }
    return add(had(ld3(m->color), diff), scale(spec, m->specular));
}

/* Scene::TraceRay, Scene.h:131-198 (recursive, as the reference) with fresnel Scene.h:26-28 */
static V trace(Ctx* c, V o, V d, int depth) {
    const double bias = c->opt->bias;
    if (depth >= c->opt->max_recursion) return sky(d);
    c->ntrace++;
    Hit h;
    if (!closest(c->sc, o, d, &h)) return sky(d);
    const o_material* m = h.m;
    V inc = unit(d);
    int front = dot(h.n, inc) < 0.0;
    V n = front ? h.n : neg(h.n);
    V view = neg(inc);
    double cos_t = smax(0.0, dot(n, view));
    double eta_t = m->ior;
    double f0 = pow((eta_t - 1.0) / (eta_t + 1.0), 2.0);
    double F = f0 + (1.0 - f0) * pow(1.0 - cos_t, 5.0);
    double tr = sclamp(m->transparency, 0.0, 1.0);
    V local = direct(c, &h, view, n, bias, depth);
    V fin = mk(0.0, 0.0, 0.0);
    if (tr < 1.0) fin = add(fin, scale(local, 1.0 - tr));
    if (tr > 0.0) {
        double eta = front ? (1.0 / eta_t) : (eta_t / 1.0);
        V rd = refract(inc, n, eta);
        if (len(rd) > bias) {
            rd = unit(rd);
            V col = trace(c, add(h.p, scale(rd, bias * 1e2)), rd, depth + 1);
            fin = add(fin, scale(col, tr * (1.0 - F)));
        } else {
            F = 1.0;
        }
    }
    double refl = (tr > 0.0) ? F : m->specular;
    if (refl > bias) {
        V R = unit(reflect(inc, n));
        V col = trace(c, add(h.p, scale(R, bias)), R, depth + 1);
        fin = add(fin, scale(col, refl));
    }
    return fin;
}

/* Camera::getRay, Math.h:99-121 */
static void get_ray(const o_camera* cam, uint32_t x, uint32_t y, int aa, uint64_t seed,
                    uint32_t sample, V* o, V* d) {
    double sx = (double)x - (double)cam->width / 2.0;
    double sy = (double)cam->height / 2.0 - (double)y;
    double jx = 0.0, jy = 0.0;
    if (aa) {
        const double inv_aa = 1.0 / 1.0; /* 1.0/double(bool aa): always 1 (Math.h:106) */
        uint64_t pix = (uint64_t)y * cam->width + x;
        jx = oracle_u01(seed, pix, sample, 0u) * inv_aa;
        jy = oracle_u01(seed, pix, sample, 1u) * inv_aa;
    }
    sx += jx;
    sy += jy;
    V pos = ld3(cam->position);
    V screen = mk(sx, sy, pos.z + cam->focal);
    *o = pos;
    *d = unit(sub(screen, pos));
}

void oracle_get_ray(const o_camera* cam, uint32_t x, uint32_t y, int aa, uint64_t seed,
                    uint32_t sample, double* ray_out) {
    V o, d;
    get_ray(cam, x, y, aa, seed, sample, &o, &d);
    ray_out[0] = o.x; ray_out[1] = o.y; ray_out[2] = o.z;
    ray_out[3] = d.x; ray_out[4] = d.y; ray_out[5] = d.z;
}

/* Scene::GeneratePixelAt / GenerateAntiAliasing, Scene.h:283-309 */
static V pixel(Ctx* c, const o_camera* cam, uint32_t x, uint32_t y) {
    V acc = mk(0.0, 0.0, 0.0);
    int samples = 0;
    const int n = cam->aa_samples;
    for (int s = 0; s < n; ++s) {
        V o, d;
        c->sample = (uint32_t)s;
        get_ray(cam, x, y, s > 0 && n > 1, c->opt->seed, (uint32_t)s, &o, &d);
        acc = add(acc, trace(c, o, d, 0));
        samples += 1;
    }
    if (samples > 0) return divs(acc, (double)samples);
    return mk(0.0, 0.0, 0.0);
}

/* Scene::RenderImage, Scene.h:311-328 (rows [row_begin,row_end)) */
int oracle_render(const o_scene* sc, const o_camera* cam, const o_opts* opt, double* out,
                  uint64_t* trace_rays, uint64_t* shadow_rays) {
    const uint32_t W = cam->width;
    const uint32_t r0 = opt->row_begin;
    const uint32_t r1 = opt->row_end ? opt->row_end : cam->height;
    if (r1 < r0 || r1 > cam->height) return -1;
    const long long total = (long long)(r1 - r0) * (long long)W;
    uint64_t nt = 0, ns = 0;
#ifdef _OPENMP
    int threads = opt->nthreads > 0 ? opt->nthreads : omp_get_max_threads();
#pragma omp parallel num_threads(threads) reduction(+ : nt, ns)
#endif
    {
        Ctx c;
        memset(&c, 0, sizeof c);
        c.sc = sc;
        c.opt = opt;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
        for (long long i = 0; i < total; ++i) {
            uint32_t x = (uint32_t)(i % W);
            uint32_t y = r0 + (uint32_t)(i / W);
            c.pixel = (uint64_t)y * W + x;
            V v = pixel(&c, cam, x, y);
            out[3 * i + 0] = v.x;
            out[3 * i + 1] = v.y;
            out[3 * i + 2] = v.z;
        }
        nt += c.ntrace;
        ns += c.nshadow;
    }
    if (trace_rays) *trace_rays += nt;
    if (shadow_rays) *shadow_rays += ns;
    return 0;
}

/* ---------------------------------------------------------------- tonemap (RaytracingEngine.cpp) */
/* ClampVec3 :70-76 */
static V clamp3(V v, double lo, double hi) {
    return mk(smin(hi, smax(lo, v.x)), smin(hi, smax(lo, v.y)), smin(hi, smax(lo, v.z)));
}
/* uncharted2_tonemap_partial :78-87 — products/quotients of two float constants are
 * formed in float, then promoted. */
static V u2_partial(V x) {
    const float A = 0.15f, B = 0.50f, C = 0.10f, D = 0.20f, E = 0.02f, F = 0.30f;
    const float CB = C * B, DE = D * E, DF = D * F, EF = E / F;
    V num = addsc(had(x, addsc(scale(x, (double)A), (double)CB)), (double)DE);
    V den = addsc(had(x, addsc(scale(x, (double)A), (double)B)), (double)DF);
    return subsc(hdiv(num, den), (double)EF);
}
/* aces_approx :89-98 */
static V aces(V v) {
    v = scale(v, (double)0.6f);
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    V num = had(v, addsc(scale(v, (double)a), (double)b));
    V den = addsc(had(v, addsc(scale(v, (double)c), (double)d)), (double)e);
    return clamp3(hdiv(num, den), (double)0.0f, (double)1.0f);
}
/* luminance :100-104, change_luminance :106-110 */
static double lum(V c) { return dot(c, mk(0.2126, 0.7152, 0.0722)); }
static V change_lum(V c, double l_out) { return scale(c, l_out / lum(c)); }

static V tonemap_op(V c, int op) {
    switch (op) {
    case 0: /* simple :123-131 */
        return mk(smin(1.0, smax(0.0, c.x)), smin(1.0, smax(0.0, c.y)), smin(1.0, smax(0.0, c.z)));
    case 1: /* reinhardSimple :133-135 */
        return hdiv(c, addsc(c, 1.0));
    case 2: { /* reinhardExtended(c, 5.0) :137-141 */
        const double ws = 5.0 * 5.0;
        V num = had(c, addsc(hdiv(c, mk(ws, ws, ws)), 1.0));
        return hdiv(num, addsc(c, 1.0));
    }
    case 3: { /* reinhardExtendedLuminance(c, 5.0) :143-148 */
        double lo = lum(c);
        double num = lo * (1.0 + (lo / (5.0 * 5.0)));
        return change_lum(c, num / (1.0 + lo));
    }
    case 4: { /* reinhardJodie(c, 0.18) :150-154 */
        double L = lum(c);
        double lm = (0.18 / log(2.0 + pow((L / 0.85), 1.7))) * log(1.0 + L);
        return change_lum(c, lm);
    }
    case 5: { /* uncharted2 :156-163 */
        const double bias = (double)2.0f;
        V cur = u2_partial(scale(c, bias));
        V ws = hdiv(mk(1.0, 1.0, 1.0), u2_partial(mk(11.2, 11.2, 11.2)));
        return had(cur, ws);
    }
    default: /* aces_approx :89-98 (also tonemap() :165-174) */
        return aces(c);
    }
}

/* toColor :113-121 — clamp to [0,1], then truncating uint8 cast of x*255 */
static void to_color(V v, uint8_t* o) {
    V c = clamp3(v, 0.0, 1.0);
    o[0] = (uint8_t)(c.x * 255.0);
    o[1] = (uint8_t)(c.y * 255.0);
    o[2] = (uint8_t)(c.z * 255.0);
}

int oracle_tonemap(const double* hdr, size_t n, int op, uint8_t* out) {
    if (op < 0 || op > 6) return -1;
    for (size_t i = 0; i < n; ++i) to_color(tonemap_op(ld3(hdr + 3 * i), op), out + 3 * i);
    return 0;
}

/* ---------------------------------------------------------------- known-answer helpers */
int oracle_sphere_intersect(const double* ray, const o_sphere* s, double* t) {
    return sphere_hit(ld3(ray), ld3(ray + 3), s, t);
}
int oracle_plane_intersect(const double* ray, const o_plane* p, double* t) {
    return plane_hit(ld3(ray), ld3(ray + 3), p, t);
}
int oracle_triangle_intersect(const double* ray, const o_triangle* tr, double* t) {
    return tri_hit(ld3(ray), ld3(ray + 3), tr, t);
}
int oracle_closest(const o_scene* sc, const double* ray, double* out, int32_t* index) {
    Hit h;
    if (!closest(sc, ld3(ray), ld3(ray + 3), &h)) {
        *index = -1;
        return 0;
    }
    out[0] = h.t;
    out[1] = h.n.x; out[2] = h.n.y; out[3] = h.n.z;
    out[4] = h.p.x; out[5] = h.p.y; out[6] = h.p.z;
    *index = h.index;
    return h.type;
}
double oracle_transmittance(const o_scene* sc, const double* ray, double max_dist, double bias) {
    return transmittance(sc, ld3(ray), ld3(ray + 3), max_dist, bias);
}
