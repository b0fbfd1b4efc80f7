/*
 * oracle.c — CPU restatement (C99, f64) of the reference's per-(pixel, sample)
 * `ray_color` hot path and of everything it calls, plus the scene builders that
 * define its inputs. Every function cites the reference file:line it restates
 * (paths relative to /root/reference/src).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker for tests/, smoke() and
 * the CPU baseline of bench.py. The product path never links or loads it.
 *
 * Deliberate, documented departures from the reference:
 *   - RNG: `rand::thread_rng()` (ChaCha12 from OS entropy, math.rs:268-276) is
 *     replaced by one stream per (pixel, sample) path — a Philox4x32-10 block of
 *     (pixel, sample) seeding xoshiro128++ (rt_numerics.h rt_pstream) — drawn in
 *     the reference's order; the medium's in-`hit` draw (hittable.rs:446) is keyed
 *     per (pixel, sample, bounce, medium id) through Philox so the outcome is
 *     independent of traversal order; scene construction uses a sequential Philox
 *     stream. The `rand` 0.8 float mappings (Standard, UniformFloat inclusive) are
 *     restated.
 *   - libm: sin/log/atan2/acos/pow come from rt_numerics.h (fdlibm algorithms)
 *     so that host and device agree bit-for-bit; host-only set-up math (tan in
 *     Camera::new, sin/cos in new_rotate_y) uses the platform libm, as Rust does.
 *   - Image size: width and height are explicit and the camera aspect is
 *     width/height (main.rs:467 computes height = width*aspect).
 *   - Work split: threads take pixels round-robin (or the reference's sample split)
 *     and every pixel always receives exactly spp samples (main.rs:516 truncates).
 */
#define _GNU_SOURCE
#include "oracle.h"
#include "../include/rt/rt_numerics.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#ifdef ORC_LIBM
/* The independent-numerics build (liboracle_libm.so, tests/test_oracle.py): the platform libm's
 * transcendentals in place of rt_numerics.h's restatements, which the kernel and this oracle
 * share. A bug in those restatements would be invisible to GPU-vs-oracle parity; against this
 * build it would show (the two agree wherever glibc and the restatement round alike). */
#define rt_sin(x) sin(x)
#define rt_cos(x) cos(x)
#define rt_log(x) log(x)
#define rt_acos(x) acos(x)
#define rt_atan2(y, x) atan2(y, x)
#define rt_pow5(x) pow((x), 5.0)   /* (1 - cosine).powf(5.0), material.rs:93 */
#endif

/* ------------------------------------------------------------------------- */
/* math.rs — Vector3                                                          */
/* ------------------------------------------------------------------------- */
typedef struct { double x, y, z; } V3;

static inline V3 v3(double x, double y, double z) { V3 r = {x, y, z}; return r; }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }      /* math.rs:147-157 */
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }      /* math.rs:175-185 */
static inline V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }                            /* math.rs:187-209 */
static inline V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }      /* math.rs:211-221 */
static inline V3 vscale(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }      /* math.rs:223-257 */
static inline V3 vdiv(V3 a, double s) { return vscale(a, 1.0 / s); }                   /* math.rs:260-266 */
static inline double vdot(V3 u, V3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }    /* math.rs:82-84 */
static inline double vlen2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }         /* math.rs:86-88 */
static inline double vlen(V3 a) { return sqrt(vlen2(a)); }                              /* math.rs:90-92 */
static inline V3 vcross(V3 u, V3 v)                                                     /* math.rs:94-100 */
{
    return v3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
static inline V3 vnormalize(V3 v) { return vdiv(v, vlen(v)); }                         /* math.rs:102-104 */
static inline V3 vreflect(V3 v, V3 n) { return vsub(v, vscale(n, 2.0 * vdot(v, n))); } /* math.rs:106-108 */
static inline V3 vrefract(V3 uv, V3 n, double etai_over_etat)                          /* math.rs:110-117 */
{
    double cos_theta = fmin(vdot(vneg(uv), n), 1.0);
    V3 r_out_perp = vscale(vadd(uv, vscale(n, cos_theta)), etai_over_etat);
    double r_out_perp_length = vlen2(r_out_perp);
    V3 r_out_parallel = vscale(n, -sqrt(fabs(1.0 - r_out_perp_length)));
    return vadd(r_out_perp, r_out_parallel);
}
static inline int vnear_zero(V3 a)                                                      /* math.rs:134-137 */
{
    const double s = 1e-8;
    return fabs(a.x) < s && fabs(a.y) < s && fabs(a.z) < s;
}
static inline double degrees_to_radians(double d) { return d * RT_PI / 180.0; }        /* math.rs:8-10 */
static inline double clampd(double x, double mn, double mx)                             /* math.rs:282-286 */
{
    if (x < mn) return mn;
    if (x > mx) return mx;
    return x;
}

/* math.rs:288-300 */
static void sphere_uv(V3 p, double* u, double* v)
{
    double theta = rt_acos(-p.y);
    double phi = rt_atan2(-p.z, p.x) + RT_PI;
    *u = phi / (2.0 * RT_PI);
    *v = theta / RT_PI;
}

/* ------------------------------------------------------------------------- */
/* RNG (math.rs:268-280 -> seeded Philox, rt_numerics.h)                      */
/* ------------------------------------------------------------------------- */
typedef struct {
    rt_stream s;            /* scene construction: sequential Philox stream (thread_rng replacement) */
    rt_pstream ps;          /* rendering: the path stream of (pixel, sample) (rt_numerics.h) */
    int render;             /* 1: draws come from ps */
    uint64_t seed;
    uint32_t pixel, sample; /* keyed-draw coordinates */
    uint32_t bounce;
} OrcRng;

static __thread OrcRng* tl_rng;

static inline uint64_t rng_u64(void)
{
    return tl_rng->render ? rt_pstream_u64(&tl_rng->ps) : rt_stream_next_u64(&tl_rng->s);
}
static inline double random_double(void) { return rt_unit53(rng_u64()); }
static inline double random_double_range(double a, double b)
{
    return rt_uniform_sample(rng_u64(), a, rt_uniform_incl_scale(a, b));
}
static inline int random_int_range(int a, int b)                                         /* math.rs:278-280 */
{
    return rt_sat_i32(random_double_range((double)a, (double)(b + 1)));
}
static inline V3 v3_random(void)                                                         /* math.rs:35-41 */
{
    double x = random_double();
    double y = random_double();
    double z = random_double();
    return v3(x, y, z);
}
static inline V3 v3_random_range(double a, double b)                                     /* math.rs:43-49 */
{
    double x = random_double_range(a, b);
    double y = random_double_range(a, b);
    double z = random_double_range(a, b);
    return v3(x, y, z);
}
static V3 random_in_unit_sphere(void)                                                    /* math.rs:51-58 */
{
    for (;;) {
        V3 p = v3_random_range(-1.0, 1.0);
        if (vlen2(p) < 1.0) return p;
    }
}
static V3 random_in_unit_disk(void)                                                      /* math.rs:69-76 */
{
    for (;;) {
        double x = random_double_range(-1.0, 1.0);
        double y = random_double_range(-1.0, 1.0);
        V3 p = v3(x, y, 0.0);
        if (vlen2(p) < 1.0) return p;
    }
}
static V3 random_unit_vector(void) { return vnormalize(random_in_unit_sphere()); }       /* math.rs:78-80 */

/* The medium's draw inside hit (hittable.rs:446), keyed so it does not depend on
 * which objects were tested before it. */
static inline double medium_random_double(int medium_id)
{
    return rt_unit53(rt_keyed_u64(tl_rng->seed, tl_rng->pixel, tl_rng->sample, tl_rng->bounce,
                                  RT_STREAM_MEDIUM + (uint32_t)medium_id));
}

/* ------------------------------------------------------------------------- */
/* ray.rs                                                                     */
/* ------------------------------------------------------------------------- */
typedef struct { V3 origin, direction; double time; } Ray;
static inline Ray ray_with_time(V3 o, V3 d, double t) { Ray r = {o, d, t}; return r; }   /* ray.rs:9-15 */
static inline V3 ray_at(const Ray* r, double t) { return vadd(r->origin, vscale(r->direction, t)); } /* ray.rs:19-21 */

/* ------------------------------------------------------------------------- */
/* perlin.rs                                                                  */
/* ------------------------------------------------------------------------- */
#define POINT_COUNT 256
typedef struct {
    V3 ranvec[POINT_COUNT];
    int32_t perm_x[POINT_COUNT], perm_y[POINT_COUNT], perm_z[POINT_COUNT];
} Perlin;

static void perlin_permute(int32_t* p, int n)                                            /* perlin.rs:122-129 */
{
    for (int i = n - 1; i >= 0; --i) {
        int target = random_int_range(0, i);
        if (target < 0) target = 0;
        if (target > n - 1) target = n - 1; /* Rust would panic on n (probability ~2^-52) */
        int32_t tmp = p[i];
        p[i] = target;                       /* Q10: writes the index, not p[target] */
        p[target] = tmp;
    }
}
static void perlin_generate_perm(int32_t* p)                                             /* perlin.rs:110-120 */
{
    for (int i = 0; i < POINT_COUNT; ++i) p[i] = i;
    perlin_permute(p, POINT_COUNT);
}
static Perlin* perlin_new(void)                                                          /* perlin.rs:13-30 */
{
    Perlin* pr = (Perlin*)calloc(1, sizeof(Perlin));
    for (int i = 0; i < POINT_COUNT; ++i) pr->ranvec[i] = vnormalize(v3_random_range(-1.0, 1.0));
    perlin_generate_perm(pr->perm_x);
    perlin_generate_perm(pr->perm_y);
    perlin_generate_perm(pr->perm_z);
    return pr;
}
static double perlin_interp(V3 c[2][2][2], double u, double v, double w)                 /* perlin.rs:70-94 */
{
    double uu = u * u * (3.0 - 2.0 * u);
    double vv = v * v * (3.0 - 2.0 * v);
    double ww = w * w * (3.0 - 2.0 * w);
    double accum = 0.0;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
                double fi = (double)i, fj = (double)j, fk = (double)k;
                V3 weight_v = v3(u - fi, v - fj, w - fk);
                accum += (fi * uu + (1.0 - fi) * (1.0 - uu)) * (fj * vv + (1.0 - fj) * (1.0 - vv)) *
                         (fk * ww + (1.0 - fk) * (1.0 - ww)) * vdot(c[i][j][k], weight_v);
            }
    return accum;
}
static double perlin_noise(const Perlin* pr, V3 p)                                       /* perlin.rs:32-68 */
{
    double x = floor(p.x), y = floor(p.y), z = floor(p.z);
    double u = p.x - x, v = p.y - y, w = p.z - z;
    u = u * u * (3.0 - 2.0 * u);                                                         /* Q9: first smoothing */
    v = v * v * (3.0 - 2.0 * v);
    w = w * w * (3.0 - 2.0 * w);
    int32_t i = rt_sat_i32(x), j = rt_sat_i32(y), k = rt_sat_i32(z);
    V3 c[2][2][2];
    for (int di = 0; di < 2; ++di)
        for (int dj = 0; dj < 2; ++dj)
            for (int dk = 0; dk < 2; ++dk) {
                uint32_t xi = ((uint32_t)i + (uint32_t)di) & 255u;
                uint32_t yi = ((uint32_t)j + (uint32_t)dj) & 255u;
                uint32_t zi = ((uint32_t)k + (uint32_t)dk) & 255u;
                c[di][dj][dk] = pr->ranvec[(uint32_t)(pr->perm_x[xi] ^ pr->perm_y[yi] ^ pr->perm_z[zi]) & 255u];
            }
    return perlin_interp(c, u, v, w);
}
static double perlin_turb(const Perlin* pr, V3 p, int depth)                             /* perlin.rs:96-108 */
{
    double accum = 0.0;
    V3 temp_p = p;
    double weight = 1.0;
    for (int i = 0; i < depth; ++i) {
        accum += weight * perlin_noise(pr, temp_p);
        weight *= 0.5;
        temp_p = vscale(temp_p, 2.0);
    }
    return fabs(accum);
}

/* ------------------------------------------------------------------------- */
/* texture.rs                                                                 */
/* ------------------------------------------------------------------------- */
enum { TEX_SOLID, TEX_CHECKER, TEX_NOISE, TEX_IMAGE };
typedef struct {
    int kind;
    V3 c0, c1;            /* solid: c0; checker: even = c0, odd = c1 */
    const Perlin* perlin; /* noise */
    double scale;
    int w, h, bps;        /* image */
    const uint8_t* data;
} Texture;

static Texture tex_solid(V3 c) { Texture t; memset(&t, 0, sizeof t); t.kind = TEX_SOLID; t.c0 = c; return t; }
static Texture tex_checker(V3 even, V3 odd)
{
    Texture t; memset(&t, 0, sizeof t); t.kind = TEX_CHECKER; t.c0 = even; t.c1 = odd; return t;
}
static Texture tex_noise(const Perlin* p, double scale)
{
    Texture t; memset(&t, 0, sizeof t); t.kind = TEX_NOISE; t.perlin = p; t.scale = scale; return t;
}
static Texture tex_image(const uint8_t* data, int w, int h)                              /* texture.rs:12-22 */
{
    Texture t; memset(&t, 0, sizeof t); t.kind = TEX_IMAGE; t.data = data; t.w = w; t.h = h; t.bps = 3 * w;
    return t;
}

static V3 tex_value(const Texture* t, double u, double v, V3 p)                          /* texture.rs:30-75 */
{
    switch (t->kind) {
    case TEX_SOLID: return t->c0;
    case TEX_CHECKER: {
        double sines = rt_sin(10.0 * p.x) * rt_sin(10.0 * p.y) * rt_sin(10.0 * p.z);
        return sines < 0.0 ? t->c1 : t->c0;
    }
    case TEX_NOISE: {
        double s = 1.0 + rt_sin(t->scale * p.z + 10.0 * perlin_turb(t->perlin, p, 7));
        return vscale(vscale(v3(1.0, 1.0, 1.0), 0.5), s);
    }
    default: {
        if (!t->data || t->w <= 0 || t->h <= 0) return v3(0.0, 1.0, 1.0);
        double uu = clampd(u, 0.0, 1.0);
        double vv = 1.0 - clampd(v, 0.0, 1.0);
        uint64_t i = rt_sat_u64(uu * (double)t->w);
        uint64_t j = rt_sat_u64(vv * (double)t->h);
        if (i >= (uint64_t)t->w) i = (uint64_t)t->w - 1;
        if (j >= (uint64_t)t->h) j = (uint64_t)t->h - 1;
        const double color_scale = 1.0 / 255.0;
        const uint8_t* px = t->data + j * (uint64_t)t->bps + i * 3;
        return v3(color_scale * (double)px[0], color_scale * (double)px[1], color_scale * (double)px[2]);
    }
    }
}

/* ------------------------------------------------------------------------- */
/* material.rs                                                                */
/* ------------------------------------------------------------------------- */
enum { MAT_LAMBERTIAN, MAT_METAL, MAT_DIELECTRIC, MAT_DIFFUSE_LIGHT, MAT_ISOTROPIC };
typedef struct {
    int kind;
    Texture tex;   /* lambertian albedo / light emit / isotropic albedo */
    V3 albedo;     /* metal */
    double fuzz;   /* metal */
    double ir;     /* dielectric */
} Material;

/* hittable.rs:6-27 */
typedef struct {
    V3 point, normal;
    double t;
    int front_face;
    int mat_handle; /* 1-based (material.rs:97-98, main.rs:46-49) */
    double u, v;
} HitRecord;

static inline void set_face_normal(HitRecord* rec, const Ray* r, V3 outward_normal)      /* hittable.rs:23-26 */
{
    rec->front_face = vdot(r->direction, outward_normal) < 0.0;
    rec->normal = rec->front_face ? outward_normal : vneg(outward_normal);
}

static double reflectance(double cosine, double ref_idx)                                 /* material.rs:89-94 */
{
    double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
    r0 = r0 * r0;
    return r0 + (1.0 - r0) * rt_pow5(1.0 - cosine);
}

static V3 mat_emitted(const Material* m, double u, double v, V3 p)                       /* material.rs:25-34 */
{
    if (m->kind == MAT_DIFFUSE_LIGHT) return tex_value(&m->tex, u, v, p);
    return v3(0.0, 0.0, 0.0);
}

/* material.rs:15-23 and the per-kind functions :36-87 */
static int mat_scatter(const Material* m, const Ray* r, const HitRecord* rec, Ray* scattered, V3* attenuation)
{
    switch (m->kind) {
    case MAT_LAMBERTIAN: {                                                               /* :36-48 */
        V3 dir = vadd(rec->normal, random_unit_vector());
        if (vnear_zero(dir)) dir = rec->normal;
        *scattered = ray_with_time(rec->point, dir, r->time);
        *attenuation = tex_value(&m->tex, rec->u, rec->v, rec->point);
        return 1;
    }
    case MAT_METAL: {                                                                    /* :50-60 */
        V3 reflected = vreflect(vnormalize(r->direction), rec->normal);
        V3 with_fuzz = vadd(reflected, vscale(random_in_unit_sphere(), m->fuzz));
        *scattered = ray_with_time(rec->point, with_fuzz, r->time);
        if (vdot(scattered->direction, rec->normal) > 0.0) { *attenuation = m->albedo; return 1; }
        return 0;
    }
    case MAT_DIELECTRIC: {                                                               /* :62-82 */
        double refraction_ratio = rec->front_face ? (1.0 / m->ir) : m->ir;
        V3 unit_direction = vnormalize(r->direction);
        double cos_theta = fmin(vdot(vneg(unit_direction), rec->normal), 1.0);
        double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
        int cannot_refract = refraction_ratio * sin_theta > 1.0;
        V3 direction;
        if (cannot_refract || reflectance(cos_theta, refraction_ratio) > random_double())
            direction = vreflect(unit_direction, rec->normal);
        else
            direction = vrefract(unit_direction, rec->normal, refraction_ratio);
        *scattered = ray_with_time(rec->point, direction, r->time);
        *attenuation = v3(1.0, 1.0, 1.0);
        return 1;
    }
    case MAT_ISOTROPIC: {                                                                /* :84-87 */
        *scattered = ray_with_time(rec->point, random_in_unit_sphere(), r->time);
        *attenuation = tex_value(&m->tex, rec->u, rec->v, rec->point);
        return 1;
    }
    default: return 0;                                                                   /* DiffuseLight */
    }
}

/* ------------------------------------------------------------------------- */
/* aabb.rs                                                                    */
/* ------------------------------------------------------------------------- */
typedef struct { V3 minimum, maximum; } AABB;

static AABB aabb_new(V3 a, V3 b) { AABB r = {a, b}; return r; }
static AABB surrounding_box(AABB b0, AABB b1)                                            /* aabb.rs:19-33 */
{
    V3 small = v3(fmin(b0.minimum.x, b1.minimum.x), fmin(b0.minimum.y, b1.minimum.y), fmin(b0.minimum.z, b1.minimum.z));
    V3 big = v3(fmax(b0.maximum.x, b1.maximum.x), fmax(b0.maximum.y, b1.maximum.y), fmax(b0.maximum.z, b1.maximum.z));
    return aabb_new(small, big);
}
static int aabb_hit(const AABB* b, const Ray* r, double t_min, double t_max)            /* aabb.rs:77-103 */
{
    double mn = t_min, mx = t_max;
    const double bmin[3] = {b->minimum.x, b->minimum.y, b->minimum.z};
    const double bmax[3] = {b->maximum.x, b->maximum.y, b->maximum.z};
    const double o[3] = {r->origin.x, r->origin.y, r->origin.z};
    const double d[3] = {r->direction.x, r->direction.y, r->direction.z};
    for (int a = 0; a < 3; ++a) {
        double inv_d = 1.0 / d[a];
        double t0 = (bmin[a] - o[a]) * inv_d;
        double t1 = (bmax[a] - o[a]) * inv_d;
        if (inv_d < 0.0) { double tmp = t0; t0 = t1; t1 = tmp; }
        mn = t0 > mn ? t0 : mn;
        mx = t1 < mx ? t1 : mx;
        if (mx <= mn) return 0;
    }
    return 1;
}

/* ------------------------------------------------------------------------- */
/* hittable.rs                                                                */
/* ------------------------------------------------------------------------- */
enum { H_SPHERE, H_MOVING_SPHERE, H_BVH, H_XY, H_XZ, H_YZ, H_BOX, H_TRANSLATE, H_ROTATE_Y, H_MEDIUM };

typedef struct Hittable Hittable;
struct Hittable {                                                                        /* hittable.rs:29-41 */
    int kind;
    int mat;                          /* 1-based handle; medium: phase function */
    V3 center0, center1;              /* spheres */
    double time0, time1, radius;
    const Hittable *left, *right;     /* bvh */
    AABB box;                         /* bvh: aabb_box; rotate_y: bbox */
    double a0, a1, b0, b1, k;         /* rects: x0 x1 y0 y1 / x0 x1 z0 z1 / y0 y1 z0 z1, k */
    V3 bmin, bmax;                    /* box */
    Hittable* sides;                  /* box: 6 rects */
    V3 offset;                        /* translate */
    const Hittable* ptr;              /* translate / rotate_y / medium boundary */
    double sin_theta, cos_theta;      /* rotate_y */
    int has_box;
    double neg_inv_density;           /* medium */
    int medium_id;
};

/* Arena of every allocation a world makes (freed with the world). */
typedef struct {
    void** ptrs;
    size_t n, cap;
} Arena;
static void* arena_alloc(Arena* a, size_t sz)
{
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 64;
        a->ptrs = (void**)realloc(a->ptrs, a->cap * sizeof(void*));
    }
    void* p = calloc(1, sz);
    a->ptrs[a->n++] = p;
    return p;
}
static void arena_free(Arena* a)
{
    for (size_t i = 0; i < a->n; ++i) free(a->ptrs[i]);
    free(a->ptrs);
    a->ptrs = NULL; a->n = a->cap = 0;
}

typedef struct {                                                                          /* main.rs:40-50 */
    Material* materials; int n_materials, cap_materials;
    const Hittable** hittables; int n_hittables, cap_hittables;
    Arena arena;
    int n_media;
    const uint8_t* image; int image_w, image_h;
} World;

static int register_material(World* w, Material m)                                       /* main.rs:46-49 */
{
    if (w->n_materials == w->cap_materials) {
        w->cap_materials = w->cap_materials ? 2 * w->cap_materials : 16;
        w->materials = (Material*)realloc(w->materials, (size_t)w->cap_materials * sizeof(Material));
    }
    w->materials[w->n_materials++] = m;
    return w->n_materials;
}
static void world_push(World* w, const Hittable* h)
{
    if (w->n_hittables == w->cap_hittables) {
        w->cap_hittables = w->cap_hittables ? 2 * w->cap_hittables : 16;
        w->hittables = (const Hittable**)realloc(w->hittables, (size_t)w->cap_hittables * sizeof(void*));
    }
    w->hittables[w->n_hittables++] = h;
}
static void world_free(World* w)
{
    free(w->materials);
    free(w->hittables);
    arena_free(&w->arena);
    memset(w, 0, sizeof *w);
}
static Hittable* hnew(World* w, int kind) { Hittable* h = (Hittable*)arena_alloc(&w->arena, sizeof(Hittable)); h->kind = kind; return h; }

static Material mat_lambertian(Texture t) { Material m; memset(&m, 0, sizeof m); m.kind = MAT_LAMBERTIAN; m.tex = t; return m; }
static Material mat_metal(V3 albedo, double fuzz) { Material m; memset(&m, 0, sizeof m); m.kind = MAT_METAL; m.albedo = albedo; m.fuzz = fuzz; return m; }
static Material mat_dielectric(double ir) { Material m; memset(&m, 0, sizeof m); m.kind = MAT_DIELECTRIC; m.ir = ir; return m; }
static Material mat_light(Texture t) { Material m; memset(&m, 0, sizeof m); m.kind = MAT_DIFFUSE_LIGHT; m.tex = t; return m; }
static Material mat_isotropic(Texture t) { Material m; memset(&m, 0, sizeof m); m.kind = MAT_ISOTROPIC; m.tex = t; return m; }

static Hittable* h_sphere(World* w, int mat, V3 c, double r)
{
    Hittable* h = hnew(w, H_SPHERE); h->mat = mat; h->center0 = c; h->radius = r; return h;
}
static Hittable* h_moving_sphere(World* w, int mat, V3 c0, V3 c1, double t0, double t1, double r)
{
    Hittable* h = hnew(w, H_MOVING_SPHERE);
    h->mat = mat; h->center0 = c0; h->center1 = c1; h->time0 = t0; h->time1 = t1; h->radius = r;
    return h;
}
static Hittable* h_rect(World* w, int kind, int mat, double a0, double a1, double b0, double b1, double k)
{
    Hittable* h = hnew(w, kind); h->mat = mat; h->a0 = a0; h->a1 = a1; h->b0 = b0; h->b1 = b1; h->k = k; return h;
}
static Hittable* h_box(World* w, V3 mn, V3 mx, int mat)                                   /* hittable.rs:132-145 */
{
    Hittable* h = hnew(w, H_BOX);
    h->mat = mat; h->bmin = mn; h->bmax = mx;
    h->sides = (Hittable*)arena_alloc(&w->arena, 6 * sizeof(Hittable));
    Hittable s[6];
    memset(s, 0, sizeof s);
    s[0].kind = H_XY; s[0].a0 = mn.x; s[0].a1 = mx.x; s[0].b0 = mn.y; s[0].b1 = mx.y; s[0].k = mx.z;
    s[1].kind = H_XY; s[1].a0 = mn.x; s[1].a1 = mx.x; s[1].b0 = mn.y; s[1].b1 = mx.y; s[1].k = mn.z;
    s[2].kind = H_XZ; s[2].a0 = mn.x; s[2].a1 = mx.x; s[2].b0 = mn.z; s[2].b1 = mx.z; s[2].k = mx.y;
    s[3].kind = H_XZ; s[3].a0 = mn.x; s[3].a1 = mx.x; s[3].b0 = mn.z; s[3].b1 = mx.z; s[3].k = mn.y;
    s[4].kind = H_YZ; s[4].a0 = mn.y; s[4].a1 = mx.y; s[4].b0 = mn.z; s[4].b1 = mx.z; s[4].k = mx.x;
    s[5].kind = H_YZ; s[5].a0 = mn.y; s[5].a1 = mx.y; s[5].b0 = mn.z; s[5].b1 = mx.z; s[5].k = mn.x;
    for (int i = 0; i < 6; ++i) { s[i].mat = mat; h->sides[i] = s[i]; }
    return h;
}
static Hittable* h_translate(World* w, const Hittable* p, V3 off)
{
    Hittable* h = hnew(w, H_TRANSLATE); h->ptr = p; h->offset = off; return h;
}

static V3 center_at_time(V3 c0, V3 c1, double t0, double t1, double time)               /* hittable.rs:556-558 */
{
    return vadd(c0, vscale(vsub(c1, c0), (time - t0) / (t1 - t0)));
}

static int bounding_box(const Hittable* h, double t0, double t1, AABB* out);

static Hittable* h_rotate_y(World* w, double angle, const Hittable* p)                  /* hittable.rs:147-199 */
{
    Hittable* h = hnew(w, H_ROTATE_Y);
    double radians = degrees_to_radians(angle);
    h->sin_theta = sin(radians);
    h->cos_theta = cos(radians);
    AABB bbox;
    if (bounding_box(p, 0.0, 1.0, &bbox)) h->has_box = 1;
    else { h->has_box = 0; bbox = aabb_new(v3(0, 0, 0), v3(0, 0, 0)); }
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
                double fi = i, fj = j, fk = k;
                double x = fi * bbox.maximum.x + (1.0 - fi) * bbox.minimum.x;
                double y = fj * bbox.maximum.y + (1.0 - fj) * bbox.minimum.y;
                double z = fk * bbox.maximum.z + (1.0 - fk) * bbox.minimum.z;
                double newx = h->cos_theta * x + h->sin_theta * z;
                double newz = -h->sin_theta * x + h->cos_theta * z;
                double tester[3] = {newx, y, newz};
                for (int c = 0; c < 3; ++c) { mn[c] = fmin(mn[c], tester[c]); mx[c] = fmax(mx[c], tester[c]); }
            }
    h->box = aabb_new(v3(mn[0], mn[1], mn[2]), v3(mx[0], mx[1], mx[2]));
    h->ptr = p;
    return h;
}
static Hittable* h_constant_medium(World* w, const Hittable* boundary, double d, int mat) /* hittable.rs:201-207 */
{
    Hittable* h = hnew(w, H_MEDIUM);
    h->mat = mat; h->ptr = boundary; h->neg_inv_density = -1.0 / d;
    h->medium_id = w->n_media++;
    return h;
}

static int bounding_box(const Hittable* h, double time0, double time1, AABB* out)       /* hittable.rs:475-554 */
{
    switch (h->kind) {
    case H_SPHERE: {
        V3 r = v3(h->radius, h->radius, h->radius);
        *out = aabb_new(vsub(h->center0, r), vadd(h->center0, r));
        return 1;
    }
    case H_MOVING_SPHERE: {
        V3 c0 = center_at_time(h->center0, h->center1, h->time0, h->time1, h->time0);
        V3 c1 = center_at_time(h->center0, h->center1, h->time0, h->time1, h->time1);
        V3 r = v3(h->radius, h->radius, h->radius);
        *out = surrounding_box(aabb_new(vsub(c0, r), vadd(c0, r)), aabb_new(vsub(c1, r), vadd(c1, r)));
        return 1;
    }
    case H_BVH: *out = h->box; return 1;
    case H_XY: *out = aabb_new(v3(h->a0, h->b0, h->k - 0.0001), v3(h->a1, h->b1, h->k + 0.0001)); return 1;
    case H_XZ: *out = aabb_new(v3(h->a0, h->k - 0.0001, h->b0), v3(h->a1, h->k + 0.0001, h->b1)); return 1;
    case H_YZ: *out = aabb_new(v3(h->k - 0.0001, h->a0, h->b0), v3(h->k + 0.0001, h->a1, h->b1)); return 1;
    case H_BOX: *out = aabb_new(h->bmin, h->bmax); return 1;
    case H_TRANSLATE: {
        AABB b;
        if (!bounding_box(h->ptr, time0, time1, &b)) return 0;
        *out = aabb_new(vadd(b.minimum, h->offset), vadd(b.maximum, h->offset));
        return 1;
    }
    case H_ROTATE_Y:
        if (!h->has_box) return 0;
        *out = h->box;
        return 1;
    default: return bounding_box(h->ptr, time0, time1, out);                              /* medium */
    }
}

/* aabb.rs:35-48: Less iff the minimum along axis is smaller; otherwise Greater (never Equal
 * when both boxes exist). `sort_by` is stable, so the order is the stable sort by key. */
static int box_is_less(const Hittable* a, const Hittable* b, int axis)
{
    AABB ba, bb;
    if (!bounding_box(a, 0.0, 0.0, &ba) || !bounding_box(b, 0.0, 0.0, &bb)) return 0;
    double am[3] = {ba.minimum.x, ba.minimum.y, ba.minimum.z};
    double bm[3] = {bb.minimum.x, bb.minimum.y, bb.minimum.z};
    return am[axis] < bm[axis];
}
static void stable_sort(const Hittable** v, int n, int axis, const Hittable** tmp)
{
    if (n < 2) return;
    int mid = n / 2;
    stable_sort(v, mid, axis, tmp);
    stable_sort(v + mid, n - mid, axis, tmp);
    int i = 0, j = mid, k = 0;
    while (i < mid && j < n) {
        if (box_is_less(v[j], v[i], axis)) tmp[k++] = v[j++];
        else tmp[k++] = v[i++];
    }
    while (i < mid) tmp[k++] = v[i++];
    while (j < n) tmp[k++] = v[j++];
    memcpy(v, tmp, (size_t)n * sizeof(*v));
}

static const Hittable* new_bvh_node(World* w, const Hittable* const* list, int start, int end,
                                    double time0, double time1)                           /* hittable.rs:77-130 */
{
    int n = end;
    const Hittable** cpy = (const Hittable**)malloc((size_t)(n > 0 ? n : 1) * sizeof(void*));
    memcpy(cpy, list, (size_t)n * sizeof(void*));
    Hittable* node = hnew(w, H_BVH);
    int axis = random_int_range(0, 2);
    if (axis != 0 && axis != 1) axis = 2;                                                  /* `_ =>` arm */
    int span = end - start;
    if (span == 1) {
        node->left = cpy[start];
        node->right = cpy[start];
    } else if (span == 2) {
        if (box_is_less(cpy[start], cpy[start + 1], axis)) { node->left = cpy[start]; node->right = cpy[start + 1]; }
        else { node->left = cpy[start + 1]; node->right = cpy[start]; }
    } else {
        const Hittable** tmp = (const Hittable**)malloc((size_t)span * sizeof(void*));
        stable_sort(cpy + start, span, axis, tmp);
        free(tmp);
        int mid = start + span / 2;
        node->left = new_bvh_node(w, cpy, start, mid, time0, time1);
        node->right = new_bvh_node(w, cpy, mid, end, time0, time1);
    }
    AABB bl, br;
    if (bounding_box(node->left, time0, time1, &bl) && bounding_box(node->right, time0, time1, &br))
        node->box = surrounding_box(bl, br);
    else
        node->box = aabb_new(v3(0, 0, 0), v3(0, 0, 0));
    free(cpy);
    return node;
}

static int hittable_hit(const Hittable* h, const Ray* r, double t_min, double t_max, HitRecord* rec);

static int hit_list(const Hittable* const* list, int n, const Ray* r, double t_min, double t_max,
                    HitRecord* rec)                                                       /* hittable.rs:43-55 */
{
    double closest_so_far = t_max;
    int any = 0;
    HitRecord tmp;
    for (int i = 0; i < n; ++i) {
        if (hittable_hit(list[i], r, t_min, closest_so_far, &tmp)) {
            closest_so_far = tmp.t;
            *rec = tmp;
            any = 1;
        }
    }
    return any;
}

static int sphere_hit(V3 center, double radius, const Ray* r, double t_min, double t_max, int mat,
                      HitRecord* rec)                                                     /* hittable.rs:254-288 */
{
    V3 oc = vsub(r->origin, center);
    double a = vlen2(r->direction);
    double half_b = vdot(oc, r->direction);
    double c = vlen2(oc) - radius * radius;
    double discriminant = half_b * half_b - a * c;
    if (discriminant < 0.0) return 0;
    double sqrtd = sqrt(discriminant);
    double root = (-half_b - sqrtd) / a;
    if (root < t_min || t_max < root) {
        root = (-half_b + sqrtd) / a;
        if (root < t_min || t_max < root) return 0;
    }
    memset(rec, 0, sizeof *rec);
    rec->mat_handle = mat;
    rec->t = root;
    rec->point = ray_at(r, rec->t);
    V3 outward_normal = vdiv(vsub(rec->point, center), radius);
    set_face_normal(rec, r, outward_normal);
    sphere_uv(outward_normal, &rec->u, &rec->v);
    return 1;
}

static int bvh_node_hit(const Hittable* h, const Ray* r, double t_min, double t_max, HitRecord* rec) /* :290-306 */
{
    if (!aabb_hit(&h->box, r, t_min, t_max)) return 0;
    HitRecord hl, hr;
    if (hittable_hit(h->left, r, t_min, t_max, &hl)) {
        if (hittable_hit(h->right, r, t_min, hl.t, &hr)) *rec = hr;
        else *rec = hl;
        return 1;
    }
    if (hittable_hit(h->right, r, t_min, t_max, &hr)) { *rec = hr; return 1; }
    return 0;
}

/* hittable.rs:308-384; axis 0: XY (k along z), 1: XZ (k along y), 2: YZ (k along x) */
static int rect_hit(const Hittable* h, const Ray* r, double t_min, double t_max, int mat, HitRecord* rec)
{
    double o[3] = {r->origin.x, r->origin.y, r->origin.z};
    double d[3] = {r->direction.x, r->direction.y, r->direction.z};
    int ka, aa, ba;
    V3 n;
    if (h->kind == H_XY) { ka = 2; aa = 0; ba = 1; n = v3(0, 0, 1); }
    else if (h->kind == H_XZ) { ka = 1; aa = 0; ba = 2; n = v3(0, 1, 0); }
    else { ka = 0; aa = 1; ba = 2; n = v3(1, 0, 0); }
    double t = (h->k - o[ka]) / d[ka];
    if (t < t_min || t > t_max) return 0;
    double x = o[aa] + t * d[aa];
    double y = o[ba] + t * d[ba];
    if (x < h->a0 || x > h->a1 || y < h->b0 || y > h->b1) return 0;
    memset(rec, 0, sizeof *rec);
    rec->u = (x - h->a0) / (h->a1 - h->a0);
    rec->v = (y - h->b0) / (h->b1 - h->b0);
    rec->t = t;
    set_face_normal(rec, r, n);
    rec->mat_handle = mat;
    rec->point = ray_at(r, t);
    return 1;
}

static int rotate_y_hit(const Hittable* h, const Ray* r, double t_min, double t_max, HitRecord* rec) /* :386-415 */
{
    V3 origin = r->origin, direction = r->direction;
    double s = h->sin_theta, c = h->cos_theta;
    origin.x = c * r->origin.x - s * r->origin.z;
    origin.z = s * r->origin.x + c * r->origin.z;
    direction.x = c * r->direction.x - s * r->direction.z;
    direction.z = s * r->direction.x + c * r->direction.z;
    Ray rotated = ray_with_time(origin, direction, r->time);
    if (!hittable_hit(h->ptr, &rotated, t_min, t_max, rec)) return 0;
    V3 p = rec->point, normal = rec->normal;
    p.x = c * rec->point.x + s * rec->point.z;
    p.z = -s * rec->point.x + c * rec->point.z;
    normal.x = c * rec->normal.x + s * rec->normal.z;
    normal.z = -s * rec->normal.x + c * rec->normal.z;
    rec->point = p;
    set_face_normal(rec, &rotated, normal);                                               /* Q7 */
    return 1;
}

static int medium_hit(const Hittable* h, const Ray* r, double t_min, double t_max, HitRecord* rec) /* :417-473 */
{
    HitRecord rec1, rec2;
    if (!hittable_hit(h->ptr, r, -INFINITY, INFINITY, &rec1)) return 0;
    if (!hittable_hit(h->ptr, r, rec1.t + 0.0001, INFINITY, &rec2)) return 0;
    if (rec1.t < t_min) rec1.t = t_min;
    if (rec2.t > t_max) rec2.t = t_max;
    if (rec1.t >= rec2.t) return 0;
    if (rec1.t < 0.0) rec1.t = 0.0;
    double ray_length = vlen(r->direction);
    double distance_inside_boundary = (rec2.t - rec1.t) * ray_length;
    double hit_distance = h->neg_inv_density * rt_log(medium_random_double(h->medium_id));
    if (hit_distance > distance_inside_boundary) return 0;
    memset(rec, 0, sizeof *rec);
    rec->t = rec1.t + hit_distance / ray_length;
    rec->point = ray_at(r, rec->t);
    rec->normal = v3(1.0, 0.0, 0.0);
    rec->front_face = 1;
    rec->mat_handle = h->mat;
    return 1;
}

static int hittable_hit(const Hittable* h, const Ray* r, double t_min, double t_max, HitRecord* rec) /* :209-252 */
{
    switch (h->kind) {
    case H_SPHERE: return sphere_hit(h->center0, h->radius, r, t_min, t_max, h->mat, rec);
    case H_MOVING_SPHERE:
        return sphere_hit(center_at_time(h->center0, h->center1, h->time0, h->time1, r->time), h->radius, r,
                          t_min, t_max, h->mat, rec);
    case H_BVH: return bvh_node_hit(h, r, t_min, t_max, rec);
    case H_XY: case H_XZ: case H_YZ: return rect_hit(h, r, t_min, t_max, h->mat, rec);
    case H_BOX: {
        const Hittable* sides[6];
        for (int i = 0; i < 6; ++i) sides[i] = &h->sides[i];
        return hit_list(sides, 6, r, t_min, t_max, rec);
    }
    case H_TRANSLATE: {                                                                   /* :232-244 */
        Ray moved = ray_with_time(vsub(r->origin, h->offset), r->direction, r->time);
        if (!hittable_hit(h->ptr, &moved, t_min, t_max, rec)) return 0;
        rec->point = vadd(rec->point, h->offset);
        V3 normal = rec->normal;
        set_face_normal(rec, &moved, normal);                                             /* Q6 */
        return 1;
    }
    case H_ROTATE_Y: return rotate_y_hit(h, r, t_min, t_max, rec);
    default: return medium_hit(h, r, t_min, t_max, rec);
    }
}

/* ------------------------------------------------------------------------- */
/* camera.rs                                                                  */
/* ------------------------------------------------------------------------- */
typedef struct {
    V3 origin, lower_left_corner, horizontal, vertical, u, v, w;
    double lens_radius, time0, time1;
} Camera;

static Camera camera_new(V3 look_from, V3 look_at, V3 vup, double vfov, double aspect_ratio,
                         double aperture, double focus_dist, double time0, double time1) /* camera.rs:18-56 */
{
    Camera c;
    double theta = degrees_to_radians(vfov);
    double h = tan(theta / 2.0);
    double viewport_height = 2.0 * h;
    double viewport_width = aspect_ratio * viewport_height;
    c.w = vnormalize(vsub(look_from, look_at));
    c.u = vnormalize(vcross(vup, c.w));
    c.v = vcross(c.w, c.u);
    c.origin = look_from;
    c.horizontal = vscale(c.u, focus_dist * viewport_width);
    c.vertical = vscale(c.v, focus_dist * viewport_height);
    c.lower_left_corner = vsub(vsub(vsub(c.origin, vscale(c.horizontal, 0.5)), vscale(c.vertical, 0.5)),
                               vscale(c.w, focus_dist));
    c.lens_radius = aperture * 0.5;
    c.time0 = time0;
    c.time1 = time1;
    return c;
}

static Ray camera_get_ray(const Camera* c, double s, double t)                           /* camera.rs:58-66 */
{
    V3 rd = vscale(random_in_unit_disk(), c->lens_radius);
    V3 offset = vadd(vscale(c->u, rd.x), vscale(c->v, rd.y));
    V3 origin = vadd(c->origin, offset);
    V3 dir = vsub(vsub(vadd(vadd(c->lower_left_corner, vscale(c->horizontal, s)), vscale(c->vertical, t)),
                       c->origin),
                  offset);
    double time = random_double_range(c->time0, c->time1);
    return ray_with_time(origin, dir, time);
}

/* ------------------------------------------------------------------------- */
/* main.rs — scene builders                                                   */
/* ------------------------------------------------------------------------- */
static void two_spheres_scene(World* w)                                                  /* main.rs:52-63 */
{
    int ground = register_material(w, mat_lambertian(tex_checker(v3(0.2, 0.3, 0.1), v3(0.9, 0.9, 0.9))));
    world_push(w, h_sphere(w, ground, v3(0.0, -10.0, 0.0), 10.0));
    world_push(w, h_sphere(w, ground, v3(0.0, 10.0, 0.0), 10.0));
}
static void arena_adopt(Arena* a, void* p)
{
    void* q = arena_alloc(a, 1);
    free(q);
    a->ptrs[a->n - 1] = p;
}
static Perlin* world_perlin(World* w)
{
    Perlin* p = perlin_new();
    arena_adopt(&w->arena, p);
    return p;
}
static void two_perlin_spheres_scene(World* w)                                           /* main.rs:65-76 */
{
    int ground = register_material(w, mat_lambertian(tex_noise(world_perlin(w), 4.0)));
    world_push(w, h_sphere(w, ground, v3(0.0, -1000.0, 0.0), 1000.0));
    world_push(w, h_sphere(w, ground, v3(0.0, 2.0, 0.0), 2.0));
}
static void earth_scene(World* w)                                                        /* main.rs:78-89 */
{
    int earth = register_material(w, mat_lambertian(tex_image(w->image, w->image_w, w->image_h)));
    world_push(w, h_sphere(w, earth, v3(0.0, 0.0, 0.0), 2.0));
}
static void simple_light_scene(World* w)                                                 /* main.rs:91-105 */
{
    int ground = register_material(w, mat_lambertian(tex_noise(world_perlin(w), 4.0)));
    world_push(w, h_sphere(w, ground, v3(0.0, -1000.0, 0.0), 1000.0));
    world_push(w, h_sphere(w, ground, v3(0.0, 2.0, 0.0), 2.0));
    int light = register_material(w, mat_light(tex_solid(v3(4.0, 4.0, 4.0))));
    world_push(w, h_rect(w, H_XY, light, 3.0, 5.0, 1.0, 3.0, -2.0));
}
static void cornell_walls(World* w, int red, int white, int green, int light, double lx0, double lx1,
                          double lz0, double lz1)                                         /* main.rs:118-123 */
{
    world_push(w, h_rect(w, H_YZ, green, 0.0, 555.0, 0.0, 555.0, 555.0));
    world_push(w, h_rect(w, H_YZ, red, 0.0, 555.0, 0.0, 555.0, 0.0));
    world_push(w, h_rect(w, H_XZ, light, lx0, lx1, lz0, lz1, 554.0));
    world_push(w, h_rect(w, H_XZ, white, 0.0, 555.0, 0.0, 555.0, 0.0));
    world_push(w, h_rect(w, H_XZ, white, 0.0, 555.0, 0.0, 555.0, 555.0));
    world_push(w, h_rect(w, H_XY, white, 0.0, 555.0, 0.0, 555.0, 555.0));
}
static void cornell_box_scene(World* w)                                                  /* main.rs:107-136 */
{
    int red = register_material(w, mat_lambertian(tex_solid(v3(0.65, 0.05, 0.05))));
    int white = register_material(w, mat_lambertian(tex_solid(v3(0.73, 0.73, 0.73))));
    int green = register_material(w, mat_lambertian(tex_solid(v3(0.12, 0.45, 0.15))));
    int light = register_material(w, mat_light(tex_solid(v3(15.0, 15.0, 15.0))));
    cornell_walls(w, red, white, green, light, 213.0, 343.0, 227.0, 332.0);
    const Hittable* box1 = h_box(w, v3(0, 0, 0), v3(165.0, 330.0, 165.0), white);
    box1 = h_rotate_y(w, 15.0, box1);
    box1 = h_translate(w, box1, v3(265.0, 0.0, 295.0));
    world_push(w, box1);
    const Hittable* box2 = h_box(w, v3(0, 0, 0), v3(165.0, 165.0, 165.0), white);
    box2 = h_rotate_y(w, -18.0, box2);
    box2 = h_translate(w, box2, v3(130.0, 0.0, 65.0));
    world_push(w, box2);
}
static void cornell_box_smoke_scene(World* w)                                            /* main.rs:138-171 */
{
    int red = register_material(w, mat_lambertian(tex_solid(v3(0.65, 0.05, 0.05))));
    int white = register_material(w, mat_lambertian(tex_solid(v3(0.73, 0.73, 0.73))));
    int green = register_material(w, mat_lambertian(tex_solid(v3(0.12, 0.45, 0.15))));
    int light = register_material(w, mat_light(tex_solid(v3(7.0, 7.0, 7.0))));
    cornell_walls(w, red, white, green, light, 113.0, 443.0, 127.0, 432.0);
    int box1_phase = register_material(w, mat_isotropic(tex_solid(v3(0.0, 0.0, 0.0))));
    const Hittable* box1 = h_box(w, v3(0, 0, 0), v3(165.0, 330.0, 165.0), white);
    box1 = h_rotate_y(w, 15.0, box1);
    box1 = h_translate(w, box1, v3(265.0, 0.0, 295.0));
    box1 = h_constant_medium(w, box1, 0.01, box1_phase);
    world_push(w, box1);
    int box2_phase = register_material(w, mat_isotropic(tex_solid(v3(1.0, 1.0, 1.0))));
    const Hittable* box2 = h_box(w, v3(0, 0, 0), v3(165.0, 165.0, 165.0), white);
    box2 = h_rotate_y(w, -18.0, box2);
    box2 = h_translate(w, box2, v3(130.0, 0.0, 65.0));
    box2 = h_constant_medium(w, box2, 0.01, box2_phase);
    world_push(w, box2);
}
static void final_scene(World* w)                                                        /* main.rs:173-243 */
{
    enum { BOXES_PER_SIDE = 20 };
    const Hittable* boxes1[BOXES_PER_SIDE * BOXES_PER_SIDE];
    int nb = 0;
    int ground = register_material(w, mat_lambertian(tex_solid(v3(0.48, 0.83, 0.53))));
    for (int i = 0; i < BOXES_PER_SIDE; ++i)
        for (int j = 0; j < BOXES_PER_SIDE; ++j) {
            double wd = 100.0;
            double x0 = -1000.0 + (double)i * wd;
            double z0 = -1000.0 + (double)j * wd;
            double y0 = 0.0;
            double x1 = x0 + wd;
            double y1 = random_double_range(1.0, 101.0);
            double z1 = z0 + wd;
            boxes1[nb++] = h_box(w, v3(x0, y0, z0), v3(x1, y1, z1), ground);
        }
    world_push(w, new_bvh_node(w, boxes1, 0, nb, 0.0, 1.0));
    int light = register_material(w, mat_light(tex_solid(v3(7.0, 7.0, 7.0))));
    world_push(w, h_rect(w, H_XZ, light, 123.0, 423.0, 147.0, 412.0, 554.0));
    V3 center_1 = v3(400.0, 400.0, 200.0);
    V3 center_2 = vadd(center_1, v3(30.0, 0.0, 0.0));
    int msm = register_material(w, mat_lambertian(tex_solid(v3(0.7, 0.3, 0.1))));
    world_push(w, h_moving_sphere(w, msm, center_1, center_2, 0.0, 1.0, 50.0));
    int dielectric = register_material(w, mat_dielectric(1.5));
    world_push(w, h_sphere(w, dielectric, v3(260.0, 150.0, 45.0), 50.0));
    int metal = register_material(w, mat_metal(v3(0.8, 0.8, 0.9), 1.0));
    world_push(w, h_sphere(w, metal, v3(0.0, 150.0, 145.0), 50.0));
    const Hittable* boundary = h_sphere(w, dielectric, v3(360.0, 150.0, 145.0), 70.0);
    world_push(w, boundary);
    int phase = register_material(w, mat_isotropic(tex_solid(v3(0.2, 0.4, 0.9))));
    world_push(w, h_constant_medium(w, boundary, 0.2, phase));
    boundary = h_sphere(w, dielectric, v3(0.0, 0.0, 0.0), 5000.0);
    phase = register_material(w, mat_isotropic(tex_solid(v3(1.0, 1.0, 1.0))));
    world_push(w, h_constant_medium(w, boundary, 0.0001, phase));
    int emat = register_material(w, mat_lambertian(tex_image(w->image, w->image_w, w->image_h)));
    world_push(w, h_sphere(w, emat, v3(400.0, 200.0, 400.0), 100.0));
    int pertext = register_material(w, mat_lambertian(tex_noise(world_perlin(w), 0.1)));
    world_push(w, h_sphere(w, pertext, v3(220.0, 280.0, 300.0), 80.0));
    const Hittable* boxes2[1000];
    int white = register_material(w, mat_lambertian(tex_solid(v3(0.73, 0.73, 0.73))));
    for (int j = 0; j < 1000; ++j) boxes2[j] = h_sphere(w, white, v3_random_range(0.0, 165.0), 10.0);
    const Hittable* bvh2 = new_bvh_node(w, boxes2, 0, 1000, 0.0, 1.0);
    world_push(w, h_translate(w, h_rotate_y(w, 15.0, bvh2), v3(-100.0, 270.0, 395.0)));
}
static void random_scene(World* w)                                                       /* main.rs:245-289 */
{
    int ground = register_material(w, mat_lambertian(tex_checker(v3(0.2, 0.5, 0.5), v3(0.9, 0.9, 0.9))));
    world_push(w, h_sphere(w, ground, v3(0.0, -1000.0, 0.0), 1000.0));
    for (int a = -11; a < 11; ++a)
        for (int b = -11; b < 11; ++b) {
            double choose_mat = random_double();
            double cx = (double)a + 0.9 * random_double();
            double cz = (double)b + 0.9 * random_double();
            V3 center = v3(cx, 0.2, cz);
            if (vlen(vsub(center, v3(4.0, 0.2, 0.0))) > 0.9) {
                if (choose_mat < 0.8) {
                    V3 albedo = v3_random();
                    int m = register_material(w, mat_lambertian(tex_solid(albedo)));
                    V3 center2 = vadd(center, v3(0.0, random_double_range(0.0, 0.5), 0.0));
                    world_push(w, h_moving_sphere(w, m, center, center2, 0.0, 1.0, 0.2));
                } else if (choose_mat < 0.95) {
                    V3 albedo = v3_random_range(0.5, 1.0);
                    double fuzz = random_double_range(0.0, 0.5);
                    int m = register_material(w, mat_metal(albedo, fuzz));
                    world_push(w, h_sphere(w, m, center, 0.2));
                } else {
                    int m = register_material(w, mat_dielectric(1.5));
                    world_push(w, h_sphere(w, m, center, 0.2));
                }
            }
        }
    int m1 = register_material(w, mat_dielectric(1.5));
    world_push(w, h_sphere(w, m1, v3(0.0, 1.0, 0.0), 1.0));
    int m2 = register_material(w, mat_lambertian(tex_solid(v3(0.4, 0.2, 0.1))));
    world_push(w, h_sphere(w, m2, v3(-4.0, 1.0, 0.0), 1.0));
    int m3 = register_material(w, mat_metal(v3(0.7, 0.6, 0.5), 0.0));
    world_push(w, h_sphere(w, m3, v3(4.0, 1.0, 0.0), 1.0));
}

/* main.rs:296-305, 314-464: per-scene camera and background. */
typedef struct { V3 look_from, look_at, background; double vfov; } ScenePreset;
static int scene_preset(int id, ScenePreset* p)
{
    switch (id) {
    case 0: case 1: case 2: case 3:
        p->look_from = v3(13.0, 2.0, 3.0); p->look_at = v3(0.0, 0.0, 0.0);
        p->background = v3(0.7, 0.8, 1.0); p->vfov = 20.0; return 0;
    case 4:
        p->look_from = v3(26.0, 3.0, 6.0); p->look_at = v3(0.0, 2.0, 0.0);
        p->background = v3(0.0, 0.0, 0.0); p->vfov = 20.0; return 0;
    case 5: case 6:
        p->look_from = v3(278.0, 278.0, -800.0); p->look_at = v3(278.0, 278.0, 0.0);
        p->background = v3(0.0, 0.0, 0.0); p->vfov = 40.0; return 0;
    case 7:
        p->look_from = v3(478.0, 278.0, -600.0); p->look_at = v3(278.0, 278.0, 0.0);
        p->background = v3(0.0, 0.0, 0.0); p->vfov = 40.0; return 0;
    default: return -1;                                                                   /* main.rs:461-463 */
    }
}

static int build_world(World* w, int scene_id, uint64_t scene_seed, const uint8_t* img, int iw, int ih)
{
    OrcRng rng;
    memset(&rng, 0, sizeof rng);
    rt_stream_init(&rng.s, scene_seed, 0, 0, RT_STREAM_SCENE);
    rng.seed = scene_seed;
    OrcRng* saved = tl_rng;
    tl_rng = &rng;
    memset(w, 0, sizeof *w);
    w->image = img; w->image_w = iw; w->image_h = ih;
    int rc = 0;
    switch (scene_id) {
    case 0: random_scene(w); break;
    case 1: two_spheres_scene(w); break;
    case 2: two_perlin_spheres_scene(w); break;
    case 3: earth_scene(w); break;
    case 4: simple_light_scene(w); break;
    case 5: cornell_box_scene(w); break;
    case 6: cornell_box_smoke_scene(w); break;
    case 7: final_scene(w); break;
    default: rc = -1;
    }
    tl_rng = saved;
    return rc;
}

/* ------------------------------------------------------------------------- */
/* main.rs:19-38 — the integrator                                             */
/* ------------------------------------------------------------------------- */
typedef struct {
    const World* world;
    V3 background;
    int max_depth;
    uint64_t casts;
} RenderCtx;

static V3 ray_color(RenderCtx* ctx, const Ray* r, int depth)
{
    if (depth <= 0) return v3(0.0, 0.0, 0.0);
    tl_rng->bounce = (uint32_t)(ctx->max_depth - depth);
    ctx->casts++;
    HitRecord rec;
    if (hit_list(ctx->world->hittables, ctx->world->n_hittables, r, 0.001, INFINITY, &rec)) {
        const Material* m = &ctx->world->materials[rec.mat_handle - 1];
        V3 emitted = mat_emitted(m, rec.u, rec.v, rec.point);
        Ray scattered;
        V3 attenuation;
        if (mat_scatter(m, r, &rec, &scattered, &attenuation))
            return vadd(emitted, vmul(attenuation, ray_color(ctx, &scattered, depth - 1)));
        return emitted;
    }
    return ctx->background;
}

/* ------------------------------------------------------------------------- */
/* main.rs:497-551 — the driver loop, threaded                                */
/* ------------------------------------------------------------------------- */
typedef struct {
    const orc_params* p;
    const World* world;
    const Camera* cam;
    V3 background;
    double* out;      /* rows_local x W x 3 */
    int n_rows;
    int tid, nthreads;
    int s_begin, s_end;  /* sample range (sample split) */
    uint64_t casts;
} Job;

static void render_pixel(Job* job, RenderCtx* ctx, OrcRng* rng, int x, int y, int s_begin, int s_end, V3* acc)
{
    const orc_params* p = job->p;
    const int chunk = p->spp_chunk > 0 ? p->spp_chunk : p->spp;
    V3 total = *acc;
    V3 part = v3(0, 0, 0);
    int in_chunk = 0;
    for (int s = s_begin; s < s_end; ++s) {
        rng->pixel = (uint32_t)y * (uint32_t)p->width + (uint32_t)x;
        rng->sample = (uint32_t)s;
        rt_pstream_init(&rng->ps, p->render_seed, rng->pixel, rng->sample);
        rng->render = 1;
        double u = ((double)x + random_double()) / ((double)p->width - 1.0);              /* main.rs:517 */
        double v = ((double)y + random_double()) / ((double)p->height - 1.0);             /* main.rs:518 */
        Ray r = camera_get_ray(job->cam, u, v);                                           /* main.rs:520 */
        V3 c = ray_color(ctx, &r, p->max_depth);                                          /* main.rs:522 */
        part = vadd(part, c);
        if (++in_chunk == chunk) { total = vadd(total, part); part = v3(0, 0, 0); in_chunk = 0; }
    }
    if (in_chunk) total = vadd(total, part);
    *acc = total;
}

static void* worker(void* arg)
{
    Job* job = (Job*)arg;
    const orc_params* p = job->p;
    OrcRng rng;
    memset(&rng, 0, sizeof rng);
    rng.seed = p->render_seed;
    tl_rng = &rng;
    RenderCtx ctx = {job->world, job->background, p->max_depth, 0};
    for (int k = 0; k < job->n_rows; ++k) {
        int y = p->row_begin + k * p->row_stride;
        for (int x = 0; x < p->width; ++x) {
            /* the row split deals pixels round-robin (a pixel's sum does not depend on the
               thread that computes it), so a render of a few rows still uses every thread */
            if (p->split == ORC_SPLIT_ROWS && ((size_t)k * p->width + x) % job->nthreads != (size_t)job->tid) continue;
            V3 acc = v3(0, 0, 0);
            render_pixel(job, &ctx, &rng, x, y, job->s_begin, job->s_end, &acc);
            double* o = job->out + ((size_t)k * p->width + x) * 3;
            o[0] = acc.x; o[1] = acc.y; o[2] = acc.z;
        }
    }
    job->casts = ctx.casts;
    tl_rng = NULL;
    return NULL;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int render_world(const orc_params* p, const World* w, const Camera* cam, V3 background, double* out_mean,
                        orc_stats* stats);

int orc_render(const orc_params* p, double* out_mean, orc_stats* stats)
{
    if (!p || !out_mean || p->width < 2 || p->height < 2 || p->spp < 1 || p->row_stride < 1 || p->row_begin < 0)
        return -1;
    if ((p->scene_id == 3 || p->scene_id == 7) && !p->image_rgb) return -2;
    ScenePreset sp;
    if (scene_preset(p->scene_id, &sp)) return -1;
    World w;
    if (build_world(&w, p->scene_id, p->scene_seed, p->image_rgb, p->image_w, p->image_h)) return -1;
    double aspect = (double)p->width / (double)p->height;
    Camera cam = camera_new(sp.look_from, sp.look_at, v3(0.0, 1.0, 0.0), sp.vfov, aspect, 0.1, 10.0, 0.0, 1.0);
    int rc = render_world(p, &w, &cam, sp.background, out_mean, stats);
    world_free(&w);
    return rc;
}

/* main.rs:466-551 for a built world, camera and background */
static int render_world(const orc_params* p, const World* wp, const Camera* camp, V3 background, double* out_mean,
                        orc_stats* stats)
{
    const World w = *wp;
    const Camera cam = *camp;
    const ScenePreset sp = {v3(0, 0, 0), v3(0, 0, 0), background, 0.0};
    int n_rows = p->row_begin < p->height ? (p->height - p->row_begin + p->row_stride - 1) / p->row_stride : 0;
    int T = p->threads > 0 ? p->threads : 1;
    double t0 = now_s();
    Job* jobs = (Job*)calloc((size_t)T, sizeof(Job));
    pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
    double** bufs = (double**)calloc((size_t)T, sizeof(double*));
    size_t n_out = (size_t)n_rows * p->width * 3;
    for (int t = 0; t < T; ++t) {
        jobs[t].p = p; jobs[t].world = &w; jobs[t].cam = &cam; jobs[t].background = sp.background;
        jobs[t].n_rows = n_rows; jobs[t].tid = t; jobs[t].nthreads = T;
        if (p->split == ORC_SPLIT_SAMPLES) {
            jobs[t].s_begin = (int)((long long)p->spp * t / T);
            jobs[t].s_end = (int)((long long)p->spp * (t + 1) / T);
            bufs[t] = (double*)calloc(n_out ? n_out : 1, sizeof(double));
            jobs[t].out = bufs[t];
        } else {
            jobs[t].s_begin = 0;
            jobs[t].s_end = p->spp;
            jobs[t].out = out_mean;
        }
        if (T == 1) worker(&jobs[t]);
        else pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    if (T > 1)
        for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
    if (p->split == ORC_SPLIT_SAMPLES) {                                                  /* main.rs:542-547 */
        memset(out_mean, 0, n_out * sizeof(double));
        for (int t = 0; t < T; ++t) {
            for (size_t i = 0; i < n_out; ++i) out_mean[i] += bufs[t][i];
            free(bufs[t]);
        }
    }
    const double scale = 1.0 / (double)p->spp;                                            /* math.rs:120 */
    for (size_t i = 0; i < n_out; ++i) out_mean[i] = out_mean[i] * scale;
    double t1 = now_s();
    if (stats) {
        stats->casts = 0;
        for (int t = 0; t < T; ++t) stats->casts += jobs[t].casts;
        stats->samples = (uint64_t)n_rows * p->width * p->spp;
        stats->seconds = t1 - t0;
    }
    free(jobs); free(th); free(bufs);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* probes                                                                     */
/* ------------------------------------------------------------------------- */
static void count_leaves(const Hittable* h, int* n, double* cs)
{
    switch (h->kind) {
    case H_BVH:
        count_leaves(h->left, n, cs);
        if (h->right != h->left) count_leaves(h->right, n, cs);
        return;
    case H_TRANSLATE: case H_ROTATE_Y: case H_MEDIUM:
        count_leaves(h->ptr, n, cs);
        return;
    default:
        (*n)++;
        *cs += h->center0.x + 2.0 * h->center0.y + 3.0 * h->center0.z + h->radius + h->k + h->bmax.y +
               h->center1.y;
        return;
    }
}

int orc_scene_info(int scene_id, uint64_t scene_seed, const uint8_t* image_rgb, int iw, int ih,
                   int* n_hittables, int* n_materials, int* n_leaf_prims, double* checksum)
{
    World w;
    if (build_world(&w, scene_id, scene_seed, image_rgb, iw, ih)) return -1;
    int n = 0;
    double cs = 0.0;
    for (int i = 0; i < w.n_hittables; ++i) count_leaves(w.hittables[i], &n, &cs);
    for (int i = 0; i < w.n_materials; ++i)
        cs += 0.5 * (w.materials[i].albedo.x + w.materials[i].tex.c0.y + w.materials[i].fuzz + w.materials[i].ir);
    if (n_hittables) *n_hittables = w.n_hittables;
    if (n_materials) *n_materials = w.n_materials;
    if (n_leaf_prims) *n_leaf_prims = n;
    if (checksum) *checksum = cs;
    world_free(&w);
    return 0;
}

int orc_eval(int fn, const double* x, const double* y, const double* z, double* out, int n)
{
    for (int i = 0; i < n; ++i) {
        double u, v;
        switch (fn) {
        case 0: out[i] = rt_sin(x[i]); break;
        case 1: out[i] = rt_cos(x[i]); break;
        case 2: out[i] = rt_log(x[i]); break;
        case 3: out[i] = rt_atan2(x[i], y[i]); break;
        case 4: out[i] = rt_acos(x[i]); break;
        case 5: sphere_uv(v3(x[i], y[i], z[i]), &u, &v); out[i] = u; break;
        case 6: sphere_uv(v3(x[i], y[i], z[i]), &u, &v); out[i] = v; break;
        case 7: out[i] = rt_pow5(x[i]); break;
        case 8: out[i] = sqrt(x[i]); break;
        case 9: out[i] = x[i] / y[i]; break;
        case 10: out[i] = rt_unit53(rt_f64_bits(x[i])); break;
        case 11: out[i] = rt_uniform_sample(rt_f64_bits(x[i]), -1.0, rt_uniform_incl_scale(-1.0, 1.0)); break;
        case 12: out[i] = (double)rt_sin_sign(x[i]); break;
        case 13: out[i] = x[i] / y[i]; break;   /* the kernel's reciprocal division (div_rcp) */
        default: return -1;
        }
    }
    return 0;
}

void orc_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out)
{
    rt_u32x4 c;
    for (int i = 0; i < 4; ++i) c.v[i] = ctr[i];
    rt_u32x4 r = rt_philox4x32_10(c, key[0], key[1]);
    for (int i = 0; i < 4; ++i) out[i] = r.v[i];
}

void orc_pstream(uint64_t seed, uint32_t pixel, uint32_t sample, int n, uint64_t* out)
{
    rt_pstream ps;
    rt_pstream_init(&ps, seed, pixel, sample);
    for (int i = 0; i < n; ++i) out[i] = rt_pstream_u64(&ps);
}

int orc_camera(int scene_id, int width, int height, double* o)
{
    ScenePreset sp;
    if (scene_preset(scene_id, &sp) || width < 1 || height < 1) return -1;
    Camera c = camera_new(sp.look_from, sp.look_at, v3(0.0, 1.0, 0.0), sp.vfov, (double)width / (double)height,
                          0.1, 10.0, 0.0, 1.0);
    V3 vs[7] = {c.origin, c.lower_left_corner, c.horizontal, c.vertical, c.u, c.v, c.w};
    for (int i = 0; i < 7; ++i) { o[3 * i] = vs[i].x; o[3 * i + 1] = vs[i].y; o[3 * i + 2] = vs[i].z; }
    o[21] = c.lens_radius;
    o[22] = c.time0;
    o[23] = c.time1;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* world builder: the reference's constructor surface (main.rs:40-50,         */
/* hittable.rs:77-207, material.rs:6-12, texture.rs:4-22) for custom worlds   */
/* ------------------------------------------------------------------------- */
struct orc_world {
    World w;
    OrcRng rng;                /* construction draws: Perlin::new, the BVH's random axis */
    Texture* tex; int n_tex, cap_tex;
    const Hittable** ids; int n_ids, cap_ids;
};

static int ow_add(orc_world* o, const Hittable* h)
{
    if (o->n_ids == o->cap_ids) {
        o->cap_ids = o->cap_ids ? 2 * o->cap_ids : 64;
        o->ids = (const Hittable**)realloc(o->ids, (size_t)o->cap_ids * sizeof(void*));
    }
    o->ids[o->n_ids] = h;
    return o->n_ids++;
}
static int ow_tex(orc_world* o, Texture t)
{
    if (o->n_tex == o->cap_tex) {
        o->cap_tex = o->cap_tex ? 2 * o->cap_tex : 16;
        o->tex = (Texture*)realloc(o->tex, (size_t)o->cap_tex * sizeof(Texture));
    }
    o->tex[o->n_tex] = t;
    return o->n_tex++;
}
static const Hittable* ow_get(const orc_world* o, int id) { return (id >= 0 && id < o->n_ids) ? o->ids[id] : NULL; }

int orc_world_create(uint64_t scene_seed, orc_world** out)
{
    orc_world* o = (orc_world*)calloc(1, sizeof(orc_world));
    if (!o) return -1;
    rt_stream_init(&o->rng.s, scene_seed, 0, 0, RT_STREAM_SCENE);   /* as build_world */
    o->rng.seed = scene_seed;
    *out = o;
    return 0;
}
void orc_world_destroy(orc_world* o)
{
    if (!o) return;
    world_free(&o->w);
    free(o->tex);
    free(o->ids);
    free(o);
}
int orc_world_texture(orc_world* o, int kind, const double c0[3], const double c1[3], double scale)
{
    switch (kind) {
    case TEX_SOLID: return ow_tex(o, tex_solid(v3(c0[0], c0[1], c0[2])));
    case TEX_CHECKER: return ow_tex(o, tex_checker(v3(c0[0], c0[1], c0[2]), v3(c1[0], c1[1], c1[2])));
    case TEX_NOISE: {
        OrcRng* saved = tl_rng;
        tl_rng = &o->rng;
        Perlin* p = world_perlin(&o->w);
        tl_rng = saved;
        return ow_tex(o, tex_noise(p, scale));
    }
    default: return -1;
    }
}
int orc_world_material(orc_world* o, int kind, int tex, const double albedo[3], double fuzz, double ir)
{
    Texture t;
    memset(&t, 0, sizeof t);
    if (kind == MAT_LAMBERTIAN || kind == MAT_DIFFUSE_LIGHT || kind == MAT_ISOTROPIC) {
        if (tex < 0 || tex >= o->n_tex) return -1;
        t = o->tex[tex];
    }
    switch (kind) {
    case MAT_LAMBERTIAN: return register_material(&o->w, mat_lambertian(t));
    case MAT_METAL: return register_material(&o->w, mat_metal(v3(albedo[0], albedo[1], albedo[2]), fuzz));
    case MAT_DIELECTRIC: return register_material(&o->w, mat_dielectric(ir));
    case MAT_DIFFUSE_LIGHT: return register_material(&o->w, mat_light(t));
    case MAT_ISOTROPIC: return register_material(&o->w, mat_isotropic(t));
    default: return -1;
    }
}
int orc_world_sphere(orc_world* o, int mat, const double c[3], double r)
{
    return ow_add(o, h_sphere(&o->w, mat, v3(c[0], c[1], c[2]), r));
}
int orc_world_moving_sphere(orc_world* o, int mat, const double c0[3], const double c1[3], double t0, double t1,
                            double r)
{
    return ow_add(o, h_moving_sphere(&o->w, mat, v3(c0[0], c0[1], c0[2]), v3(c1[0], c1[1], c1[2]), t0, t1, r));
}
int orc_world_rect(orc_world* o, int axis, int mat, double a0, double a1, double b0, double b1, double k)
{
    const int kind = axis == 0 ? H_XY : axis == 1 ? H_XZ : H_YZ;
    return ow_add(o, h_rect(&o->w, kind, mat, a0, a1, b0, b1, k));
}
int orc_world_box(orc_world* o, const double mn[3], const double mx[3], int mat)
{
    return ow_add(o, h_box(&o->w, v3(mn[0], mn[1], mn[2]), v3(mx[0], mx[1], mx[2]), mat));
}
int orc_world_translate(orc_world* o, int id, const double off[3])
{
    const Hittable* p = ow_get(o, id);
    return p ? ow_add(o, h_translate(&o->w, p, v3(off[0], off[1], off[2]))) : -1;
}
int orc_world_rotate_y(orc_world* o, int id, double angle)
{
    const Hittable* p = ow_get(o, id);
    return p ? ow_add(o, h_rotate_y(&o->w, angle, p)) : -1;
}
int orc_world_constant_medium(orc_world* o, int boundary, double density, int phase)
{
    const Hittable* p = ow_get(o, boundary);
    return p ? ow_add(o, h_constant_medium(&o->w, p, density, phase)) : -1;
}
int orc_world_bvh(orc_world* o, const int* ids, int n, double t0, double t1)
{
    if (n < 1) return -1;
    const Hittable** list = (const Hittable**)malloc((size_t)n * sizeof(void*));
    for (int i = 0; i < n; ++i) {
        list[i] = ow_get(o, ids[i]);
        if (!list[i]) { free(list); return -1; }
    }
    OrcRng* saved = tl_rng;
    tl_rng = &o->rng;
    const Hittable* h = new_bvh_node(&o->w, list, 0, n, t0, t1);
    tl_rng = saved;
    free(list);
    return ow_add(o, h);
}
int orc_world_push(orc_world* o, int id)
{
    const Hittable* p = ow_get(o, id);
    if (!p) return -1;
    world_push(&o->w, p);
    return 0;
}
int orc_world_render(const orc_world* o, const orc_params* p, const double* cam24, const double bg[3],
                     double* out_mean, orc_stats* stats)
{
    if (!o || !p || !cam24 || !bg || !out_mean || p->width < 2 || p->height < 2 || p->spp < 1 ||
        p->row_stride < 1 || p->row_begin < 0)
        return -1;
    Camera cam;
    V3* vs[7] = {&cam.origin, &cam.lower_left_corner, &cam.horizontal, &cam.vertical, &cam.u, &cam.v, &cam.w};
    for (int i = 0; i < 7; ++i) *vs[i] = v3(cam24[3 * i], cam24[3 * i + 1], cam24[3 * i + 2]);
    cam.lens_radius = cam24[21];
    cam.time0 = cam24[22];
    cam.time1 = cam24[23];
    return render_world(p, &o->w, &cam, v3(bg[0], bg[1], bg[2]), out_mean, stats);
}

/* ---- output: Vector3::write_color (math.rs:119-132) and the P3 writer (main.rs:472,591-596) ---- */

/* Rust's `f64 as i32` (saturating since Rust 1.45): NaN -> 0, out of range -> the nearest
 * bound, otherwise truncation toward zero. Restated here independently of rt_numerics.h's
 * rt_sat_i32, which the product uses. */
static int rust_as_i32(double x)
{
    if (isnan(x)) return 0;
    if (x >= 2147483647.0) return 2147483647;
    if (x <= -2147483648.0) return -2147483647 - 1;
    return (int)trunc(x);
}

/* write_color(samples_per_pixel) of one channel: scale = 1.0 / spp (math.rs:120),
 * (x * scale).sqrt() (:123-125), clamp(_, 0.0, 0.999) (:127-129, clamp math.rs:282-286:
 * NaN passes through), 256.0 * c as i32. */
static int write_color_channel(double x, int samples_per_pixel)
{
    const double scale = 1.0 / (double)samples_per_pixel;
    const double r = sqrt(x * scale);
    return rust_as_i32(256.0 * clampd(r, 0.0, 0.999));
}

int orc_write_color(const double* rgb, int samples_per_pixel, int64_t n, int32_t* out)
{
    if (!rgb || !out || n < 0 || samples_per_pixel < 1) return -1;
    for (int64_t i = 0; i < 3 * n; ++i) out[i] = write_color_channel(rgb[i], samples_per_pixel);
    return 0;
}

int orc_write_ppm(const double* rgb, int samples_per_pixel, int width, int height, const char* path)
{
    if (!rgb || !path || width < 1 || height < 1 || samples_per_pixel < 1) return -1;
    FILE* f = fopen(path, "wb");
    if (!f) return -1;
    fprintf(f, "P3\n%d %d\n255\n\n", width, height);             /* main.rs:472: println! adds "\n" */
    for (int j = height - 1; j >= 0; --j)                              /* main.rs:591: rows top to bottom */
        for (int i = 0; i < width; ++i) {                              /* main.rs:592 */
            const double* px = rgb + ((size_t)j * width + i) * 3;
            fprintf(f, "%d %d %d\n", write_color_channel(px[0], samples_per_pixel),
                    write_color_channel(px[1], samples_per_pixel), write_color_channel(px[2], samples_per_pixel));
        }
    return fclose(f) == 0 ? 0 : -1;
}
