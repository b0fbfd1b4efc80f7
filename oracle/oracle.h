/*
 * oracle.h — CPU restatement of the reference's per-(pixel, sample) ray_color
 * path (themeshpotato/rust-ray-tracing-in-a-weekend, /root/reference/src).
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU
 * baseline — never as the product path.
 *
 * Parity status: the reference is Rust and cannot be
 * built here (no cargo/rustc; crates not vendored), and it has no tests. The
 * only golden data it holds is the sphere_uv table (math.rs:292-294), which
 * pins sphere_uv. Everything RNG-driven is "parity unpinned" against the
 * reference itself: `rand::thread_rng()` is unseedable (math.rs:268-276), so
 * the oracle replaces it with the seeded Philox protocol of rt_numerics.h and
 * restates every other line of the algorithm.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Scene ids follow the reference's `match` arms (main.rs:314-464). */
enum {
    ORC_SCENE_RANDOM = 0,
    ORC_SCENE_TWO_SPHERES = 1,
    ORC_SCENE_TWO_PERLIN = 2,
    ORC_SCENE_EARTH = 3,
    ORC_SCENE_SIMPLE_LIGHT = 4,
    ORC_SCENE_CORNELL = 5,
    ORC_SCENE_CORNELL_SMOKE = 6,
    ORC_SCENE_FINAL = 7
};

/* Work partition for the CPU render. */
enum {
    ORC_SPLIT_ROWS = 0,    /* thread t renders rows y with (y - row_begin)/row_stride % T == t */
    ORC_SPLIT_SAMPLES = 1  /* reference decomposition (main.rs:497-551): every thread renders
                              all pixels with spp/T samples; sums merged after join */
};

typedef struct {
    int scene_id;
    uint64_t scene_seed;
    uint64_t render_seed;
    int width, height;          /* full image; aspect = width/height */
    int spp, max_depth;
    int spp_chunk;              /* samples summed per partial before the partials are added */
    int row_begin, row_stride;  /* rows rendered: row_begin + k*row_stride < height */
    int threads;                /* 0 -> 1 */
    int split;                  /* ORC_SPLIT_* */
    const uint8_t* image_rgb;   /* earthmap RGB8 (texture.rs:12-22), may be NULL for scenes without it */
    int image_w, image_h;
} orc_params;

typedef struct {
    uint64_t casts;             /* hit_hittables calls from ray_color */
    uint64_t samples;
    double seconds;
} orc_stats;

/* Renders the selected rows. out_mean receives, for each rendered row k (in
 * order) and x, the reference's pixel value sum * (1/spp) as 3 doubles
 * (math.rs:119-126 before gamma). Returns 0 or a negative error. */
int orc_render(const orc_params* p, double* out_mean, orc_stats* stats);

/* Number of objects / materials the scene builder produces (structure probe). */
int orc_scene_info(int scene_id, uint64_t scene_seed, const uint8_t* image_rgb, int iw, int ih,
                   int* n_hittables, int* n_materials, int* n_leaf_prims, double* checksum);

/* Function-level probes used by the unit tests. fn: 0 sin, 1 cos, 2 log, 3 atan2(x, y),
 * 4 acos, 5 sphere_uv u of unit vector (x[i], y[i], z[i]), 6 sphere_uv v, 7 pow5,
 * 8 sqrt, 9 x/y, 10 unit53(bits of x), 11 uniform(-1,1) of bits of x, 12 rt_sin_sign. */
int orc_eval(int fn, const double* x, const double* y, const double* z, double* out, int n);

/* Philox4x32-10 of (ctr[4], key[2]) -> out[4]. */
void orc_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out);

/* The first n u64 draws of the path stream of (seed, pixel, sample) (rt_numerics.h rt_pstream). */
void orc_pstream(uint64_t seed, uint32_t pixel, uint32_t sample, int n, uint64_t* out);

/* Camera of scene_id at width x height (camera.rs:18-56 with main.rs parameters):
 * 24 doubles: origin, lower_left_corner, horizontal, vertical, u, v, w, lens_radius, t0, t1. */
int orc_camera(int scene_id, int width, int height, double* out24);

/* Custom worlds through the reference's constructor surface (main.rs:40-50,
 * hittable.rs:77-207, material.rs:6-12, texture.rs:4-22), built by the same calls as the
 * product's rt_world_* so tests can render one world on both sides. Ids: textures
 * 0-based, material handles 1-based (main.rs:46-49), hittables 0-based; negative = error.
 * The scene seed drives the construction draws (Perlin::new, the BVH's random axis). */
typedef struct orc_world orc_world;
int orc_world_create(uint64_t scene_seed, orc_world** out);
void orc_world_destroy(orc_world* w);
int orc_world_texture(orc_world* w, int kind, const double c0[3], const double c1[3], double scale); /* 0 solid 1 checker 2 noise */
int orc_world_material(orc_world* w, int kind, int tex, const double albedo[3], double fuzz, double ir);
int orc_world_sphere(orc_world* w, int mat, const double c[3], double r);
int orc_world_moving_sphere(orc_world* w, int mat, const double c0[3], const double c1[3], double t0, double t1,
                            double r);
int orc_world_rect(orc_world* w, int axis, int mat, double a0, double a1, double b0, double b1, double k);
int orc_world_box(orc_world* w, const double mn[3], const double mx[3], int mat);
int orc_world_translate(orc_world* w, int id, const double off[3]);
int orc_world_rotate_y(orc_world* w, int id, double angle);
int orc_world_constant_medium(orc_world* w, int boundary, double density, int phase);
int orc_world_bvh(orc_world* w, const int* ids, int n, double t0, double t1);
int orc_world_push(orc_world* w, int id);
/* p: geometry, spp, depth, seeds, rows, threads (scene_id and image unused); cam24 as
 * orc_camera's output; bg the background color. */
int orc_world_render(const orc_world* w, const orc_params* p, const double* cam24, const double bg[3],
                     double* out_mean, orc_stats* stats);

/* Output (math.rs:119-132, main.rs:472,591-596). rgb is height x width x 3 f64, row 0 =
 * the bottom image row (y = 0), holding per-pixel sums taken over samples_per_pixel samples;
 * each channel is written as (int)(256 * clamp(sqrt(x * (1.0 / spp)), 0, 0.999)) with Rust's
 * saturating `as i32` (NaN -> 0). Pass orc_render's out_mean (already sum * (1/spp)) with
 * spp = 1: x * 1.0 == x, so that equals write_color(spp) of the sums.
 * orc_write_color: the 3n channel values of n pixels, in memory order, into out. */
int orc_write_color(const double* rgb, int samples_per_pixel, int64_t n, int32_t* out);
int orc_write_ppm(const double* rgb, int samples_per_pixel, int width, int height, const char* path);

#ifdef __cplusplus
}
#endif
#endif
