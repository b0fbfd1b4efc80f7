/*
 * rt_abi.h — the drop-in boundary: a C ABI (plain pointers and sizes) over the
 * MI355X path tracer. Every entry point returns RT_OK (0) or a negative RT_ERR_*
 * code; nothing aborts and no C++ exception crosses it.
 *
 * What it replaces in the reference (paths relative to /root/reference/src):
 *
 *   rt_render                 the per-(pixel, sample) driver loop main.rs:497-551
 *                             = Camera::get_ray (camera.rs:58-66) followed by
 *                             ray_color (main.rs:19-38) per sample, summed per
 *                             pixel and divided by spp (math.rs:119-126)
 *   rt_camera_new             Camera::new (camera.rs:18-56)
 *   rt_world_*                World + register_material (main.rs:40-50) and the
 *                             Hittable / Material / Texture constructors
 *                             (hittable.rs:77-207, material.rs:6-12, texture.rs:4-22,
 *                             perlin.rs:13-30)
 *   rt_world_build_scene      the scene builders main.rs:52-289
 *   rt_scene_preset           the per-scene camera/background table main.rs:314-464
 *   rt_world_flatten          (new) lowers the Hittable tree to rt_scene_soa
 *   rt_ctx_upload_*           (new) copies the SoA tables into HBM
 *   rt_write_ppm              write_color + the P3 writer (math.rs:119-132,
 *                             main.rs:472, 591-596)
 *   rt_accum_* /              the per-thread partial sums, their merge into the shared
 *   rt_render_progressive     buffer and the progress channel (main.rs:504-582), as
 *                             resumable sample batches with a progress callback
 *   rt_comm_* /               the partition of one frame over workers (main.rs:497-551)
 *   rt_render_gather          and the merge of their buffers (main.rs:542-547), over GPUs:
 *                             8x8 tile shards, one RCCL gather to rank 0, a reorder kernel
 *
 * Threading: a context is bound to one device and is used by one host thread at
 * a time. Worlds are plain host objects.
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stddef.h>
#include <stdint.h>

#include "rt_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 6   /* v6: RT_OPT_COMM_DIRECT */

enum {
    RT_OK = 0,
    RT_ERR_INVALID = -1,      /* bad argument / handle */
    RT_ERR_HIP = -2,          /* a HIP runtime call failed (see rt_last_error) */
    RT_ERR_UNSUPPORTED = -3,  /* a Hittable nesting the flattener does not lower */
    RT_ERR_OOM = -4,
    RT_ERR_NO_DEVICE = -5,
    RT_ERR_NO_SCENE = -6,     /* render before upload */
    RT_ERR_COMM = -7,         /* an RCCL call failed, or RCCL could not be loaded (see rt_last_error) */
    RT_ERR_PEER = -8          /* a collective call failed on another rank; this rank's state is consistent */
};

typedef struct rt_ctx rt_ctx;
typedef struct rt_world rt_world;

int rt_abi_version(void);
/* Text of the last error on this thread ("" if none). */
const char* rt_last_error(void);
/* Build identity of the loaded library: the source hash it was compiled from (16 hex digits
 * of sha256 over csrc/, include/rt/ and the compile flags: __graft_entry__.source_hash()),
 * "unknown" for a build without one. Profiles and PMC records are keyed by it, so a caller can
 * check that the library it times is the build its counters describe. */
const char* rt_build_info(void);

/* ---- device context --------------------------------------------------------- */
int rt_device_count(int* count);
int rt_ctx_create(int device, rt_ctx** out);
void rt_ctx_destroy(rt_ctx* ctx);

/* ---- host scene model (the reference's World / Hittable surface) --------------- */
/* A world owns a seeded construction stream (Philox, rt_numerics.h) that replaces
 * thread_rng() during scene building (random_double in main.rs:191,233,256-268,
 * perlin.rs:16-22,123-124, hittable.rs:82). */
int rt_world_create(uint64_t scene_seed, rt_world** out);
void rt_world_destroy(rt_world* w);

/* Textures (texture.rs:4-22) -> texture id >= 0. */
int rt_world_texture_solid(rt_world* w, double r, double g, double b, int* tex_out);
int rt_world_texture_checker(rt_world* w, const double even[3], const double odd[3], int* tex_out);
/* Perlin::new() draws from the world's stream (perlin.rs:13-30). */
int rt_world_texture_noise(rt_world* w, double scale, int* tex_out);
/* RGB8 texels as stb_image returns them; the world copies them. */
int rt_world_texture_image(rt_world* w, const uint8_t* rgb, int width, int height, int* tex_out);

/* Materials (material.rs:6-12) -> 1-based MaterialHandle (main.rs:46-49). */
int rt_world_material_lambertian(rt_world* w, int tex, int* handle_out);
int rt_world_material_metal(rt_world* w, const double albedo[3], double fuzz, int* handle_out);
int rt_world_material_dielectric(rt_world* w, double ir, int* handle_out);
int rt_world_material_diffuse_light(rt_world* w, int tex, int* handle_out);
int rt_world_material_isotropic(rt_world* w, int tex, int* handle_out);

/* Hittables (hittable.rs:30-41, constructors :77-207) -> hittable id >= 0. */
int rt_world_sphere(rt_world* w, int mat, const double center[3], double radius, int* id_out);
int rt_world_moving_sphere(rt_world* w, int mat, const double c0[3], const double c1[3], double t0, double t1,
                           double radius, int* id_out);
/* axis: 0 XYRect (k on z), 1 XZRect (k on y), 2 YZRect (k on x). */
int rt_world_rect(rt_world* w, int axis, int mat, double a0, double a1, double b0, double b1, double k,
                  int* id_out);
int rt_world_box(rt_world* w, const double mn[3], const double mx[3], int mat, int* id_out);
int rt_world_translate(rt_world* w, int child, const double offset[3], int* id_out);
int rt_world_rotate_y(rt_world* w, int child, double angle_degrees, int* id_out);
int rt_world_constant_medium(rt_world* w, int boundary, double density, int phase_mat, int* id_out);
/* new_bvh_node(list, 0, n, t0, t1): random axis + median split, draws from the stream. */
int rt_world_bvh(rt_world* w, const int* ids, int n, double t0, double t1, int* id_out);
/* world.hittables.push(id) */
int rt_world_push(rt_world* w, int id);

/* Built-in scene builders, ids as the reference's match arms (main.rs:314-464):
 * 0 random, 1 two_spheres, 2 two_perlin, 3 earth, 4 simple_light, 5 cornell,
 * 6 cornell_smoke, 7 final. Scenes 3 and 7 need the earth texture (RGB8). */
int rt_world_build_scene(rt_world* w, int scene_id, const uint8_t* image_rgb, int image_w, int image_h);

typedef struct rt_world_info {
    int32_t n_hittables;     /* top-level list length */
    int32_t n_materials;
    int32_t n_leaf_prims;    /* leaves reachable from the list */
    int32_t n_media;
    double checksum;         /* same probe as the oracle's orc_scene_info */
} rt_world_info;
int rt_world_info_get(const rt_world* w, rt_world_info* out);

/* ---- camera ----------------------------------------------------------------------- */
int rt_camera_new(const double look_from[3], const double look_at[3], const double vup[3], double vfov,
                  double aspect_ratio, double aperture, double focus_dist, double time0, double time1,
                  rt_camera* out);

typedef struct rt_scene_preset {
    double look_from[3], look_at[3], background[3];
    double vfov, aperture, focus_dist, time0, time1;
    int32_t default_width, default_spp;   /* the reference's own image_width / samples_per_pixel */
    double default_aspect;
} rt_scene_preset;
int rt_scene_preset_get(int scene_id, rt_scene_preset* out);
/* Preset camera for an explicit width x height (aspect = width/height). */
int rt_scene_camera(int scene_id, int width, int height, rt_camera* cam_out, double background_out[3]);

/* ---- lowering + upload ---------------------------------------------------------------- */
/* SAH builder options of this world's rt_world_flatten (the tree changes, the image does not):
 * value < 0 (or 0 for the sizes and the cost) restores the default. Tuning knobs for A/B runs
 * (scripts/ab_variants.py --bvh); the defaults are DESIGN.md §2's. */
enum {
    RT_BUILD_C_ISECT = 1,          /* primitive-test cost relative to a node visit (default 1) */
    RT_BUILD_MAX_LEAF = 2,         /* largest leaf the cost model may pick (8) */
    RT_BUILD_FORCE_LEAF = 3,       /* a set this small is always one leaf (2) */
    RT_BUILD_ROOT_LEAF = 4,        /* a whole BVH of at most this many items is one leaf (8) */
    RT_BUILD_SPLIT_BOX_PAIRS = 5,  /* pairs holding a Box, a medium or a BLAS instance split by cost (1) */
    RT_BUILD_SPLIT_BLAS_PAIRS = 6  /* pairs inside instance BLASes split by cost (1) */
};
int rt_world_set_build_option(rt_world* w, int key, double value);
/* Flattens the world into SoA tables owned by the world (valid until the next
 * flatten or rt_world_destroy). accel: RT_ACCEL_SAH / _LINEAR / _MEDIAN (rt_scene.h). */
int rt_world_flatten(rt_world* w, int accel, const rt_scene_soa** soa_out);
/* Checks a (possibly foreign) SoA the way rt_ctx_upload_soa does before copying it: every
 * index in range, no cycle in the node graph, and the traversal stack each walk needs
 * (computed from the tables; the soa's tlas_depth / blas_depth fields are not trusted).
 * Host only, no device needed. Depth outputs may be NULL. */
int rt_scene_validate(const rt_scene_soa* soa, int32_t* tlas_depth, int32_t* blas_depth);
int rt_ctx_upload_soa(rt_ctx* ctx, const rt_scene_soa* soa);
int rt_ctx_upload_world(rt_ctx* ctx, rt_world* w, int accel);

/* ---- render ----------------------------------------------------------------------------- */
enum { RT_OUT_F32 = 0, RT_OUT_F64 = 1 };

typedef struct rt_render_params {
    int32_t width, height;       /* full image */
    int32_t spp, max_depth;
    int32_t spp_chunk;           /* samples a lane sums before its partial is written; 0 = auto */
    int32_t row_begin, row_stride; /* rows rendered: y = row_begin + k*row_stride < height (y = 0 bottom) */
    int32_t out_format;          /* RT_OUT_F32 / RT_OUT_F64 */
    int32_t out_on_device;       /* 0: out is host memory (copied back); 1: out is a device pointer */
    int32_t count_work;          /* 1: also count casts / node visits / prim tests (slower) */
    double background[3];
    uint64_t render_seed;
    void* stream;                /* hipStream_t to launch on (NULL = the context's stream) */
    int32_t row_block;           /* 0 / 1: rows as above. B > 1 (a power of two <= 64): the image is cut
                                    into bands of B rows and the shard is bands j = row_begin +
                                    m*row_stride (rows jB .. jB+B-1 < height): row-band interleave, so
                                    a multi-GPU shard keeps 8x8 work tiles contiguous in the image */
    int32_t tile_shard;          /* 0: rows as above. 1 (row_block 0 / 1): the shard is the 8x8 pixel tiles
                                    t = row_begin + m*row_stride of the frame's tile grid (ceil(width/8)
                                    tiles per tile row, t = ty*ceil(width/8) + tx), written side by side
                                    as one 8-row slab: out row k holds rows 8*ty + k of the shard's
                                    tiles, tile m in columns 8m .. 8m+7 (rt_tiles_in_shard tiles; the
                                    pixels of an edge tile past the image are rendered and meaningless).
                                    Every shard is whole 8x8 tiles, so a multi-GPU shard keeps the
                                    kernel's work tiles compact in the image at any GPU count. With a
                                    tile order set on the context (rt_ctx_set_tile_order), t is a
                                    position in that order: the shard's tile m is order[row_begin +
                                    m*row_stride]. */
} rt_render_params;

/* Renders the selected rows (or tiles) into out (rows_local x width x 3, row k = the k-th
 * selected row; tile shards: 8 x (8 * tiles_local) x 3) as the per-pixel mean radiance
 * sum * (1/spp). Synchronous unless out_on_device is set, in which case the work is only
 * enqueued on `stream`. */
int rt_render(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* p, void* out);

/* Rows rendered for (height, row_begin, row_stride). */
int rt_rows_in_shard(int height, int row_begin, int row_stride);
/* Rows rendered for (height, row_begin, row_stride, row_block) (rt_render_params.row_block). */
int rt_rows_in_band_shard(int height, int row_begin, int row_stride, int row_block);
/* 8x8 tiles rendered for (width, height, row_begin, row_stride) with tile_shard = 1. */
int rt_tiles_in_shard(int width, int height, int tile_begin, int tile_stride);

typedef struct rt_stats {
    double kernel_ms;            /* last rt_render: trace kernel time (HIP events) */
    double reduce_ms;            /* last rt_render: chunk-reduction kernel time */
    uint64_t samples;
    uint64_t casts;              /* count_work only */
    uint64_t node_visits;        /* count_work only: BVH nodes fetched */
    uint64_t prim_tests;         /* count_work only */
    uint64_t n_items;            /* work items (pixel, chunk) */
    int32_t n_chunks, spp_chunk;
    int64_t scene_bytes;         /* device bytes of the uploaded scene */
    int32_t node_bytes, prim_bytes, material_bytes;
    int32_t variant_features;    /* feature set of the kernel variant launched */
    int32_t slab32;              /* 1 if the conservative f32 slab test was used */
    int32_t lds_stack;           /* 1 if the traversal stack lived in LDS */
    int32_t lds_nodes;           /* TLAS nodes kept in LDS (0: read from L1/L2) */
    uint64_t cycles_camera;      /* count_work only: wave-cycles in camera-ray generation */
    uint64_t cycles_trace;       /* count_work only: wave-cycles in traversal + hit records */
    uint64_t cycles_shade;       /* count_work only: wave-cycles in materials / textures */
    uint64_t wave_steps;         /* count_work only: bounce-loop iterations executed per wave, summed;
                                    casts / (64 * wave_steps) = lane occupancy of the bounce loop */
    uint64_t wave_node_steps;    /* count_work only: node-visit iterations per wave, summed;
                                    node_visits / (64 * wave_node_steps) = its lane occupancy */
    uint64_t cycles_nodes;       /* count_work only: wave-cycles in BVH node-visit loops (part of trace) */
    uint64_t cycles_leaves;      /* count_work only: wave-cycles in leaf primitive tests (part of trace) */
    int32_t schedule;            /* RT_SCHED_* the last render ran with */
    int32_t n_batches;           /* trace launches it took (pool: per-sample buffer batches) */
    uint64_t wave_leaf_steps;    /* count_work only: leaf-loop iterations per wave, summed;
                                    prim_tests / (64 * wave_leaf_steps) = its lane occupancy */
    uint64_t camera_lanes;       /* count_work only: lanes starting a sample, summed over the */
    uint64_t camera_steps;       /*   wave iterations in which any lane did (camera_steps) */
    uint64_t shade_lanes;        /* count_work only: lanes shading a hit, summed over the */
    uint64_t shade_steps;        /*   wave iterations in which any lane did (shade_steps) */
    int32_t precision;           /* RT_PREC_* the last render ran with */
    int32_t waves_per_simd;      /* resident waves per SIMD of the last trace kernel (occupancy) */
    int64_t trace_buf_bytes;     /* the trace-output buffer the last render used (both halves when overlapped) */
    int32_t overlapped;          /* 1 if its buffer batches ran overlapped (two trace streams) */
    int32_t reserved0;           /* always 0 (ABI v4's wavefront-schedule iteration count; that schedule is gone) */
    int64_t ring_bytes;          /* POOL with the in-kernel reduction (ABI v3): its record ring, part of
                                    trace_buf_bytes; 0 when the per-sample buffer ran */
} rt_stats;
int rt_last_stats(rt_ctx* ctx, rt_stats* out);
/* Diagnostic: the raw count_work counters of the last render (n entries; returns how many
 * exist). 0-14 as in rt_stats; wave-cycles (s_memtime) per phase of the pool kernels: 3 ray
 * generation, 4 trace, 5 shading, 8 node loops, 9 leaf tests (both of the top-level walk),
 * 15 ray set-up, 16 walk prologue (pre-leaf test), 17 hit record, 18 media and 19 instances
 * (inside the leaf tests), 20 refill, 21 kernel total (summed over waves), 22 deferred instance
 * walks (after the top-level walk), 23 / 24 ray generation's seeding + jitter / rejection loop, 25
 * the longest wave lifetime, 26 waves. Bounce-loop lane slots that cast nothing (with casts they
 * add up to 64 x wave_steps): 27 idle, no unit left (the tail), 28 idle, every ring slot holding
 * an unfinished block, 29 the path ended in its scatter, 30 the depth cap, 31 a rejection loop
 * carried to the next iteration. */
int rt_last_counters(rt_ctx* ctx, uint64_t* out, int n);

/* ---- tile order: balancing tile shards (ABI v4; main.rs:497-551's partition, rebalanced) ------ */
/* Per 8x8 tile of the image (raster order, ceil(width/8) per tile row), the lane-cycles
 * (s_memtime) its samples took in the last render, if that render had count_work set and ran
 * a pool schedule (POOL, ITEMS; any shard mode). Copies min(n, tiles) entries; returns the
 * tile count, or 0 when the last render counted none. A cost estimate for
 * rt_ctx_set_tile_order: e.g. a few samples per pixel of the frame with count_work. */
int rt_last_tile_costs(rt_ctx* ctx, uint64_t* out, int64_t n);
/* The order in which tile shards (rt_render_params.tile_shard = 1) take the frame's tiles:
 * order[t] is the raster tile at position t, a permutation of the frame's n tiles (checked:
 * RT_ERR_INVALID otherwise). Shards then take positions row_begin + m*row_stride; a frame of
 * another tile count fails with RT_ERR_INVALID. Under a tile order the pool schedules also deal
 * their work blocks tile-major (all of a tile's sample groups before the next tile's) instead
 * of sample-group-major. The tiles sorted by cost, most expensive first, then give round-robin
 * shards of nearly equal cost, each finishing its expensive tiles first and ending on its
 * cheapest ones (a shard's launch otherwise ends on the last sample group of its most
 * expensive tiles). Only which pixels a shard renders, and when, changes, not their bits.
 * n = 0: raster order again (the default). Waits for the device. */
int rt_ctx_set_tile_order(rt_ctx* ctx, const uint32_t* order, int64_t n);

/* ---- multi-GPU render: tile shards, one RCCL gather, on-device reassembly (ABI v5) ------------
 * The reference splits one frame over 10 threads (main.rs:497-551: every thread all pixels,
 * spp/10 samples) and merges their buffers under a mutex (main.rs:542-547). Here a frame is split
 * over GPUs by 8x8 tiles: rank r of `world` renders the tiles at positions r, r + world, ... of the
 * frame's tile order (rt_render_params.tile_shard), RCCL gathers every rank's slab to rank 0 over
 * xGMI in one collective, and a reorder kernel on rank 0 writes the frame. Every draw is keyed by
 * (pixel, sample), so the frame is bit-identical to rt_render's at any world size and tile order.
 *
 * A communicator binds one context (one device) to one rank. Two ways to make them:
 *   one process per GPU:     rank 0 calls rt_comm_unique_id and sends the 128 bytes to the other
 *                            ranks (any channel: MPI, a socket, torch.distributed); every rank then
 *                            calls rt_comm_init_rank with its own context (ncclCommInitRank);
 *   one process, N GPUs:     rt_comm_init_all over N contexts on N distinct devices
 *                            (ncclCommInitAll), then the *_all calls drive every rank from one
 *                            host thread (RCCL group calls).
 * RCCL (librccl.so.1) is loaded when the first communicator is made; the rest of the library does
 * not need it. Collective calls (rt_comm_tile_order, rt_render_gather) must be made by every rank
 * of the communicator with the same camera and frame parameters. */
typedef struct rt_comm rt_comm;
enum { RT_COMM_ID_BYTES = 128 };   /* ncclUniqueId */
int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]);
int rt_comm_init_rank(rt_ctx* ctx, int rank, int world, const uint8_t id[RT_COMM_ID_BYTES], rt_comm** out);
int rt_comm_init_all(rt_ctx* const* ctxs, int n, rt_comm** comms_out);
/* Destroys the RCCL communicator (after the rank's enqueued work is done); the context stays. */
void rt_comm_destroy(rt_comm* comm);
int rt_comm_rank(const rt_comm* comm, int* rank, int* world);

/* Collective: the cost-ordered tile deal (rt_ctx_set_tile_order) on every rank. Each rank renders
 * its raster-order tile shard of the frame p describes (its shard fields are ignored) at cost_spp
 * samples per pixel with count_work — f64 and a pool schedule, whatever the context is set to —
 * one RCCL all-reduce sums the per-tile lane-cycles (each tile counted by one rank), and every
 * rank sets the same order, rt_cost_tile_order's, on its context. A rank whose pass fails (and,
 * with RT_ERR_PEER, every other rank) falls back to raster order. The cost pass is 1/world of a
 * cost_spp frame per rank. */
int rt_comm_tile_order(rt_comm* comm, const rt_camera* cam, const rt_render_params* p, int cost_spp);
int rt_comm_tile_order_all(rt_comm* const* comms, int n, const rt_camera* cam, const rt_render_params* p,
                           int cost_spp);

/* Collective: one frame over the communicator's ranks. p describes the whole frame (its shard
 * fields row_begin / row_stride / row_block / tile_shard are ignored: rank r renders the tile
 * shard r of `world` in the context's tile order). Rank 0 receives the frame (height x width x 3
 * of p->out_format, row 0 = bottom), as rt_render's: on the device if p->out_on_device (the work
 * is then only enqueued on p->stream or the context's stream), else in host memory (synchronous).
 * Other ranks ignore `frame` (may be NULL) and, without out_on_device, return once their slab
 * has been sent. */
int rt_render_gather(rt_comm* comm, const rt_camera* cam, const rt_render_params* p, void* frame);
/* The same for the n ranks of one process (rt_comm_init_all; comms[i] is rank i): every rank's
 * render is enqueued on its context's stream, then the n gathers as one RCCL group. p->stream must
 * be NULL; with out_on_device, frame is a device pointer on comms[0]'s device. */
int rt_render_gather_all(rt_comm* const* comms, int n, const rt_camera* cam, const rt_render_params* p,
                         void* frame);

typedef struct rt_comm_stats {
    double render_ms;     /* last rt_render_gather: this rank's shard render (HIP events on its stream) */
    double gather_ms;     /* its RCCL gather: from the end of its render to the gather's end (includes the
                             wait for slower ranks) */
    double assemble_ms;   /* rank 0: the reorder kernel */
    double kernel_ms;     /* the trace kernel's part of render_ms (rt_stats.kernel_ms) */
    int64_t slab_bytes;   /* bytes each rank sent (its slab, padded to the largest shard) */
    int32_t tiles;        /* this rank's tiles */
    int32_t tile_order;   /* 1: a cost order was set by the last rt_comm_tile_order; 0: raster */
    double cost_pass_ms;  /* last rt_comm_tile_order on this rank: wall time of the count pass + all-reduce */
    int32_t peer_failed;  /* rank 0: ranks whose shard render failed in the last gather (their status words,
                             sent with the slabs; a host-bound rt_render_gather returns RT_ERR_PEER then) */
} rt_comm_stats;
int rt_comm_last_stats(rt_comm* comm, rt_comm_stats* out);

/* The reorder kernel alone, for callers with their own transport: `world` tile slabs at
 * `slabs` (device memory of ctx's device, rank r's at r * slab_elems elements; slab_elems >=
 * 8 * 8 * rt_tiles_in_shard(width, height, 0, world) * 3) -> frame (device, height x width x 3) of
 * p->out_format for the frame p describes, in ctx's tile order. Enqueued on p->stream (or the
 * context's stream). */
int rt_tiles_assemble(rt_ctx* ctx, const void* slabs, int64_t slab_elems, int world, const rt_render_params* p,
                      void* frame);
/* The same on the host (no device): elem_bytes 4 (f32) or 8 (f64), order NULL (raster) or the
 * n-tile permutation rt_ctx_set_tile_order takes. */
int rt_tiles_assemble_host(const void* slabs, int64_t slab_elems, int world, int width, int height, int elem_bytes,
                           const uint32_t* order, void* frame);
/* The cost order from per-tile costs (rt_last_tile_costs): raster tiles sorted by cost, most
 * expensive first, ties in raster order. Host only. */
int rt_cost_tile_order(const uint64_t* costs, int64_t n, uint32_t* order);

/* ---- progressive / resumable accumulation ------------------------------------ */
/* A device f64 running sum per pixel of one row shard. Batches render consecutive sample
 * ranges [done, done + n) and add their per-pixel sums; rt_accum_resolve divides. When
 * every batch boundary is a multiple of the chunk size (rt_render_params.spp_chunk at
 * create time; 0 = rt_render's auto choice for p->spp), the result is bit-identical to
 * one rt_render of the same total spp: the sums are added in the same order.
 * The reference's version of this is each thread's local_pixel_colors merged into the
 * mutex-guarded buffer (main.rs:508-547) plus the progress channel (main.rs:504-582). */
typedef struct rt_accum rt_accum;
/* p: width, height, row_begin, row_stride, spp (for the auto chunk) and spp_chunk. */
int rt_accum_create(rt_ctx* ctx, const rt_render_params* p, rt_accum** out);
void rt_accum_destroy(rt_accum* acc);
/* Renders samples [done, done + sample_count) of the shard with p's camera-independent
 * settings (max_depth, background, render_seed, count_work, stream; its geometry fields
 * must match the accumulator's) and adds them. Enqueued on the stream; rt_last_stats
 * describes the batch. */
int rt_accum_add(rt_ctx* ctx, rt_accum* acc, const rt_camera* cam, const rt_render_params* p, int sample_count);
/* Checkpoint: samples done, and (if sums is not NULL) the rows_local x width x 3 f64 sums. */
int rt_accum_get(rt_accum* acc, double* sums, int64_t* samples_done);
/* Restore a checkpoint taken with rt_accum_get (same geometry and chunk size). */
int rt_accum_set(rt_accum* acc, const double* sums, int64_t samples_done);
/* out = sums * (1/divisor) (divisor 0: the samples done), as rt_render writes it. The
 * reference divides by its nominal spp even when spp/thread_count truncated the samples
 * actually taken (main.rs:516, 596): pass that spp as divisor to reproduce it. */
int rt_accum_resolve(rt_ctx* ctx, rt_accum* acc, double divisor, int out_format, int out_on_device, void* out);

/* Progress callback: return 0 to continue, nonzero to stop after this batch. */
typedef int (*rt_progress_fn)(void* user, int64_t samples_done, int64_t samples_total);
/* rt_render in batches of batch_spp samples (rounded up to the chunk size), calling
 * progress after each batch; out as rt_render (sums / samples done if stopped early). */
int rt_render_progressive(rt_ctx* ctx, const rt_camera* cam, const rt_render_params* p, int batch_spp,
                          rt_progress_fn progress, void* user, void* out);

/* ---- output ------------------------------------------------------------------------------ */
/* P3 PPM byte for byte as the reference writes it (write_color, math.rs:119-132; main.rs:472,
 * 591-596): header "P3\nW H\n255\n\n", rows top to bottom, each channel
 * (int)(256 * clamp(sqrt(x * (1.0 / samples_per_pixel)), 0, 0.999)) in f64, with Rust's
 * saturating `as i32` (NaN -> 0). rgb is height x width x 3 f64 with row 0 = bottom (y = 0):
 * per-pixel sums over samples_per_pixel samples (rt_accum_get), or rt_render's RT_OUT_F64 mean
 * (already sum * (1/spp)) with samples_per_pixel = 1 — x * 1.0 == x, so both give the
 * reference's bytes. */
int rt_write_ppm_f64(const double* rgb, int samples_per_pixel, int width, int height, const char* path);
/* The same channel values without the file: out[i] for the 3n channels of n pixels, in memory order. */
int rt_write_color(const double* rgb, int samples_per_pixel, int64_t n, int32_t* out);
/* The f32 frame's writer (RT_OUT_F32 output, the f32 mode): as rt_write_ppm_f64 with spp = 1, but
 * the mean was rounded to f32 before the sqrt, so a channel whose 256*sqrt(mean) lies within
 * ~1e-5 of an integer can differ by one from the reference's f64 write_color. */
int rt_write_ppm(const float* mean_rgb, int width, int height, const char* path);

/* Kernel variant knobs of a context: slab32 (conservative f32 BVH slab tests),
 * lds_stack (traversal stack in LDS instead of scratch), lds_nodes (keep the TLAS in LDS
 * when it fits). Defaults 1/1/1. Results do not depend on them (tests check this). */
int rt_ctx_set_variant(rt_ctx* ctx, int slab32, int lds_stack, int lds_nodes);

/* Context options (rt_ctx_set_option / rt_ctx_get_option). The library reads no environment
 * variable: every behaviour switch is one of these or a setter above. Images do not depend on
 * any of them (the tests check this); they trade speed and memory.
 *   RT_OPT_TRACE_BUF_BYTES  bound of the trace-output buffer (below, default 64 GiB); 0 restores the default
 *   RT_OPT_BATCH_OVERLAP    1 (default): buffer batches overlap on two streams; 0: one buffer, in order
 *   RT_OPT_BLOCK_SAMPLES    per-sample pool: samples per work block (0: auto, 16 down to 4 for small shards)
 *   RT_OPT_BLOCK_CHUNKS     item pool: chunks per work block (0: auto = 2)
 *   RT_OPT_EXTRA_FEATURES   feature bits OR-ed into the scene's, so a scene runs on a larger
 *                           feature-set variant than it needs (tests: the all-features variant)
 *   RT_OPT_HOIST            1 (default): the spheres variants test a huge root-child leaf before
 *                           the walk (SceneDev.pre_leaf); takes effect at the next upload
 *   RT_OPT_POOL_RING        1 (default): POOL reduces each finished (tile, chunk) block inside the
 *                           trace kernel into chunk partials when its per-sample buffer would not
 *                           fit the bound in one batch; 2: whenever its blocks allow; 0: never (the
 *                           per-sample buffer and reduce_samples; see RT_SCHED_POOL)
 *   RT_OPT_COMM_DIRECT      1 (default): rt_render_gather on a communicator of one rank, with the
 *                           context in raster tile order, is rt_render straight into the frame (a
 *                           world of one has nothing to gather); 0: the tile shard, the RCCL gather
 *                           and the reorder kernel as at any other world size (tests) */
enum {
    RT_OPT_TRACE_BUF_BYTES = 1,
    RT_OPT_BATCH_OVERLAP = 2,
    RT_OPT_BLOCK_SAMPLES = 3,
    RT_OPT_BLOCK_CHUNKS = 4,
    RT_OPT_EXTRA_FEATURES = 5,
    RT_OPT_HOIST = 6,
    /* 7, 8: ABI v4's wavefront-schedule options, removed with it (RT_ERR_INVALID) */
    RT_OPT_POOL_RING = 9,
    RT_OPT_COMM_DIRECT = 10
};
int rt_ctx_set_option(rt_ctx* ctx, int key, int64_t value);
int rt_ctx_get_option(rt_ctx* ctx, int key, int64_t* value);

/* Work schedule of a context (default RT_SCHED_AUTO). Images are bit-identical under all of
 * them.
 *   CHUNKS: a wave owns an 8x8 tile x one chunk of samples, each lane one pixel's chunk,
 *           written as one partial per (pixel, chunk); the wave waits for its slowest lane.
 *   POOL:   persistent waves take (tile, chunk) blocks from a device counter and a lane
 *           whose path ended takes the block's next (pixel, sample) at once. Every sample's
 *           radiance goes to a per-sample buffer ([8x8 tile][sample][pixel of the tile]) summed
 *           per pixel in sample order by a second kernel. When that buffer does not fit the bound
 *           in one batch (RT_OPT_POOL_RING), a block belongs to one wave instead: its samples wait
 *           in that wave's ring of 4 blocks, and when the block's last sample ends the wave sums
 *           every pixel's samples in order into the chunk partial (1/chunk of the per-sample
 *           bytes, as ITEMS). Same bits either way.
 *   ITEMS:  persistent waves as POOL, but a lane takes a whole (pixel, chunk) item, traces
 *           its samples in order and writes one partial, as CHUNKS does (1/chunk of POOL's
 *           buffer bytes); a lane whose item ended takes the next item at once.
 *   AUTO:   ITEMS for the Cornell-box variant (rects, boxes and instances without media: measured
 *           fastest there); otherwise POOL when it can reduce in the kernel or its
 *           per-sample radiance is at most 4 x the buffer bound, else ITEMS; rt_stats.schedule
 *           reports which ran.
 * Schedule 4 (ABI v4's wavefront split: wf_logic / wf_trace kernels over a path pool in HBM) was
 * measured 2.3x slower than POOL on the final scene and removed; rt_ctx_set_schedule(4) returns
 * RT_ERR_UNSUPPORTED (the code: scripts/experiments/r05_wavefront.patch).
 * The trace-output buffer (POOL's ring included) is bounded by RT_OPT_TRACE_BUF_BYTES (default
 * 64 GiB, or half the device's free memory if that is less; allocated lazily, as large as a
 * render needs). A larger render runs in buffer
 * batches whose sums are carried across, in two halves of the bound: batch k traces into half
 * k & 1 on one of two context streams while the render's stream reduces batch k - 1, so
 * consecutive traces overlap (RT_OPT_BATCH_OVERLAP 0: one buffer, in order). Under the default
 * bound C2 (11.5 GB) and C4 (49.8 GB) render through the per-sample buffer in one batch, C5
 * (1.6 TB of records) through the ring's chunk partials in a few. */
enum { RT_SCHED_CHUNKS = 0, RT_SCHED_POOL = 1, RT_SCHED_ITEMS = 2, RT_SCHED_AUTO = 3 };
int rt_ctx_set_schedule(rt_ctx* ctx, int schedule);

/* Arithmetic of a context's renders (default RT_PREC_F64).
 *   F64: the reference's f64 everywhere (math.rs:13-17), path-identical to the oracle: the
 *        same rays, hits and draws; the per-pixel means differ only in the last ulps (the
 *        throughput product T = a0*a1*...*e associates left here, right in the recursive
 *        ray_color, main.rs:31; L_inf ~3e-16 at full C2 spp). Exact-t ties between two
 *        primitives resolve by test order, which a BVH (and the hoisted root leaf) changes
 *        against the reference's list order — a measure-zero event for spheres.
 *   F32: a fast mode: f32 rays, hit records, materials and textures (sphere tests keep
 *        |oc|^2 - r^2 in f64), one 32-bit draw per uniform; per-pixel sums
 *        stay f64. Statistically equal to F64 (independent-seed tests), not bitwise; never
 *        the headline metric. count_work is not available in it. */
enum { RT_PREC_F64 = 0, RT_PREC_F32 = 1 };
int rt_ctx_set_precision(rt_ctx* ctx, int precision);

/* ---- self test ------------------------------------------------------------------------------ */
/* Evaluates rt_numerics.h functions on the device (same fn ids as the oracle's
 * orc_eval) so tests can check host/device bit equality. */
int rt_device_eval(rt_ctx* ctx, int fn, const double* x, const double* y, const double* z, double* out, int n);

#ifdef __cplusplus
}
#endif
#endif
