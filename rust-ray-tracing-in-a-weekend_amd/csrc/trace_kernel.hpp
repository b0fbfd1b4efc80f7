// trace_kernel.hpp — launch interface of the megakernel (trace_kernel.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "rt/rt_scene.h"

// The first instance a cast's top-level walk reaches is tested after that walk (trace_world's
// DeferInst), its BLAS walk then starting at stack entry 0; shared with the host, which sizes the
// stack from it (abi.cpp: a scene where no other nested walk can happen needs max(TLAS, BLAS)
// entries instead of their sum)
#ifndef RT_DEFER_INST
#define RT_DEFER_INST 1
#endif

// Threads per workgroup of the final-scene variant's kernels (the others: 256). 512 (8 waves)
// shares one LDS copy of the TLAS and materials among twice the waves, which leaves room for
// the instanced BLAS in LDS (SceneDev.n_lds_blas; the host sizes that budget with it): the
// final scene's 1000-sphere BLAS 512 of 548 nodes staged instead of 64, C4 1920x1080x100
// 110.95 -> 108.23 ms; 512 threads with 64 staged 111.27 (profiles/r03r_ab_c4.log)
// Round 6: 1024 (16 waves, one workgroup per CU at 4 waves per SIMD) stages the whole BLAS and
// shares one copy of everything among the CU's waves: C4 1920x1080x1000 979.1 -> 976.4 ms, f32 mode
// at 100 spp 86.33 -> 84.98, images bit-identical (profiles/r06u_ab_b1024_c4*.log; at 100 spp
// 105.15 -> 104.71, r06t_ab_b1024_c4.log)
#ifndef RT_BLOCK_FINAL
#define RT_BLOCK_FINAL 1024
#endif

namespace rtk {

// Threads per workgroup of the f32 mode's spheres variant: its 76 VGPRs allow 6 waves per SIMD,
// which 256-thread blocks cannot reach (each holds its own 22.7 KB copy of the random scene's
// TLAS, 6 x 28.8 KB > 160 KB per CU); 512-thread blocks share one copy among 8 waves (3 blocks,
// 105 KB).
#ifndef RT_BLOCK_F32_FINAL
#define RT_BLOCK_F32_FINAL RT_BLOCK_FINAL
#endif
// Threads per workgroup of the f64 spheres variant (C1, C2, C5): 768 (12 waves, two workgroups per
// CU) at 6 waves per SIMD (RT_MIN_WAVES_SPHERES_S16: 80 VGPRs, 32-40 B of scratch), two LDS copies
// of the TLAS per CU instead of five. C2 1200x800x500 74.55 -> 72.00 ms, images identical; 512
// threads at 6 waves 72.24, 384 at 6 81.12, 448 at 7 (96 B of scratch) 89.86, 512 at 5 (two
// workgroups: 4 waves per SIMD) 82.42 (profiles/r06w_ab_sph_c2.log, r06x_ab_sph_c2.log)
#ifndef RT_BLOCK_SPHERES
#define RT_BLOCK_SPHERES 768
#endif
#ifndef RT_BLOCK_F32_SPHERES
#define RT_BLOCK_F32_SPHERES 512
#endif

// workgroup threads of a kernel variant (host and device): see RT_BLOCK_FINAL, RT_BLOCK_SPHERES,
// RT_BLOCK_F32_SPHERES. s16: the spheres variant's 16-bit-stack configuration (slab32, LDS stack,
// whole TLAS in LDS: Stack16Cfg), the one those workgroup sizes and their wave counts are for;
// its other configurations keep 256-thread workgroups
#ifndef RT_STACK16
#define RT_STACK16 1
#endif
__host__ __device__ constexpr int block_threads_of(uint32_t variant_features, bool f32, bool s16 = false)
{
    return variant_features == 287u /* FEAT_SET_FINAL */            ? (f32 ? RT_BLOCK_F32_FINAL : RT_BLOCK_FINAL)
           : variant_features == 0u /* FEAT_SET_SPHERES */ && s16 ? (f32 ? RT_BLOCK_F32_SPHERES : RT_BLOCK_SPHERES)
                                                                   : 256;
}

// Device view of the uploaded rt_scene_soa tables.
struct SceneDev {
    const rt_prim* prims;
    const int32_t* prim_refs;
    const rt_prim* leaf_prims;  // prims[prim_refs[j]] for every leaf slot j (copied at upload):
                                // a primitive test reads its record directly, not through prim_refs
    const rt_bvh_node* nodes;
    const rt_instance* instances;
    const rt_material* materials;
    const rt_texture* textures;
    const double* perlin_ranvec;
    const int32_t* perlin_perm;
    const uint8_t* image;
    int32_t tlas_root;
    int32_t blas_base;      // first stack entry of a BLAS walk nested in the top-level walk
    int32_t stack_entries;  // traversal stack entries per lane (TLAS + nested BLAS walk, or the
                            // larger of the two when every BLAS walk is a deferred one: abi.cpp)
    int32_t n_lds_nodes;    // the first n TLAS nodes (BFS order, nodes[0, n)) are copied into LDS
    int32_t n_tlas_nodes;   // TLAS size (its nodes are nodes[0, n_tlas_nodes))
    int32_t has_spheres;    // any Sphere / MovingSphere: rays need 1/|d|^2 for the root divisions
    int32_t has_lights;     // any DiffuseLight material (else no hit emits: the random scene)
    int32_t n_lds_materials;  // > 0: the material and texture tables are staged in LDS after the
    int32_t n_lds_textures;   // TLAS nodes (the kernel variants with rects or media; small tables)
    // A leaf the cast tests before the TLAS walk (0: none): a root child holding a primitive
    // far larger than the rest of the scene (the random scene's r = 1000 ground, the final
    // scene's r = 5000 fog), whose test then runs once per cast with the whole wave instead
    // of whenever each lane's walk reaches it; the walk starts below the root with t_max from
    // it. Its (padded) box gates the test; the walk then starts at pre_root, the other root
    // child. Only the spheres variants use it (PreLeaf: elsewhere the extra inlined leaf code
    // costs the variant its occupancy); the others walk from tlas_root as before.
    int32_t pre_leaf, pre_root;
    float pre_lo[3], pre_hi[3];
    // the TLAS walk's stack entries fit 16 bits (Stack16: node records at LDS byte addresses
    // < 32 KB, i.e. <= 409 TLAS nodes, and leaf codes of <= 1023 leaf slots); set at upload
    int32_t stack16_ok;
    // BLAS nodes staged in LDS after the TLAS records (variants with instanced BLASes): the device
    // node array holds one instance BLAS's nodes in BFS order right after the TLAS prefix,
    // nodes[n_tlas_nodes, n_tlas_nodes + n_blas_bfs) (abi.cpp), and a launch stages the first
    // n_lds_blas of them (its LDS budget): the nested walk's top levels then read LDS
    int32_t n_blas_bfs, n_lds_blas;
    int32_t pad0;           // (unused: keeps the kernel-argument layout the kernels were timed with)
};

struct KParams {
    rt_camera cam;
    double bg[3];
    double scale_m11;   // rand UniformFloat::new_inclusive(-1, 1) scale
    double scale_time;  // rand UniformFloat::new_inclusive(time0, time1) scale
    double wm1, hm1;    // width - 1, height - 1 (the jitter divisors of main.rs:517-518)
    double inv_wm1, inv_hm1;  // 1 / (width - 1), 1 / (height - 1), correctly rounded
    uint64_t seed;
    int32_t width, height, spp, max_depth;   // width: of the shard's pixel grid (the image's, or a tile slab's)
    int32_t spp_chunk, n_chunks;
    int32_t row_begin, row_stride, n_rows;
    int32_t row_block_shift;    // rows in bands of 2^shift (rt_render_params.row_block); 0: single rows
    int32_t tiles_x, tiles_y;   // 8x8 pixel tiles over (width, n_rows)
    int32_t sample_begin;       // chunk c covers samples [sample_begin + c*spp_chunk, ..) up to spp
    int32_t block_chunks;       // item pool: chunks per work block (a block = one tile x this many chunks)
    int32_t block_samples;      // per-sample pool: samples per work block (one tile x this many samples)
    uint32_t n_work_blocks;     // pool schedules: tiles x sample groups of this launch (host-computed: in
                                // the kernel the division's VGPR result stayed live through the loop)
    int32_t img_width;          // the image's width (pixel keys)
    int32_t tile_shard;         // rt_render_params.tile_shard: grid tile m = the frame's tile at position
                                // row_begin + m*row_stride of tile_order (raster order if null)
    int32_t img_tiles_x;        // tiles per tile row of the image
    // tile shards: ty = t / img_tiles_x as umulhi(t, tile_div_magic), exact for every tile t of the
    // frame (host-checked: t * (magic * img_tiles_x - 2^32) < 2^32); 0: a plain division
    uint32_t tile_div_magic;
    int32_t ring_waves;         // per-sample pool, in-kernel reduction: waves the ring holds (0: off)
    double* ring;               // per-sample pool, in-kernel reduction: kPoolRing blocks of records per wave
    // tile shards: the frame's tile order (rt_ctx_set_tile_order), position -> raster tile; null: raster
    const uint32_t* tile_order;
    // pool schedules: work blocks dealt tile-major (all of a tile's sample groups, then the next
    // tile: set with a tile order, so the most expensive tiles are done first and entirely) rather
    // than group-major; deal_div = the block index's inner extent: tiles (group-major) or sample
    // (chunk) groups per tile (tile-major)
    int32_t tile_major;
    uint32_t deal_div;
    // count_work renders (COUNT kernels): per raster tile of the image, the lane-cycles its samples took
    unsigned long long* tile_cost;
};

// Per-sample pool with the reduction in the kernel (round 5): a wave's work block (one tile x
// one chunk of samples) is owned by that wave alone, so the wave counts its finished samples
// and, when the block's last one ends, sums every pixel's samples in order and writes the
// chunk partial (reduce_chunks' input). The records wait in a ring of kPoolRing blocks per
// wave (record j of a block: sample j / 64, pixel j % 64 of the 8x8 tile). Needs chunks of at
// most 16 samples and samples below 2^20 (the host checks both).
constexpr int kPoolRing = 4;
constexpr unsigned kRingSlot = 16 * 64;        // records per ring slot: chunks of at most 16 samples
constexpr int kRingCur = kPoolRing;            // lanes of the wave's ring-state VGPR (trace_pool):
constexpr int kRingOcc = kPoolRing + 1;        //   the slot units are taken from, the occupied slots
constexpr size_t kRingWaveDoubles = (size_t)kPoolRing * kRingSlot * 3 + 8;   // a wave's records + header
constexpr int kRingSampleBits = 20;            // ring: samples below 2^20, the record index above
constexpr uint32_t kRingSampleMask = (1u << kRingSampleBits) - 1;
static_assert(kPoolRing * kRingSlot <= (1u << (32 - kRingSampleBits)), "ring record index bits");

// Scene features (which code a kernel variant must contain).
enum : uint32_t {
    FEAT_RECT = 1,      // XY/XZ/YZ rects and boxes
    FEAT_INST = 2,      // Translate / RotateY instances
    FEAT_MEDIUM = 4,    // ConstantMedium
    FEAT_NOISE = 8,     // Perlin noise texture
    FEAT_IMAGE = 16,    // image texture
    FEAT_INST_RECT = 32,    // rects or boxes inside an instance (its child prim or BLAS)
    FEAT_MEDIUM_INST = 64,  // a medium boundary that is not a sphere (box, rect, instance)
    FEAT_INST_MEDIUM = 128, // a medium inside an instance (nested Translate/RotateY over a ConstantMedium)
    FEAT_INST_BLAS = 256,   // an instance over a BVH (a nested walk; instances over one primitive need none)
    FEAT_SHUTTER = 512,     // a MovingSphere whose shutter is not [0, 1] (its centre needs a division)
    FEAT_NEST_MOVING = 1024, // a MovingSphere (nonzero velocity) under an instance or in a medium boundary
    FEAT_IMAGE_UV = 2048,    // an image texture on a rect / box or an instanced primitive (its uv is stored at
                             // the hit; else it is a top-level sphere's, recomputed from the hit normal)
    FEAT_ALL = 4095,
    FEAT_STATIC = 1u << 16,  // kernel-internal (InstC / BoundC): every sphere reached here is static
    FEAT_SET_SPHERES = 0,                                          // compiled variant: spheres + solid/checker
    FEAT_SET_RECTINST = FEAT_RECT | FEAT_INST | FEAT_INST_RECT,    // + rects, boxes, instances of one prim (Cornell)
    FEAT_SET_MEDIA = FEAT_SET_RECTINST | FEAT_MEDIUM | FEAT_MEDIUM_INST,  // + constant media (Cornell smoke)
    // + Perlin and image textures, instances over spheres, media bounded by spheres (final scene)
    FEAT_SET_FINAL = FEAT_RECT | FEAT_INST | FEAT_MEDIUM | FEAT_NOISE | FEAT_IMAGE | FEAT_INST_BLAS
};
static_assert(FEAT_SET_FINAL == 287u, "block_threads_of");

struct LaunchOpts {
    uint32_t features;  // scene features (FEAT_*)
    int slab32;         // conservative f32 slab tests
    int lds_stack;      // traversal stack in LDS (1) or scratch (0)
    int count;          // count_work variant
    int pool;           // RT_SCHED_*: 0 chunks, 1 per-sample pool (per-sample output), 2 item pool (partials)
    int f32;            // the f32 fast mode (RT_PREC_F32)
    int* waves_per_simd = nullptr;  // out (optional): resident waves per SIMD of the launched trace kernel
};

// Per-sample pool output: [8x8 tile][sample of the batch][64 pixels of the tile, row-major]
// radiance records (f64 x 3). A wave's work block is one tile x consecutive samples and its
// lanes take the block's units in order, so records written close in time lie close in memory
// and fill whole cache lines while those sit in L2; the earlier [sample][pixel] layout spread
// each (tile, sample)'s 64 records over 8 image rows written ~1 ms apart, and L2 evicted the
// lines half written (C2 DRAM writes 1.22x the radiance bytes, C4 1.29x; profiles/r03o_*).
// Edge tiles keep all 64 slots (unused ones are never written or read).
struct SampleTiles {
    int32_t width, n_rows, tiles_x;
    int32_t f32_records;   // the f32 mode's records: f32 x 3 (12 B) instead of f64 x 3 (24 B)
};
__host__ __device__ inline size_t tiled_record(int tiles_x, int n_samples, int x, int k, int s)
{
    const size_t tile = (size_t)(k >> 3) * (size_t)tiles_x + (size_t)(x >> 3);
    return (tile * (size_t)n_samples + (size_t)s) * 64 + (size_t)(((k & 7) << 3) | (x & 7));
}
__host__ __device__ inline size_t tiled_pixels(int width, int n_rows)   // records per sample, padded tiles
{
    return (size_t)((width + 7) / 8) * (size_t)((n_rows + 7) / 8) * 64;
}

uint32_t variant_features(uint32_t scene_features);
// Ph: host copy of the params (grid size); P: the same params in device memory
// chunk schedule: out = chunk partials [n_chunks][n_px][3]; pool schedule: out = per-sample
// radiance, tiled_record order over spp - sample_begin samples; work = one device counter
hipError_t launch_trace(const SceneDev& S, const KParams& Ph, const KParams* P, double* out,
                        unsigned long long* counters, unsigned* work, const LaunchOpts& o, hipStream_t stream);
// pool schedule: per pixel, chunk sums of its samples (sample order) added to 0.0, scaled to out
// (out and the carried sums are in pixel order k * width + x)
hipError_t launch_reduce_samples(const double* samples, void* out, bool f64, SampleTiles g, int n_samples,
                                 int chunk, double scale, hipStream_t stream);
// the same across buffer batches: acc = closed chunks' total, open = the chunk in progress
// (pos of its samples seen before this batch); close ends the last chunk
hipError_t launch_reduce_samples_carry(const double* samples, double* acc, double* open, SampleTiles g,
                                       int n_samples, int chunk, int pos, bool close, hipStream_t stream);
hipError_t launch_reduce(const double* partial, void* out, bool f64, long long n_px, int n_chunks, double scale,
                         hipStream_t stream);
// acc[i] += chunk partials in chunk order (progressive accumulation, rt_accum_add)
hipError_t launch_accumulate(const double* partial, double* acc, long long n_px, int n_chunks, hipStream_t stream);
// tile shards gathered from `world` ranks (rank r's slab at r * slab_elems elements) -> the frame
// (height x width x 3, row 0 = bottom) in the tile order `order` (null: raster); rt_tiles_assemble
hipError_t launch_assemble_tiles(const void* gathered, void* frame, bool f64, int world, long long slab_elems,
                                 int width, int height, const uint32_t* order, hipStream_t stream);
hipError_t launch_eval(int fn, const double* x, const double* y, const double* z, double* out, int n,
                       hipStream_t stream);

}  // namespace rtk
