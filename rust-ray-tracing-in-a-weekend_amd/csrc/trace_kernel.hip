// trace_kernel.hip — host-side dispatch of the megakernel (the variants live in
// trace_v*.hip over trace_device.hpp), the per-pixel reductions of the schedules, and the
// device numerics probe. See trace_device.hpp for the execution model.
#include "trace_device.hpp"

namespace rtk {

// One thread per record slot of a tile (tiled_record order: a wave reads one tile's 64
// consecutive records per sample); slots of an edge tile outside the image return. Sets the
// pixel's output index and the record base of sample 0.
__device__ __forceinline__ bool tile_slot(SampleTiles g, int n_samples, long long i, long long& px, size_t& rec)
{
    const long long tile = i >> 6;
    const int lp = (int)(i & 63);
    const int x = (int)(tile % g.tiles_x) * 8 + (lp & 7);
    const int k = (int)(tile / g.tiles_x) * 8 + (lp >> 3);
    if (x >= g.width || k >= g.n_rows) return false;
    px = (long long)k * g.width + x;
    rec = tiled_record(g.tiles_x, n_samples, x, k, 0);
    return true;
}

// Per pixel: chunk sums of consecutive samples (chunk order, each from 0.0), added in
// chunk order to 0.0 and scaled into out: the same additions, in the same order, as the
// chunk schedule's lane sums + reduce_chunks.
template <typename T, typename Rec = double>
__global__ void __launch_bounds__(256) reduce_samples(const Rec* __restrict__ samples, T* __restrict__ out,
                                                      SampleTiles g, long long n_slots, int n_samples, int chunk,
                                                      double scale)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long px;
    size_t rec;
    if (i >= n_slots || !tile_slot(g, n_samples, i, px, rec)) return;
    double r = 0.0, g_ = 0.0, b = 0.0;
    for (int c0 = 0; c0 < n_samples; c0 += chunk) {
        const int c1 = min(n_samples, c0 + chunk);
        double cr = 0.0, cg = 0.0, cb = 0.0;
        for (int j = c0; j < c1; ++j) {
            const Rec* p = samples + (rec + (size_t)j * 64) * 3;
            cr = cr + (double)p[0];
            cg = cg + (double)p[1];
            cb = cb + (double)p[2];
        }
        r = r + cr;
        g_ = g_ + cg;
        b = b + cb;
    }
    out[3 * px + 0] = (T)(r * scale);
    out[3 * px + 1] = (T)(g_ * scale);
    out[3 * px + 2] = (T)(b * scale);
}

// reduce_samples with one block per 8x8 tile: wave w of kReduceWaves sums chunks w, w + W, ... of
// the tile's 64 pixels (each chunk from 0.0, its samples in order, four samples' loads in flight),
// parks the chunk sums in LDS, and wave 0 adds a round's W chunk sums in chunk order to the running
// total: reduce_samples' additions in reduce_samples' order (bit-identical), with W waves' loads
// in flight per tile instead of one lane's walk over every sample, and no tail of long per-pixel
// loops at the end of the launch.
#ifndef RT_REDUCE_TILED
#define RT_REDUCE_TILED 1
#endif
constexpr int kReduceWaves = 8;
template <typename T, typename Rec = double>
__global__ void __launch_bounds__(64 * kReduceWaves) reduce_samples_tiled(const Rec* __restrict__ samples,
                                                                          T* __restrict__ out, SampleTiles g,
                                                                          int n_samples, int chunk, double scale)
{
    __shared__ double part[kReduceWaves][3][64];
    const unsigned tile = blockIdx.x;
    const int lane = (int)(threadIdx.x & 63u), w = (int)(threadIdx.x >> 6);
    const Rec* base = samples + ((size_t)tile * (size_t)n_samples * 64 + (size_t)lane) * 3;
    const int n_chunks = (n_samples + chunk - 1) / chunk;
    double r = 0.0, g_ = 0.0, b = 0.0;
    for (int c0 = 0; c0 < n_chunks; c0 += kReduceWaves) {
        const int c = c0 + w;
        if (c < n_chunks) {
            const int j0 = c * chunk, j1 = min(n_samples, j0 + chunk);
            double cr = 0.0, cg = 0.0, cb = 0.0;
            int j = j0;
            for (; j + 4 <= j1; j += 4) {
                Rec v[4][3];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const Rec* p = base + (size_t)(j + q) * 192;
                    v[q][0] = p[0];
                    v[q][1] = p[1];
                    v[q][2] = p[2];
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    cr = cr + (double)v[q][0];
                    cg = cg + (double)v[q][1];
                    cb = cb + (double)v[q][2];
                }
            }
            for (; j < j1; ++j) {
                const Rec* p = base + (size_t)j * 192;
                cr = cr + (double)p[0];
                cg = cg + (double)p[1];
                cb = cb + (double)p[2];
            }
            part[w][0][lane] = cr;
            part[w][1][lane] = cg;
            part[w][2][lane] = cb;
        }
        __syncthreads();
        if (w == 0) {
            const int nc = min(kReduceWaves, n_chunks - c0);
            for (int q = 0; q < nc; ++q) {
                r = r + part[q][0][lane];
                g_ = g_ + part[q][1][lane];
                b = b + part[q][2][lane];
            }
        }
        __syncthreads();
    }
    if (w == 0) {
        const int x = (int)(tile % (unsigned)g.tiles_x) * 8 + (lane & 7);
        const int k = (int)(tile / (unsigned)g.tiles_x) * 8 + (lane >> 3);
        if (x < g.width && k < g.n_rows) {
            const size_t px = (size_t)k * (size_t)g.width + (size_t)x;
            out[3 * px + 0] = (T)(r * scale);
            out[3 * px + 1] = (T)(g_ * scale);
            out[3 * px + 2] = (T)(b * scale);
        }
    }
}

// The same sums over a render split into buffer batches that need not end on a chunk
// boundary: acc holds the closed chunks' total, open the chunk in progress (pos samples
// in at batch start, uniform); `close` ends the render's last chunk.
template <typename Rec = double>
__global__ void __launch_bounds__(256) reduce_samples_carry(const Rec* __restrict__ samples,
                                                            double* __restrict__ acc, double* __restrict__ open,
                                                            SampleTiles g, long long n_slots, int n_samples,
                                                            int chunk, int pos, int close)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long px;
    size_t rec;
    if (i >= n_slots || !tile_slot(g, n_samples, i, px, rec)) return;
    double r = acc[3 * px + 0], g_ = acc[3 * px + 1], b = acc[3 * px + 2];
    double cr = 0.0, cg = 0.0, cb = 0.0;
    if (pos > 0) {
        cr = open[3 * px + 0];
        cg = open[3 * px + 1];
        cb = open[3 * px + 2];
    }
    for (int j = 0; j < n_samples; ++j) {
        const Rec* p = samples + (rec + (size_t)j * 64) * 3;
        cr = cr + (double)p[0];
        cg = cg + (double)p[1];
        cb = cb + (double)p[2];
        if (++pos == chunk) {
            r = r + cr;
            g_ = g_ + cg;
            b = b + cb;
            cr = cg = cb = 0.0;
            pos = 0;
        }
    }
    if (close && pos > 0) {
        r = r + cr;
        g_ = g_ + cg;
        b = b + cb;
    }
    acc[3 * px + 0] = r;
    acc[3 * px + 1] = g_;
    acc[3 * px + 2] = b;
    open[3 * px + 0] = cr;
    open[3 * px + 1] = cg;
    open[3 * px + 2] = cb;
}

// sum of partials in chunk order, times 1/spp (math.rs:120-125 before sqrt).
template <typename T>
__global__ void __launch_bounds__(256) reduce_chunks(const double* __restrict__ partial, T* __restrict__ out,
                                                     long long n_px, int n_chunks, double scale)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_px) return;
    double r = 0.0, g = 0.0, b = 0.0;
    for (int c = 0; c < n_chunks; ++c) {
        const double* p = partial + ((size_t)c * n_px + i) * 3;
        r = r + p[0];
        g = g + p[1];
        b = b + p[2];
    }
    out[3 * i + 0] = (T)(r * scale);
    out[3 * i + 1] = (T)(g * scale);
    out[3 * i + 2] = (T)(b * scale);
}

// Progressive accumulation: continues reduce_chunks' running sum across batches, so a
// render split at chunk boundaries sums in the same order as one launch.
__global__ void __launch_bounds__(256) accumulate_chunks(const double* __restrict__ partial,
                                                         double* __restrict__ acc, long long n_px, int n_chunks)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_px) return;
    double r = acc[3 * i + 0], g = acc[3 * i + 1], b = acc[3 * i + 2];
    for (int c = 0; c < n_chunks; ++c) {
        const double* p = partial + ((size_t)c * n_px + i) * 3;
        r = r + p[0];
        g = g + p[1];
        b = b + p[2];
    }
    acc[3 * i + 0] = r;
    acc[3 * i + 1] = g;
    acc[3 * i + 2] = b;
}

// Multi-GPU reassembly (rt_tiles_assemble, rt_render_gather; the merge of main.rs:542-547): the
// gathered tile slabs of `world` ranks, rank r's at r * slab_elems (8 rows x 8 * n_r tiles x 3,
// its tiles m at positions r + m * world of the tile order), written into the frame (row 0 =
// bottom). One thread per slab pixel: 8 consecutive threads read one tile row's 24 contiguous
// elements and write them to one frame row; pixels of an edge tile outside the image are dropped.
template <typename T>
__global__ void __launch_bounds__(256) assemble_tiles(const T* __restrict__ gathered, T* __restrict__ frame,
                                                      int world, long long slab_elems, int n_max, int width,
                                                      int height, int tiles_x, long long n_tiles,
                                                      const uint32_t* __restrict__ order)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // (rank, row k, column)
    const long long per_rank = 64LL * n_max;
    if (i >= per_rank * world) return;
    const int r = (int)(i / per_rank);
    const long long j = i - (long long)r * per_rank;
    const int n_r = (int)((n_tiles - r + world - 1) / world);   // rt_tiles_in_shard
    const int k = (int)(j / (8LL * n_max));
    const int col = (int)(j - (long long)k * 8 * n_max);
    const int m = col >> 3;
    if (m >= n_r) return;
    const long long pos = r + (long long)m * world;
    const long long t = order ? (long long)order[pos] : pos;
    const int x = (int)(t % tiles_x) * 8 + (col & 7);
    const int y = (int)(t / tiles_x) * 8 + k;
    if (x >= width || y >= height) return;
    const T* src = gathered + (long long)r * slab_elems + ((long long)k * 8 * n_r + col) * 3;
    T* dst = frame + ((long long)y * width + x) * 3;
    dst[0] = src[0];
    dst[1] = src[1];
    dst[2] = src[2];
}

struct StoredUV {   // hit_uv's config for the eval kernel: uv inputs held in the record
    static constexpr uint32_t F = FEAT_ALL;
};

__global__ void eval_numerics(int fn, const double* x, const double* y, const double* z, double* out, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double r = 0.0;
    switch (fn) {
    case 0: r = rt_sin(x[i]); break;
    case 1: r = rt_cos(x[i]); break;
    case 2: r = rt_log(x[i]); break;
    case 3: r = rt_atan2(x[i], y[i]); break;
    case 4: r = rt_acos(x[i]); break;
    case 5: case 6: {
        HitT<double> h;
        h.uvkind = 1;
        h.uv0 = x[i]; h.uv1 = y[i]; h.uv2 = z[i];
        double u, v;
        hit_uv<StoredUV>(h, u, v);   // uv inputs held in the record
        r = fn == 5 ? u : v;
        break;
    }
    case 7: r = rt_pow5(x[i]); break;
    case 8: r = __builtin_sqrt(x[i]); break;
    case 9: r = x[i] / y[i]; break;
    case 10: r = rt_unit53(rt_f64_bits(x[i])); break;
    case 11: r = rt_uniform_sample(rt_f64_bits(x[i]), -1.0, rt_uniform_incl_scale(-1.0, 1.0)); break;
    case 12: r = (double)rt_sin_sign(x[i]); break;
    case 13: r = div_rcp(x[i], y[i], rcp_for_div(y[i])); break;   // must equal x / y bit for bit
    default: break;
    }
    out[i] = r;
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
uint32_t variant_features(uint32_t scene_features)
{
    if ((scene_features & ~FEAT_SET_SPHERES) == 0) return FEAT_SET_SPHERES;
    if ((scene_features & ~FEAT_SET_RECTINST) == 0) return FEAT_SET_RECTINST;
    if ((scene_features & ~FEAT_SET_MEDIA) == 0) return FEAT_SET_MEDIA;
    if ((scene_features & ~FEAT_SET_FINAL) == 0) return FEAT_SET_FINAL;
    return FEAT_ALL;
}

hipError_t launch_trace(const SceneDev& S, const KParams& Ph, const KParams* P, double* out,
                        unsigned long long* counters, unsigned* work, const LaunchOpts& o, hipStream_t stream)
{
    Launch L;
    L.S = &S;
    L.P = P;
    L.out = out;
    L.counters = counters;
    L.work = work;
    L.pool = o.pool;
    L.waves_per_simd = o.waves_per_simd;
    L.max_waves = o.pool == 1 && Ph.ring ? (unsigned)Ph.ring_waves : 0u;
    // waves of the chunk schedule / work blocks of the pools
    const long long groups = o.pool == 2   ? (Ph.n_chunks + std::max(1, Ph.block_chunks) - 1) / std::max(1, Ph.block_chunks)
                             : o.pool == 1 ? ((long long)Ph.spp - Ph.sample_begin + std::max(1, Ph.block_samples) - 1) /
                                                 std::max(1, Ph.block_samples)
                                           : Ph.n_chunks;
    L.n_blocks = (unsigned long long)Ph.tiles_x * Ph.tiles_y * groups;
    if (L.n_blocks == 0) return hipSuccess;
    if (L.n_blocks > 0xfffffff0ULL) return hipErrorInvalidValue;
    if (o.pool) {
        const hipError_t e = hipMemsetAsync(work, 0, sizeof(unsigned), stream);
        if (e != hipSuccess) return e;
    }
    const uint32_t f = variant_features(o.features);
    if (o.f32 && o.count) {
        if (f == FEAT_SET_SPHERES) return launch_variant_f32_count<FEAT_SET_SPHERES>(L, o, stream);
        if (f == FEAT_SET_FINAL) return launch_variant_f32_count<FEAT_SET_FINAL>(L, o, stream);
        return hipErrorNotSupported;
    }
    if (o.f32) {
        if (f == FEAT_SET_SPHERES) return launch_variant_f32<FEAT_SET_SPHERES>(L, o, stream);
        if (f == FEAT_SET_RECTINST) return launch_variant_f32<FEAT_SET_RECTINST>(L, o, stream);
        if (f == FEAT_SET_MEDIA) return launch_variant_f32<FEAT_SET_MEDIA>(L, o, stream);
        if (f == FEAT_SET_FINAL) return launch_variant_f32<FEAT_SET_FINAL>(L, o, stream);
        return launch_variant_f32<FEAT_ALL>(L, o, stream);
    }
    if (o.count) {
        if (f == FEAT_SET_SPHERES) return launch_variant<FEAT_SET_SPHERES, true>(L, o, stream);
        if (f == FEAT_SET_RECTINST) return launch_variant<FEAT_SET_RECTINST, true>(L, o, stream);
        if (f == FEAT_SET_MEDIA) return launch_variant<FEAT_SET_MEDIA, true>(L, o, stream);
        if (f == FEAT_SET_FINAL) return launch_variant<FEAT_SET_FINAL, true>(L, o, stream);
        return launch_variant<FEAT_ALL, true>(L, o, stream);
    }
    if (f == FEAT_SET_SPHERES) return launch_variant<FEAT_SET_SPHERES, false>(L, o, stream);
    if (f == FEAT_SET_RECTINST) return launch_variant<FEAT_SET_RECTINST, false>(L, o, stream);
    if (f == FEAT_SET_MEDIA) return launch_variant<FEAT_SET_MEDIA, false>(L, o, stream);
    if (f == FEAT_SET_FINAL) return launch_variant<FEAT_SET_FINAL, false>(L, o, stream);
    return launch_variant<FEAT_ALL, false>(L, o, stream);
}


hipError_t launch_reduce_samples(const double* samples, void* out, bool f64, SampleTiles g, int n_samples,
                                 int chunk, double scale, hipStream_t stream)
{
    const long long n_slots = (long long)tiled_pixels(g.width, g.n_rows);
    const float* rec32 = reinterpret_cast<const float*>(samples);
    if (RT_REDUCE_TILED) {   // one block per tile
        const long long tiles = n_slots / 64;
        if (tiles <= 0 || chunk < 1) return tiles <= 0 ? hipSuccess : hipErrorInvalidValue;
        const dim3 grid((unsigned)tiles), block(64 * kReduceWaves);
        if (g.f32_records && f64)
            hipLaunchKernelGGL((reduce_samples_tiled<double, float>), grid, block, 0, stream, rec32, (double*)out, g,
                               n_samples, chunk, scale);
        else if (g.f32_records)
            hipLaunchKernelGGL((reduce_samples_tiled<float, float>), grid, block, 0, stream, rec32, (float*)out, g,
                               n_samples, chunk, scale);
        else if (f64)
            hipLaunchKernelGGL(reduce_samples_tiled<double>, grid, block, 0, stream, samples, (double*)out, g, n_samples,
                               chunk, scale);
        else
            hipLaunchKernelGGL(reduce_samples_tiled<float>, grid, block, 0, stream, samples, (float*)out, g, n_samples,
                               chunk, scale);
        return hipGetLastError();
    }
    const long long blocks = (n_slots + 255) / 256;
    if (blocks <= 0) return hipSuccess;
    if (g.f32_records && f64)
        hipLaunchKernelGGL((reduce_samples<double, float>), dim3((unsigned)blocks), dim3(256), 0, stream, rec32,
                           (double*)out, g, n_slots, n_samples, chunk, scale);
    else if (g.f32_records)
        hipLaunchKernelGGL((reduce_samples<float, float>), dim3((unsigned)blocks), dim3(256), 0, stream, rec32,
                           (float*)out, g, n_slots, n_samples, chunk, scale);
    else if (f64)
        hipLaunchKernelGGL(reduce_samples<double>, dim3((unsigned)blocks), dim3(256), 0, stream, samples, (double*)out,
                           g, n_slots, n_samples, chunk, scale);
    else
        hipLaunchKernelGGL(reduce_samples<float>, dim3((unsigned)blocks), dim3(256), 0, stream, samples, (float*)out,
                           g, n_slots, n_samples, chunk, scale);
    return hipGetLastError();
}

hipError_t launch_reduce_samples_carry(const double* samples, double* acc, double* open, SampleTiles g,
                                       int n_samples, int chunk, int pos, bool close, hipStream_t stream)
{
    const long long n_slots = (long long)tiled_pixels(g.width, g.n_rows);
    const long long blocks = (n_slots + 255) / 256;
    if (blocks <= 0) return hipSuccess;
    if (g.f32_records)
        hipLaunchKernelGGL(reduce_samples_carry<float>, dim3((unsigned)blocks), dim3(256), 0, stream,
                           reinterpret_cast<const float*>(samples), acc, open, g, n_slots, n_samples, chunk, pos,
                           (int)close);
    else
        hipLaunchKernelGGL(reduce_samples_carry<double>, dim3((unsigned)blocks), dim3(256), 0, stream, samples, acc,
                           open, g, n_slots, n_samples, chunk, pos, (int)close);
    return hipGetLastError();
}

hipError_t launch_reduce(const double* partial, void* out, bool f64, long long n_px, int n_chunks, double scale,
                         hipStream_t stream)
{
    const long long blocks = (n_px + 255) / 256;
    if (blocks <= 0) return hipSuccess;
    if (f64)
        hipLaunchKernelGGL(reduce_chunks<double>, dim3((unsigned)blocks), dim3(256), 0, stream, partial, (double*)out,
                           n_px, n_chunks, scale);
    else
        hipLaunchKernelGGL(reduce_chunks<float>, dim3((unsigned)blocks), dim3(256), 0, stream, partial, (float*)out,
                           n_px, n_chunks, scale);
    return hipGetLastError();
}

hipError_t launch_accumulate(const double* partial, double* acc, long long n_px, int n_chunks, hipStream_t stream)
{
    const long long blocks = (n_px + 255) / 256;
    if (blocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(accumulate_chunks, dim3((unsigned)blocks), dim3(256), 0, stream, partial, acc, n_px, n_chunks);
    return hipGetLastError();
}

hipError_t launch_assemble_tiles(const void* gathered, void* frame, bool f64, int world, long long slab_elems,
                                 int width, int height, const uint32_t* order, hipStream_t stream)
{
    const int tiles_x = (width + 7) / 8;
    const long long n_tiles = (long long)tiles_x * ((height + 7) / 8);
    const int n_max = (int)((n_tiles + world - 1) / world);
    const long long n = 64LL * n_max * world;
    const long long blocks = (n + 255) / 256;
    if (blocks <= 0) return hipSuccess;
    if (blocks > 0x7fffffffLL || slab_elems < 192LL * n_max) return hipErrorInvalidValue;
    if (f64)
        hipLaunchKernelGGL(assemble_tiles<double>, dim3((unsigned)blocks), dim3(256), 0, stream, (const double*)gathered,
                           (double*)frame, world, slab_elems, n_max, width, height, tiles_x, n_tiles, order);
    else
        hipLaunchKernelGGL(assemble_tiles<float>, dim3((unsigned)blocks), dim3(256), 0, stream, (const float*)gathered,
                           (float*)frame, world, slab_elems, n_max, width, height, tiles_x, n_tiles, order);
    return hipGetLastError();
}

hipError_t launch_eval(int fn, const double* x, const double* y, const double* z, double* out, int n,
                       hipStream_t stream)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(eval_numerics, dim3((n + 255) / 256), dim3(256), 0, stream, fn, x, y, z, out, n);
    return hipGetLastError();
}

}  // namespace rtk
