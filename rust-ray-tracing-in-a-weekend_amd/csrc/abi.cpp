// abi.cpp — the extern "C" boundary (include/rt/rt_abi.h). No exception and no
// C++ type crosses it; every entry point returns RT_OK or a negative RT_ERR_*.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <limits>
#include <functional>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "rt/rt_abi.h"
#include "ctx_internal.hpp"
#include "scene_model.hpp"
#include "trace_kernel.hpp"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg)
{
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what)
{
    return fail(RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return hip_fail(e_, #expr); \
    } while (0)

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// device slots for launch params (a ring: a render's params stay intact while later
// renders are enqueued behind it on the same stream)
constexpr int kParamSlots = 16;

// LDS stack entries per lane above which the scratch stack is used (48 KB per block)
constexpr int kMaxLdsStack = 48;
// TLAS nodes kept in LDS (32 KB per block): the first kMaxLdsNodes in BFS order, i.e.
// the top levels; deeper ones are read from L1/L2
constexpr int kMaxLdsNodes = 512;
// waves per SIMD of the final-scene variant (trace_device.hpp min_waves: its LDS budget is per
// workgroup of the workgroups those waves make)
#ifndef RT_MIN_WAVES_FINAL
#define RT_MIN_WAVES_FINAL 4
#endif
// instance BLAS nodes staged in LDS at most (64 B each)
#ifndef RT_LDS_BLAS_MAX
#define RT_LDS_BLAS_MAX 1024   // the LDS budget decides (512-thread final variant: 512 of the final scene's 548
                               // BLAS nodes, 110.95 -> 108.23 ms at C4 1920x1080x100, r03r_ab_c4.log; with 256-thread
                               // workgroups the budget held ~95: 64 staged 132.15 ms, 16 133.31, none 132.98, r03h)
#endif
constexpr int kMaxLdsBlas = RT_LDS_BLAS_MAX;
// material (64 B) and texture (96 B) tables staged in LDS when both are this small (10 KB)
constexpr int kMaxLdsMaterials = 64;

}  // namespace

struct rt_world {
    explicit rt_world(uint64_t seed) : w(seed) {}
    rtw::World w;
};

constexpr int kCounters = 32;  // count_work counters (trace_device.hpp: the trace kernels' epilogues; rt_last_counters)

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    void* scene_buf = nullptr;
    size_t scene_bytes = 0;
    rtk::SceneDev S{};
    bool has_scene = false;
    double* partial = nullptr;
    size_t partial_cap = 0;
    void* out_buf = nullptr;
    size_t out_cap = 0;
    unsigned long long* counters = nullptr;
    rtk::KParams* params = nullptr;     // ring of kParamSlots device copies of the launch params
    int param_slot = 0;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    // Cross-stream ordering: the scratch buffers (partial, work counter, acc_tmp, counters,
    // params ring, staging) are per context, so work enqueued on a new stream must wait for
    // everything the context enqueued on the previous one. ev_done is recorded after each
    // enqueue; a call on another stream first makes that stream wait for it.
    hipEvent_t ev_done = nullptr;
    hipStream_t last_stream = nullptr;
    bool any_enqueued = false;
    bool pending_stats = false;
    bool pending_counts = false;
    rt_stats stats{};
    uint32_t features = rtk::FEAT_ALL;  // of the uploaded scene
    int n_materials = 0, n_textures = 0;
    int block_chunks = 0;               // RT_OPT_BLOCK_CHUNKS: chunks per item-pool work block (0: auto)
    int block_samples = 0;              // RT_OPT_BLOCK_SAMPLES: samples per per-sample-pool work block (0: auto)
    int opt_ring = 1;                   // RT_OPT_POOL_RING: POOL reduces finished blocks in the kernel (0 never,
                                        // 1 when its per-sample buffer would not fit the bound, 2 always)
    int opt_comm_direct = 1;            // RT_OPT_COMM_DIRECT: a world-1 rt_render_gather renders straight into the frame
    double* ring = nullptr;             // its per-wave record ring (kPoolRing blocks per wave)
    size_t ring_cap = 0;
    unsigned long long raw_counters[kCounters] = {};   // the last count_work render's counters (rt_last_counters)
    uint32_t* tile_order = nullptr;     // rt_ctx_set_tile_order: tile shards' position -> raster tile (device)
    int64_t tile_order_n = 0;           //   its length (0: raster order)
    unsigned long long* tile_cost = nullptr;   // count_work pool renders: lane-cycles per raster tile
    int64_t tile_cost_cap = 0;          //   tiles allocated
    int64_t tile_cost_n = 0;            //   tiles of the last count_work render (rt_last_tile_costs)
    uint32_t extra_features = 0;        // RT_OPT_EXTRA_FEATURES: a larger kernel variant than the scene needs (tests)
    double pad_extent = 0.0;
    int opt_slab32 = 1;                 // rt_ctx_set_variant
    int opt_lds = 1;                    // rt_ctx_set_variant
    int opt_lds_nodes = 1;              // rt_ctx_set_variant: keep the TLAS in LDS when it fits
    int opt_hoist = 1;                  // RT_OPT_HOIST: test a huge root-child leaf before the walk (pre_leaf)
    int opt_pool = RT_SCHED_AUTO;       // rt_ctx_set_schedule: RT_SCHED_*
    int opt_precision = RT_PREC_F64;    // rt_ctx_set_precision: RT_PREC_*
    size_t sample_buf_cap = (size_t)32 << 30;  // RT_OPT_TRACE_BUF_BYTES: bound of the trace-output buffer
    unsigned* work = nullptr;           // pool / item schedules: work-block counters (one per overlapped batch)
    // Overlapped buffer batches (RT_OPT_BATCH_OVERLAP): batch k traces on tstream[k & 1] into half k & 1
    // of the trace-output buffer while the caller's stream reduces batch k - 1
    hipStream_t tstream[2] = {nullptr, nullptr};
    hipEvent_t ev_in = nullptr, ev_tr[2] = {nullptr, nullptr}, ev_rd[2] = {nullptr, nullptr};
    int opt_overlap = 1;
    double* acc_tmp = nullptr;          // running sums when a render takes several buffer batches
    size_t acc_tmp_cap = 0;
    int n_tlas_nodes = 0;
    int n_nodes = 0;                    // BVH nodes of the uploaded scene (TLAS + BLASes)
    int n_cus = 256;
    size_t lds_per_cu = 160 * 1024;     // the device's LDS per CU and per workgroup (read at creation)
    size_t lds_per_block = 160 * 1024;
};

// The trace-output buffer's default bound: 64 GiB, or half the device's free memory if that is
// less (round 6). The per-sample buffer is as fast as the in-kernel ring reduction on the random
// scene and 1.4 % faster on the final scene, whose ring reductions stall a wave holding 4 waves'
// worth of path state per SIMD (interleaved medians, kernel + reduce ms: C2 74.47 vs 74.41, C2 f32
// 64.46 vs 64.38, C4 982.1 vs 996.2; profiles/r06c_ab_*.log), and a 288 GB device holds C4's
// 49.8 GB of records in one batch. The ring stays for renders the bound does not hold in one
// batch (C5: 1.6 TB of records), where its chunk partials are 1/16 of the bytes.
static size_t default_buf_cap()
{
    size_t fr = 0, tot = 0;
    size_t cap = (size_t)64 << 30;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr > 0) cap = std::min(cap, fr / 2);
    return std::max(cap >> 20, (size_t)1) << 20;
}

#ifndef RT_SRC_HASH
#define RT_SRC_HASH "unknown"
#endif

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }
const char* rt_last_error(void) { return g_last_error.c_str(); }
const char* rt_build_info(void) { return RT_SRC_HASH; }

int rt_device_count(int* count)
{
    if (!count) return fail(RT_ERR_INVALID, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return hip_fail(e, "hipGetDeviceCount");
    }
    *count = n;
    return RT_OK;
}

int rt_ctx_create(int device, rt_ctx** out)
{
    if (!out) return fail(RT_ERR_INVALID, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RT_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return fail(RT_ERR_INVALID, "device index out of range");
    HIP_TRY(hipSetDevice(device));
    rt_ctx* c = new (std::nothrow) rt_ctx();
    if (!c) return fail(RT_ERR_OOM, "rt_ctx");
    c->device = device;
    c->sample_buf_cap = default_buf_cap();
    {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) == hipSuccess && v > 0)
            c->lds_per_cu = (size_t)v;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && v > 0)
            c->lds_per_block = (size_t)v;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && v > 0)
            c->n_cus = v;
        c->lds_per_block = std::min(c->lds_per_block, c->lds_per_cu);
    }
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    for (int i = 0; i < 3 && e == hipSuccess; ++i) e = hipEventCreate(&c->ev[i]);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMalloc((void**)&c->counters, kCounters * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMalloc((void**)&c->params, kParamSlots * sizeof(rtk::KParams));
    if (e == hipSuccess) e = hipMalloc((void**)&c->work, 2 * sizeof(unsigned));
    for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipStreamCreateWithFlags(&c->tstream[i], hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->ev_tr[i], hipEventDisableTiming);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->ev_rd[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming);
    if (e != hipSuccess) {
        rt_ctx_destroy(c);
        return hip_fail(e, "rt_ctx_create");
    }
    *out = c;
    return RT_OK;
}

void rt_ctx_destroy(rt_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->ev_done && c->any_enqueued) (void)hipEventSynchronize(c->ev_done);  // work on a caller's stream
    (void)hipFree(c->scene_buf);
    (void)hipFree(c->partial);
    (void)hipFree(c->ring);
    (void)hipFree(c->out_buf);
    (void)hipFree(c->counters);
    (void)hipFree(c->tile_order);
    (void)hipFree(c->tile_cost);
    (void)hipFree(c->params);
    (void)hipFree(c->work);
    (void)hipFree(c->acc_tmp);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    for (int i = 0; i < 2; ++i) {
        if (c->tstream[i]) (void)hipStreamSynchronize(c->tstream[i]);
        if (c->tstream[i]) (void)hipStreamDestroy(c->tstream[i]);
        if (c->ev_tr[i]) (void)hipEventDestroy(c->ev_tr[i]);
        if (c->ev_rd[i]) (void)hipEventDestroy(c->ev_rd[i]);
    }
    if (c->ev_in) (void)hipEventDestroy(c->ev_in);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

// ---- world -------------------------------------------------------------------
int rt_world_create(uint64_t scene_seed, rt_world** out)
{
    if (!out) return fail(RT_ERR_INVALID, "null out");
    *out = new (std::nothrow) rt_world(scene_seed);
    return *out ? RT_OK : fail(RT_ERR_OOM, "rt_world");
}
void rt_world_destroy(rt_world* w) { delete w; }

#define CHECK_WORLD(w, o)                                              \
    do {                                                               \
        if (!(w) || !(o)) return fail(RT_ERR_INVALID, "null argument"); \
    } while (0)

static rtw::V3 vec(const double* a) { return rtw::v3(a[0], a[1], a[2]); }

int rt_world_texture_solid(rt_world* w, double r, double g, double b, int* o)
{
    CHECK_WORLD(w, o);
    *o = w->w.texture_solid(rtw::v3(r, g, b));
    return RT_OK;
}
int rt_world_texture_checker(rt_world* w, const double even[3], const double odd[3], int* o)
{
    CHECK_WORLD(w, o);
    if (!even || !odd) return fail(RT_ERR_INVALID, "null color");
    *o = w->w.texture_checker(vec(even), vec(odd));
    return RT_OK;
}
int rt_world_texture_noise(rt_world* w, double scale, int* o)
{
    CHECK_WORLD(w, o);
    *o = w->w.texture_noise(scale);
    return RT_OK;
}
int rt_world_texture_image(rt_world* w, const uint8_t* rgb, int width, int height, int* o)
{
    CHECK_WORLD(w, o);
    if (width < 0 || height < 0 || (!rgb && width * height > 0)) return fail(RT_ERR_INVALID, "bad image");
    *o = w->w.texture_image(rgb, width, height);
    return RT_OK;
}

int rt_world_material_lambertian(rt_world* w, int tex, int* o)
{
    CHECK_WORLD(w, o);
    if (!w->w.valid_texture(tex)) return fail(RT_ERR_INVALID, "bad texture id");
    *o = w->w.lambertian(tex);
    return RT_OK;
}
int rt_world_material_metal(rt_world* w, const double albedo[3], double fuzz, int* o)
{
    CHECK_WORLD(w, o);
    if (!albedo) return fail(RT_ERR_INVALID, "null albedo");
    *o = w->w.metal(vec(albedo), fuzz);
    return RT_OK;
}
int rt_world_material_dielectric(rt_world* w, double ir, int* o)
{
    CHECK_WORLD(w, o);
    *o = w->w.dielectric(ir);
    return RT_OK;
}
int rt_world_material_diffuse_light(rt_world* w, int tex, int* o)
{
    CHECK_WORLD(w, o);
    if (!w->w.valid_texture(tex)) return fail(RT_ERR_INVALID, "bad texture id");
    *o = w->w.diffuse_light(tex);
    return RT_OK;
}
int rt_world_material_isotropic(rt_world* w, int tex, int* o)
{
    CHECK_WORLD(w, o);
    if (!w->w.valid_texture(tex)) return fail(RT_ERR_INVALID, "bad texture id");
    *o = w->w.isotropic(tex);
    return RT_OK;
}

int rt_world_sphere(rt_world* w, int mat, const double c[3], double r, int* o)
{
    CHECK_WORLD(w, o);
    if (!c || !w->w.valid_material(mat)) return fail(RT_ERR_INVALID, "bad sphere");
    *o = w->w.sphere(mat, vec(c), r);
    return RT_OK;
}
int rt_world_moving_sphere(rt_world* w, int mat, const double c0[3], const double c1[3], double t0, double t1,
                           double r, int* o)
{
    CHECK_WORLD(w, o);
    if (!c0 || !c1 || !w->w.valid_material(mat)) return fail(RT_ERR_INVALID, "bad moving sphere");
    *o = w->w.moving_sphere(mat, vec(c0), vec(c1), t0, t1, r);
    return RT_OK;
}
int rt_world_rect(rt_world* w, int axis, int mat, double a0, double a1, double b0, double b1, double k, int* o)
{
    CHECK_WORLD(w, o);
    if (axis < 0 || axis > 2 || !w->w.valid_material(mat)) return fail(RT_ERR_INVALID, "bad rect");
    rtw::HKind kind = axis == 0 ? rtw::HKind::XYRect : axis == 1 ? rtw::HKind::XZRect : rtw::HKind::YZRect;
    *o = w->w.rect(kind, mat, a0, a1, b0, b1, k);
    return RT_OK;
}
int rt_world_box(rt_world* w, const double mn[3], const double mx[3], int mat, int* o)
{
    CHECK_WORLD(w, o);
    if (!mn || !mx || !w->w.valid_material(mat)) return fail(RT_ERR_INVALID, "bad box");
    *o = w->w.box(vec(mn), vec(mx), mat);
    return RT_OK;
}
int rt_world_translate(rt_world* w, int child, const double off[3], int* o)
{
    CHECK_WORLD(w, o);
    if (!off || !w->w.valid_hittable(child)) return fail(RT_ERR_INVALID, "bad translate");
    *o = w->w.translate(child, vec(off));
    return RT_OK;
}
int rt_world_rotate_y(rt_world* w, int child, double angle, int* o)
{
    CHECK_WORLD(w, o);
    if (!w->w.valid_hittable(child)) return fail(RT_ERR_INVALID, "bad rotate_y");
    *o = w->w.rotate_y(child, angle);
    return RT_OK;
}
int rt_world_constant_medium(rt_world* w, int boundary, double density, int phase, int* o)
{
    CHECK_WORLD(w, o);
    if (!w->w.valid_hittable(boundary) || !w->w.valid_material(phase)) return fail(RT_ERR_INVALID, "bad medium");
    *o = w->w.constant_medium(boundary, density, phase);
    return RT_OK;
}
int rt_world_bvh(rt_world* w, const int* ids, int n, double t0, double t1, int* o)
{
    CHECK_WORLD(w, o);
    if (!ids || n <= 0) return fail(RT_ERR_INVALID, "empty bvh list");
    std::vector<int> list(ids, ids + n);
    for (int id : list)
        if (!w->w.valid_hittable(id)) return fail(RT_ERR_INVALID, "bad id in bvh list");
    *o = w->w.bvh(list, 0, n, t0, t1);
    return RT_OK;
}
int rt_world_push(rt_world* w, int id)
{
    if (!w || !w->w.valid_hittable(id)) return fail(RT_ERR_INVALID, "bad hittable id");
    w->w.push(id);
    return RT_OK;
}

int rt_world_build_scene(rt_world* w, int scene_id, const uint8_t* img, int iw, int ih)
{
    if (!w) return fail(RT_ERR_INVALID, "null world");
    int rc = rtw::build_scene(w->w, scene_id, img, iw, ih);
    if (rc) return fail(rc, "unknown scene id or missing image texture");
    return RT_OK;
}

// Same structure probe as the oracle's orc_scene_info (leaves through BVHs,
// instances and media; span-1 duplicates counted once).
static void count_leaves(const rtw::World& w, int id, int& n, double& cs)
{
    const rtw::HNode& h = w.nodes[id];
    switch (h.kind) {
    case rtw::HKind::BvhNode:
        count_leaves(w, h.left, n, cs);
        if (h.right != h.left) count_leaves(w, h.right, n, cs);
        return;
    case rtw::HKind::Translate: case rtw::HKind::RotateY: case rtw::HKind::ConstantMedium:
        count_leaves(w, h.ptr, n, cs);
        return;
    default: {
        n++;
        double cy1 = h.kind == rtw::HKind::MovingSphere ? h.c1.y : 0.0;
        double rad = (h.kind == rtw::HKind::Sphere || h.kind == rtw::HKind::MovingSphere) ? h.radius : 0.0;
        double k = (h.kind == rtw::HKind::XYRect || h.kind == rtw::HKind::XZRect || h.kind == rtw::HKind::YZRect) ? h.k : 0.0;
        double by = h.kind == rtw::HKind::Box ? h.bmax.y : 0.0;
        double c0x = (h.kind == rtw::HKind::Sphere || h.kind == rtw::HKind::MovingSphere) ? h.c0.x : 0.0;
        double c0y = (h.kind == rtw::HKind::Sphere || h.kind == rtw::HKind::MovingSphere) ? h.c0.y : 0.0;
        double c0z = (h.kind == rtw::HKind::Sphere || h.kind == rtw::HKind::MovingSphere) ? h.c0.z : 0.0;
        cs += c0x + 2.0 * c0y + 3.0 * c0z + rad + k + by + cy1;
        return;
    }
    }
}

int rt_world_info_get(const rt_world* w, rt_world_info* out)
{
    if (!w || !out) return fail(RT_ERR_INVALID, "null argument");
    int n = 0;
    double cs = 0.0;
    for (int id : w->w.hittables) count_leaves(w->w, id, n, cs);
    for (const rtw::Material& m : w->w.materials) {
        double tex_c0y = m.tex >= 0 ? w->w.textures[m.tex].c0.y : 0.0;
        double albedo_x = m.kind == RT_MAT_METAL ? m.albedo.x : 0.0;
        cs += 0.5 * (albedo_x + tex_c0y + m.fuzz + m.ir);
    }
    out->n_hittables = (int32_t)w->w.hittables.size();
    out->n_materials = (int32_t)w->w.materials.size();
    out->n_leaf_prims = n;
    out->n_media = w->w.n_media;
    out->checksum = cs;
    return RT_OK;
}

// ---- camera -----------------------------------------------------------------------
int rt_camera_new(const double look_from[3], const double look_at[3], const double vup[3], double vfov,
                  double aspect, double aperture, double focus_dist, double t0, double t1, rt_camera* out)
{
    if (!look_from || !look_at || !vup || !out) return fail(RT_ERR_INVALID, "null argument");
    *out = rtw::camera_new(vec(look_from), vec(look_at), vec(vup), vfov, aspect, aperture, focus_dist, t0, t1);
    return RT_OK;
}

int rt_scene_preset_get(int scene_id, rt_scene_preset* out)
{
    if (!out) return fail(RT_ERR_INVALID, "null out");
    rtw::Preset p;
    if (!rtw::scene_preset(scene_id, p)) return fail(RT_ERR_INVALID, "unknown scene id");
    auto put = [](double* d, rtw::V3 a) { d[0] = a.x; d[1] = a.y; d[2] = a.z; };
    put(out->look_from, p.look_from);
    put(out->look_at, p.look_at);
    put(out->background, p.background);
    out->vfov = p.vfov;
    out->aperture = 0.1;     // main.rs:469
    out->focus_dist = 10.0;  // main.rs:312
    out->time0 = 0.0;
    out->time1 = 1.0;
    out->default_width = p.width;
    out->default_spp = p.spp;
    out->default_aspect = p.aspect;
    return RT_OK;
}

int rt_scene_camera(int scene_id, int width, int height, rt_camera* cam, double bg[3])
{
    if (!cam || width < 1 || height < 1) return fail(RT_ERR_INVALID, "bad argument");
    rtw::Preset p;
    if (!rtw::scene_preset(scene_id, p)) return fail(RT_ERR_INVALID, "unknown scene id");
    *cam = rtw::camera_new(p.look_from, p.look_at, rtw::v3(0.0, 1.0, 0.0), p.vfov, (double)width / (double)height,
                           0.1, 10.0, 0.0, 1.0);
    if (bg) {
        bg[0] = p.background.x;
        bg[1] = p.background.y;
        bg[2] = p.background.z;
    }
    return RT_OK;
}

// ---- lowering + upload ---------------------------------------------------------------
int rt_world_set_build_option(rt_world* w, int key, double v)
{
    if (!w) return fail(RT_ERR_INVALID, "null world");
    if (!std::isfinite(v)) return fail(RT_ERR_INVALID, "build option value not finite");
    rtw::BuildOptions& b = w->w.build;
    const int iv = v < 0 ? -1 : (int)std::min(v, 1e6);
    switch (key) {
    case RT_BUILD_C_ISECT: b.c_isect = v > 0 ? v : 0.0; return RT_OK;
    case RT_BUILD_MAX_LEAF: b.max_leaf = std::max(iv, 0); return RT_OK;
    case RT_BUILD_FORCE_LEAF: b.force_leaf = std::max(iv, 0); return RT_OK;
    case RT_BUILD_ROOT_LEAF: b.root_leaf = iv; return RT_OK;
    case RT_BUILD_SPLIT_BOX_PAIRS: b.split_box_pairs = iv; return RT_OK;
    case RT_BUILD_SPLIT_BLAS_PAIRS: b.split_blas_pairs = iv; return RT_OK;
    default: return fail(RT_ERR_INVALID, "unknown build option");
    }
}

int rt_world_flatten(rt_world* w, int accel, const rt_scene_soa** soa_out)
{
    if (!w || !soa_out) return fail(RT_ERR_INVALID, "null argument");
    std::string err;
    int rc = rtw::flatten(w->w, accel, err);
    if (rc) return fail(rc, err);
    *soa_out = &w->w.flat.soa;
    return RT_OK;
}

// Stack entries a walk from `ref` needs, the way the kernel's visit uses its stack (push
// the farther child when both are hit; with two identical child boxes child 0 is always
// taken first, so only it stacks above the pushed child 1) — the rule flatten.cpp's
// stack_need builds with, recomputed here from the tables alone. Iterative post-order
// with three colours, so a cycle in a foreign node graph is found instead of walked
// forever (the persistent kernel would spin on it). Returns -1 on a cycle.
static int walk_need(const rt_scene_soa* s, int ref, std::vector<int>& need, std::vector<uint8_t>& colour)
{
    if (ref < 0) return 0;
    std::vector<int> todo{ref};
    while (!todo.empty()) {
        const int i = todo.back();
        if (colour[i] == 2) {
            todo.pop_back();
            continue;
        }
        const rt_bvh_node& nd = s->nodes[i];
        if (colour[i] == 0) {
            colour[i] = 1;  // on the current path
            for (int ch : nd.child) {
                if (ch < 0 || colour[ch] == 2) continue;
                if (colour[ch] == 1) return -1;  // back edge
                todo.push_back(ch);
            }
            continue;
        }
        todo.pop_back();  // both children done
        auto nc = [&](int ch) { return ch < 0 ? 0 : need[ch]; };
        const bool same = std::memcmp(nd.lo0, nd.lo1, 12) == 0 && std::memcmp(nd.hi0, nd.hi1, 12) == 0;
        need[i] = same ? std::max(1 + nc(nd.child[0]), nc(nd.child[1])) : 1 + std::max(nc(nd.child[0]), nc(nd.child[1]));
        colour[i] = 2;
    }
    return need[ref];
}

// SceneDev.pre_leaf: a root child that is a leaf of <= 2 primitives whose box holds at least
// 8x the volume of its sibling's (a ground or fog sphere around the whole scene) is tested
// before the walk, which then starts at the sibling (in the kernel variants that do this). The closest hit does not depend on the
// order of the tests, so the image does not change (tests/test_gpu_parity.py); only SAH
// tables (the LINEAR / MEDIAN modes keep the reference's structures as they are).
static void hoist_root_leaf(const rt_scene_soa* s, rtk::SceneDev& S)
{
    if (s->accel != RT_ACCEL_SAH || s->tlas_root < 0 || s->tlas_root >= s->n_nodes) return;
    const rt_bvh_node& root = s->nodes[s->tlas_root];
    auto volume = [](const float* lo, const float* hi) {
        double v = 1.0;
        for (int a = 0; a < 3; ++a) v *= std::max(0.0, (double)hi[a] - (double)lo[a]);
        return v;
    };
    for (int c = 0; c < 2; ++c) {
        const int leaf = root.child[c], other = root.child[1 - c];
        if (leaf >= 0 || (~leaf & 31) > 2) continue;
        const float* lo = c ? root.lo1 : root.lo0;
        const float* hi = c ? root.hi1 : root.hi0;
        const double v = volume(lo, hi), vo = volume(c ? root.lo0 : root.lo1, c ? root.hi0 : root.hi1);
        if (!(v >= 8.0 * vo) || !std::isfinite(v)) continue;
        S.pre_leaf = leaf;
        for (int a = 0; a < 3; ++a) {
            S.pre_lo[a] = lo[a];
            S.pre_hi[a] = hi[a];
        }
        S.pre_root = other;
        return;
    }
}

// Validates a (possibly foreign) SoA so the kernel never indexes out of bounds, never
// overruns its traversal stack and never walks a cycle; computes the stack needs itself
// (the tlas_depth / blas_depth fields are not trusted) and whether the TLAS really lies in
// nodes[0, n_tlas_nodes) (the kernel copies that prefix into LDS and then reads only LDS).
static int validate_soa(const rt_scene_soa* s, int& tlas_depth, int& blas_depth, int& n_tlas_nodes)
{
    if (s->n_prim_refs >= (1 << 26) - 64) return fail(RT_ERR_UNSUPPORTED, "too many primitive references");
    if (s->n_prims < 0 || s->n_prim_refs < 0 || s->n_nodes < 0 || s->n_instances < 0 || s->n_materials < 0 ||
        s->n_textures < 0 || s->n_perlin < 0 || s->image_bytes < 0)
        return fail(RT_ERR_INVALID, "negative table size");
    if ((s->n_prims && !s->prims) || (s->n_prim_refs && !s->prim_refs) || (s->n_nodes && !s->nodes) ||
        (s->n_instances && !s->instances) || (s->n_materials && !s->materials) || (s->n_textures && !s->textures) ||
        (s->n_perlin && (!s->perlin_ranvec || !s->perlin_perm)) || (s->image_bytes && !s->image_data))
        return fail(RT_ERR_INVALID, "null table");
    auto simple_kind = [](int k) { return k >= RT_PRIM_SPHERE && k <= RT_PRIM_BOX; };
    for (int i = 0; i < s->n_prims; ++i) {
        const rt_prim& p = s->prims[i];
        if (p.kind < RT_PRIM_SPHERE || p.kind > RT_PRIM_MEDIUM) return fail(RT_ERR_INVALID, "bad prim kind");
        if (p.kind == RT_PRIM_INSTANCE && (p.a < 0 || p.a >= s->n_instances)) return fail(RT_ERR_INVALID, "bad instance");
        if (p.kind == RT_PRIM_MEDIUM) {
            if (p.a < 0 || p.a >= s->n_prims) return fail(RT_ERR_INVALID, "bad boundary");
            const int bk = s->prims[p.a].kind;  // boundary_t: a simple prim or an instance
            if (!simple_kind(bk) && bk != RT_PRIM_INSTANCE) return fail(RT_ERR_UNSUPPORTED, "medium boundary kind");
        }
        if (p.kind != RT_PRIM_INSTANCE && (p.mat < 0 || p.mat >= s->n_materials)) return fail(RT_ERR_INVALID, "bad material");
    }
    for (int i = 0; i < s->n_materials; ++i) {
        const rt_material& m = s->materials[i];
        if (m.kind < RT_MAT_LAMBERTIAN || m.kind > RT_MAT_ISOTROPIC) return fail(RT_ERR_INVALID, "bad material kind");
        bool needs_tex = m.kind == RT_MAT_LAMBERTIAN || m.kind == RT_MAT_DIFFUSE_LIGHT || m.kind == RT_MAT_ISOTROPIC;
        if (needs_tex && (m.tex < 0 || m.tex >= s->n_textures)) return fail(RT_ERR_INVALID, "bad texture ref");
    }
    for (int i = 0; i < s->n_textures; ++i) {
        const rt_texture& t = s->textures[i];
        if (t.kind < RT_TEX_SOLID || t.kind > RT_TEX_IMAGE) return fail(RT_ERR_INVALID, "bad texture kind");
        if (t.kind == RT_TEX_NOISE && (t.perlin < 0 || t.perlin >= s->n_perlin)) return fail(RT_ERR_INVALID, "bad perlin");
        if (t.kind == RT_TEX_IMAGE && t.img_w > 0 &&
            (t.img_h <= 0 || t.img_offset < 0 || t.img_bps < 3 * (int64_t)t.img_w ||
             t.img_offset + t.img_bps * (int64_t)(t.img_h - 1) + 3 * (int64_t)t.img_w > s->image_bytes))
            return fail(RT_ERR_INVALID, "image texture out of range");
    }
    for (int i = 0; i < s->n_prim_refs; ++i)
        if (s->prim_refs[i] < 0 || s->prim_refs[i] >= s->n_prims) return fail(RT_ERR_INVALID, "bad prim ref");
    auto check_ref = [&](int ref) {
        if (ref >= 0) return ref < s->n_nodes;
        int code = ~ref;
        return (code >> 5) + (code & 31) <= s->n_prim_refs;
    };
    for (int i = 0; i < s->n_nodes; ++i)
        if (!check_ref(s->nodes[i].child[0]) || !check_ref(s->nodes[i].child[1])) return fail(RT_ERR_INVALID, "bad node");
    if (!check_ref(s->tlas_root)) return fail(RT_ERR_INVALID, "bad tlas root");
    for (int i = 0; i < s->n_instances; ++i) {
        const rt_instance& in = s->instances[i];
        if (in.n_ops < 0 || in.n_ops > 4) return fail(RT_ERR_INVALID, "bad instance ops");
        if (in.child_kind != RT_CHILD_PRIM && in.child_kind != RT_CHILD_BVH) return fail(RT_ERR_INVALID, "bad instance child kind");
        if (in.child_kind == RT_CHILD_PRIM ? (in.child < 0 || in.child >= s->n_prims) : !check_ref(in.child))
            return fail(RT_ERR_INVALID, "bad instance child");
        if (in.child_kind == RT_CHILD_PRIM && !simple_kind(s->prims[in.child].kind) &&
            s->prims[in.child].kind != RT_PRIM_MEDIUM)
            return fail(RT_ERR_UNSUPPORTED, "instance child must be a primitive, a medium or a BVH");
    }
    // what the kernel's nested calls assume (flatten.cpp lowers any nesting into this shape):
    // a medium's boundary instance has no medium child (no recursion), and an instance BLAS
    // holds simple primitives only
    for (int i = 0; i < s->n_prims; ++i) {
        const rt_prim& p = s->prims[i];
        if (p.kind != RT_PRIM_MEDIUM || s->prims[p.a].kind != RT_PRIM_INSTANCE) continue;
        const rt_instance& in = s->instances[s->prims[p.a].a];
        if (in.child_kind == RT_CHILD_PRIM && s->prims[in.child].kind == RT_PRIM_MEDIUM)
            return fail(RT_ERR_UNSUPPORTED, "a medium's boundary holds a medium");
    }
    // stack needs (the kernel: TLAS walk in entries [0, tlas), a nested BLAS walk above it)
    std::vector<int> need((size_t)s->n_nodes, 0);
    std::vector<uint8_t> colour((size_t)s->n_nodes, 0);
    const int t = walk_need(s, s->tlas_root, need, colour);
    if (t < 0) return fail(RT_ERR_INVALID, "cycle in the TLAS node graph");
    tlas_depth = t + 1;  // + 1 as flatten.cpp records it
    blas_depth = 0;
    // Each node's need depends only on its subtree, and a completed walk leaves every node it
    // reached done (colour 2) with its need recorded, so the walks of instance BLASes share
    // one colour array: a BLAS shared by many instances, or a subtree of one already walked,
    // costs nothing the second time (O(nodes) in total, not O(instances x nodes)). Likewise
    // `checked` marks subtrees whose leaves were already found to hold simple primitives.
    std::vector<uint8_t> checked((size_t)s->n_nodes, 0);
    for (int i = 0; i < s->n_instances; ++i) {
        const rt_instance& in = s->instances[i];
        if (in.child_kind != RT_CHILD_BVH) continue;
        const int b = walk_need(s, in.child, need, colour);
        if (b < 0) return fail(RT_ERR_INVALID, "cycle in an instance BVH");
        blas_depth = std::max(blas_depth, b + 1);
        std::vector<int> todo{in.child};   // acyclic (checked above): every leaf slot is a simple prim
        while (!todo.empty()) {
            const int ref = todo.back();
            todo.pop_back();
            if (ref >= 0) {
                if (checked[ref]) continue;
                checked[ref] = 1;
                todo.push_back(s->nodes[ref].child[0]);
                todo.push_back(s->nodes[ref].child[1]);
                continue;
            }
            const int code = ~ref;
            for (int j = code >> 5; j < (code >> 5) + (code & 31); ++j)
                if (!simple_kind(s->prims[s->prim_refs[j]].kind))
                    return fail(RT_ERR_UNSUPPORTED, "an instance BVH holds a non-primitive");
        }
    }
    if (tlas_depth > 32 || blas_depth > 32) return fail(RT_ERR_UNSUPPORTED, "BVH too deep for the traversal stack");
    // the TLAS-in-LDS claim: every node reachable from the root lies in [0, n_tlas_nodes)
    n_tlas_nodes = 0;
    if (s->n_tlas_nodes > 0 && s->n_tlas_nodes <= s->n_nodes && s->tlas_root == 0) {
        bool inside = true;
        std::vector<int> todo{0};
        std::fill(colour.begin(), colour.end(), 0);
        while (!todo.empty() && inside) {
            const int i = todo.back();
            todo.pop_back();
            if (i >= s->n_tlas_nodes) inside = false;
            if (!inside || colour[i]) continue;
            colour[i] = 1;
            for (int ch : s->nodes[i].child)
                if (ch >= 0) todo.push_back(ch);
        }
        if (inside) n_tlas_nodes = s->n_tlas_nodes;
    }
    return RT_OK;
}

int rt_scene_validate(const rt_scene_soa* s, int32_t* tlas_depth, int32_t* blas_depth)
{
    if (!s) return fail(RT_ERR_INVALID, "null argument");
    int t = 0, b = 0, n = 0;
    int rc = validate_soa(s, t, b, n);
    if (rc) return rc;
    if (tlas_depth) *tlas_depth = t;
    if (blas_depth) *blas_depth = b;
    return RT_OK;
}

int rt_ctx_upload_soa(rt_ctx* c, const rt_scene_soa* s)
{
    if (!c || !s) return fail(RT_ERR_INVALID, "null argument");
    int tlas_depth = 0, blas_depth = 0, n_tlas_nodes = 0;
    int vrc = validate_soa(s, tlas_depth, blas_depth, n_tlas_nodes);
    if (vrc) return vrc;

    // The device's primitive records. A Sphere is stored as a MovingSphere that does not
    // move (velocity 0, a = 1: the centre c0 + 0 * time is c0 bit for bit), so the kernel's
    // sphere test reads no kind and selects nothing (sphere_center). Then the records in
    // leaf-slot order (prims[prim_refs[j]]): the leaf loops read a record without first
    // loading its index.
    // A MovingSphere's a says whether its shutter is [0, 1] ((time - 0) / (1 - 0) is time
    // exactly); it is recomputed here rather than trusted from a foreign SoA. Only a scene
    // with another shutter needs FEAT_SHUTTER (the per-primitive flag and the division);
    // without it a sphere test issues all its loads at once.
    std::vector<rt_prim> prims(s->prims, s->prims + s->n_prims);
    bool general_shutter = false;
    for (rt_prim& p : prims) {
        if (p.kind == RT_PRIM_SPHERE) {
            p.a = 1;
            p.p[5] = p.p[6] = p.p[7] = 0.0;
            p.p[8] = 0.0;
            p.p[9] = 1.0;
        } else if (p.kind == RT_PRIM_MOVING_SPHERE) {
            p.a = (p.p[8] == 0.0 && p.p[9] == 1.0) ? 1 : 0;
            if (!p.a) general_shutter = true;
        } else if (p.kind == RT_PRIM_INSTANCE) {
            // b = 1: the instance's child is a BVH (the kernel defers the first such walk of a
            // cast, RT_DEFER_INST); a single child primitive is tested where the walk meets it
            p.b = s->instances[p.a].child_kind == RT_CHILD_BVH ? 1 : 0;
        }
    }
    std::vector<rt_prim> leaf_prims((size_t)s->n_prim_refs);
    for (int j = 0; j < s->n_prim_refs; ++j) leaf_prims[(size_t)j] = prims[(size_t)s->prim_refs[j]];
    // Device copies of the nodes and instances in which every instance BLAS's leaf codes count
    // slots from that BLAS's first leaf slot (kept in the device rt_instance.pad): the codes of
    // both walks then stay small enough for 16-bit stack entries (Stack16: the final scene's
    // 1000-sphere BLAS has slots 410..1409, relative 0..999). Only when every BLAS is disjoint
    // from the TLAS and from the other BLASes (or shares a BLAS with its base); otherwise the
    // codes stay absolute and the scene takes the 32-bit stack (stack16_ok 0).
    std::vector<rt_bvh_node> nodes_dev(s->nodes, s->nodes + s->n_nodes);
    std::vector<rt_instance> inst_dev(s->instances, s->instances + s->n_instances);
    for (rt_instance& in : inst_dev) in.pad = 0;
    int max_code = 0;             // the largest leaf code ((first slot << 5) | count) either walk pushes
    bool rel_ok = true;
    {
        auto leaf_first = [](int ref) { return (~ref) >> 5; };
        std::vector<int> owner((size_t)s->n_nodes, -1);   // -2: TLAS; else the BLAS base
        std::vector<int> todo;
        if (s->tlas_root >= 0) todo.push_back(s->tlas_root);
        else max_code = std::max(max_code, ~s->tlas_root);
        while (!todo.empty()) {   // validate_soa checked refs and acyclicity
            const int i = todo.back();
            todo.pop_back();
            if (owner[(size_t)i] == -2) continue;
            owner[(size_t)i] = -2;
            for (int ch : s->nodes[i].child) {
                if (ch >= 0) todo.push_back(ch);
                else max_code = std::max(max_code, ~ch);
            }
        }
        // each BLAS root is walked once however many instances share it (memo: root -> base),
        // over one epoch-stamped visited array
        std::unordered_map<int, int> root_base;
        std::vector<uint32_t> seen((size_t)s->n_nodes, 0);
        uint32_t epoch = 0;
        for (size_t ii = 0; ii < inst_dev.size() && rel_ok; ++ii) {
            rt_instance& in = inst_dev[ii];
            if (in.child_kind != RT_CHILD_BVH) continue;
            if (in.child >= 0) {
                const auto m = root_base.find(in.child);
                if (m != root_base.end()) {
                    in.pad = m->second;
                    continue;
                }
            }
            std::vector<int> blas;   // the BLAS's nodes, and its smallest leaf slot
            int base = 1 << 30;
            const int root = in.child;
            if (in.child < 0) base = leaf_first(in.child);
            else todo.push_back(in.child);
            ++epoch;
            while (!todo.empty()) {
                const int i = todo.back();
                todo.pop_back();
                if (seen[(size_t)i] == epoch) continue;
                seen[(size_t)i] = epoch;
                blas.push_back(i);
                for (int ch : s->nodes[i].child) {
                    if (ch >= 0) todo.push_back(ch);
                    else base = std::min(base, leaf_first(ch));
                }
            }
            for (int i : blas)
                if (owner[(size_t)i] == -2 || (owner[(size_t)i] >= 0 && owner[(size_t)i] != base)) rel_ok = false;
            if (!rel_ok) break;
            auto rel = [&](int ref) {
                const int code = ~ref;
                const int first = (code >> 5) - base;
                const int rcode = (first << 5) | (code & 31);
                max_code = std::max(max_code, rcode);
                return ~rcode;
            };
            for (int i : blas) {
                if (owner[(size_t)i] == base) continue;   // shared with an instance already rewritten
                owner[(size_t)i] = base;
                for (int& ch : nodes_dev[(size_t)i].child)
                    if (ch < 0) ch = rel(ch);
            }
            if (in.child < 0) in.child = rel(in.child);
            else root_base.emplace(root, base);
            in.pad = base;
        }
        if (!rel_ok) {   // absolute codes everywhere
            nodes_dev.assign(s->nodes, s->nodes + s->n_nodes);
            inst_dev.assign(s->instances, s->instances + s->n_instances);
            for (rt_instance& in : inst_dev) in.pad = 0;
            max_code = (s->n_prim_refs << 5) | 31;
        }
    }
    // The largest instance BLAS in BFS order right after the TLAS prefix (device node order
    // only): a launch stages its top levels in LDS (SceneDev.n_lds_blas), where the nested
    // walk reads them instead of waiting on L2 for every level. Needs the TLAS prefix and a
    // BLAS disjoint from it (validate_soa's n_tlas_nodes); otherwise nothing is staged.
    int n_blas_bfs = 0;
    {
        int best_root = -1;
        size_t best_n = 0;
        std::vector<int> bfs;
        std::unordered_set<int> walked;   // each BLAS root once, over one epoch-stamped array
        std::vector<uint32_t> seen((size_t)s->n_nodes, 0);
        uint32_t epoch = 0;
        for (const rt_instance& in : inst_dev) {
            if (in.child_kind != RT_CHILD_BVH || in.child < n_tlas_nodes) continue;
            if (!walked.insert(in.child).second) continue;
            std::vector<int> order{in.child};
            ++epoch;
            seen[(size_t)in.child] = epoch;
            bool disjoint = true;
            for (size_t i = 0; i < order.size(); ++i)
                for (int ch : nodes_dev[(size_t)order[i]].child)
                    if (ch >= 0 && seen[(size_t)ch] != epoch) {
                        seen[(size_t)ch] = epoch;
                        if (ch < n_tlas_nodes) disjoint = false;
                        order.push_back(ch);
                    }
            if (disjoint && order.size() > best_n) {
                best_n = order.size();
                best_root = in.child;
                bfs.swap(order);
            }
        }
        if (best_root >= 0 && (n_tlas_nodes > 0 || s->tlas_root < 0)) {
            std::vector<int> perm((size_t)s->n_nodes, -1);
            for (int i = 0; i < n_tlas_nodes; ++i) perm[(size_t)i] = i;
            int next = n_tlas_nodes;
            for (int b : bfs) perm[(size_t)b] = next++;
            for (int i = 0; i < s->n_nodes; ++i)
                if (perm[(size_t)i] < 0) perm[(size_t)i] = next++;
            std::vector<rt_bvh_node> moved((size_t)s->n_nodes);
            for (int i = 0; i < s->n_nodes; ++i) {
                rt_bvh_node nd = nodes_dev[(size_t)i];
                for (int& ch : nd.child)
                    if (ch >= 0) ch = perm[(size_t)ch];
                moved[(size_t)perm[(size_t)i]] = nd;
            }
            nodes_dev.swap(moved);
            for (rt_instance& in : inst_dev)
                if (in.child_kind == RT_CHILD_BVH && in.child >= 0) in.child = perm[(size_t)in.child];
            n_blas_bfs = (int)bfs.size();
        }
    }
    size_t off[10], bytes[10] = {
        (size_t)s->n_nodes * sizeof(rt_bvh_node), (size_t)s->n_prim_refs * 4, (size_t)s->n_prims * sizeof(rt_prim),
        (size_t)s->n_instances * sizeof(rt_instance), (size_t)s->n_materials * sizeof(rt_material),
        (size_t)s->n_textures * sizeof(rt_texture), (size_t)s->n_perlin * 768 * 8, (size_t)s->n_perlin * 768 * 4,
        (size_t)s->image_bytes, (size_t)s->n_prim_refs * sizeof(rt_prim)};
    const void* src[10] = {nodes_dev.data(), s->prim_refs, prims.data(), inst_dev.data(), s->materials, s->textures,
                           s->perlin_ranvec, s->perlin_perm, s->image_data, leaf_prims.data()};
    size_t total = 0;
    for (int i = 0; i < 10; ++i) {
        off[i] = total;
        total = align_up(total + bytes[i], 256);
    }
    total = std::max<size_t>(total, 256);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->any_enqueued) HIP_TRY(hipEventSynchronize(c->ev_done));  // renders still reading the scene
    if (total > c->scene_bytes) {
        (void)hipFree(c->scene_buf);
        c->scene_buf = nullptr;
        c->scene_bytes = 0;
        HIP_TRY(hipMalloc(&c->scene_buf, total));
        c->scene_bytes = total;
    }
    char* base = (char*)c->scene_buf;
    for (int i = 0; i < 10; ++i)
        if (bytes[i]) HIP_TRY(hipMemcpy(base + off[i], src[i], bytes[i], hipMemcpyHostToDevice));
    c->S.nodes = (const rt_bvh_node*)(base + off[0]);
    c->S.prim_refs = (const int32_t*)(base + off[1]);
    c->S.prims = (const rt_prim*)(base + off[2]);
    c->S.instances = (const rt_instance*)(base + off[3]);
    c->S.materials = (const rt_material*)(base + off[4]);
    c->S.textures = (const rt_texture*)(base + off[5]);
    c->S.perlin_ranvec = (const double*)(base + off[6]);
    c->S.perlin_perm = (const int32_t*)(base + off[7]);
    c->S.image = (const uint8_t*)(base + off[8]);
    c->S.leaf_prims = (const rt_prim*)(base + off[9]);
    c->S.tlas_root = s->tlas_root;
    c->S.pre_leaf = 0;
    if (c->opt_hoist) hoist_root_leaf(s, c->S);
    // Stack16 (trace_device.hpp): node records at LDS addresses < 32 KB (80 B each), BLAS node
    // indices < 32768, and leaf codes ((first slot << 5) | count, stored complemented; BLAS slots
    // relative, above) strictly above the -32768 = ~32767 sentinel: every code < 32767 (a leaf
    // at first slot 1023 holding 31 primitives would complement to the sentinel itself)
    c->S.stack16_ok = (n_tlas_nodes * (int64_t)80 <= 32767 - 80 && max_code < 32767 && s->n_nodes <= 32767) ? 1 : 0;
    c->S.n_lds_nodes = 0;
    c->S.n_blas_bfs = n_blas_bfs;
    c->S.n_lds_blas = 0;
    // traversal stack: TLAS walk, then a nested BLAS walk (instances) above it, sized from the
    // depths validate_soa measured (<= 32 each), each walk's bottom entry holding its RT_DONE
    // sentinel (traverse): the 66-entry scratch stack always fits
    c->S.blas_base = tlas_depth + 1;
    c->S.stack_entries = tlas_depth + 1 + (blas_depth > 0 ? blas_depth + 1 : 0);
    // A BLAS walk nests in the top-level walk only for a cast's second instance over a BVH (the
    // first is deferred until the top-level walk ends, then walks from entry 0: RT_DEFER_INST),
    // an instance over a medium, or a medium whose boundary is an instance. A scene whose top
    // level holds one instance over a BVH and none of the others (the final scene) needs the
    // larger of the two walks, not their sum: 13 entries instead of 25 per lane, 12 KB less LDS
    // per block.
    if (RT_DEFER_INST && blas_depth > 0) {
        int n_inst = 0;
        bool inst_boundary = false;
        std::vector<int> todo{s->tlas_root};
        while (!todo.empty()) {
            const int ref = todo.back();
            todo.pop_back();
            if (ref >= 0) {   // acyclic and in range (validate_soa)
                todo.push_back(s->nodes[ref].child[0]);
                todo.push_back(s->nodes[ref].child[1]);
                continue;
            }
            const int code = ~ref;
            for (int j = code >> 5; j < (code >> 5) + (code & 31); ++j) {
                const rt_prim& p = s->prims[s->prim_refs[j]];
                if (p.kind == RT_PRIM_INSTANCE) {   // an instance that may walk a BLAS
                    const rt_instance& in = s->instances[p.a];
                    if (in.child_kind == RT_CHILD_BVH) ++n_inst;
                    else if (s->prims[in.child].kind == RT_PRIM_MEDIUM) inst_boundary = true;   // never deferred
                }
                if (p.kind == RT_PRIM_MEDIUM && s->prims[p.a].kind == RT_PRIM_INSTANCE) inst_boundary = true;
            }
        }
        if (n_inst <= 1 && !inst_boundary) c->S.stack_entries = std::max(tlas_depth + 1, blas_depth + 1);
    }
    c->n_tlas_nodes = n_tlas_nodes;
    c->n_nodes = s->n_nodes;
    c->n_materials = s->n_materials;
    c->n_textures = s->n_textures;
    c->S.n_tlas_nodes = c->n_tlas_nodes;
    c->has_scene = true;
    uint32_t feat = 0;
    for (int i = 0; i < s->n_prims; ++i) {
        const int k = s->prims[i].kind;
        if (k == RT_PRIM_XY_RECT || k == RT_PRIM_XZ_RECT || k == RT_PRIM_YZ_RECT || k == RT_PRIM_BOX) feat |= rtk::FEAT_RECT;
        if (k == RT_PRIM_INSTANCE) feat |= rtk::FEAT_INST;
        if (k == RT_PRIM_MEDIUM) feat |= rtk::FEAT_MEDIUM;
    }
    // what instances and medium boundaries reach (the kernel variant drops the rest there):
    // rects / boxes under an instance, and medium boundaries other than spheres
    auto is_rect = [](int k) {
        return k == RT_PRIM_XY_RECT || k == RT_PRIM_XZ_RECT || k == RT_PRIM_YZ_RECT || k == RT_PRIM_BOX;
    };
    for (int i = 0; i < s->n_instances; ++i) {
        const rt_instance& in = s->instances[i];
        if (in.child_kind == RT_CHILD_PRIM) {
            const int ck = s->prims[in.child].kind;
            if (is_rect(ck)) feat |= rtk::FEAT_INST_RECT;
            if (ck == RT_PRIM_MEDIUM) {
                feat |= rtk::FEAT_INST_MEDIUM | rtk::FEAT_MEDIUM;
                const int bk = s->prims[s->prims[in.child].a].kind;   // its boundary, tested in object space
                if (bk != RT_PRIM_SPHERE && bk != RT_PRIM_MOVING_SPHERE) feat |= rtk::FEAT_MEDIUM_INST;
            }
            continue;
        }
        feat |= rtk::FEAT_INST_BLAS;
        std::vector<int> todo{in.child};   // validate_soa checked refs and acyclicity
        while (!todo.empty() && !(feat & rtk::FEAT_INST_RECT)) {
            const int ref = todo.back();
            todo.pop_back();
            if (ref >= 0) {
                todo.push_back(s->nodes[ref].child[0]);
                todo.push_back(s->nodes[ref].child[1]);
                continue;
            }
            const int code = ~ref, first = code >> 5, count = code & 31;
            for (int j = first; j < first + count; ++j)
                if (is_rect(s->prims[s->prim_refs[j]].kind)) feat |= rtk::FEAT_INST_RECT;
        }
    }
    for (int i = 0; i < s->n_prims; ++i)
        if (s->prims[i].kind == RT_PRIM_MEDIUM) {
            const int bk = s->prims[s->prims[i].a].kind;
            if (bk != RT_PRIM_SPHERE && bk != RT_PRIM_MOVING_SPHERE) feat |= rtk::FEAT_MEDIUM_INST;
        }
    for (int i = 0; i < s->n_textures; ++i) {
        if (s->textures[i].kind == RT_TEX_NOISE) feat |= rtk::FEAT_NOISE;
        if (s->textures[i].kind == RT_TEX_IMAGE) feat |= rtk::FEAT_IMAGE;
    }
    // FEAT_IMAGE_UV: an image-textured primitive whose hit record must carry its uv inputs (a rect
    // or box, or anything under an instance); otherwise uv comes from a top-level sphere's normal
    if (feat & rtk::FEAT_IMAGE) {
        auto imaged = [&](const rt_prim& p) {
            if (p.kind == RT_PRIM_INSTANCE || p.kind == RT_PRIM_MEDIUM) return false;
            const int m = p.mat;
            return m >= 0 && m < s->n_materials && s->materials[m].kind != RT_MAT_METAL &&
                   s->materials[m].kind != RT_MAT_DIELECTRIC && s->materials[m].tex >= 0 &&
                   s->materials[m].tex < s->n_textures && s->textures[s->materials[m].tex].kind == RT_TEX_IMAGE;
        };
        std::vector<uint8_t> under((size_t)s->n_prims, 0);   // reached through an instance
        for (int i = 0; i < s->n_instances; ++i) {
            const rt_instance& in = s->instances[i];
            if (in.child_kind == RT_CHILD_PRIM) {
                under[(size_t)in.child] = 1;
                continue;
            }
            std::vector<int> todo{in.child};
            while (!todo.empty()) {
                const int ref = todo.back();
                todo.pop_back();
                if (ref >= 0) {
                    todo.push_back(s->nodes[ref].child[0]);
                    todo.push_back(s->nodes[ref].child[1]);
                    continue;
                }
                const int code = ~ref;
                for (int j = code >> 5; j < (code >> 5) + (code & 31); ++j) under[(size_t)s->prim_refs[j]] = 1;
            }
        }
        for (int i = 0; i < s->n_prims; ++i) {
            const rt_prim& p = s->prims[i];
            if (imaged(p) && (under[(size_t)i] || (p.kind != RT_PRIM_SPHERE && p.kind != RT_PRIM_MOVING_SPHERE)))
                feat |= rtk::FEAT_IMAGE_UV;
        }
    }
    if (general_shutter) feat |= rtk::FEAT_SHUTTER;
    // FEAT_NEST_MOVING: a sphere that really moves (nonzero velocity, or a shutter other than
    // [0, 1], whose centre may not be c0) under an instance or inside a medium boundary; without
    // it the kernel tests spheres there as static (FEAT_STATIC: c0, no velocity loads)
    {
        auto moving = [&](int i) {
            const rt_prim& q = prims[(size_t)i];
            return q.kind == RT_PRIM_MOVING_SPHERE && (!q.a || q.p[5] != 0.0 || q.p[6] != 0.0 || q.p[7] != 0.0);
        };
        std::vector<uint8_t> seen((size_t)s->n_nodes, 0);
        auto bvh_moving = [&](int root) {   // validate_soa checked refs and acyclicity
            std::vector<int> todo{root};
            while (!todo.empty()) {
                const int ref = todo.back();
                todo.pop_back();
                if (ref >= 0) {
                    if (seen[(size_t)ref]) continue;
                    seen[(size_t)ref] = 1;
                    todo.push_back(s->nodes[ref].child[0]);
                    todo.push_back(s->nodes[ref].child[1]);
                    continue;
                }
                const int code = ~ref;
                for (int j = code >> 5; j < (code >> 5) + (code & 31); ++j)
                    if (moving(s->prim_refs[j])) return true;
            }
            return false;
        };
        // an instance's child prim (a medium: its boundary, which holds no medium) or BLAS
        std::function<bool(int)> inst_moving = [&](int ii) {
            const rt_instance& in = s->instances[ii];
            if (in.child_kind == RT_CHILD_BVH) return bvh_moving(in.child);
            const rt_prim& cp = s->prims[in.child];
            if (cp.kind == RT_PRIM_MEDIUM) {
                const rt_prim& b = s->prims[cp.a];
                return b.kind == RT_PRIM_INSTANCE ? inst_moving(b.a) : moving(cp.a);
            }
            return moving(in.child);
        };
        bool nest = false;
        for (int i = 0; i < s->n_instances && !nest; ++i) nest = inst_moving(i);
        for (int i = 0; i < s->n_prims && !nest; ++i) {
            if (s->prims[i].kind != RT_PRIM_MEDIUM) continue;
            const int b = s->prims[i].a;
            nest = s->prims[b].kind == RT_PRIM_INSTANCE ? inst_moving(s->prims[b].a) : moving(b);
        }
        if (nest) feat |= rtk::FEAT_NEST_MOVING;
    }
    c->features = feat;
    c->S.has_lights = 0;   // any DiffuseLight: without one, a hit never emits (shade_begin skips its material read)
    for (int i = 0; i < s->n_materials; ++i)
        if (s->materials[i].kind == RT_MAT_DIFFUSE_LIGHT) c->S.has_lights = 1;
    c->S.has_spheres = 0;
    for (int i = 0; i < s->n_prims; ++i)
        if (s->prims[i].kind == RT_PRIM_SPHERE || s->prims[i].kind == RT_PRIM_MOVING_SPHERE) c->S.has_spheres = 1;
    c->pad_extent = s->pad_extent > 0.0 && std::isfinite(s->pad_extent) ? s->pad_extent : 0.0;
    c->stats.scene_bytes = (int64_t)total;
    return RT_OK;
}

int rt_ctx_upload_world(rt_ctx* c, rt_world* w, int accel)
{
    const rt_scene_soa* soa = nullptr;
    int rc = rt_world_flatten(w, accel, &soa);
    if (rc) return rc;
    return rt_ctx_upload_soa(c, soa);
}

// ---- render ----------------------------------------------------------------------------
int rt_rows_in_shard(int height, int row_begin, int row_stride)
{
    if (height <= 0 || row_stride <= 0 || row_begin < 0 || row_begin >= height) return 0;
    return (height - row_begin + row_stride - 1) / row_stride;
}

// ceil(spp/16), at most 16 samples per work block (measured, pool schedule: C2 16 vs 32
// 99.4 / 100.4 ms, C4 16 vs 63 1565 / 1636 ms, C3 flat); a function of spp only, so the
// summation order (and the image) does not depend on launch geometry or sharding
static int auto_chunk(int spp) { return std::min(16, std::max(1, (spp + 15) / 16)); }

int rt_rows_in_band_shard(int height, int row_begin, int row_stride, int row_block)
{
    if (row_block <= 1) return rt_rows_in_shard(height, row_begin, row_stride);
    if (height <= 0 || row_stride <= 0 || row_begin < 0 || (row_block & (row_block - 1)) || row_block > 64) return 0;
    const int bands = (height + row_block - 1) / row_block;
    const int mine = rt_rows_in_shard(bands, row_begin, row_stride);
    if (!mine) return 0;
    const int last = row_begin + (mine - 1) * row_stride;   // its last band may be cut by the image
    return (mine - 1) * row_block + std::min(row_block, height - last * row_block);
}

int rt_tiles_in_shard(int width, int height, int tile_begin, int tile_stride)
{
    if (width <= 0 || height <= 0) return 0;
    const long long tiles = (long long)((width + 7) / 8) * ((height + 7) / 8);
    if (tiles > 0x7fffffffLL) return 0;
    return rt_rows_in_shard((int)tiles, tile_begin, tile_stride);
}

static int row_block_of(const rt_render_params* p) { return p->row_block > 1 ? p->row_block : 1; }
static int shard_rows(const rt_render_params* p)
{
    return rt_rows_in_band_shard(p->height, p->row_begin, p->row_stride, row_block_of(p));
}
// The shard's output layout (the kernel's pixel grid): its rows of the image, or (tile_shard)
// its 8x8 tiles side by side in one 8-row slab
struct Layout {
    int w, rows;
};
static Layout layout_of(const rt_render_params* p)
{
    if (p->tile_shard) {
        const int n = rt_tiles_in_shard(p->width, p->height, p->row_begin, p->row_stride);
        return Layout{8 * n, n > 0 ? 8 : 0};
    }
    return Layout{p->width, shard_rows(p)};
}

static bool bad_geometry(const rt_render_params* p)
{
    const int b = row_block_of(p);
    return p->width < 2 || p->height < 2 || p->row_stride < 1 || p->row_begin < 0 || p->spp_chunk < 0 ||
           (b & (b - 1)) || b > 64 || (long long)p->width * p->height > 0xffffffffLL ||
           (p->tile_shard != 0 && (p->tile_shard != 1 || b > 1));
}

static int grow(rt_ctx* c, hipStream_t stream, double*& buf, size_t& cap, size_t need, bool* oom = nullptr)
{
    if (need <= cap) return RT_OK;
    HIP_TRY(hipStreamSynchronize(stream));
    (void)hipFree(buf);
    buf = nullptr;
    cap = 0;
    const hipError_t e = hipMalloc((void**)&buf, need);
    if (e == hipErrorOutOfMemory && oom) {   // the caller retries with a smaller batch
        (void)hipGetLastError();
        buf = nullptr;
        *oom = true;
        return RT_ERR_HIP;
    }
    HIP_TRY(e);
    cap = need;
    return RT_OK;
}

// Where a sample range's per-pixel sums go: added to acc (n_px x 3 f64), or (acc null)
// written as sum * scale to out (f32 / f64).
struct Sink {
    double* acc = nullptr;
    void* out = nullptr;
    bool f64 = true;
    double scale = 1.0;
};

// Traces samples [s_begin, s_end) of the shard in chunks of `chunk` and reduces them into
// the sink. Events: ev[0] before the first trace launch, ev[1] after the last one, ev[2]
// after the last reduction. Chunk and item schedules: chunk partials per launch, reduced in
// chunk order (or added to the sink's / a running accumulator across buffer batches).
// Per-sample pool: per-sample radiance in batches; with more than one batch (or an acc
// sink) the sums run through an accumulator plus the open chunk's sum (carried across
// batches), which keeps the additions in the one-batch order.
static int run_range(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, int s_begin, int s_end, int chunk,
                     hipStream_t stream, const Sink& sink)
{
    const Layout lay = layout_of(p);
    const int n_rows = lay.rows;
    const long long n_px = (long long)n_rows * lay.w;
    const size_t px = (size_t)std::max<long long>(n_px, 1);
    if (n_px == 0 || s_end <= s_begin) {
        // an empty shard (rt_rows_in_shard / rt_tiles_in_shard 0: a rank past the tile count)
        // or an empty sample range: nothing to trace or write; the events still bracket the
        // (empty) work so rt_last_stats resolves
        for (int i = 0; i < 3; ++i) HIP_TRY(hipEventRecord(c->ev[i], stream));
        c->stats.n_batches = 0;
        c->stats.trace_buf_bytes = 0;
        c->stats.overlapped = 0;
        c->stats.ring_bytes = 0;
        c->stats.samples = 0;
        c->stats.n_items = 0;
        c->stats.n_chunks = 0;
        c->stats.spp_chunk = chunk;
        c->pending_stats = true;
        c->pending_counts = false;
        return RT_OK;
    }

    rtk::KParams K;
    std::memset(&K, 0, sizeof K);
    K.cam = *cam;
    for (int i = 0; i < 3; ++i) K.bg[i] = p->background[i];
    K.scale_m11 = rt_uniform_incl_scale(-1.0, 1.0);
    K.scale_time = rt_uniform_incl_scale(cam->time0, cam->time1);
    K.wm1 = (double)p->width - 1.0;
    K.hm1 = (double)p->height - 1.0;
    K.inv_wm1 = 1.0 / K.wm1;
    K.inv_hm1 = 1.0 / K.hm1;
    K.seed = p->render_seed;
    K.width = lay.w;
    K.height = p->height;
    K.img_width = p->width;
    K.max_depth = p->max_depth;
    K.spp_chunk = chunk;
    K.row_begin = p->row_begin;
    K.row_stride = p->row_stride;
    K.row_block_shift = 0;
    while ((1 << K.row_block_shift) < row_block_of(p)) K.row_block_shift++;
    K.tile_shard = p->tile_shard;
    K.img_tiles_x = (p->width + 7) / 8;
    const int64_t img_tiles = (int64_t)K.img_tiles_x * ((p->height + 7) / 8);
    {   // t / img_tiles_x by multiply-high: m = floor(2^32 / d) + 1 gives floor(t * m / 2^32) =
        // floor(t / d) whenever t * (m d - 2^32) < 2^32 (the excess stays under one step of t / d)
        const uint64_t d = (uint64_t)K.img_tiles_x, m = ((uint64_t)1 << 32) / std::max<uint64_t>(d, 1) + 1;
        const uint64_t e = m * d - ((uint64_t)1 << 32);
        K.tile_div_magic = (d >= 2 && m < ((uint64_t)1 << 32) && (uint64_t)img_tiles * e < ((uint64_t)1 << 32))
                               ? (uint32_t)m : 0u;
    }
    if (p->tile_shard && c->tile_order_n > 0) {   // the context's tile order: every tile shard takes it
        if (c->tile_order_n != img_tiles)
            return fail(RT_ERR_INVALID, "the tile order has " + std::to_string(c->tile_order_n) + " tiles, the frame " +
                                            std::to_string(img_tiles));
        K.tile_order = c->tile_order;
        K.tile_major = 1;   // the order's first tiles done first and entirely (rt_abi.h rt_ctx_set_tile_order)
    }
    K.n_rows = n_rows;
    K.tiles_x = (lay.w + 7) / 8;
    K.tiles_y = (n_rows + 7) / 8;

    const bool count = p->count_work != 0;
    // conservative f32 slab tests need every ray origin within 2M of the origin (flatten.cpp):
    // hit points are inside the scene bounds; check the camera (+ lens) here
    const double cam_mag = std::sqrt(cam->origin[0] * cam->origin[0] + cam->origin[1] * cam->origin[1] +
                                     cam->origin[2] * cam->origin[2]) + std::fabs(cam->lens_radius) *
                           (1.0 + std::sqrt(cam->u[0] * cam->u[0] + cam->u[1] * cam->u[1] + cam->u[2] * cam->u[2]) +
                            std::sqrt(cam->v[0] * cam->v[0] + cam->v[1] * cam->v[1] + cam->v[2] * cam->v[2]));
    rtk::LaunchOpts o;
    o.features = c->features | c->extra_features;
    o.slab32 = c->opt_slab32 && c->pad_extent > 0.0 && cam_mag <= 2.0 * c->pad_extent;
    o.lds_stack = c->opt_lds && c->S.stack_entries <= kMaxLdsStack;
    o.count = count;
    o.f32 = c->opt_precision == RT_PREC_F32;
    if (o.f32 && count && rtk::variant_features(o.features) != rtk::FEAT_SET_SPHERES &&
        rtk::variant_features(o.features) != rtk::FEAT_SET_FINAL)
        return fail(RT_ERR_UNSUPPORTED, "count_work in the f32 mode: the spheres and final-scene variants only");
    if (o.f32) o.slab32 = 1;   // statistical mode: f32 boxes whatever the camera
    // a scene with no BVH node (the Cornell scenes: one top-level leaf, instances over one
    // box) tests no slab: the f64-slab instantiation then, which holds no f32 ray terms
    // (rects + instances variant 125 vs 130 VGPRs: 4 vs 3 waves per SIMD)
    if (c->n_nodes == 0 && !o.f32) o.slab32 = 0;
    const long long total = s_end - s_begin;
    const size_t px_bytes = px * 3 * sizeof(double);
    // one sample's records in the per-sample buffer: whole 8x8 tiles (trace_kernel.hpp, tiled_record)
    // (the f32 mode's records are f32: SampleTiles.f32_records; trace_pool writes them so)
    const rtk::SampleTiles tiles{lay.w, n_rows, (lay.w + 7) / 8, o.f32 ? 1 : 0};
    const size_t sample_bytes = rtk::tiled_pixels(lay.w, n_rows) * 3 * (o.f32 ? sizeof(float) : sizeof(double));
    // the TLAS in LDS (read-only, shared by the block) when it fits the per-block budget
    rtk::SceneDev S = c->S;
    S.n_lds_nodes = c->opt_lds_nodes ? std::min(c->n_tlas_nodes, kMaxLdsNodes) : 0;
    // small material and texture tables in LDS too (the variants with rects or media)
    const bool stage = c->opt_lds_nodes && c->n_materials <= kMaxLdsMaterials && c->n_textures <= kMaxLdsMaterials &&
                       c->n_materials > 0;
    S.n_lds_materials = stage ? c->n_materials : 0;
    S.n_lds_textures = stage ? c->n_textures : 0;
    // the top levels of the BFS-ordered instance BLAS in LDS too (variants with nested walks),
    // as many as the LDS left over at the block count the rest of the layout allows
    S.n_lds_blas = 0;
    if (c->S.n_blas_bfs > 0 && c->opt_lds_nodes && (rtk::variant_features(o.features) & rtk::FEAT_INST_BLAS) != 0) {
        const bool oct = o.slab32 && S.n_lds_nodes == c->n_tlas_nodes && S.n_lds_nodes > 0;
        const uint32_t variant = rtk::variant_features(o.features);
        const int bt = rtk::block_threads_of(variant, o.f32 != 0);   // workgroup threads (RT_BLOCK_FINAL)
        const size_t base = (size_t)S.n_lds_nodes * (oct ? 80 : 64) +
                            (o.lds_stack ? (size_t)c->S.stack_entries * (size_t)bt * 4 : 0) +
                            (size_t)S.n_lds_materials * 64 + (size_t)S.n_lds_textures * 96;
        // the CU's 160 KB shared by `blocks` workgroups, each allocation rounded up to the LDS
        // granule (taken as 1 KB; the occupancy API does not round: a layout it rated at 3
        // blocks per CU ran 2 and took 174 instead of 133 ms, r03g_ab_c4.log), and no more
        // workgroups than the variant's registers allow (final scene 4 waves per SIMD, the
        // all-features variant 3: 16 or 12 waves per CU)
        const size_t lds_cu = c->lds_per_cu, granule = 1024;
        const size_t wave_blocks = std::max<size_t>(1, (size_t)(variant == rtk::FEAT_SET_FINAL ? 4 * RT_MIN_WAVES_FINAL : 12) /
                                                           (size_t)(bt / 64));
        const size_t blocks = std::max<size_t>(1, std::min(wave_blocks,
            lds_cu / (((std::max<size_t>(base, 1) + granule - 1) / granule) * granule)));
        const size_t budget = std::min(lds_cu / blocks, c->lds_per_block) / granule * granule;
        const size_t spare = budget > base ? budget - base : 0;
        S.n_lds_blas = (int32_t)std::min<size_t>({(size_t)c->S.n_blas_bfs, spare / 64, (size_t)kMaxLdsBlas});
    }
    // work blocks of one tile: 16-sample chunks, per-sample pool one chunk per block, item pool
    // two (C2 kernel ms, pool 1/2/4 chunks: 99.8/100.2/103.2; items 1/2/4: 106.8/104.1/105.0;
    // profiles/r02f_*, r02g_*)
    K.block_chunks = c->block_chunks > 0 ? c->block_chunks : 2;
    // Schedule and buffer batches, from the context's trace-output bound (sample_buf_cap). The
    // bound is sized from the free HBM when the context is created; if the device has less by
    // now (another context, torch or RCCL allocated since), the allocation below fails and the
    // bound is halved until it fits: more batches (or the item pool), the same image.
    // per-sample pool blocks: the chunk's 16 samples per tile while that leaves >= 160 k blocks
    // (~40 per resident wave), else halved down to 4: a small shard's last blocks would
    // otherwise leave waves idle (C2 rows of 1 of 8 GPUs: 16 / 8 / 4 samples 14.06 / 13.70 /
    // 13.57 ms; the whole frame 99.9 / 100.0 / 101.4; scripts/shard_coherence.py, r02p)
    if (c->block_samples > 0) {
        K.block_samples = c->block_samples;
    } else {
        const long long tiles = (long long)K.tiles_x * K.tiles_y;
        int bs = chunk;
        while (bs > 4 && tiles * ((total + bs - 1) / bs) < 160000) bs = (bs + 1) / 2;
        K.block_samples = bs;
    }
    // the pool's in-kernel reduction needs blocks of exactly one chunk (a block's sum is the
    // chunk's) and batches on chunk boundaries; its ring: kPoolRing blocks for each wave of the
    // persistent grid (at most 24 per CU: the spheres variant's 6 per SIMD, f64 and f32; the
    // launch clamps its grid to ring_waves)
    bool ring_ok = c->opt_ring && K.block_samples == chunk && chunk <= (int)(rtk::kRingSlot / 64) &&
                   s_end <= (int)rtk::kRingSampleMask;
    // (the spheres variant runs 6 waves per SIMD: RT_BLOCK_SPHERES, RT_BLOCK_F32_SPHERES)
    const int ring_waves = c->n_cus * (rtk::variant_features(o.features) == rtk::FEAT_SET_SPHERES ? 24 : 20);
    const size_t ring_bytes = (size_t)ring_waves * rtk::kRingWaveDoubles * sizeof(double);
    bool ring = false;
    bool per_sample = false;
    long long batch = 0;
    int n_batches = 0;
    double* acc = sink.acc;
    double* open = nullptr;
    bool own_acc = false;
    // halved on an out-of-memory retry for this render only: the context's bound stays, so a
    // later render on it uses the memory freed since
    size_t buf_cap = c->sample_buf_cap;
    bool overlap = false;
    for (;;) {
        // AUTO: the per-sample pool when its per-sample radiance is at most 4 times the bound,
        // else the item pool, whose partials take 1/chunk of those bytes (C5's 1.6 TB: one launch).
        // Round 2, pool vs items: C2 101.6 vs 106.7 ms per frame, C4 1492 vs 1571 (r02d_*, r02e_*);
        // round 4: C2 74.75 vs 76.06, C4 1018.5 vs 1074.7; C5 in 25 overlapped pool batches of
        // 64 GB halves 10,578 ms vs the item pool 10,649 in 64 batches at a 4 GB bound (r04f_*)
        // AUTO, measured per variant (round 5, profiles/r05x_*, r05w_*, r05y_*): the Cornell box takes
        // the item pool (C3 800x800x1000: items 204.5 ms, per-sample buffer 209.9, ring 215.0); the
        // others the per-sample pool — its buffer while that fits the bound in one batch (C1: 2.03 ms,
        // ring 2.06), else the ring (C2: 74.0 vs 74.7 unbounded; C4 x256: 267.3, items 291.8) — and
        // the item pool only when neither fits
        const uint32_t variant = rtk::variant_features(o.features);
        // (the media variant, Cornell smoke 600x600x200: items 31.72 ms, per-sample buffer 30.28: pool)
        const bool cornell = variant == rtk::FEAT_SET_RECTINST;
        const bool fits_one = (size_t)total * sample_bytes <= buf_cap;
        o.pool = c->opt_pool != RT_SCHED_AUTO ? c->opt_pool
                 : cornell && !o.f32 ? RT_SCHED_ITEMS
                 : (ring_ok || (size_t)total * sample_bytes <= 4 * buf_cap ? RT_SCHED_POOL : RT_SCHED_ITEMS);
        // POOL with the in-kernel reduction: chunk partials like ITEMS (the ring takes its share of
        // the bound first, the partials at least one chunk)
        ring = o.pool == RT_SCHED_POOL && ring_ok && (c->opt_ring == 2 || !fits_one);
        // overlapped batches trace two launches at once, a ring each: a render that does not fit
        // one batch beside one ring budgets two
        size_t out_cap = buf_cap;
        if (ring) {
            const size_t all = (size_t)((total + chunk - 1) / chunk) * px_bytes;
            const int rings = c->opt_overlap && all + ring_bytes > buf_cap ? 2 : 1;
            out_cap = std::max(buf_cap > rings * ring_bytes ? buf_cap - rings * ring_bytes : 0, px_bytes);
        }
        // Buffer batches: the trace output is bounded by sample_buf_cap. Per-sample pool: samples x
        // pixels x 24 B; chunk and item schedules: chunks x pixels x 24 B, batches on chunk
        // boundaries (relative to s_begin), so the partials add in one-launch order. A render that
        // does not fit in one batch takes two buffers of half the bound: batch k traces into half
        // k & 1 on stream tstream[k & 1] while the caller's stream reduces batch k - 1, so the
        // next trace fills the CUs its predecessor's last waves leave (no tail per batch).
        per_sample = o.pool == RT_SCHED_POOL && !ring;
        const size_t unit = per_sample ? sample_bytes : px_bytes;
        long long fit = (long long)std::max<size_t>(1, out_cap / unit);
        batch = std::min<long long>(total, per_sample ? fit : fit * chunk);
        // (only with 256-thread workgroups: a batch's launch of the large-workgroup variants —
        // the spheres variant's 768 threads, the final scene's 1024 — takes a CU only when a whole
        // workgroup of its predecessor has left, and the two persistent grids then contend instead:
        // C5 4096x4096x4096 overlapped 11,471 ms per frame, in order 10,474, profiles/r06zz_c5_*)
        const bool big_wg = rtk::block_threads_of(variant, o.f32 != 0,
                                                  o.slab32 && o.lds_stack && S.n_lds_nodes > 0 &&
                                                      S.n_lds_nodes == c->n_tlas_nodes && S.stack16_ok) > 256;
        overlap = c->opt_overlap && !big_wg && batch < total && o.pool != RT_SCHED_CHUNKS;
        if (overlap) {
            fit = (long long)std::max<size_t>(1, out_cap / 2 / unit);
            batch = std::min<long long>(total, per_sample ? fit : fit * chunk);
        }
        n_batches = (int)((total + batch - 1) / batch);
        acc = sink.acc;
        open = nullptr;
        own_acc = false;
        bool oom = false;
        int rc = RT_OK;
        if (per_sample && (n_batches > 1 || acc)) {  // acc_tmp = [open chunk sums | running total (no acc sink)]
            rc = grow(c, stream, c->acc_tmp, c->acc_tmp_cap, 2 * px_bytes);
            if (rc) return rc;
            open = c->acc_tmp;
            if (!acc) {
                acc = c->acc_tmp + px * 3;
                own_acc = true;
            }
        } else if (!per_sample && n_batches > 1 && !acc) {  // running total of the chunk partials
            rc = grow(c, stream, c->acc_tmp, c->acc_tmp_cap, px_bytes);
            if (rc) return rc;
            acc = c->acc_tmp;
            own_acc = true;
        }
        const int max_chunks = (int)((batch + chunk - 1) / chunk);
        const size_t half = per_sample ? (size_t)batch * sample_bytes : (size_t)max_chunks * px_bytes;
        const size_t need = overlap ? 2 * half : half;
        rc = grow(c, stream, c->partial, c->partial_cap, need, &oom);
        if (rc == RT_OK && ring) {
            rc = grow(c, stream, c->ring, c->ring_cap, (overlap ? 2 : 1) * ring_bytes, &oom);
            if (rc != RT_OK && oom) {   // no room for the ring: the per-sample buffer, as before
                ring_ok = false;
                continue;
            }
        }
        if (rc == RT_OK) break;
        if (!oom) return rc;
        if (buf_cap <= ((size_t)1 << 20) || need <= (per_sample ? sample_bytes : px_bytes))
            return hip_fail(hipErrorOutOfMemory, "trace output buffer (smallest batch)");
        buf_cap = std::max<size_t>(buf_cap / 2, (size_t)1 << 20);
    }
    if (own_acc) HIP_TRY(hipMemsetAsync(acc, 0, px_bytes, stream));
    K.ring_waves = ring ? ring_waves : 0;
    if (count) {
        HIP_TRY(hipMemsetAsync(c->counters, 0, kCounters * sizeof(unsigned long long), stream));
        if (img_tiles > c->tile_cost_cap) {   // (a render's first use: no work on the context's streams reads it)
            HIP_TRY(hipStreamSynchronize(stream));
            (void)hipFree(c->tile_cost);
            c->tile_cost = nullptr;
            c->tile_cost_cap = 0;
            HIP_TRY(hipMalloc((void**)&c->tile_cost, (size_t)img_tiles * sizeof(unsigned long long)));
            c->tile_cost_cap = img_tiles;
        }
        HIP_TRY(hipMemsetAsync(c->tile_cost, 0, (size_t)img_tiles * sizeof(unsigned long long), stream));
        K.tile_cost = c->tile_cost;
        // (the pool kernels count them; the chunk schedule does not)
        c->tile_cost_n = o.pool == RT_SCHED_POOL || o.pool == RT_SCHED_ITEMS ? img_tiles : 0;
    }
    int waves_per_simd = 0;
    o.waves_per_simd = &waves_per_simd;
    HIP_TRY(hipEventRecord(c->ev[0], stream));
    // overlapped batches: both trace streams start after everything enqueued on `stream` so far
    if (overlap) {
        HIP_TRY(hipEventRecord(c->ev_in, stream));
        for (int i = 0; i < 2; ++i) HIP_TRY(hipStreamWaitEvent(c->tstream[i], c->ev_in, 0));
    }
    const size_t half_elems = overlap ? (per_sample ? (size_t)batch * sample_bytes
                                                    : (size_t)((batch + chunk - 1) / chunk) * px_bytes) / sizeof(double)
                                      : 0;
    for (int bi = 0; bi < n_batches; ++bi) {
        const int b0 = s_begin + (int)(bi * batch);
        const int b1 = (int)std::min<long long>(s_end, b0 + batch);
        K.sample_begin = b0;
        K.spp = b1;
        K.n_chunks = (b1 - b0 + chunk - 1) / chunk;
        {
            const unsigned g = o.pool == RT_SCHED_ITEMS ? (unsigned)K.block_chunks : (unsigned)K.block_samples;   // (POOL: samples)
            const unsigned n = o.pool == RT_SCHED_ITEMS ? (unsigned)K.n_chunks : (unsigned)(K.spp - K.sample_begin);
            const unsigned n_groups = (n + g - 1) / std::max(g, 1u);
            K.n_work_blocks = (unsigned)K.tiles_x * (unsigned)K.tiles_y * n_groups;
            K.deal_div = K.tile_major ? n_groups : (unsigned)K.tiles_x * (unsigned)K.tiles_y;
        }
        // batch bi's buffer half, trace stream and work counter (one of each per overlapped batch)
        const int h = overlap ? (bi & 1) : 0;
        double* buf = c->partial + (size_t)h * half_elems;
        hipStream_t ts = overlap ? c->tstream[h] : stream;
        K.ring = ring ? c->ring + (size_t)h * (ring_bytes / sizeof(double)) : nullptr;   // one ring per trace stream
        if (overlap && bi >= 2) HIP_TRY(hipStreamWaitEvent(ts, c->ev_rd[h], 0));   // batch bi - 2 reduced: half free
        rtk::KParams* dK = c->params + c->param_slot;
        c->param_slot = (c->param_slot + 1) % kParamSlots;
        HIP_TRY(hipMemcpyAsync(dK, &K, sizeof K, hipMemcpyHostToDevice, ts));
        HIP_TRY(rtk::launch_trace(S, K, dK, buf, c->counters, c->work + h, o, ts));
        if (bi == n_batches - 1) HIP_TRY(hipEventRecord(c->ev[1], ts));
        if (overlap) {   // reduce in batch order on `stream`, after this batch's trace
            HIP_TRY(hipEventRecord(c->ev_tr[h], ts));
            HIP_TRY(hipStreamWaitEvent(stream, c->ev_tr[h], 0));
        }
        if (!per_sample) {
            if (acc) HIP_TRY(rtk::launch_accumulate(buf, acc, n_px, K.n_chunks, stream));
            else HIP_TRY(rtk::launch_reduce(buf, sink.out, sink.f64, n_px, K.n_chunks, sink.scale, stream));
        } else if (!open) {
            HIP_TRY(rtk::launch_reduce_samples(buf, sink.out, sink.f64, tiles, b1 - b0, chunk, sink.scale, stream));
        } else {
            HIP_TRY(rtk::launch_reduce_samples_carry(buf, acc, open, tiles, b1 - b0, chunk,
                                                     (int)(((long long)b0 - s_begin) % chunk), bi == n_batches - 1,
                                                     stream));
        }
        if (overlap) HIP_TRY(hipEventRecord(c->ev_rd[h], stream));
    }
    if (own_acc)  // resolve the running sums: 0.0 + sum, times scale, as one batch does
        HIP_TRY(rtk::launch_reduce(acc, sink.out, sink.f64, n_px, 1, sink.scale, stream));
    HIP_TRY(hipEventRecord(c->ev[2], stream));

    c->stats.lds_nodes = S.n_lds_nodes;
    c->stats.variant_features = (int32_t)rtk::variant_features(o.features);
    c->stats.slab32 = o.slab32;
    c->stats.lds_stack = o.lds_stack;
    c->stats.schedule = o.pool;
    c->stats.precision = o.f32 ? RT_PREC_F32 : RT_PREC_F64;
    c->stats.waves_per_simd = waves_per_simd;
    c->stats.n_batches = n_batches;
    c->stats.ring_bytes = ring ? (int64_t)((overlap ? 2 : 1) * ring_bytes) : 0;
    c->stats.trace_buf_bytes = (int64_t)(overlap ? 2 * half_elems * sizeof(double)
                                                 : (per_sample ? (size_t)batch * sample_bytes
                                                               : (size_t)((batch + chunk - 1) / chunk) * px_bytes)) +
                               c->stats.ring_bytes;
    c->stats.overlapped = overlap ? 1 : 0;
    c->stats.samples = (uint64_t)n_px * (uint64_t)total;
    c->stats.n_chunks = (int32_t)((total + chunk - 1) / chunk);
    c->stats.n_items = (uint64_t)n_px * (uint64_t)c->stats.n_chunks;
    c->stats.spp_chunk = chunk;
    c->stats.node_bytes = (int32_t)sizeof(rt_bvh_node);
    c->stats.prim_bytes = (int32_t)sizeof(rt_prim);
    c->stats.material_bytes = (int32_t)sizeof(rt_material);
    c->pending_stats = true;
    c->pending_counts = count;
    if (!c->stats.samples) c->stats.casts = c->stats.node_visits = c->stats.prim_tests = 0;
    return RT_OK;
}

// Orders work about to be enqueued on `stream` after everything this context enqueued on
// another stream before (the context's scratch buffers are shared between its renders).
static int begin_on(rt_ctx* c, hipStream_t stream)
{
    if (c->any_enqueued && stream != c->last_stream) HIP_TRY(hipStreamWaitEvent(stream, c->ev_done, 0));
    return RT_OK;
}
static int end_on(rt_ctx* c, hipStream_t stream)
{
    HIP_TRY(hipEventRecord(c->ev_done, stream));
    c->last_stream = stream;
    c->any_enqueued = true;
    return RT_OK;
}
// begin_on ... end_on around every call that enqueues: once begin_on has run, end_on runs on
// every way out, an early error return included — work already queued on `stream` before the
// error still reads the context's buffers, and the next call on another stream must wait
// for it (ev_done, last_stream), not for the call before
struct StreamScope {
    rt_ctx* c;
    hipStream_t stream;
    bool open = false;
    StreamScope(rt_ctx* c_, hipStream_t s_) : c(c_), stream(s_) {}
    int begin()
    {
        const int rc = begin_on(c, stream);
        open = rc == RT_OK;
        return rc;
    }
    int end()
    {
        open = false;
        return end_on(c, stream);
    }
    ~StreamScope()
    {
        if (open) (void)end_on(c, stream);
    }
};

// Device buffer for a host-bound result (grown on demand).
static int out_staging(rt_ctx* c, hipStream_t stream, size_t out_bytes, void*& dev_out)
{
    if (out_bytes > c->out_cap) {
        HIP_TRY(hipStreamSynchronize(stream));  // ordered after every earlier use (begin_on)
        (void)hipFree(c->out_buf);
        c->out_buf = nullptr;
        c->out_cap = 0;
        HIP_TRY(hipMalloc(&c->out_buf, std::max<size_t>(out_bytes, 16)));
        c->out_cap = std::max<size_t>(out_bytes, 16);
    }
    dev_out = c->out_buf;
    return RT_OK;
}

int rt_render(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, void* out)
{
    if (!c || !cam || !p || !out) return fail(RT_ERR_INVALID, "null argument");
    if (!c->has_scene) return fail(RT_ERR_NO_SCENE, "no scene uploaded");
    if (bad_geometry(p) || p->spp < 1 || p->max_depth < 0 || (p->out_format != RT_OUT_F32 && p->out_format != RT_OUT_F64))
        return fail(RT_ERR_INVALID, "bad render params");
    const Layout lay = layout_of(p);
    const int chunk = p->spp_chunk > 0 ? std::min(p->spp_chunk, p->spp) : auto_chunk(p->spp);
    const long long n_px = (long long)lay.rows * lay.w;

    HIP_TRY(hipSetDevice(c->device));
    hipStream_t stream = p->stream ? (hipStream_t)p->stream : c->stream;
    StreamScope scope(c, stream);
    int rc = scope.begin();
    if (rc) return rc;
    const size_t out_bytes = (size_t)n_px * 3 * (p->out_format == RT_OUT_F64 ? 8 : 4);
    void* dev_out = out;
    if (!p->out_on_device) {
        rc = out_staging(c, stream, out_bytes, dev_out);
        if (rc) return rc;
    }
    Sink sink;
    sink.out = dev_out;
    sink.f64 = p->out_format == RT_OUT_F64;
    sink.scale = 1.0 / (double)p->spp;
    rc = run_range(c, cam, p, 0, p->spp, chunk, stream, sink);
    if (rc) return rc;
    if (!p->out_on_device) HIP_TRY(hipMemcpyAsync(out, dev_out, out_bytes, hipMemcpyDeviceToHost, stream));
    rc = scope.end();
    if (rc) return rc;
    if (!p->out_on_device) HIP_TRY(hipStreamSynchronize(stream));
    return RT_OK;
}

// ---- progressive accumulation -----------------------------------------------------------------
struct rt_accum {
    rt_ctx* ctx = nullptr;
    int width = 0, height = 0, row_begin = 0, row_stride = 1, row_block = 1, tile_shard = 0, n_rows = 0, chunk = 1;
    long long n_px = 0;
    int64_t done = 0;
    double* sums = nullptr;             // device, n_px x 3
    hipStream_t last_stream = nullptr;  // the stream the last batch was enqueued on
};

int rt_accum_create(rt_ctx* c, const rt_render_params* p, rt_accum** out)
{
    if (!c || !p || !out) return fail(RT_ERR_INVALID, "null argument");
    *out = nullptr;
    if (bad_geometry(p) || p->spp < 0 || (p->spp_chunk == 0 && p->spp < 1))
        return fail(RT_ERR_INVALID, "bad accumulator geometry");
    auto* a = new (std::nothrow) rt_accum;
    if (!a) return fail(RT_ERR_OOM, "out of host memory");
    a->ctx = c;
    a->width = p->width;
    a->height = p->height;
    a->row_begin = p->row_begin;
    a->row_stride = p->row_stride;
    a->row_block = row_block_of(p);
    a->tile_shard = p->tile_shard;
    const Layout lay = layout_of(p);
    a->n_rows = lay.rows;
    a->chunk = p->spp_chunk > 0 ? p->spp_chunk : auto_chunk(p->spp);
    a->n_px = (long long)lay.rows * lay.w;
    a->last_stream = c->stream;
    const size_t bytes = (size_t)std::max<long long>(a->n_px, 1) * 3 * sizeof(double);
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = hipMalloc((void**)&a->sums, bytes);
    if (e == hipSuccess) e = hipMemset(a->sums, 0, bytes);
    if (e != hipSuccess) {
        (void)hipFree(a->sums);
        delete a;
        return hip_fail(e, "rt_accum_create");
    }
    *out = a;
    return RT_OK;
}

void rt_accum_destroy(rt_accum* a)
{
    if (!a) return;
    (void)hipSetDevice(a->ctx->device);
    (void)hipStreamSynchronize(a->last_stream);
    (void)hipFree(a->sums);
    delete a;
}

int rt_accum_add(rt_ctx* c, rt_accum* a, const rt_camera* cam, const rt_render_params* p, int sample_count)
{
    if (!c || !a || !cam || !p) return fail(RT_ERR_INVALID, "null argument");
    if (a->ctx != c) return fail(RT_ERR_INVALID, "accumulator belongs to another context");
    if (!c->has_scene) return fail(RT_ERR_NO_SCENE, "no scene uploaded");
    if (p->width != a->width || p->height != a->height || p->row_begin != a->row_begin ||
        p->row_stride != a->row_stride || row_block_of(p) != a->row_block || p->tile_shard != a->tile_shard)
        return fail(RT_ERR_INVALID, "render params do not match the accumulator's shard");
    if (sample_count < 0 || p->max_depth < 0 || a->done + sample_count > 0x7fffffffLL)
        return fail(RT_ERR_INVALID, "bad sample range");
    if (sample_count == 0) return RT_OK;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t stream = p->stream ? (hipStream_t)p->stream : c->stream;
    if (stream != a->last_stream) HIP_TRY(hipStreamSynchronize(a->last_stream));
    StreamScope scope(c, stream);
    int rc = scope.begin();
    if (rc) return rc;
    a->last_stream = stream;   // the sums' stream from here on, even if a launch below fails
    Sink sink;
    sink.acc = a->sums;
    rc = run_range(c, cam, p, (int)a->done, (int)(a->done + sample_count), a->chunk, stream, sink);
    if (rc) return rc;
    rc = scope.end();
    if (rc) return rc;
    a->done += sample_count;
    return RT_OK;
}

int rt_accum_get(rt_accum* a, double* sums, int64_t* samples_done)
{
    if (!a) return fail(RT_ERR_INVALID, "null argument");
    if (samples_done) *samples_done = a->done;
    if (!sums) return RT_OK;
    HIP_TRY(hipSetDevice(a->ctx->device));
    HIP_TRY(hipStreamSynchronize(a->last_stream));
    HIP_TRY(hipMemcpy(sums, a->sums, (size_t)a->n_px * 3 * sizeof(double), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_accum_set(rt_accum* a, const double* sums, int64_t samples_done)
{
    if (!a || !sums) return fail(RT_ERR_INVALID, "null argument");
    if (samples_done < 0 || samples_done > 0x7fffffffLL) return fail(RT_ERR_INVALID, "bad sample count");
    HIP_TRY(hipSetDevice(a->ctx->device));
    HIP_TRY(hipStreamSynchronize(a->last_stream));
    HIP_TRY(hipMemcpy(a->sums, sums, (size_t)a->n_px * 3 * sizeof(double), hipMemcpyHostToDevice));
    a->done = samples_done;
    return RT_OK;
}

int rt_accum_resolve(rt_ctx* c, rt_accum* a, double divisor, int out_format, int out_on_device, void* out)
{
    if (!c || !a || !out) return fail(RT_ERR_INVALID, "null argument");
    if (a->ctx != c) return fail(RT_ERR_INVALID, "accumulator belongs to another context");
    if (out_format != RT_OUT_F32 && out_format != RT_OUT_F64) return fail(RT_ERR_INVALID, "bad output format");
    if (divisor == 0.0) divisor = (double)a->done;
    if (!(divisor > 0.0) || !std::isfinite(divisor)) return fail(RT_ERR_INVALID, "nothing accumulated / bad divisor");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t stream = a->last_stream;
    StreamScope scope(c, stream);
    int rc = scope.begin();
    if (rc) return rc;
    const size_t out_bytes = (size_t)a->n_px * 3 * (out_format == RT_OUT_F64 ? 8 : 4);
    void* dev_out = out;
    if (!out_on_device) {
        rc = out_staging(c, stream, out_bytes, dev_out);
        if (rc) return rc;
    }
    // one "chunk" holding the running sums: 0.0 + sum = sum, then * (1/divisor) as rt_render
    HIP_TRY(rtk::launch_reduce(a->sums, dev_out, out_format == RT_OUT_F64, a->n_px, 1, 1.0 / divisor, stream));
    if (!out_on_device) HIP_TRY(hipMemcpyAsync(out, dev_out, out_bytes, hipMemcpyDeviceToHost, stream));
    rc = scope.end();
    if (rc) return rc;
    if (!out_on_device) HIP_TRY(hipStreamSynchronize(stream));
    return RT_OK;
}

int rt_render_progressive(rt_ctx* c, const rt_camera* cam, const rt_render_params* p, int batch_spp,
                          rt_progress_fn progress, void* user, void* out)
{
    if (!c || !cam || !p || !out) return fail(RT_ERR_INVALID, "null argument");
    if (p->spp < 1 || batch_spp < 1) return fail(RT_ERR_INVALID, "bad spp / batch");
    rt_accum* a = nullptr;
    int rc = rt_accum_create(c, p, &a);
    if (rc) return rc;
    const int batch = (batch_spp + a->chunk - 1) / a->chunk * a->chunk;  // keep chunk boundaries
    while (rc == RT_OK && a->done < p->spp) {
        const int n = (int)std::min<int64_t>(batch, p->spp - a->done);
        rc = rt_accum_add(c, a, cam, p, n);
        if (rc) break;
        if (progress) {
            hipError_t e = hipStreamSynchronize(a->last_stream);
            if (e != hipSuccess) {
                rc = hip_fail(e, "rt_render_progressive");
                break;
            }
            if (progress(user, a->done, p->spp)) break;
        }
    }
    if (rc == RT_OK)
        rc = rt_accum_resolve(c, a, a->done == p->spp ? (double)p->spp : 0.0, p->out_format, p->out_on_device, out);
    if (rc == RT_OK && p->out_on_device) {
        hipError_t e = hipStreamSynchronize(a->last_stream);  // the accumulator is freed below
        if (e != hipSuccess) rc = hip_fail(e, "rt_render_progressive");
    }
    rt_accum_destroy(a);
    return rc;
}

int rt_last_stats(rt_ctx* c, rt_stats* out)
{
    if (!c || !out) return fail(RT_ERR_INVALID, "null argument");
    if (c->pending_stats) {
        HIP_TRY(hipSetDevice(c->device));
        HIP_TRY(hipEventSynchronize(c->ev[2]));
        float a = 0, b = 0;
        HIP_TRY(hipEventElapsedTime(&a, c->ev[0], c->ev[1]));
        HIP_TRY(hipEventElapsedTime(&b, c->ev[1], c->ev[2]));
        c->stats.kernel_ms = a;
        c->stats.reduce_ms = b;
        if (c->pending_counts) {
            unsigned long long h[kCounters];
            HIP_TRY(hipMemcpy(h, c->counters, sizeof h, hipMemcpyDeviceToHost));
            c->stats.casts = h[0];
            c->stats.node_visits = h[1];
            c->stats.prim_tests = h[2];
            c->stats.cycles_camera = h[3];
            c->stats.cycles_trace = h[4];
            c->stats.cycles_shade = h[5];
            c->stats.wave_steps = h[6];
            c->stats.wave_node_steps = h[7];
            c->stats.cycles_nodes = h[8];
            c->stats.cycles_leaves = h[9];
            c->stats.wave_leaf_steps = h[10];
            c->stats.camera_lanes = h[11];
            c->stats.camera_steps = h[12];
            c->stats.shade_lanes = h[13];
            c->stats.shade_steps = h[14];
            for (int i = 0; i < kCounters; ++i) c->raw_counters[i] = h[i];
        } else {
            c->stats.casts = c->stats.node_visits = c->stats.prim_tests = 0;
            c->stats.cycles_camera = c->stats.cycles_trace = c->stats.cycles_shade = 0;
            c->stats.wave_steps = c->stats.wave_node_steps = 0;
            c->stats.cycles_nodes = c->stats.cycles_leaves = 0;
            c->stats.wave_leaf_steps = c->stats.camera_lanes = c->stats.camera_steps = 0;
            c->stats.shade_lanes = c->stats.shade_steps = 0;
            for (int i = 0; i < kCounters; ++i) c->raw_counters[i] = 0;
        }
        c->pending_stats = false;
    }
    *out = c->stats;
    return RT_OK;
}

int rt_last_tile_costs(rt_ctx* c, uint64_t* out, int64_t n)
{
    if (!c || (!out && n > 0) || n < 0) return fail(RT_ERR_INVALID, "bad argument");
    rt_stats st;
    const int rc = rt_last_stats(c, &st);   // the last render done
    if (rc) return rc;
    if (!c->pending_counts || c->tile_cost_n == 0) return 0;   // the last render counted no tile costs
    const int64_t m = std::min<int64_t>(n, c->tile_cost_n);
    if (m > 0) HIP_TRY(hipMemcpy(out, c->tile_cost, (size_t)m * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return (int)c->tile_cost_n;
}

int rt_ctx_set_tile_order(rt_ctx* c, const uint32_t* order, int64_t n)
{
    if (!c || n < 0 || (n > 0 && !order)) return fail(RT_ERR_INVALID, "bad argument");
    if (n > ((int64_t)1 << 30)) return fail(RT_ERR_INVALID, "tile order too long");
    std::vector<uint8_t> seen((size_t)n, 0);
    for (int64_t i = 0; i < n; ++i) {
        if ((int64_t)order[i] >= n || seen[order[i]]) return fail(RT_ERR_INVALID, "the tile order is not a permutation of 0..n-1");
        seen[order[i]] = 1;
    }
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());   // no render still reads the old order
    (void)hipFree(c->tile_order);
    c->tile_order = nullptr;
    c->tile_order_n = 0;
    if (n == 0) return RT_OK;
    HIP_TRY(hipMalloc((void**)&c->tile_order, (size_t)n * sizeof(uint32_t)));
    HIP_TRY(hipMemcpy(c->tile_order, order, (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice));
    c->tile_order_n = n;
    return RT_OK;
}

int rt_last_counters(rt_ctx* c, uint64_t* out, int n)
{
    if (!c || !out || n < 0) return fail(RT_ERR_INVALID, "null argument");
    rt_stats st;
    const int rc = rt_last_stats(c, &st);   // resolves a pending render's counters
    if (rc) return rc;
    for (int i = 0; i < n; ++i) out[i] = i < kCounters ? (uint64_t)c->raw_counters[i] : 0;
    return std::min(n, kCounters);
}

// ---- output ---------------------------------------------------------------------------------
// write_color (math.rs:119-131) of one f64 channel summed over spp samples: scale = 1.0/spp,
// sqrt(x * scale), clamp to [0, 0.999] (NaN passes through, math.rs:282-286), 256 * c with
// Rust's saturating `as i32` (NaN -> 0). All in f64, as the reference: with rt_render's
// RT_OUT_F64 mean (sum * (1/spp)) and spp = 1 this is write_color(spp) of the sums bit for bit.
static inline int write_color_f64(double x, double scale)
{
    const double r = std::sqrt(x * scale);
    const double c = r < 0.0 ? 0.0 : r > 0.999 ? 0.999 : r;
    return (int)rt_sat_i32(256.0 * c);
}

int rt_write_color(const double* rgb, int samples_per_pixel, int64_t n, int32_t* out)
{
    if (!rgb || !out || n < 0 || samples_per_pixel < 1) return fail(RT_ERR_INVALID, "bad argument");
    const double scale = 1.0 / (double)samples_per_pixel;
    for (int64_t i = 0; i < 3 * n; ++i) out[i] = write_color_f64(rgb[i], scale);
    return RT_OK;
}

int rt_write_ppm_f64(const double* rgb, int samples_per_pixel, int width, int height, const char* path)
{
    if (!rgb || !path || width < 1 || height < 1 || samples_per_pixel < 1) return fail(RT_ERR_INVALID, "bad argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(RT_ERR_INVALID, std::string("cannot open ") + path);
    const double scale = 1.0 / (double)samples_per_pixel;           // math.rs:120
    std::fprintf(f, "P3\n%d %d\n255\n\n", width, height);          // main.rs:472 (println! adds the blank line)
    for (int j = height - 1; j >= 0; --j)                          // main.rs:591-596: rows top to bottom
        for (int i = 0; i < width; ++i) {
            const double* px = rgb + ((size_t)j * width + i) * 3;
            std::fprintf(f, "%d %d %d\n", write_color_f64(px[0], scale), write_color_f64(px[1], scale),
                         write_color_f64(px[2], scale));
        }
    if (std::fclose(f) != 0) return fail(RT_ERR_INVALID, std::string("cannot write ") + path);
    return RT_OK;
}

// The f32 frame's writer (RT_OUT_F32 renders, the f32 mode): the mean is rounded to f32
// before the sqrt, so a channel whose 256*sqrt(mean) lies within ~1e-5 of an integer may
// differ by one from the reference's f64 write_color; rt_write_ppm_f64 is the exact one.
int rt_write_ppm(const float* mean, int width, int height, const char* path)
{
    if (!mean || !path || width < 1 || height < 1) return fail(RT_ERR_INVALID, "bad argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(RT_ERR_INVALID, std::string("cannot open ") + path);
    std::fprintf(f, "P3\n%d %d\n255\n\n", width, height);  // main.rs:472 (println! adds the blank line)
    auto to_byte = [](double x) {                           // math.rs:119-131
        double r = std::sqrt(x);
        double c = r < 0.0 ? 0.0 : r > 0.999 ? 0.999 : r;   // clamp (NaN passes through)
        return (int)rt_sat_i32(256.0 * c);                  // `as i32`: NaN -> 0
    };
    for (int j = height - 1; j >= 0; --j)                   // main.rs:591-596
        for (int i = 0; i < width; ++i) {
            const float* px = mean + ((size_t)j * width + i) * 3;
            std::fprintf(f, "%d %d %d\n", to_byte(px[0]), to_byte(px[1]), to_byte(px[2]));
        }
    std::fclose(f);
    return RT_OK;
}

// ---- self test ----------------------------------------------------------------------------------
int rt_ctx_set_variant(rt_ctx* c, int slab32, int lds_stack, int lds_nodes)
{
    if (!c || slab32 < 0 || slab32 > 1 || lds_stack < 0 || lds_stack > 1 || lds_nodes < 0 || lds_nodes > 1)
        return fail(RT_ERR_INVALID, "bad variant");
    c->opt_slab32 = slab32;
    c->opt_lds = lds_stack;
    c->opt_lds_nodes = lds_nodes;
    return RT_OK;
}

int rt_ctx_set_precision(rt_ctx* c, int precision)
{
    if (!c || (precision != RT_PREC_F64 && precision != RT_PREC_F32)) return fail(RT_ERR_INVALID, "bad precision");
    c->opt_precision = precision;
    return RT_OK;
}

int rt_ctx_set_option(rt_ctx* c, int key, int64_t v)
{
    if (!c) return fail(RT_ERR_INVALID, "null context");
    switch (key) {
    case RT_OPT_TRACE_BUF_BYTES:
        if (v < 0) return fail(RT_ERR_INVALID, "negative buffer bound");
        c->sample_buf_cap = v == 0 ? default_buf_cap() : std::max<size_t>((size_t)v, (size_t)1 << 20);
        return RT_OK;
    case RT_OPT_BATCH_OVERLAP: c->opt_overlap = v != 0; return RT_OK;
    case RT_OPT_BLOCK_SAMPLES:
        if (v < 0 || v > 1024) return fail(RT_ERR_INVALID, "block samples out of range (0..1024)");
        c->block_samples = (int)v;
        return RT_OK;
    case RT_OPT_BLOCK_CHUNKS:
        if (v < 0 || v > 64) return fail(RT_ERR_INVALID, "block chunks out of range (0..64)");
        c->block_chunks = (int)v;
        return RT_OK;
    case RT_OPT_EXTRA_FEATURES:
        if (v < 0 || (v & ~(int64_t)rtk::FEAT_ALL)) return fail(RT_ERR_INVALID, "unknown feature bits");
        c->extra_features = (uint32_t)v;
        return RT_OK;
    case RT_OPT_HOIST: c->opt_hoist = v != 0; return RT_OK;
    case RT_OPT_POOL_RING:
        if (v < 0 || v > 2) return fail(RT_ERR_INVALID, "pool ring mode out of range (0 never, 1 when needed, 2 always)");
        c->opt_ring = (int)v;
        return RT_OK;
    case RT_OPT_COMM_DIRECT: c->opt_comm_direct = v != 0; return RT_OK;
    default: return fail(RT_ERR_INVALID, "unknown option");
    }
}

int rt_ctx_get_option(rt_ctx* c, int key, int64_t* v)
{
    if (!c || !v) return fail(RT_ERR_INVALID, "null argument");
    switch (key) {
    case RT_OPT_TRACE_BUF_BYTES: *v = (int64_t)c->sample_buf_cap; return RT_OK;
    case RT_OPT_BATCH_OVERLAP: *v = c->opt_overlap; return RT_OK;
    case RT_OPT_BLOCK_SAMPLES: *v = c->block_samples; return RT_OK;
    case RT_OPT_BLOCK_CHUNKS: *v = c->block_chunks; return RT_OK;
    case RT_OPT_EXTRA_FEATURES: *v = c->extra_features; return RT_OK;
    case RT_OPT_HOIST: *v = c->opt_hoist; return RT_OK;
    case RT_OPT_POOL_RING: *v = c->opt_ring; return RT_OK;
    case RT_OPT_COMM_DIRECT: *v = c->opt_comm_direct; return RT_OK;
    default: return fail(RT_ERR_INVALID, "unknown option");
    }
}

int rt_ctx_set_schedule(rt_ctx* c, int schedule)
{
    if (c && schedule == 4)   // the wavefront schedule of ABI v4 (rejected, scripts/experiments/r05_wavefront.patch)
        return fail(RT_ERR_UNSUPPORTED, "schedule 4 (wavefront) was removed: 2.3x slower than the pool on C4 (DESIGN.md 5.7)");
    if (!c || schedule < RT_SCHED_CHUNKS || schedule > RT_SCHED_AUTO) return fail(RT_ERR_INVALID, "bad schedule");
    c->opt_pool = schedule;
    return RT_OK;
}

int rt_device_eval(rt_ctx* c, int fn, const double* x, const double* y, const double* z, double* out, int n)
{
    if (!c || !x || !out || n < 0 || fn < 0 || fn > 13) return fail(RT_ERR_INVALID, "bad argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(c->device));
    double* d = nullptr;
    const size_t b = (size_t)n * sizeof(double);
    HIP_TRY(hipMalloc((void**)&d, 4 * b));
    hipError_t e = hipMemcpy(d, x, b, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + n, y ? y : x, b, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + 2 * n, z ? z : x, b, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rtk::launch_eval(fn, d, d + n, d + 2 * n, d + 3 * n, n, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(out, d + 3 * n, b, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "rt_device_eval");
    return RT_OK;
}

}  // extern "C"

// ---- what comm.cpp reads of a context (ctx_internal.hpp) ---------------------------------------
namespace rtx {
int fail(int code, const std::string& msg) { return ::fail(code, msg); }
int hip_fail(hipError_t e, const char* what) { return ::hip_fail(e, what); }
int ctx_device(const rt_ctx* c) { return c->device; }
hipStream_t ctx_stream(const rt_ctx* c) { return c->stream; }
const uint32_t* ctx_tile_order(const rt_ctx* c, int64_t* n)
{
    *n = c->tile_order_n;
    return c->tile_order;
}
int ctx_schedule(const rt_ctx* c) { return c->opt_pool; }
int ctx_precision(const rt_ctx* c) { return c->opt_precision; }
bool ctx_comm_direct(const rt_ctx* c) { return c->opt_comm_direct != 0; }
}  // namespace rtx
