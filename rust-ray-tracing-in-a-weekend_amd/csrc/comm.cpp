// comm.cpp — the multi-GPU render behind the C ABI (rt_abi.h, "multi-GPU render"; ABI v5).
//
// The reference splits one frame over 10 std::threads, each tracing every pixel with spp/10
// samples into its own buffer, and sums the buffers under a mutex (main.rs:497-551, merge at
// :542-547). Here the split is over GPUs and by image area: rank r of `world` renders the 8x8
// tiles at positions r, r + world, ... of the frame's tile order (one slab per rank, rt_render's
// tile_shard layout), one RCCL gather moves the slabs to rank 0 over xGMI, and a reorder kernel
// (trace_kernel.hip, assemble_tiles) writes the frame there. Every draw is keyed by (pixel,
// sample), so the frame equals rt_render's bit for bit at any world size or tile order.
//
// RCCL is loaded with dlopen when the first communicator is made (librccl.so.1: the process's
// copy if one is loaded already — torch's, say — else the ROCm install's), so the library and
// every single-GPU entry point load and run without it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <new>
#include <numeric>
#include <string>
#include <vector>

#include "ctx_internal.hpp"
#include "rt/rt_abi.h"
#include "trace_kernel.hpp"

namespace {

using rtx::fail;

#define HIP_TRY(expr)                                          \
    do {                                                       \
        hipError_t e_ = (expr);                                \
        if (e_ != hipSuccess) return rtx::hip_fail(e_, #expr); \
    } while (0)

// ---- RCCL, resolved at run time ------------------------------------------------------------------
struct Rccl {
    void* h = nullptr;
    std::string err;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGather) Gather = nullptr;
    decltype(&ncclAllReduce) AllReduce = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

const Rccl& rccl()
{
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"}) {
            R.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (R.h) break;
            const char* e = dlerror();
            R.err = e ? e : "dlopen failed";
        }
        if (!R.h) return;
        bool ok = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(R.h, name));
            if (!fn) {
                ok = false;
                R.err = std::string("librccl.so.1 has no ") + name;
            }
        };
        sym(R.GetUniqueId, "ncclGetUniqueId");
        sym(R.CommInitRank, "ncclCommInitRank");
        sym(R.CommInitAll, "ncclCommInitAll");
        sym(R.CommDestroy, "ncclCommDestroy");
        sym(R.Gather, "ncclGather");
        sym(R.AllReduce, "ncclAllReduce");
        sym(R.GroupStart, "ncclGroupStart");
        sym(R.GroupEnd, "ncclGroupEnd");
        sym(R.GetErrorString, "ncclGetErrorString");
        if (!ok) R.h = nullptr;
    });
    return R;
}

int load_rccl(const Rccl*& R)
{
    R = &rccl();
    if (!R->h) return fail(RT_ERR_COMM, "RCCL not available: " + R->err);
    return RT_OK;
}

int nccl_fail(const Rccl& R, ncclResult_t r, const char* what)
{
    return fail(RT_ERR_COMM, std::string(what) + ": " + (R.GetErrorString ? R.GetErrorString(r) : "RCCL error"));
}

#define NCCL_TRY(R, expr)                                              \
    do {                                                               \
        ncclResult_t r_ = (expr);                                      \
        if (r_ != ncclSuccess) return nccl_fail((R), r_, #expr);       \
    } while (0)

}  // namespace

struct rt_comm {
    rt_ctx* ctx = nullptr;
    int rank = 0, world = 1, device = 0;
    ncclComm_t nc = nullptr;
    // this rank's tile slab (+ an 8-byte status trailer, sent with it), rank 0's gathered slabs,
    // rank 0's frame for a host-bound result, and the tile-cost vector of rt_comm_tile_order
    void* slab = nullptr;
    size_t slab_cap = 0;
    void* recv = nullptr;
    size_t recv_cap = 0;
    void* stage = nullptr;
    size_t stage_cap = 0;
    uint64_t* cost = nullptr;
    size_t cost_cap = 0;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};   // render start / end, gathered, assembled
    rt_comm_stats stats{};
    bool pending = false;       // a gather's events not yet read into stats
    bool direct = false;        // the last frame was a world-1 direct render (no slabs gathered)
    size_t status_off = 0;      // byte offset of the status trailer in a slab (rank 0: to check the peers')
    size_t slab_stride = 0;     // bytes per rank in recv
};

namespace {

int grow(hipStream_t s, void*& buf, size_t& cap, size_t need)
{
    if (need <= cap) return RT_OK;
    HIP_TRY(hipStreamSynchronize(s));   // no earlier frame still reads it
    (void)hipFree(buf);
    buf = nullptr;
    cap = 0;
    HIP_TRY(hipMalloc(&buf, need));
    cap = need;
    return RT_OK;
}

bool bad_frame(const rt_render_params* p)
{
    return !p || p->width < 2 || p->height < 2 || p->spp < 1 || p->max_depth < 0 ||
           (p->out_format != RT_OUT_F32 && p->out_format != RT_OUT_F64) ||
           (long long)p->width * p->height > 0xffffffffLL;
}

// One frame's shard on one rank: the render params of its tile shard and the slab geometry
// (every rank's slab is padded to the largest shard's, rank 0's; + the 8-byte status trailer).
struct Shard {
    rt_render_params q;
    int n_max = 0, n_mine = 0;
    long long slab_elems = 0;   // 8 x 8 n_max x 3
    size_t esz = 8;
    size_t slab_bytes = 0;      // slab_elems * esz + 8
};

int shard_of(const rt_comm* m, const rt_render_params* p, hipStream_t s, Shard& f)
{
    if (bad_frame(p)) return fail(RT_ERR_INVALID, "bad render params");
    f.q = *p;
    f.q.row_block = 0;
    f.q.tile_shard = 1;
    f.q.row_begin = m->rank;
    f.q.row_stride = m->world;
    f.q.out_on_device = 1;
    f.q.stream = s;
    f.n_max = rt_tiles_in_shard(p->width, p->height, 0, m->world);
    f.n_mine = rt_tiles_in_shard(p->width, p->height, m->rank, m->world);
    if (f.n_max <= 0) return fail(RT_ERR_INVALID, "frame too large for a tile shard");
    f.esz = p->out_format == RT_OUT_F64 ? 8 : 4;
    f.slab_elems = 192LL * f.n_max;
    f.slab_bytes = (size_t)f.slab_elems * f.esz + 8;
    return RT_OK;
}

hipStream_t stream_of(const rt_comm* m, const rt_render_params* p)
{
    return p && p->stream ? (hipStream_t)p->stream : rtx::ctx_stream(m->ctx);
}

// Renders this rank's shard into its slab and writes the status trailer (0, or -rc when the
// render could not be enqueued: the rank still takes part in the gather, so no peer waits
// forever, and rank 0 sees the failure in the trailer). Returns the render's rc.
int enqueue_shard(rt_comm* m, const rt_camera* cam, const Shard& f, hipStream_t s)
{
    HIP_TRY(hipSetDevice(m->device));
    int rc = grow(s, m->slab, m->slab_cap, f.slab_bytes);
    if (rc) return rc;
    if (m->rank == 0) {
        rc = grow(s, m->recv, m->recv_cap, f.slab_bytes * (size_t)m->world);
        if (rc) return rc;
    }
    HIP_TRY(hipEventRecord(m->ev[0], s));
    rc = rt_render(m->ctx, cam, &f.q, m->slab);
    HIP_TRY(hipSetDevice(m->device));
    HIP_TRY(hipEventRecord(m->ev[1], s));
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)((char*)m->slab + f.slab_bytes - 8), rc ? -rc : 0, 2, s));
    m->status_off = f.slab_bytes - 8;
    m->slab_stride = f.slab_bytes;
    return rc;
}

int enqueue_gather(const Rccl& R, rt_comm* m, const Shard& f, hipStream_t s)
{
    NCCL_TRY(R, R.Gather(m->slab, m->rank == 0 ? m->recv : nullptr, f.slab_bytes, ncclUint8, 0, m->nc, s));
    HIP_TRY(hipEventRecord(m->ev[2], s));
    return RT_OK;
}

// Rank 0: the reorder kernel into the frame (the caller's device buffer, or the staging buffer
// copied to the caller's host memory), in the context's tile order.
int enqueue_assemble(rt_comm* m, const rt_render_params* p, const Shard& f, hipStream_t s, void* frame)
{
    int64_t n_order = 0;
    const uint32_t* order = rtx::ctx_tile_order(m->ctx, &n_order);
    const size_t frame_bytes = (size_t)p->width * p->height * 3 * f.esz;
    void* dst = frame;
    if (!p->out_on_device) {
        const int rc = grow(s, m->stage, m->stage_cap, frame_bytes);
        if (rc) return rc;
        dst = m->stage;
    }
    HIP_TRY(rtk::launch_assemble_tiles(m->recv, dst, f.esz == 8, m->world, (long long)(f.slab_bytes / f.esz),
                                       p->width, p->height, n_order > 0 ? order : nullptr, s));
    HIP_TRY(hipEventRecord(m->ev[3], s));
    if (!p->out_on_device) HIP_TRY(hipMemcpyAsync(frame, dst, frame_bytes, hipMemcpyDeviceToHost, s));
    return RT_OK;
}

// Rank 0 after its stream is synchronized: the peers' status trailers (RT_ERR_PEER if any failed).
int peer_status(rt_comm* m)
{
    for (int r = 0; r < m->world; ++r) {
        int32_t st = 0;
        HIP_TRY(hipMemcpy(&st, (char*)m->recv + (size_t)r * m->slab_stride + m->status_off, 4,
                          hipMemcpyDeviceToHost));
        if (st != 0)
            return fail(RT_ERR_PEER, "rank " + std::to_string(r) + "'s shard render failed (" + std::to_string(-st) +
                                         "): the frame is incomplete");
    }
    return RT_OK;
}

void note_gather(rt_comm* m, const Shard& f)
{
    m->pending = true;
    m->direct = false;
    m->stats.slab_bytes = (int64_t)f.slab_bytes;
    m->stats.tiles = f.n_mine;
}

// A world of one (RT_OPT_COMM_DIRECT, raster tile order): rt_render straight into the frame.
// The frame is the tile path's bit for bit (every draw keyed by (pixel, sample)); it skips the
// slab, the one-rank gather and the reorder pass (C2 at N = 1: 75.09 -> 74.70-74.92 ms per step,
// profiles/r06e_c2_*.log). The stats' gather and assemble times are 0.
bool direct_ok(const rt_comm* m)
{
    int64_t n_order = 0;
    (void)rtx::ctx_tile_order(m->ctx, &n_order);
    return m->world == 1 && n_order == 0 && rtx::ctx_comm_direct(m->ctx);
}

int render_direct(rt_comm* m, const rt_camera* cam, const rt_render_params* p, hipStream_t s, void* frame)
{
    if (bad_frame(p)) return fail(RT_ERR_INVALID, "bad render params");
    rt_render_params q = *p;
    q.row_begin = 0;
    q.row_stride = 1;
    q.row_block = 0;
    q.tile_shard = 0;
    q.stream = s;
    HIP_TRY(hipSetDevice(m->device));
    HIP_TRY(hipEventRecord(m->ev[0], s));
    const int rc = rt_render(m->ctx, cam, &q, frame);
    HIP_TRY(hipSetDevice(m->device));
    for (int i = 1; i < 4; ++i) HIP_TRY(hipEventRecord(m->ev[i], s));
    m->pending = true;
    m->direct = true;
    m->stats.slab_bytes = 0;
    m->stats.tiles = rt_tiles_in_shard(p->width, p->height, 0, 1);
    return rc;
}

int check_comms(rt_comm* const* comms, int n)
{
    if (!comms || n < 1) return fail(RT_ERR_INVALID, "no communicators");
    for (int i = 0; i < n; ++i)
        if (!comms[i] || comms[i]->rank != i || comms[i]->world != n)
            return fail(RT_ERR_INVALID, "comms[i] must be rank i of a world of n (rt_comm_init_all)");
    return RT_OK;
}

// ---- rt_comm_tile_order's phases -------------------------------------------------------------------
struct CostPass {
    int rc = RT_OK;
    int schedule = RT_SCHED_AUTO, precision = RT_PREC_F64;
    int64_t n_tiles = 0;
    std::chrono::steady_clock::time_point t0;
};

// The count pass of this rank's raster shard, its tile costs (+ a failure flag) into m->cost.
// Returns an error only when the all-reduce could not be fed (then the caller must not enter it:
// the peers see no contribution... which RCCL cannot express, so this is limited to argument
// errors every rank shares).
int cost_local(rt_comm* m, const rt_camera* cam, const rt_render_params* p, int cost_spp, hipStream_t s, CostPass& cp)
{
    cp.t0 = std::chrono::steady_clock::now();
    if (bad_frame(p) || cost_spp < 1) return fail(RT_ERR_INVALID, "bad render params or cost_spp");
    cp.n_tiles = (int64_t)((p->width + 7) / 8) * ((p->height + 7) / 8);
    HIP_TRY(hipSetDevice(m->device));
    int rc = grow(s, (void*&)m->cost, m->cost_cap, (size_t)(cp.n_tiles + 1) * sizeof(uint64_t));
    if (rc) return rc;
    cp.schedule = rtx::ctx_schedule(m->ctx);
    cp.precision = rtx::ctx_precision(m->ctx);
    std::vector<uint64_t> h((size_t)cp.n_tiles + 1, 0);
    // raster shards, f64 (count_work's tile costs), a pool schedule (the chunk schedule counts none)
    rc = rt_ctx_set_tile_order(m->ctx, nullptr, 0);
    if (!rc && cp.precision != RT_PREC_F64) rc = rt_ctx_set_precision(m->ctx, RT_PREC_F64);
    if (!rc && cp.schedule == RT_SCHED_CHUNKS) rc = rt_ctx_set_schedule(m->ctx, RT_SCHED_POOL);
    Shard f;
    rt_render_params q = *p;
    q.spp = cost_spp;
    q.count_work = 1;
    q.out_format = RT_OUT_F32;
    if (!rc) rc = shard_of(m, &q, s, f);
    if (!rc) rc = grow(s, m->slab, m->slab_cap, f.slab_bytes);
    if (!rc) rc = rt_render(m->ctx, cam, &f.q, m->slab);
    if (!rc) {
        const int got = rt_last_tile_costs(m->ctx, h.data(), cp.n_tiles);   // synchronizes the render
        if (got < 0) rc = got;
        else if (got != cp.n_tiles) rc = fail(RT_ERR_UNSUPPORTED, "the count pass recorded no tile costs");
    }
    (void)rt_ctx_set_precision(m->ctx, cp.precision);
    (void)rt_ctx_set_schedule(m->ctx, cp.schedule);
    cp.rc = rc;
    if (rc) std::fill(h.begin(), h.end(), 0);
    h[(size_t)cp.n_tiles] = rc ? 1 : 0;   // failures, summed over the ranks
    HIP_TRY(hipSetDevice(m->device));
    HIP_TRY(hipMemcpyAsync(m->cost, h.data(), h.size() * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));   // (h is pageable and local)
    return RT_OK;
}

int cost_finish(rt_comm* m, hipStream_t s, CostPass& cp)
{
    HIP_TRY(hipSetDevice(m->device));
    std::vector<uint64_t> h((size_t)cp.n_tiles + 1, 0);
    HIP_TRY(hipMemcpyAsync(h.data(), m->cost, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    int rc = RT_OK;
    if (h[(size_t)cp.n_tiles] != 0) {   // some rank's pass failed: every rank keeps raster order
        (void)rt_ctx_set_tile_order(m->ctx, nullptr, 0);
        rc = cp.rc ? cp.rc : fail(RT_ERR_PEER, "another rank's cost pass failed: raster tile order");
        m->stats.tile_order = 0;
    } else {
        std::vector<uint32_t> order((size_t)cp.n_tiles);
        rc = rt_cost_tile_order(h.data(), cp.n_tiles, order.data());
        if (!rc) rc = rt_ctx_set_tile_order(m->ctx, order.data(), cp.n_tiles);
        m->stats.tile_order = rc ? 0 : 1;
    }
    m->stats.cost_pass_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - cp.t0).count();
    return rc;
}

}  // namespace

extern "C" {

int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES])
{
    if (!id) return fail(RT_ERR_INVALID, "null id");
    const Rccl* R;
    int rc = load_rccl(R);
    if (rc) return rc;
    ncclUniqueId u;
    NCCL_TRY(*R, R->GetUniqueId(&u));
    static_assert(sizeof u == RT_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof u);
    return RT_OK;
}

static int comm_new(rt_ctx* ctx, int rank, int world, rt_comm** out)
{
    rt_comm* m = new (std::nothrow) rt_comm();
    if (!m) return fail(RT_ERR_OOM, "rt_comm");
    m->ctx = ctx;
    m->rank = rank;
    m->world = world;
    m->device = rtx::ctx_device(ctx);
    hipError_t e = hipSetDevice(m->device);
    for (int i = 0; i < 4 && e == hipSuccess; ++i) e = hipEventCreate(&m->ev[i]);
    if (e != hipSuccess) {
        for (auto& v : m->ev)
            if (v) (void)hipEventDestroy(v);
        delete m;
        return rtx::hip_fail(e, "rt_comm events");
    }
    *out = m;
    return RT_OK;
}

int rt_comm_init_rank(rt_ctx* ctx, int rank, int world, const uint8_t id[RT_COMM_ID_BYTES], rt_comm** out)
{
    if (!ctx || !id || !out || world < 1 || rank < 0 || rank >= world) return fail(RT_ERR_INVALID, "bad argument");
    *out = nullptr;
    const Rccl* R;
    int rc = load_rccl(R);
    if (rc) return rc;
    rt_comm* m = nullptr;
    rc = comm_new(ctx, rank, world, &m);
    if (rc) return rc;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    const ncclResult_t r = R->CommInitRank(&m->nc, world, u, rank);
    if (r != ncclSuccess) {
        rt_comm_destroy(m);
        return nccl_fail(*R, r, "ncclCommInitRank");
    }
    *out = m;
    return RT_OK;
}

int rt_comm_init_all(rt_ctx* const* ctxs, int n, rt_comm** comms_out)
{
    if (!ctxs || !comms_out || n < 1) return fail(RT_ERR_INVALID, "bad argument");
    const Rccl* R;
    int rc = load_rccl(R);
    if (rc) return rc;
    std::vector<int> dev((size_t)n);
    for (int i = 0; i < n; ++i) {
        comms_out[i] = nullptr;
        if (!ctxs[i]) return fail(RT_ERR_INVALID, "null context");
        dev[(size_t)i] = rtx::ctx_device(ctxs[i]);
        for (int j = 0; j < i; ++j)
            if (dev[(size_t)j] == dev[(size_t)i]) return fail(RT_ERR_INVALID, "two contexts on one device");
    }
    std::vector<ncclComm_t> nc((size_t)n, nullptr);
    NCCL_TRY(*R, R->CommInitAll(nc.data(), n, dev.data()));
    for (int i = 0; i < n; ++i) {
        rc = comm_new(ctxs[i], i, n, &comms_out[i]);
        if (rc) {
            for (int j = 0; j < n; ++j) {
                if (comms_out[j]) rt_comm_destroy(comms_out[j]);
                else if (nc[(size_t)j]) (void)R->CommDestroy(nc[(size_t)j]);
                comms_out[j] = nullptr;
            }
            return rc;
        }
        comms_out[i]->nc = nc[(size_t)i];
    }
    return RT_OK;
}

void rt_comm_destroy(rt_comm* m)
{
    if (!m) return;
    (void)hipSetDevice(m->device);
    for (auto& e : m->ev)
        if (e) (void)hipEventSynchronize(e);
    (void)hipStreamSynchronize(rtx::ctx_stream(m->ctx));
    if (m->nc) {
        const Rccl& R = rccl();
        if (R.CommDestroy) (void)R.CommDestroy(m->nc);
    }
    (void)hipFree(m->slab);
    (void)hipFree(m->recv);
    (void)hipFree(m->stage);
    (void)hipFree(m->cost);
    for (auto& e : m->ev)
        if (e) (void)hipEventDestroy(e);
    delete m;
}

int rt_comm_rank(const rt_comm* m, int* rank, int* world)
{
    if (!m) return fail(RT_ERR_INVALID, "null communicator");
    if (rank) *rank = m->rank;
    if (world) *world = m->world;
    return RT_OK;
}

int rt_comm_tile_order(rt_comm* m, const rt_camera* cam, const rt_render_params* p, int cost_spp)
{
    if (!m || !cam || !p) return fail(RT_ERR_INVALID, "null argument");
    const Rccl* R;
    int rc = load_rccl(R);
    if (rc) return rc;
    const hipStream_t s = stream_of(m, p);
    CostPass cp;
    rc = cost_local(m, cam, p, cost_spp, s, cp);
    if (rc) return rc;
    NCCL_TRY(*R, R->AllReduce(m->cost, m->cost, (size_t)cp.n_tiles + 1, ncclUint64, ncclSum, m->nc, s));
    return cost_finish(m, s, cp);
}

int rt_comm_tile_order_all(rt_comm* const* comms, int n, const rt_camera* cam, const rt_render_params* p,
                           int cost_spp)
{
    int rc = check_comms(comms, n);
    if (rc) return rc;
    if (!cam || !p) return fail(RT_ERR_INVALID, "null argument");
    if (p->stream) return fail(RT_ERR_INVALID, "the *_all calls run on each context's stream: p->stream must be NULL");
    const Rccl* R;
    rc = load_rccl(R);
    if (rc) return rc;
    std::vector<CostPass> cp((size_t)n);
    for (int i = 0; i < n; ++i) {
        rc = cost_local(comms[i], cam, p, cost_spp, rtx::ctx_stream(comms[i]->ctx), cp[(size_t)i]);
        if (rc) return rc;
    }
    NCCL_TRY(*R, R->GroupStart());
    for (int i = 0; i < n; ++i) {
        rt_comm* m = comms[i];
        const ncclResult_t r = R->AllReduce(m->cost, m->cost, (size_t)cp[(size_t)i].n_tiles + 1, ncclUint64, ncclSum,
                                            m->nc, rtx::ctx_stream(m->ctx));
        if (r != ncclSuccess) {
            (void)R->GroupEnd();
            return nccl_fail(*R, r, "ncclAllReduce");
        }
    }
    NCCL_TRY(*R, R->GroupEnd());
    int first = RT_OK;
    for (int i = 0; i < n; ++i) {
        rc = cost_finish(comms[i], rtx::ctx_stream(comms[i]->ctx), cp[(size_t)i]);
        if (rc && !first) first = rc;
    }
    return first;
}

int rt_render_gather(rt_comm* m, const rt_camera* cam, const rt_render_params* p, void* frame)
{
    if (!m || !cam || !p) return fail(RT_ERR_INVALID, "null argument");
    if (m->rank == 0 && !frame) return fail(RT_ERR_INVALID, "rank 0 needs a frame");
    if (direct_ok(m)) return render_direct(m, cam, p, stream_of(m, p), frame);
    const Rccl* R;
    int rc = load_rccl(R);
    if (rc) return rc;
    const hipStream_t s = stream_of(m, p);
    Shard f;
    rc = shard_of(m, p, s, f);   // (argument errors: every rank has the same p and fails alike)
    if (rc) return rc;
    const int rc_render = enqueue_shard(m, cam, f, s);
    if (m->slab_cap < f.slab_bytes || (m->rank == 0 && m->recv_cap < f.slab_bytes * (size_t)m->world))
        return rc_render;   // no buffers to send from: nothing was enqueued for the peers either
    rc = enqueue_gather(*R, m, f, s);
    if (rc) return rc;
    note_gather(m, f);
    if (m->rank == 0) {
        rc = enqueue_assemble(m, p, f, s, frame);
        if (rc) return rc;
    }
    if (p->out_on_device) return rc_render;
    HIP_TRY(hipStreamSynchronize(s));
    if (rc_render) return rc_render;
    return m->rank == 0 ? peer_status(m) : RT_OK;
}

int rt_render_gather_all(rt_comm* const* comms, int n, const rt_camera* cam, const rt_render_params* p, void* frame)
{
    int rc = check_comms(comms, n);
    if (rc) return rc;
    if (!cam || !p || !frame) return fail(RT_ERR_INVALID, "null argument");
    if (p->stream) return fail(RT_ERR_INVALID, "the *_all calls run on each context's stream: p->stream must be NULL");
    const Rccl* R;
    rc = load_rccl(R);
    if (rc) return rc;
    if (n == 1 && direct_ok(comms[0])) return render_direct(comms[0], cam, p, rtx::ctx_stream(comms[0]->ctx), frame);
    std::vector<Shard> f((size_t)n);
    for (int i = 0; i < n; ++i) {
        rc = shard_of(comms[i], p, rtx::ctx_stream(comms[i]->ctx), f[(size_t)i]);
        if (rc) return rc;
    }
    int rc_render = RT_OK;
    for (int i = 0; i < n; ++i) {   // every render enqueued before any gather: the GPUs trace at once
        rc = enqueue_shard(comms[i], cam, f[(size_t)i], rtx::ctx_stream(comms[i]->ctx));
        if (rc && !rc_render) rc_render = rc;
        if (comms[i]->slab_cap < f[(size_t)i].slab_bytes ||
            (i == 0 && comms[0]->recv_cap < f[0].slab_bytes * (size_t)n))
            return rc;   // no buffers: nothing to gather
    }
    NCCL_TRY(*R, R->GroupStart());
    for (int i = 0; i < n; ++i) {
        rt_comm* m = comms[i];
        const ncclResult_t r = R->Gather(m->slab, i == 0 ? m->recv : nullptr, f[(size_t)i].slab_bytes, ncclUint8, 0,
                                         m->nc, rtx::ctx_stream(m->ctx));
        if (r != ncclSuccess) {
            (void)R->GroupEnd();
            return nccl_fail(*R, r, "ncclGather");
        }
    }
    NCCL_TRY(*R, R->GroupEnd());
    for (int i = 0; i < n; ++i) {
        HIP_TRY(hipSetDevice(comms[i]->device));
        HIP_TRY(hipEventRecord(comms[i]->ev[2], rtx::ctx_stream(comms[i]->ctx)));
        note_gather(comms[i], f[(size_t)i]);
    }
    HIP_TRY(hipSetDevice(comms[0]->device));
    rc = enqueue_assemble(comms[0], p, f[0], rtx::ctx_stream(comms[0]->ctx), frame);
    if (rc) return rc;
    if (p->out_on_device) return rc_render;
    for (int i = 0; i < n; ++i) {
        HIP_TRY(hipSetDevice(comms[i]->device));
        HIP_TRY(hipStreamSynchronize(rtx::ctx_stream(comms[i]->ctx)));
    }
    if (rc_render) return rc_render;
    HIP_TRY(hipSetDevice(comms[0]->device));
    return peer_status(comms[0]);
}

int rt_comm_last_stats(rt_comm* m, rt_comm_stats* out)
{
    if (!m || !out) return fail(RT_ERR_INVALID, "null argument");
    if (m->pending) {
        HIP_TRY(hipSetDevice(m->device));
        HIP_TRY(hipEventSynchronize(m->ev[2]));
        float a = 0, b = 0, c = 0;
        HIP_TRY(hipEventElapsedTime(&a, m->ev[0], m->ev[1]));
        HIP_TRY(hipEventElapsedTime(&b, m->ev[1], m->ev[2]));
        if (m->rank == 0) {
            HIP_TRY(hipEventSynchronize(m->ev[3]));
            HIP_TRY(hipEventElapsedTime(&c, m->ev[2], m->ev[3]));
        }
        m->stats.render_ms = a;
        m->stats.gather_ms = b;
        m->stats.assemble_ms = c;
        rt_stats st;
        if (rt_last_stats(m->ctx, &st) == RT_OK) m->stats.kernel_ms = st.kernel_ms;
        m->stats.peer_failed = 0;
        for (int r = 0; m->rank == 0 && !m->direct && r < m->world; ++r) {
            int32_t v = 0;
            HIP_TRY(hipMemcpy(&v, (char*)m->recv + (size_t)r * m->slab_stride + m->status_off, 4, hipMemcpyDeviceToHost));
            m->stats.peer_failed += v != 0;
        }
        m->pending = false;
    }
    *out = m->stats;
    return RT_OK;
}

int rt_tiles_assemble(rt_ctx* ctx, const void* slabs, int64_t slab_elems, int world, const rt_render_params* p,
                      void* frame)
{
    if (!ctx || !slabs || !frame || world < 1 || bad_frame(p)) return fail(RT_ERR_INVALID, "bad argument");
    const int n_max = rt_tiles_in_shard(p->width, p->height, 0, world);
    if (n_max <= 0 || slab_elems < 192LL * n_max) return fail(RT_ERR_INVALID, "slab_elems below the largest shard's");
    int64_t n_order = 0;
    const uint32_t* order = rtx::ctx_tile_order(ctx, &n_order);
    const int64_t n_tiles = (int64_t)((p->width + 7) / 8) * ((p->height + 7) / 8);
    if (n_order > 0 && n_order != n_tiles) return fail(RT_ERR_INVALID, "the context's tile order is for another frame");
    HIP_TRY(hipSetDevice(rtx::ctx_device(ctx)));
    const hipStream_t s = p->stream ? (hipStream_t)p->stream : rtx::ctx_stream(ctx);
    HIP_TRY(rtk::launch_assemble_tiles(slabs, frame, p->out_format == RT_OUT_F64, world, (long long)slab_elems,
                                       p->width, p->height, n_order > 0 ? order : nullptr, s));
    return RT_OK;
}

int rt_tiles_assemble_host(const void* slabs, int64_t slab_elems, int world, int width, int height, int elem_bytes,
                           const uint32_t* order, void* frame)
{
    if (!slabs || !frame || world < 1 || width < 1 || height < 1 || (elem_bytes != 4 && elem_bytes != 8))
        return fail(RT_ERR_INVALID, "bad argument");
    const int tx = (width + 7) / 8;
    const int64_t n_tiles = (int64_t)tx * ((height + 7) / 8);
    const int n_max = rt_tiles_in_shard(width, height, 0, world);
    if (n_max <= 0 || slab_elems < 192LL * n_max) return fail(RT_ERR_INVALID, "slab_elems below the largest shard's");
    if (order) {
        std::vector<uint8_t> seen((size_t)n_tiles, 0);
        for (int64_t i = 0; i < n_tiles; ++i) {
            if ((int64_t)order[i] >= n_tiles || seen[order[i]]) return fail(RT_ERR_INVALID, "order is not a permutation");
            seen[order[i]] = 1;
        }
    }
    const size_t px = 3 * (size_t)elem_bytes;
    const char* in = (const char*)slabs;
    char* out = (char*)frame;
    for (int r = 0; r < world; ++r) {
        const int n_r = rt_tiles_in_shard(width, height, r, world);
        for (int m = 0; m < n_r; ++m) {
            const int64_t pos = r + (int64_t)m * world;
            const int64_t t = order ? (int64_t)order[pos] : pos;
            const int x0 = (int)(t % tx) * 8, y0 = (int)(t / tx) * 8;
            for (int k = 0; k < 8 && y0 + k < height; ++k) {
                const int w = std::min(8, width - x0);
                std::memcpy(out + ((size_t)(y0 + k) * width + x0) * px,
                            in + ((size_t)r * slab_elems + ((size_t)k * 8 * n_r + 8 * (size_t)m) * 3) * elem_bytes,
                            (size_t)w * px);
            }
        }
    }
    return RT_OK;
}

int rt_cost_tile_order(const uint64_t* costs, int64_t n, uint32_t* order)
{
    if (n < 0 || (n > 0 && (!costs || !order)) || n > ((int64_t)1 << 32)) return fail(RT_ERR_INVALID, "bad argument");
    std::iota(order, order + n, 0u);
    std::stable_sort(order, order + n, [costs](uint32_t a, uint32_t b) { return costs[a] > costs[b]; });
    return RT_OK;
}

}  // extern "C"
