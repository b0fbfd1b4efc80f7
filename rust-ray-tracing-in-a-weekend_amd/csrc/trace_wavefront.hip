// trace_wavefront.hip — the wavefront schedule (RT_SCHED_WAVEFRONT) of the final-scene
// feature set: the megakernel's per-(pixel, sample) arithmetic (trace_device.hpp), split
// into two kernels over a pool of path slots in HBM so that the BVH walks run over a
// compacted ray queue with per-lane ray fetch instead of inside the bounce loop.
//
// Why: in the megakernel a wave's lanes each walk one
// cast per bounce-loop iteration and the wave waits for its longest walk, so the node loop
// runs at lane occupancy 0.21 and the leaf loop at 0.34 on C4; the 1000-sphere BLAS walk
// (deferred to the end of the top-level walk) runs for the few lanes that need it.
//
//   wf_logic   one thread per slot (256-thread blocks, one 64-slot queue segment per wave):
//              the hit record of the slot's last cast (finish_hit), emission or background
//              (main.rs:25-37), the material's draws and scattered ray (material.rs:15-94); a
//              slot with no path takes the next (pixel, sample) unit of its wave's work block
//              (tile x samples, the per-sample pool's blocks) and its camera ray (camera.rs:
//              58-66); the camera's and the materials' rejection tries in one loop, as the pool
//              does. Live slots go to the wave's queue segment; a finished sample's radiance to
//              the per-sample buffer (tiled_record, reduced by reduce_samples as the pool's).
//   wf_trace   a persistent grid (one 1024-thread block per CU, every TLAS and BLAS node staged
//              in LDS as 80-B LdsNode records): each lane walks one ray; a lane whose walk ends
//              writes (t, leaf slot, sub, side) and takes the next queued ray at once. The top-
//              level walk and the deferred instance BLAS walk (trace_world's DeferInst) are one
//              step loop over one node format, so lanes in either phase share the node visits
//              and the sphere test. Per ray the tests run in the megakernel's order, so the
//              closest hit — and the image — is the same bit for bit.
//
// Per cast HBM traffic (bytes): wf_trace reads the queue entry, the ray and the
// medium key (72) and writes the hit (16); wf_logic reads the slot state, hit and ray (<= 128)
// and writes the next ray and state (<= 104).
#include "trace_device.hpp"

namespace rtk {

// A kernel configuration with its own workgroup size (the LDS stack stride and staging loops
// follow BT): the final-scene feature set, f32 slabs, f64 arithmetic
template <uint32_t F_, bool S32_, bool LDS_, bool NALL_, bool COUNT_, int BT_>
struct WfCfg : Cfg<F_, S32_, LDS_, NALL_, COUNT_, false> {
    static constexpr int BT = BT_;
};
constexpr int kWfTraceThreads = 1024;   // one block per CU: the LDS holds one copy of every node
constexpr int kWfLogicThreads = 256;
#ifndef RT_WF_CHUNK
#define RT_WF_CHUNK 16   // iterations enqueued between two polls of the live flag
#endif

__device__ __forceinline__ __attribute__((address_space(3))) int* lds_int(uint32_t a)
{
    return (__attribute__((address_space(3))) int*)(uintptr_t)a;
}

// ---------------------------------------------------------------------------------------------
// wf_trace
// ---------------------------------------------------------------------------------------------
template <class C>
__global__ void __launch_bounds__(kWfTraceThreads, 1) wf_trace(SceneDev S, const KParams* __restrict__ Pp, WfPaths W,
                                                              unsigned long long* __restrict__ counters, int parity)
{
    using R = double;
    const KParams& P = *Pp;
    // every node (the TLAS, then the instanced BLAS in BFS order) as an LdsNode: per axis both
    // children's lower, upper and lower planes again; child references as LDS byte addresses
    const int n_nodes = S.n_tlas_nodes + S.n_blas_bfs;
    LdsNode* const nodes = reinterpret_cast<LdsNode*>(rt_lds);
    const uint32_t nb0 = lds_addr(nodes);
    for (int i = threadIdx.x; i < n_nodes; i += kWfTraceThreads) {
        const rt_bvh_node n = S.nodes[i];
        LdsNode o;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            o.ax[a][0] = n.lo0[a]; o.ax[a][1] = n.lo1[a];
            o.ax[a][2] = n.hi0[a]; o.ax[a][3] = n.hi1[a];
            o.ax[a][4] = n.lo0[a]; o.ax[a][5] = n.lo1[a];
        }
#pragma unroll
        for (int c = 0; c < 2; ++c)
            o.child[c] = n.child[c] >= 0 ? (int)(nb0 + (uint32_t)n.child[c] * (uint32_t)sizeof(LdsNode)) : n.child[c];
        nodes[i] = o;
    }
    // the deferred instance's record after the nodes (S.defer_inst: the scene's one instance over a
    // BVH, abi.cpp), then the stacks
    char* const lds_inst = reinterpret_cast<char*>(nodes + n_nodes);
    if (threadIdx.x < sizeof(rt_instance) / 8 && S.defer_inst >= 0)
        reinterpret_cast<uint64_t*>(lds_inst)[threadIdx.x] =
            reinterpret_cast<const uint64_t*>(S.instances + S.defer_inst)[threadIdx.x];
    __syncthreads();
    // the lane's stack column: entry e at stack0 + e * (block threads * 4)
    const uint32_t stack0 = nb0 + (uint32_t)n_nodes * (uint32_t)sizeof(LdsNode) + (uint32_t)sizeof(rt_instance) +
                            (uint32_t)threadIdx.x * 4u;
    constexpr uint32_t SSTR = kWfTraceThreads * 4u;
    StackT<C> nostack;   // (medium boundaries and single-primitive instances walk no BVH here)
    nostack.init(0);
    Count cnt{};
    uint64_t t_start = 0;
    if (C::COUNT) t_start = __builtin_amdgcn_s_memtime();
    const R t_min = (R)0.001;
    const float tmin_f = f32_down(t_min);
    float ninf;
    asm("s_mov_b32 %0, 0xff800000" : "=s"(ninf));
    const uint32_t n = (uint32_t)W.n;
    const uint32_t n_seg = n >> 6, seg_per_shard = n_seg / kWfShards;
    const int lane = threadIdx.x & 63;

    // wave state: a window of two queue segments (128 entries) being drained
    // this iteration's queue buffer: entry e of component c at [c * n + e]
    const double* const qo = W.qo + (size_t)parity * 3 * n;
    const double* const qd = W.qd + (size_t)parity * 3 * n;
    const double* const qtime = W.qtime + (size_t)parity * n;
    const uint4* const qkey = W.qkey + (size_t)parity * n;
    double* const ht = W.ht + (size_t)parity * n;
    int2* const hp = W.hp + (size_t)parity * n;
    const uint32_t refill_min = (uint32_t)max(1, P.wf_refill);
    // static windows: wave g drains windows g, g + n_waves, ... (the queue is dense: every logic
    // wave fills its segment with its live slots), each window's counts loaded one window ahead
    const uint32_t n_win = n_seg / 2, n_waves = gridDim.x * (kWfTraceThreads / 64);
    uint32_t nxt = blockIdx.x * (kWfTraceThreads / 64) + (threadIdx.x >> 6);
    uint2 pre = make_uint2(0u, 0u);
    if (nxt < n_win) pre = *reinterpret_cast<const uint2*>(W.qn + 2 * nxt);
    uint32_t win_a = 0, cnt_a = 0, win_b = 0, cnt_b = 0, win_next = 0;
    bool exhausted = false;
    // lane state
    bool busy = false, blas = false, any = false;
    uint32_t pos = 0, sp = 0;
    int cur = RT_DONE, pend = -1, base = 0;
    RayT<R> r;
    R t_max = (R)RT_INF;
    float tmax_f = 0.0f;
    HitRefT<R> best;
    best.t = (R)0; best.prim = 0; best.sub = 0; best.side = 0;
    Keyed key{P.seed, 0, 0, 0};

    auto push = [&](int v) { *lds_int(sp) = v; sp += SSTR; };
    auto pop = [&]() -> int { sp -= SSTR; return *lds_int(sp); };
    auto visit = [&](int node) -> int {   // traverse's OctNodes visit (trace_device.hpp)
        if (C::COUNT) cnt.nodes++;
        const uint32_t nb = (uint32_t)node;
        typedef int i2v __attribute__((ext_vector_type(2)));
        auto pairs = [&](uint32_t off, f2v& nn, f2v& ff) {
            const auto q = lds_ptr<f2v>(nb + off);   // one ds_read2_b64
            nn = q[0];
            ff = q[1];
        };
        f2v npx, fpx, npy, fpy, npz, fpz;
        pairs(r.onx, npx, fpx);
        pairs(r.ony, npy, fpy);
        pairs(r.onz, npz, fpz);
        const i2v ch = *lds_ptr<i2v>(nb + (uint32_t)offsetof(LdsNode, child));
        float tn[2], tf[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const float nx = __builtin_fmaf(c ? npx.y : npx.x, r.sx.x, r.sx.y);
            const float ny = __builtin_fmaf(c ? npy.y : npy.x, r.sy.x, r.sy.y);
            const float nz = __builtin_fmaf(c ? npz.y : npz.x, r.sz.x, r.sz.y);
            const float fx = __builtin_fmaf(c ? fpx.y : fpx.x, r.sx.x, r.sx.y);
            const float fy = __builtin_fmaf(c ? fpy.y : fpy.x, r.sy.x, r.sy.y);
            const float fz = __builtin_fmaf(c ? fpz.y : fpz.x, r.sz.x, r.sz.y);
            tn[c] = fmaxf(fmaxf(nx, ny), fmaxf(nz, tmin_f));
            tf[c] = fminf(fminf(fx, fy), __builtin_amdgcn_fmed3f(fz, tmax_f, ninf));
        }
        const bool h0 = tn[0] <= tf[0], h1 = tn[1] <= tf[1], near0 = tn[0] <= tn[1];
        if (h0 && h1) {
            push(near0 ? ch.y : ch.x);
            return near0 ? ch.x : ch.y;
        }
        if (h0) return ch.x;
        if (h1) return ch.y;
        return pop();
    };
    auto root_ref = [&](int ref) { return ref >= 0 ? (int)(nb0 + (uint32_t)ref * (uint32_t)sizeof(LdsNode)) : ref; };

    uint64_t tp = 0;   // COUNT: phase stamps (wave-cycles, s_memtime)
    if (C::COUNT) tp = __builtin_amdgcn_s_memtime();
    for (;;) {
        // ---- refill: idle lanes take the next queued rays (ballot + mbcnt over the segment)
        if (C::COUNT) tp = __builtin_amdgcn_s_memtime();
        uint64_t idle = __ballot(!busy);
        if (idle != 0 && !exhausted && ((uint32_t)__popcll(idle) >= refill_min || idle == ~0ull)) {
            while (idle != 0) {
                uint64_t tf = 0;
                if (C::COUNT) tf = __builtin_amdgcn_s_memtime();
                if (win_next == cnt_a + cnt_b) {
                    // the next window: the prefetched one, whose successor's counts are loaded now
                    if (nxt >= n_win) {
                        exhausted = true;
                        break;
                    }
                    win_a = nxt << 7;
                    win_b = win_a + 64;
                    cnt_a = __builtin_amdgcn_readfirstlane(pre.x);
                    cnt_b = __builtin_amdgcn_readfirstlane(pre.y);
                    win_next = 0;
                    nxt += n_waves;
                    if (nxt < n_win) pre = *reinterpret_cast<const uint2*>(W.qn + 2 * nxt);
                    RT_STAMP(cnt.t_pre, tf);   // window changes
                    continue;
                }
                const unsigned rank = lanes_below(idle);
                const unsigned take = min((unsigned)__popcll(idle), cnt_a + cnt_b - win_next);
                if (!busy && rank < take) {
                    const uint32_t e = win_next + rank;
                    pos = e < cnt_a ? win_a + e : win_b + (e - cnt_a);
                    // non-temporal: the queue streams through once and must not evict the scene
                    r.ox = __builtin_nontemporal_load(&qo[pos]);
                    r.oy = __builtin_nontemporal_load(&qo[n + pos]);
                    r.oz = __builtin_nontemporal_load(&qo[2 * n + pos]);
                    r.dx = __builtin_nontemporal_load(&qd[pos]);
                    r.dy = __builtin_nontemporal_load(&qd[n + pos]);
                    r.dz = __builtin_nontemporal_load(&qd[2 * n + pos]);
                    r.time = __builtin_nontemporal_load(&qtime[pos]);
                    typedef unsigned u4v __attribute__((ext_vector_type(4)));
                    const u4v kq = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(&qkey[pos]));
                    key.pixel = kq.x;
                    key.sample = kq.y;
                    key.bounce = kq.z;
                    finish_ray<C>(r, S.has_spheres != 0);
                    t_max = (R)RT_INF;
                    tmax_f = f32_up(t_max);
                    any = false;
                    blas = false;
                    pend = -1;
                    base = 0;
                    sp = stack0;
                    push(RT_DONE);
                    cur = root_ref(S.tlas_root);
                    busy = true;
                    if (C::COUNT) cnt.casts++;
                }
                RT_STAMP(cnt.t_setup, tf);   // lanes' ray loads and set-up
                win_next += take;
                idle = __ballot(!busy);
            }
        }
        RT_STAMP(cnt.t_refill, tp);
        if (!__any(busy)) {
            if (exhausted) break;
            continue;
        }
        if (C::COUNT) {
            const uint32_t nbusy = (uint32_t)__popcll(__ballot(busy));
            if (first_active_lane()) {
                cnt.wave_steps++;
                cnt.shade_lanes += nbusy;   // busy lanes summed over the wave's steps
            }
        }
        if (!busy) continue;
        // ---- one while-while step: node visits until a leaf (or the end), then the leaf
        while (cur >= 0) {
            if (C::COUNT && first_active_lane()) cnt.wave_nodes++;
            cur = visit(cur);
        }
        RT_STAMP(cnt.t_nodes, tp);
        if (cur != RT_DONE) {
            const int code = ~cur, first = code >> 5, count = code & 31;
            for (int i = 0; i < count; ++i) {
                if (C::COUNT && first_active_lane()) cnt.wave_leaves++;
                const int j = base + first + i;   // the leaf slot (BLAS codes count from in.pad)
                const rt_prim& p = S.leaf_prims[j];
                R tt = (R)0;
                int side = 0, sub = 0;
                bool h = false;
                if (p.kind == RT_PRIM_INSTANCE) {   // top level only (the BLAS holds spheres)
                    if (pend < 0 && p.b != 0) {
                        pend = j;   // trace_world's DeferInst: walked after the top-level walk
                    } else {
                        HitRefT<R> b;
                        b.sub = 0;
                        b.side = 0;
                        h = instance_t<C>(S, S.instances[p.a], r, t_min, t_max, b, nostack, 0, key, cnt);
                        tt = b.t;
                        sub = b.sub;
                        side = b.side;
                    }
                } else if (p.kind == RT_PRIM_MEDIUM) {
                    h = medium_t<C>(S, p, r, t_min, t_max, tt, nostack, 0, key, cnt);
                } else {
                    h = simple_t<C>(p, r, t_min, t_max, tt, side, cnt, (C::F & FEAT_SHUTTER) != 0);
                }
                if (h) {
                    t_max = tt;
                    tmax_f = f32_up(t_max);
                    any = true;
                    best.t = tt;
                    if (blas) {   // trace_world: best = instance_t's ref, best.prim = pend
                        best.prim = pend;
                        best.sub = j;   // in.pad + the BLAS's own slot
                        best.side = side;
                    } else {
                        best.prim = j;
                        if (p.kind == RT_PRIM_INSTANCE) best.sub = sub;
                        best.side = side;
                    }
                }
            }
            cur = pop();
            RT_STAMP(cnt.t_leaves, tp);
        } else if (!blas && pend >= 0) {
            // the deferred instance (the scene's one instance over a BVH, staged in LDS): its BLAS
            // walked in object space with the walk's t_max
            const rt_instance& in = *reinterpret_cast<const rt_instance*>(lds_inst);
            instance_ray(in, r);
            finish_ray<C>(r, S.has_spheres != 0);
            t_max = any ? best.t : (R)RT_INF;
            tmax_f = f32_up(t_max);
            blas = true;
            base = in.pad;
            sp = stack0;
            push(RT_DONE);
            cur = root_ref(in.child);
            RT_STAMP(cnt.t_defer, tp);
        } else {
            __builtin_nontemporal_store(best.t, &ht[pos]);
            typedef int i2w __attribute__((ext_vector_type(2)));
            const i2w hv = {any ? best.prim : -1, (best.sub << 3) | (best.side & 7)};
            __builtin_nontemporal_store(hv, reinterpret_cast<i2w*>(&hp[pos]));
            busy = false;
            RT_STAMP(cnt.t_rec, tp);
        }
    }
    if (C::COUNT) {
        atomicAdd(&counters[0], (unsigned long long)cnt.casts);
        atomicAdd(&counters[1], (unsigned long long)cnt.nodes);
        atomicAdd(&counters[2], (unsigned long long)cnt.prims);
        atomicAdd(&counters[6], (unsigned long long)cnt.wave_steps);
        atomicAdd(&counters[7], (unsigned long long)cnt.wave_nodes);
        atomicAdd(&counters[10], (unsigned long long)cnt.wave_leaves);
        atomicAdd(&counters[13], (unsigned long long)cnt.shade_lanes);
        atomicAdd(&counters[8], (unsigned long long)cnt.t_nodes);
        atomicAdd(&counters[9], (unsigned long long)cnt.t_leaves);
        atomicAdd(&counters[17], (unsigned long long)cnt.t_rec);
        atomicAdd(&counters[20], (unsigned long long)cnt.t_refill);
        atomicAdd(&counters[22], (unsigned long long)cnt.t_defer);
        atomicAdd(&counters[15], (unsigned long long)cnt.t_setup);
        atomicAdd(&counters[16], (unsigned long long)cnt.t_pre);
        if (lane == 0) atomicAdd(&counters[21], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
    }
}

// ---------------------------------------------------------------------------------------------
// wf_logic
// ---------------------------------------------------------------------------------------------
template <class C>
__global__ void __launch_bounds__(kWfLogicThreads) wf_logic(SceneDev S, const KParams* __restrict__ Pp, WfPaths W,
                                                           double* __restrict__ samples, unsigned* __restrict__ work,
                                                           int iter)
{
    using R = double;
    const KParams& P = *Pp;
    stage_lds<C>(S);   // the material and texture tables (S: no nodes, no BLAS, no stack)
    if (blockIdx.x == 0 && threadIdx.x < kWfShards) W.tctr[threadIdx.x] = 0u;   // this iteration's wf_trace
    if (blockIdx.x == 0 && threadIdx.x == kWfShards) W.flag[(iter + kWfFlags / 2) % kWfFlags] = 0;
    const uint32_t n = (uint32_t)W.n;
    const uint32_t slot = blockIdx.x * kWfLogicThreads + threadIdx.x;   // the grid covers n exactly
    const uint32_t w = slot >> 6;
    const int lane = threadIdx.x & 63;
    // the last iteration's queue (parity ^ 1: its rays and hits) and this one's (parity)
    const size_t lo = (size_t)((iter & 1) ^ 1) * n, cu = (size_t)(iter & 1) * n;
    const int32_t st = W.st[slot];
    const bool traced = st >= 0;   // the slot's ray was queued and traced in the last iteration
    int depth = st;
    double cr = 0.0, cg = 0.0, cb = 0.0;   // the sample's radiance (one emission or the background)
    R Tr = (R)1, Tg = (R)1, Tb = (R)1;
    rt_pstream rs{0u, 0u, 0u, 0u};
    RayT<R> r;
    HitT<R> h;
    bool pending = false, ended = false;
    int x = 0, k = 0, s = 0;
    uint32_t pixel = 0;
    // the slot's state in one round of loads (whether or not it holds a path: no load waits on st)
    const uint32_t qp = W.qpos[slot];
    const double T0 = W.T[slot], T1 = W.T[n + slot], T2 = W.T[2 * n + slot];
    const uint4 q = W.rng[slot];
    if (traced) {
        Tr = T0; Tg = T1; Tb = T2;
        rs.s0 = q.x; rs.s1 = q.y; rs.s2 = q.z; rs.s3 = q.w;
        // the slot's queue entry: its ray, key and hit (one dependent round of loads)
        const size_t e = lo + qp;
        const int2 hp = W.hp[e];
        const uint4 kq = W.qkey[e];
        pixel = kq.x;
        s = (int)kq.y;
        r.ox = W.qo[3 * lo + qp]; r.oy = W.qo[3 * lo + n + qp]; r.oz = W.qo[3 * lo + 2 * n + qp];
        r.dx = W.qd[3 * lo + qp]; r.dy = W.qd[3 * lo + n + qp]; r.dz = W.qd[3 * lo + 2 * n + qp];
        r.time = W.qtime[e];
        const double t_hit = W.ht[e];
        if (hp.x < 0) {   // main.rs:37: the background
            cr = cr + Tr * P.bg[0];
            cg = cg + Tg * P.bg[1];
            cb = cb + Tb * P.bg[2];
            ended = true;
        } else {
            r.a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;   // finish_ray's |d|^2 (shade_end's 1/sqrt)
            HitRefT<R> best;
            best.t = t_hit;
            best.prim = hp.x;
            best.sub = hp.y >> 3;
            best.side = hp.y & 7;
            finish_hit<C>(S, r, best, h);
            pending = shade_begin<C>(S, h, Tr, Tg, Tb, cr, cg, cb);   // false: a DiffuseLight ended it
            ended = !pending;
        }
    }
    auto record = [&](double vr, double vg, double vb) {   // the sample's slot of the per-sample buffer
        double* o = samples + tiled_record(P.tiles_x, P.spp - P.sample_begin, x, k, s - P.sample_begin) * 3;
        o[0] = vr;
        o[1] = vg;
        o[2] = vb;
    };
    auto load_unit = [&]() {   // (s and pixel came with the queue entry)
        const int2 xk = W.xk[slot];
        x = xk.x;
        k = xk.y;
    };
    if (ended) {
        load_unit();
        record(cr, cg, cb);
    }

    // ---- a slot with no path takes the next unit of its wave's work block (the per-sample pool's
    // refill, trace_pool): a block is one 8x8 tile x block_samples samples, units sample-major
    const unsigned n_tiles = (unsigned)P.tiles_x * (unsigned)P.tiles_y;
    const unsigned group = (unsigned)P.block_samples;
    int4 wb = W.wblk[w];
    unsigned blk = __builtin_amdgcn_readfirstlane((unsigned)wb.x);
    unsigned blk_next = __builtin_amdgcn_readfirstlane((unsigned)wb.y);
    unsigned blk_units = __builtin_amdgcn_readfirstlane((unsigned)wb.z);
    bool exhausted = __builtin_amdgcn_readfirstlane(wb.w) != 0;
    unsigned nvalid = 64;
    int tx0 = 0, tk0 = 0, vw = 8, s0 = 0;
    auto decode = [&](unsigned b) {
        const unsigned grp = b / n_tiles, tile = b - grp * n_tiles;
        tx0 = (int)(tile % (unsigned)P.tiles_x) * 8;
        tk0 = (int)(tile / (unsigned)P.tiles_x) * 8;
        vw = min(8, P.width - tx0);
        nvalid = (unsigned)(vw * min(8, P.n_rows - tk0));
        s0 = P.sample_begin + (int)(grp * group);
    };
    if (blk_next < blk_units) decode(blk);
    bool want = !pending;   // no path in the slot now
    bool new_sample = false;
    uint64_t need = __ballot(want);
    while (need != 0 && !exhausted) {
        if (blk_next == blk_units) {
            unsigned b = 0;
            if (lane == 0) b = atomicAdd(work, 1u);
            b = __builtin_amdgcn_readfirstlane(b);
            if (b >= P.n_work_blocks) {
                exhausted = true;
                break;
            }
            blk = b;
            decode(b);
            blk_units = nvalid * (unsigned)(min(P.spp, s0 + (int)group) - s0);
            blk_next = 0;
        }
        const unsigned rank = lanes_below(need);
        const unsigned take = min((unsigned)__popcll(need), blk_units - blk_next);
        if (want && rank < take) {
            const unsigned u = blk_next + rank;
            unsigned si;
            if (nvalid == 64u) {   // a full 8x8 tile: shifts, not divisions
                si = u >> 6;
                x = tx0 + (int)(u & 7u);
                k = tk0 + (int)((u >> 3) & 7u);
            } else {
                si = u / nvalid;
                const unsigned pp = u - si * nvalid;
                x = tx0 + (int)(pp % (unsigned)vw);
                k = tk0 + (int)(pp / (unsigned)vw);
            }
            s = s0 + (int)si;
            want = false;
            new_sample = true;
        }
        blk_next += take;
        need = __ballot(want);
    }
    if (lane == 0) W.wblk[w] = make_int4((int)blk, (int)blk_next, (int)blk_units, exhausted ? 1 : 0);

    // ---- ray generation: camera rays of new samples and scattered rays of pending hits, their
    // random_in_unit_disk / random_in_unit_sphere tries in one rejection loop (trace_pool)
    R u = (R)0, v = (R)0;
    if (new_sample) {
        int ix, y;
        image_xy(P, x, k, ix, y);
        pixel = (uint32_t)y * (uint32_t)P.img_width + (uint32_t)ix;
        ds_start(rs, P.seed, pixel, (uint32_t)s);
        camera_begin(P, ix, y, rs, u, v);
        Tr = Tg = Tb = (R)1;
        depth = P.max_depth;
    }
    const bool tries = new_sample || (pending && shade_draws<C>(S, h.mat));
    R qx = (R)0, qy = (R)0, qz = (R)0, l2 = (R)1;
    const bool three = !new_sample;
    while (tries && !unit_try(rs, (R)P.scale_m11, three, qx, qy, qz, l2)) {
    }
    bool go = false;
    if (new_sample) {
        camera_end(P, rs, u, v, qx, qy, r);
        go = true;
    } else if (pending) {
        go = shade_end<C, false>(S, h, r, rs, Tr, Tg, Tb, qx, qy, qz, l2);
        if (go) depth -= 1;
    }
    const bool has = new_sample || pending;
    const bool live = has && go && depth > 0;   // main.rs:21-23: depth 0 is black
    if (has && !live) {   // absorbed (Metal), or out of depth: the sample's radiance is 0
        if (!new_sample) load_unit();
        record(0.0, 0.0, 0.0);
    }
    const uint64_t lm = __ballot(live);
    if (live) {   // the ray goes to this wave's segment of this iteration's queue
        const uint32_t qp = (w << 6) + lanes_below(lm);
        W.qo[3 * cu + qp] = r.ox; W.qo[3 * cu + n + qp] = r.oy; W.qo[3 * cu + 2 * n + qp] = r.oz;
        W.qd[3 * cu + qp] = r.dx; W.qd[3 * cu + n + qp] = r.dy; W.qd[3 * cu + 2 * n + qp] = r.dz;
        W.qtime[cu + qp] = r.time;
        W.qkey[cu + qp] = make_uint4(pixel, (uint32_t)s, (uint32_t)(P.max_depth - depth), slot);
        W.qpos[slot] = qp;
        W.T[slot] = Tr; W.T[n + slot] = Tg; W.T[2 * n + slot] = Tb;
        W.rng[slot] = make_uint4(rs.s0, rs.s1, rs.s2, rs.s3);
        if (new_sample) W.xk[slot] = make_int2(x, k);
    }
    if (live || traced) W.st[slot] = live ? depth : -1;
    if (lane == 0) {
        W.qn[w] = (uint32_t)__popcll(lm);
        if (lm != 0) W.flag[iter % kWfFlags] = 1;
    }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
using WfTraceC = WfCfg<FEAT_SET_FINAL, true, true, true, false, kWfTraceThreads>;
using WfTraceCountC = WfCfg<FEAT_SET_FINAL, true, true, true, true, kWfTraceThreads>;
using WfLogicC = WfCfg<FEAT_SET_FINAL, true, false, false, false, kWfLogicThreads>;

static size_t wf_trace_lds(const SceneDev& S)
{
    return (size_t)(S.n_tlas_nodes + S.n_blas_bfs) * sizeof(LdsNode) + sizeof(rt_instance) +
           (size_t)S.stack_entries * kWfTraceThreads * sizeof(int);
}

bool wavefront_fits(const SceneDev& S, size_t lds_per_block)
{
    return S.n_tlas_nodes > 0 && wf_trace_lds(S) <= lds_per_block;
}

hipError_t launch_wavefront(const SceneDev& S, const KParams& Ph, const KParams* P, double* out, unsigned* work,
                            const WfPaths& W, unsigned long long* counters, bool count, WfHost& host,
                            hipStream_t stream)
{
    host.iterations = 0;
    if (W.n <= 0 || (W.n % (kWfLogicThreads * kWfShards)) != 0) return hipErrorInvalidValue;
    const unsigned long long units = (unsigned long long)Ph.tiles_x * Ph.tiles_y * 64ull *
                                     (unsigned long long)(Ph.spp - Ph.sample_begin);
    if (units == 0) return hipSuccess;
    hipError_t e;
    if ((e = hipMemsetAsync(W.st, 0xff, (size_t)W.n * sizeof(int32_t), stream)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(W.wblk, 0, (size_t)(W.n / 64) * sizeof(int4), stream)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(W.flag, 0, kWfFlags * sizeof(int32_t), stream)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(work, 0, sizeof(unsigned), stream)) != hipSuccess) return e;

    SceneDev SL = S;   // the logic kernel's LDS: the material and texture tables only
    SL.n_lds_nodes = 0;
    SL.n_lds_blas = 0;
    const size_t lds_logic = (size_t)SL.n_lds_materials * 64 + (size_t)SL.n_lds_textures * 96;
    const size_t lds_trace = wf_trace_lds(S);
    auto trace = count ? wf_trace<WfTraceCountC> : wf_trace<WfTraceC>;
    int per_cu = 0, cus = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, trace, kWfTraceThreads, lds_trace) != hipSuccess ||
        per_cu <= 0)
        return hipErrorNotSupported;
    host.waves_per_simd = per_cu * kWfTraceThreads / 256;
    // a multiple of the shard count: every shard's segments have their own waves
    const unsigned trace_blocks = (unsigned)std::max(kWfShards, cus * per_cu / kWfShards * kWfShards);
    const unsigned logic_blocks = (unsigned)(W.n / kWfLogicThreads);
    // an upper bound on the iterations (a path casts at most max_depth rays; a slot waits at most
    // one iteration between two paths), so a fault in the loop cannot spin forever
    const long long max_iter = (long long)((units + (unsigned long long)W.n - 1) / (unsigned long long)W.n) *
                                   (2LL * Ph.max_depth + 4) + 64;
    int it = 0, chunk = 0;
    for (;;) {
        for (int j = 0; j < RT_WF_CHUNK; ++j, ++it) {
            hipLaunchKernelGGL(wf_logic<WfLogicC>, dim3(logic_blocks), dim3(kWfLogicThreads), lds_logic, stream, SL, P,
                               W, out, work, it);
            hipLaunchKernelGGL(trace, dim3(trace_blocks), dim3(kWfTraceThreads), lds_trace, stream, S, P, W, counters,
                               it & 1);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        // the flag of this chunk's last iteration, read by the host one chunk later (pipelined)
        if ((e = hipMemcpyAsync((void*)&host.flag_host[chunk & 1], &W.flag[(it - 1) % kWfFlags], sizeof(int32_t),
                                hipMemcpyDeviceToHost, stream)) != hipSuccess)
            return e;
        if ((e = hipEventRecord(host.ev[chunk & 1], stream)) != hipSuccess) return e;
        if (chunk > 0) {
            if ((e = hipEventSynchronize(host.ev[(chunk - 1) & 1])) != hipSuccess) return e;
            if (host.flag_host[(chunk - 1) & 1] == 0) break;   // no path left after that chunk
        }
        ++chunk;
        if (it > max_iter) return hipErrorLaunchFailure;
    }
    host.iterations = it;
    return hipSuccess;
}

}  // namespace rtk
