// trace_device.hpp — the MI355X megakernel for the reference's per-(pixel, sample)
// hot path: Camera::get_ray (camera.rs:58-66) + ray_color (main.rs:19-38) and
// everything below it (hittable.rs, material.rs, texture.rs, perlin.rs), in f64
// like the reference (math.rs:13-17).
//
// Execution model:
//   * work unit = one (pixel, sample) path; work block = one 8x8 pixel tile x one chunk
//     of spp_chunk samples (a function of spp only);
//   * trace_pool (default): persistent waves take blocks from a device counter, and a
//     lane whose path ended takes the block's next unit in the same bounce-loop
//     iteration (ballot + mbcnt), so lanes do not idle until the last blocks run out;
//     each sample's radiance goes to its slot of a per-sample buffer (tiled) and
//     reduce_samples sums every pixel's samples in sample order, chunk by chunk — the
//     image does not depend on which lane computed a sample, on the launch geometry or
//     on how rows are sharded over GPUs; trace_chunks (the first schedule, kept for A/B)
//     gives a lane one pixel's chunk and adds the same partial sums;
//   * the depth-50 recursion is an iterative bounce loop; traversal carries only
//     (t, primitive slot); the HitRecord (hittable.rs:6-27) is built once per cast;
//   * TLAS nodes and the traversal stack in LDS, conservative f32 slab tests, f64
//     primitive tests; materials share their expensive steps so a wave holding several
//     kinds runs each step once;
//   * RNG: per (pixel, sample) a Philox4x32-10 block seeds a xoshiro128++ path stream
//     (rt_numerics.h); the medium's in-hit draw is keyed by (pixel, sample, bounce, medium id).
// Built with -ffp-contract=off: bit-for-bit the operation order of the reference.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "rt/rt_numerics.h"
#include "rt/rt_scene.h"
#include "trace_kernel.hpp"

namespace rtk {

// R: the path's arithmetic type — double (the reference's f64, math.rs:13-17; path-identical
// to the oracle: the same rays, hits and draws, per-pixel means within last-ulp summation
// differences) or float (the f32 fast mode; statistically equal).
typedef float f2v __attribute__((ext_vector_type(2)));
template <class R>
struct RayT {
    R ox, oy, oz;
    R dx, dy, dz;
    R time;
    R a;                      // length_squared(direction)
    R ya;                     // f64: 1 / a correctly rounded (NaN outside [2^-900, 2^900]: see div_rcp)
    R ix, iy, iz;             // 1 / direction (f64 slab tests only)
    R yx, yy, yz;             // f64, scenes with rects: RN(1 / direction) for div_rcp (NaN outside its range)
    // f32 slab terms per axis (f32 slab tests only): (1 / direction, -origin * (1 / direction)),
    // a register pair each, so one v_pk_fma_f32 takes both for the two children of a node
    // (op_sel: the pair's low half as the factor, its high half as the addend, in both lanes)
    f2v sx, sy, sz;
    uint32_t onx, ony, onz;   // byte offsets in a node of child 0's near planes (by direction sign)
};

// The HitRecord of hittable.rs:6-27 (uv deferred to texture lookup: uvkind 1 keeps the
// object-space outward normal for sphere_uv, 2 keeps (x-a0, a1-a0, y-b0, b1-b0)).
template <class R>
struct HitT {
    R t, px, py, pz, nx, ny, nz;
    R uv0, uv1, uv2, uv3;
    int front, mat, uvkind;
};
using Hit = HitT<double>;

// What traversal keeps per candidate: the parameter and which primitive produced it.
template <class R>
struct HitRefT {
    R t;
    int prim;   // prim index (top level)
    int sub;    // instance: BLAS prim index; box: winning side (0..5)
    int side;   // box inside an instance: winning side
};

struct Keyed {                 // coordinates of the medium's keyed draw
    uint64_t seed;
    uint32_t pixel, sample, bounce;
};

struct Count {
    uint32_t casts, nodes, prims;
    uint32_t wave_steps, wave_nodes;  // loop iterations the wave executed (counted by its first active lane)
    uint32_t wave_leaves;             // leaf-loop iterations the wave executed
    uint32_t cam_lanes, cam_steps;    // lanes starting a sample / iterations in which any did
    uint32_t shade_lanes, shade_steps;
    uint64_t t_nodes, t_leaves;       // wave-cycles in node-visit loops / leaf tests (same in every lane)
    // pool kernels, finer phases (wave-cycles; each added by the first active lane of the region
    // it times, so summed over lanes they are wave totals): ray set-up, the walk's prologue
    // (pre-leaf test, bounds), the hit record, and inside the leaf tests the media and instances
    uint64_t t_setup, t_pre, t_rec, t_med, t_inst, t_refill, t_defer;
    // ray generation split (pool kernels): path seeding + camera jitter, the rejection loop
    uint64_t t_seed, t_tries;
    // pool kernels, why a lane of a bounce-loop iteration casts no ray (with casts they add up to
    // 64 x wave_steps): no unit left to take (the launch's tail), every ring slot holding an
    // unfinished block (RING), a path that ended in its scatter (the material absorbed it), the
    // depth cap, a rejection loop left for the next iteration (RT_TRY_LEFT)
    uint32_t idle_tail, idle_ring, no_scatter, depth_cap, try_wait;
};
// COUNT phase stamps: tp is the lane's last stamp; the first active lane adds the interval
#define RT_STAMP(acc, tp)                                                   \
    do {                                                                    \
        if (C::COUNT) {                                                     \
            const uint64_t t_ = __builtin_amdgcn_s_memtime();               \
            if (first_active_lane()) (acc) += t_ - (tp);                    \
            (tp) = t_;                                                      \
        }                                                                   \
    } while (0)
// COUNT only: true in exactly one active lane of the wave
__device__ __forceinline__ bool first_active_lane()
{
    return (int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1;
}

// Compile-time kernel configuration (one instantiation per variant):
//   F      scene features the variant handles (trace_kernel.hpp FEAT_*); code for the
//          others is not emitted, which keeps register pressure and code size down
//   S32    conservative f32 slab tests (boxes padded on the host, see flatten.cpp)
//   LDS    traversal stack in LDS (interleaved per lane) instead of scratch
//   COUNT  diagnostic: count casts / node visits / primitive tests and time the phases
// Traversal is while-while (Aila & Laine 2009); the if-if form, speculative while-while and
// a per-lane state machine with ballot-gated shading all measured slower (DESIGN.md §5.2;
// the rejected experiments are kept as patches under scripts/experiments/).
//   NALL   every TLAS node is in LDS (no per-node LDS/global choice)
#ifndef RT_RECT_RCP
#define RT_RECT_RCP 1   // rect / box tests divide through the ray's reciprocals (rects + instances variant only): round 3, without machine LICM, Cornell 800x800x200 45.76 vs 47.04 ms (r03d_ab_c3.log); round 2 measured it slower (58.1 vs 56.5) when its registers spilled
#endif
#ifndef RT_BOX_RCP
#define RT_BOX_RCP 1   // a Box's six sides divide through three per-box reciprocals (BoxRcp)
#endif
#ifndef RT_TRY_LEFT
// pool schedules: the wave leaves its rejection loop (random_in_unit_disk /
// random_in_unit_sphere tries, math.rs:51-76) once at most RT_TRY_LEFT lanes still reject, after
// at least RT_TRY_MIN tries; those lanes keep their stream position and candidate state and go
// on drawing in the next bounce-loop iteration instead of tracing in this one. Each lane's draws
// stay in its own stream order, so the bits do not change; the wave no longer runs as many
// tries as its unluckiest lane (E[max of 64 geometric(0.52)] ~ 6.9 against a mean of 1.9).
// 0: the loop runs until every lane accepted (round 3). C2 1200x800x100 (profiles/r04b_ab_c2.log):
// off 15.28 ms, 2 15.12, 4 15.07, 8 15.37, 4 after one try 15.22; images identical.
#define RT_TRY_LEFT 4
#endif
#ifndef RT_TRY_MIN
#define RT_TRY_MIN 2
#endif
// the variants the cap applies to: the spheres ones (C2, C5) and the Cornell box's (C3 800x800x200
// 46.00 -> 45.80 ms, profiles/r04d_ab_c3.log). The final scene's is 1-2 % slower with it (C4
// 1920x1080x100 106.84 -> 109.04 ms, r04c_ab_c4.log; 107.83 -> 109.19, r04d_ab_c4.log): its
// iterations are long, so a lane that sits one out loses more than the wave saves on tries
template <class C>
constexpr bool TryLeft() { return RT_TRY_LEFT > 0 && (C::F == FEAT_SET_SPHERES || C::F == FEAT_SET_RECTINST); }
//   F32    the f32 fast mode (Real = float): statistically, not bitwise, equal
template <uint32_t F_, bool S32_, bool LDS_, bool NALL_, bool COUNT_, bool F32_ = false>
struct Cfg {
    static constexpr uint32_t F = F_;
    static constexpr bool S32 = S32_;
    static constexpr bool LDS = LDS_;
    static constexpr bool NALL = NALL_;
    static constexpr bool COUNT = COUNT_;
    static constexpr bool F32 = F32_;
    // threads per workgroup (RT_BLOCK_FINAL): a property of the launched kernel, inherited by the
    // reduced configurations of nested code (CfgDrop), which share its LDS stack
    static constexpr int BT = block_threads_of(F_, F32_, RT_STACK16 && LDS_ && NALL_ && S32_);
    using Real = typename std::conditional<F32_, float, double>::type;
};

// The configuration of code reached only through an instance or a medium boundary: the
// feature bits the scene does not need there are dropped (FEAT_INST_RECT / FEAT_MEDIUM_INST
// clear), so e.g. the final scene's instanced BLAS of spheres compiles the sphere test only.
// threads per workgroup (RT_BLOCK_FINAL; the LDS stack's lane stride)
template <class C>
constexpr int BlockThreads() { return C::BT; }

template <class C, uint32_t DROP>
struct CfgDrop : C {
    static constexpr uint32_t F = C::F & ~DROP;
};
// Spheres reached only through an instance or a medium boundary are static unless the scene
// says otherwise (FEAT_NEST_MOVING): their test then loads no velocity (FEAT_STATIC; the final
// scene's instanced cluster and its fog / glass-medium boundaries), which shortens the nested
// walk's live ranges; c0 + 0 * s is c0 bit for bit, so the result is the same.
template <class C, uint32_t DROP>
struct CfgDropStatic : C {
    static constexpr uint32_t F = (C::F & ~DROP) | ((C::F & FEAT_NEST_MOVING) ? 0u : (uint32_t)FEAT_STATIC);
};
template <class C>
using InstC = CfgDropStatic<C, (C::F & FEAT_INST_RECT) ? 0u : (uint32_t)FEAT_RECT>;
template <class C>
using BoundC = CfgDropStatic<C, FEAT_INST_MEDIUM | ((C::F & FEAT_MEDIUM_INST) ? 0u : (uint32_t)(FEAT_RECT | FEAT_INST))>;
template <class C>
using InstMedC = CfgDropStatic<C, FEAT_INST_MEDIUM>;   // a medium under an instance: no medium below it

// Traversal stack. LDS: a lane-interleaved dynamic LDS array [entry][block threads]
// (consecutive lanes hit consecutive banks) sized per scene by the host (TLAS depth +
// BLAS depth); scratch: a private array (deep scenes).
extern __shared__ int rt_lds[];  // [cached TLAS nodes] [stack entries x block lanes] [materials, textures]
// The lane's index in its wave, recomputed where it is used (volatile: not CSE'd into one
// value that stays live through the bounce loop; at 128 VGPRs the final variant spilled the
// stack base it replaces and reloaded it from scratch at every walk)
__device__ __forceinline__ int lane_remat()
{
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
template <bool LDS, bool REMAT = false, int BT = 256>
struct Stack;
template <int BT>
struct Stack<true, true, BT> {   // the variants with nested walks (128 VGPRs)
    int wave0;   // rt_lds index of this wave's lane 0, entry 0 (wave-uniform: an SGPR)
    __device__ __forceinline__ int& operator[](int i) const { return rt_lds[wave0 + lane_remat() + i * BT]; }
    __device__ __forceinline__ void init(int stack_off)
    {
        wave0 = stack_off + __builtin_amdgcn_readfirstlane((int)threadIdx.x & ~63);
    }
};
template <int BT>
struct Stack<true, false, BT> {   // (Cornell variants: the remat costs 0.3-0.9 %, nothing spills)
    int* base;
    __device__ __forceinline__ int& operator[](int i) const { return base[i * BT]; }
    __device__ __forceinline__ void init(int stack_off) { base = rt_lds + stack_off + threadIdx.x; }
};
template <int BT>
struct Stack<false, false, BT> {
    int v[66];   // 32 + 32 entries + the two walks' RT_DONE sentinels
    __device__ __forceinline__ int& operator[](int i) { return v[i]; }
};
#ifndef RT_STACK16
// 16-bit LDS stack entries in the spheres variant with the whole TLAS in LDS: its 35 KB of LDS
// per block (22.7 KB of node records + a 12-entry 32-bit stack) let only 4 blocks share a CU's
// 160 KB; with 6.1 KB of stack 5 blocks fit, and the variant runs at 5 waves per SIMD (96
// VGPRs, min_waves) — C2 1200x800x100 16.48 -> 15.40 ms, same bits (profiles/r02ao_*)
#define RT_STACK16 1
#endif
template <int BT>
struct Stack16 {   // node records at LDS addresses < 32 KB, leaf codes > -32768 (SceneDev.stack16_ok)
    short* base;
    __device__ __forceinline__ short& operator[](int i) const { return base[i * BT]; }
};
// (the final-scene variant with 16-bit entries measured ~7 % slower: C4 1920x1080x100 142.1 vs
// 132.7 ms, r03f_ab_c4.log; the spheres variant only)
template <class C>
constexpr bool Stack16Cfg()
{
    return RT_STACK16 && C::LDS && C::NALL && C::S32 && C::F == FEAT_SET_SPHERES;
}
template <class C>
using StackT = typename std::conditional<Stack16Cfg<C>(), Stack16<BlockThreads<C>()>,
                                         Stack<C::LDS, C::LDS && (C::F & FEAT_INST_BLAS) != 0, BlockThreads<C>()>>::type;

// Division by a value b used many times, through its correctly rounded reciprocal
// y = RN(1/b): q0 = RN(q*y), then one correction q1 = RN(q0 + RN-exact(q - b*q0) * y).
// With y correctly rounded this is Markstein's theorem (IBM J. R&D 34(1), 1990): q1 =
// RN(q/b), bit for bit what `q / b` gives, barring overflow / underflow in the products,
// which the range guard on b excludes (y is NaN outside it, and the division runs then);
// checked on 8e8 random and adversarial pairs on the host (all-ones / power-of-two
// significands, both signs, exponents -20..20). A zero q may come out as -0 where q / b
// gives +0 or the reverse; every caller compares the quotient with t_min > 0 first or
// has q, b >= 0, so the sign of a zero quotient changes nothing.
__device__ __forceinline__ double rcp_for_div(double b)
{
    const double m = __builtin_fabs(b);
    return (m >= 0x1.0p-900 && m <= 0x1.0p+900) ? 1.0 / b : __builtin_nan("");
}
__device__ __forceinline__ double div_rcp(double q, double b, double y)
{
    const double q0 = q * y;
    const double q1 = __builtin_fma(__builtin_fma(-b, q0, q), y, q0);
    if (__builtin_expect(q1 != q1, 0)) return q / b;  // y outside the guard (or q not finite)
    return q1;
}

__device__ __forceinline__ float f32_inv_dir(double d)
{
    // an exact 0 would give inf * 0 = NaN in the slab products; a 1e-30 component keeps the
    // interval of a ray parallel to a slab finite and correct (inside: huge, outside: empty)
    float f = (float)d;
    if (__builtin_fabsf(f) < 1e-30f) f = __builtin_copysignf(1e-30f, f);
    return __builtin_amdgcn_rcpf(f);
}

// ---- precision-generic helpers: double = the reference's libm restated (rt_numerics.h,
// bit-identical host/device), float = the device's f32 functions (f32 mode only)
__device__ __forceinline__ double r_sqrt(double x) { return __builtin_sqrt(x); }
__device__ __forceinline__ float r_sqrt(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ double r_fabs(double x) { return __builtin_fabs(x); }
__device__ __forceinline__ float r_fabs(float x) { return __builtin_fabsf(x); }
__device__ __forceinline__ double r_floor(double x) { return __builtin_floor(x); }
__device__ __forceinline__ float r_floor(float x) { return __builtin_floorf(x); }
__device__ __forceinline__ double r_fmin(double a, double b) { return fmin(a, b); }
__device__ __forceinline__ float r_fmin(float a, float b) { return fminf(a, b); }
__device__ __forceinline__ double r_sin(double x) { return rt_sin(x); }
__device__ __forceinline__ float r_sin(float x) { return sinf(x); }
__device__ __forceinline__ double r_log(double x) { return rt_log(x); }
__device__ __forceinline__ float r_log(float x) { return logf(x); }
__device__ __forceinline__ double r_acos(double x) { return rt_acos(x); }
__device__ __forceinline__ float r_acos(float x) { return acosf(x); }
__device__ __forceinline__ double r_atan2(double y, double x) { return rt_atan2(y, x); }
__device__ __forceinline__ float r_atan2(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ double r_pow5(double x) { return rt_pow5(x); }
__device__ __forceinline__ float r_pow5(float x) { const float x2 = x * x; return x2 * x2 * x; }
template <class R>
__device__ __forceinline__ int32_t r_sat_i32(R x) { return rt_sat_i32((double)x); }
template <class R>
__device__ __forceinline__ uint64_t r_sat_u64(R x) { return rt_sat_u64((double)x); }

// Rect / box tests divide through the ray's correctly rounded reciprocals (div_rcp, same
// bits, 3 FMAs instead of an f64 division per face): in the rects + instances variant only —
// the media and final-scene variants would spill the 6 VGPRs the reciprocals hold.
template <class C>
constexpr bool RectRcp()
{
    return RT_RECT_RCP && !C::F32 && (C::F & FEAT_RECT) != 0 && (C::F & (FEAT_MEDIUM | FEAT_NOISE | FEAT_IMAGE)) == 0;
}

// A Box's six sides through three per-box reciprocals (box_t): in the variants with Perlin or
// image textures (final scene: 80.0 -> 78.6 ms), whose 3 waves per SIMD the extra live values do
// not change; the 4-wave Cornell variant spills them (49.6 -> 51.6 ms) and Cornell smoke's
// media variant loses too (39.1 -> 39.5; profiles/r02_ab_boxrcp_*.log)
#ifndef RT_BOX_RCP_ALL
#define RT_BOX_RCP_ALL 0
#endif
template <class C>
constexpr bool BoxRcp()
{
    return RT_BOX_RCP && !C::F32 && (RT_BOX_RCP_ALL || (C::F & (FEAT_NOISE | FEAT_IMAGE)) != 0);
}

// spheres: the scene has spheres (wave-uniform); otherwise no root division needs 1/a.
// SLABS = false: no node-slab terms (a ray that meets one primitive, e.g. an instance's child)
template <class C, bool SLABS = true>
__device__ __forceinline__ void finish_ray(RayT<typename C::Real>& r, bool spheres)
{
    r.a = r.dx * r.dx + r.dy * r.dy + r.dz * r.dz;
    if constexpr (!C::F32) r.ya = (C::F == FEAT_SET_SPHERES || spheres) ? rcp_for_div(r.a) : __builtin_nan("");
    if constexpr (RectRcp<C>()) {
        r.yx = rcp_for_div(r.dx);
        r.yy = rcp_for_div(r.dy);
        r.yz = rcp_for_div(r.dz);
    }
    if constexpr (!SLABS) {
    } else if constexpr (C::S32) {
        r.sx.x = f32_inv_dir(r.dx);
        r.sy.x = f32_inv_dir(r.dy);
        r.sz.x = f32_inv_dir(r.dz);
        r.sx.y = -(float)r.ox * r.sx.x;
        r.sy.y = -(float)r.oy * r.sy.x;
        r.sz.y = -(float)r.oz * r.sz.x;
        // the LDS node (LdsNode): per axis [lo0 lo1 hi0 hi1 lo0 lo1] at bytes 0/24/48; the
        // near planes of both children at +0 (direction >= 0) or +8, the far ones 8 bytes on
        r.onx = r.sx.x >= 0.0f ? 0u : 8u;
        r.ony = r.sy.x >= 0.0f ? 24u : 32u;
        r.onz = r.sz.x >= 0.0f ? 48u : 56u;
    } else {
        r.ix = (typename C::Real)1 / r.dx;
        r.iy = (typename C::Real)1 / r.dy;
        r.iz = (typename C::Real)1 / r.dz;
    }
}

// hittable.rs:23-26
template <class R>
__device__ __forceinline__ void set_face_normal(HitT<R>& h, R dx, R dy, R dz, R nx, R ny, R nz)
{
    const bool front = dx * nx + dy * ny + dz * nz < (R)0;
    h.front = front;
    h.nx = front ? nx : -nx;
    h.ny = front ? ny : -ny;
    h.nz = front ? nz : -nz;
}

// ---------------------------------------------------------------------------
// primitives: a t-only test (traversal) and a finisher (once per cast)
// ---------------------------------------------------------------------------

// hittable.rs:254-273: the root in [t_min, t_max]
template <bool SMALL = false>
__device__ __forceinline__ bool sphere_t(double cx, double cy, double cz, double radius, const RayT<double>& r,
                                         double t_min, double t_max, double& t)
{
    const double ocx = r.ox - cx, ocy = r.oy - cy, ocz = r.oz - cz;
    const double half_b = ocx * r.dx + ocy * r.dy + ocz * r.dz;
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - radius * radius;
    const double disc = half_b * half_b - r.a * c;
    if (disc < 0.0) return false;
    const double sqrtd = __builtin_sqrt(disc);
    double root = div_rcp(-half_b - sqrtd, r.a, r.ya);
    if (root < t_min || t_max < root) {
        root = div_rcp(-half_b + sqrtd, r.a, r.ya);
        if (root < t_min || t_max < root) return false;
    }
    t = root;
    return true;
}

// A sphere-bounded ConstantMedium's two boundary queries (hittable.rs:430-434: hit over
// (-inf, inf), then over (t1 + 0.0001, inf)) from one quadratic: both calls of sphere_t above
// compute the same discriminant and roots, and differ only in the range the roots are checked
// against, so the pair (t1, t2) is theirs bit for bit; the second discriminant, sqrt and
// division are not computed again (round 5, VERDICT r04 item 6: the final scene's r = 5000
// fog sphere is queried by nearly every cast).
__device__ __forceinline__ bool sphere_t2(double cx, double cy, double cz, double radius, const RayT<double>& r,
                                          double& t1, double& t2)
{
    const double ocx = r.ox - cx, ocy = r.oy - cy, ocz = r.oz - cz;
    const double half_b = ocx * r.dx + ocy * r.dy + ocz * r.dz;
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - radius * radius;
    const double disc = half_b * half_b - r.a * c;
    if (disc < 0.0) return false;   // both queries miss
    const double sqrtd = __builtin_sqrt(disc);
    const double near = div_rcp(-half_b - sqrtd, r.a, r.ya);
    // first query, (-inf, inf): the near root (no double lies outside it; a NaN root passes
    // sphere_t's range test too)
    t1 = near;
    const double lo = t1 + 0.0001;
    if (near < lo || RT_INF < near) {
        const double far = div_rcp(-half_b + sqrtd, r.a, r.ya);
        if (far < lo || RT_INF < far) return false;
        t2 = far;
    } else {
        t2 = near;
    }
    return true;
}

// f32 mode: c = |oc|^2 - r^2 and b/2 = oc . d of a sphere test. c of a large sphere is taken in
// f64 (an f32 c loses everything to cancellation on the r = 1000 ground sphere, whose surface
// every bounce starts on: |oc|^2 ~ 1e6, one f32 ulp 0.06); a small one's in f32, where the
// cancellation costs at most ~r^2 2^-24 (3e-6 at r <= 8), far below the t_min = 0.001 it must
// stay under. The random scene's BVH holds only r <= 1 spheres (its ground is the pre-leaf).
// SMALL: the spheres variant only (in the final-scene variant the second path costs spills).
#ifndef RT_F32_SMALL_SPHERE
#define RT_F32_SMALL_SPHERE 8.0
#endif
// 1: the small-sphere path in every f32 variant. Off: in the final-scene variant it was no faster
// (C4 1920x1080x100 f32 89.82 ms against 89.50 without; with the fast division 87.89 against
// 86.36; profiles/r06t_ab_f32final_c4.log)
#ifndef RT_F32_SMALL_ALL
#define RT_F32_SMALL_ALL 0
#endif
template <bool SMALL = false>
__device__ __forceinline__ void sphere_cb(double cx, double cy, double cz, double radius, const RayT<float>& r,
                                          float& c, float& half_b)
{
    if (SMALL && radius <= RT_F32_SMALL_SPHERE) {
        const float ox = r.ox - (float)cx, oy = r.oy - (float)cy, oz = r.oz - (float)cz;
        const float rf = (float)radius;
        c = (ox * ox + oy * oy + oz * oz) - rf * rf;
        half_b = ox * r.dx + oy * r.dy + oz * r.dz;
        return;
    }
    const double ocx = (double)r.ox - cx, ocy = (double)r.oy - cy, ocz = (double)r.oz - cz;
    c = (float)((ocx * ocx + ocy * ocy + ocz * ocz) - radius * radius);
    half_b = (float)ocx * r.dx + (float)ocy * r.dy + (float)ocz * r.dz;
}

// f32 mode: sphere_t's f32 roots, the same selection (its second query starts at
// t1 + max(1e-4, |t1| 2^-19), medium_t)
__device__ __forceinline__ bool sphere_t2(double cx, double cy, double cz, double radius, const RayT<float>& r,
                                          float& t1, float& t2)
{
    float c, half_b;
    sphere_cb(cx, cy, cz, radius, r, c, half_b);
    const float disc = half_b * half_b - r.a * c;
    if (disc < 0.0f) return false;
    const float q = -(half_b + __builtin_copysignf(__builtin_sqrtf(disc), half_b));
    const float r0 = c / q, r1 = q / r.a;
    const float tn = fminf(r0, r1), tf = fmaxf(r0, r1);
    t1 = tn;
    const float lo = t1 + fmaxf(0.0001f, __builtin_fabsf(t1) * 0x1.0p-19f);
    float root = tn;
    if (root < lo || (float)RT_INF < root) {
        root = tf;
        if (root < lo || (float)RT_INF < root) return false;
    }
    t2 = root;
    return true;
}

// f32 mode: the same roots, robust in f32 (Haines et al., Ray Tracing Gems ch. 7): c as
// sphere_cb takes it, the near root as c / q (Vieta) instead of the cancelling -b - sqrt(disc).
template <bool SMALL = false>
__device__ __forceinline__ bool sphere_t(double cx, double cy, double cz, double radius, const RayT<float>& r,
                                         float t_min, float t_max, float& t)
{
    float c, half_b;
    sphere_cb<SMALL>(cx, cy, cz, radius, r, c, half_b);
    const float disc = half_b * half_b - r.a * c;
    if (disc < 0.0f) return false;
    const float q = -(half_b + __builtin_copysignf(__builtin_sqrtf(disc), half_b));
    const float t0 = c / q, t1 = q / r.a;
    const float tn = fminf(t0, t1), tf = fmaxf(t0, t1);
    float root = tn;
    if (root < t_min || t_max < root) {
        root = tf;
        if (root < t_min || t_max < root) return false;
    }
    t = root;
    return true;
}

// Whether hit records carry the texture coordinates' inputs (uv0..uv3). Without FEAT_IMAGE_UV
// the only image-textured primitives are top-level spheres, whose outward normal — the
// sphere_uv input — is the record's normal, negated back when the hit was on the back face
// (exact): the final scene's records then keep 8 VGPRs fewer live across the bounce loop.
template <class C>
constexpr bool UVStore()
{
    return (C::F & FEAT_IMAGE) != 0 && (C::F & FEAT_IMAGE_UV) != 0;
}

// hittable.rs:275-287
template <class C, class R = typename C::Real>
__device__ __forceinline__ void sphere_finish(R cx, R cy, R cz, R inv_r, const RayT<R>& r, R t, int mat, HitT<R>& h)
{
    h.t = t;
    h.px = r.ox + r.dx * t;
    h.py = r.oy + r.dy * t;
    h.pz = r.oz + r.dz * t;
    const R onx = (h.px - cx) * inv_r, ony = (h.py - cy) * inv_r, onz = (h.pz - cz) * inv_r;
    set_face_normal(h, r.dx, r.dy, r.dz, onx, ony, onz);
    h.mat = mat;
    h.uvkind = 1;
    if constexpr (UVStore<C>()) {
        h.uv0 = onx;
        h.uv1 = ony;
        h.uv2 = onz;
    }
}

// hittable.rs:308-320 (axis 0: XY, k on z; 1: XZ, k on y; 2: YZ, k on x)
template <class R>
__device__ __forceinline__ void rect_axes(int axis, const RayT<R>& r, R& ok, R& dk, R& oa, R& da, R& ob, R& db)
{
    if (axis == 0) { ok = r.oz; dk = r.dz; oa = r.ox; da = r.dx; ob = r.oy; db = r.dy; }
    else if (axis == 1) { ok = r.oy; dk = r.dy; oa = r.ox; da = r.dx; ob = r.oz; db = r.dz; }
    else { ok = r.ox; dk = r.dx; oa = r.oy; da = r.dy; ob = r.oz; db = r.dz; }
}

template <bool RCP = false, class R>
__device__ __forceinline__ bool rect_t(int axis, R a0, R a1, R b0, R b1, R k, const RayT<R>& r, R t_min, R t_max,
                                       R& t_out)
{
    R ok, dk, oa, da, ob, db;
    rect_axes(axis, r, ok, dk, oa, da, ob, db);
    R t;
    if constexpr (RCP) {
        // (k - o) / d through the ray's correctly rounded 1/d: the same bits (div_rcp), 3 FMAs
        // instead of a division per rect (a Box tests 6)
        const R yk = axis == 0 ? r.yz : axis == 1 ? r.yy : r.yx;
        t = div_rcp(k - ok, dk, yk);
    } else {
        t = (k - ok) / dk;
    }
    if (t < t_min || t > t_max) return false;
    const R x = oa + t * da;
    const R y = ob + t * db;
    if (x < a0 || x > a1 || y < b0 || y > b1) return false;
    t_out = t;
    return true;
}

// rect_t with the caller's RN(1 / d_axis), |d_axis| in [2^-900, 2^900] (div_rcp: the division's bits)
__device__ __forceinline__ bool rect_t_y(int axis, double a0, double a1, double b0, double b1, double k,
                                         const RayT<double>& r, double yk, double t_min, double t_max, double& t_out)
{
    double ok, dk, oa, da, ob, db;
    rect_axes(axis, r, ok, dk, oa, da, ob, db);
    const double q = k - ok, q0 = q * yk;   // div_rcp without its guard (the caller checked the range)
    const double t = __builtin_fma(__builtin_fma(-dk, q0, q), yk, q0);
    if (t < t_min || t > t_max) return false;
    const double x = oa + t * da;
    const double y = ob + t * db;
    if (x < a0 || x > a1 || y < b0 || y > b1) return false;
    t_out = t;
    return true;
}
template <class R>
__device__ __forceinline__ bool rect_t_y(int, R, R, R, R, R, const RayT<R>&, R, R, R, R&) { return false; }

// hittable.rs:322-331
template <class C, class R = typename C::Real>
__device__ __forceinline__ void rect_finish(int axis, R a0, R a1, R b0, R b1, const RayT<R>& r, R t, int mat,
                                            HitT<R>& h)
{
    R ok, dk, oa, da, ob, db;
    rect_axes(axis, r, ok, dk, oa, da, ob, db);
    h.uvkind = 2;
    if constexpr (UVStore<C>()) {
        const R x = oa + t * da;
        const R y = ob + t * db;
        h.uv0 = x - a0;
        h.uv1 = a1 - a0;
        h.uv2 = y - b0;
        h.uv3 = b1 - b0;
    }
    h.t = t;
    set_face_normal(h, r.dx, r.dy, r.dz, axis == 2 ? (R)1 : (R)0, axis == 1 ? (R)1 : (R)0, axis == 0 ? (R)1 : (R)0);
    h.mat = mat;
    h.px = r.ox + r.dx * t;
    h.py = r.oy + r.dy * t;
    h.pz = r.oz + r.dz * t;
}

// slab tests of an f32 box (BVH nodes, Box pre-tests)
template <class RayType>
__device__ __forceinline__ bool slab32(const float* lo, const float* hi, const RayType& r, float t_min, float t_max,
                                       float& t_near)
{
    const float x0 = __builtin_fmaf(lo[0], r.sx.x, r.sx.y), x1 = __builtin_fmaf(hi[0], r.sx.x, r.sx.y);
    const float y0 = __builtin_fmaf(lo[1], r.sy.x, r.sy.y), y1 = __builtin_fmaf(hi[1], r.sy.x, r.sy.y);
    const float z0 = __builtin_fmaf(lo[2], r.sz.x, r.sz.y), z1 = __builtin_fmaf(hi[2], r.sz.x, r.sz.y);
    const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), t_min));
    const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), t_max));
    t_near = tn;
    return tn <= tf;
}

// f32 bounds of a double t range, rounded outward
template <class R>
__device__ __forceinline__ float f32_down(R t)
{
    const float f = (float)t;
    return f > 0.0f ? f * (1.0f - 0x1.0p-20f) : f * (1.0f + 0x1.0p-20f);
}
template <class R>
__device__ __forceinline__ float f32_up(R t)
{
    const float f = (float)t;
    return f > 0.0f ? f * (1.0f + 0x1.0p-20f) : f * (1.0f - 0x1.0p-20f);
}

// Conservative slab test against an f32 box (rounded outward and padded on the
// host), in f64. NaN products (0 * inf) are ignored by fmin/fmax.
template <class R>
__device__ __forceinline__ bool slab(const float* lo, const float* hi, const RayT<R>& r, R t_min, R t_max, R& t_near)
{
    const R x0 = ((R)lo[0] - r.ox) * r.ix, x1 = ((R)hi[0] - r.ox) * r.ix;
    const R y0 = ((R)lo[1] - r.oy) * r.iy, y1 = ((R)hi[1] - r.oy) * r.iy;
    const R z0 = ((R)lo[2] - r.oz) * r.iz, z1 = ((R)hi[2] - r.oz) * r.iz;
    const R tn = fmax(fmax(fmin(x0, x1), fmin(y0, y1)), fmax(fmin(z0, z1), t_min));
    const R tf = fmin(fmin(fmax(x0, x1), fmax(y0, y1)), fmin(fmax(z0, z1), t_max));
    t_near = tn;
    return tn <= tf;
}

// the six sides of new_box (hittable.rs:135-142): side -> axis, (a0 a1 b0 b1 k) from min/max
template <class R>
__device__ __forceinline__ void box_side(const rt_prim& p, int side, int& axis, R& a0, R& a1, R& b0, R& b1, R& k)
{
    const R mnx = (R)p.p[0], mny = (R)p.p[1], mnz = (R)p.p[2], mxx = (R)p.p[3], mxy = (R)p.p[4], mxz = (R)p.p[5];
    if (side < 2) { axis = 0; a0 = mnx; a1 = mxx; b0 = mny; b1 = mxy; k = side == 0 ? mxz : mnz; }
    else if (side < 4) { axis = 1; a0 = mnx; a1 = mxx; b0 = mnz; b1 = mxz; k = side == 2 ? mxy : mny; }
    else { axis = 2; a0 = mny; a1 = mxy; b0 = mnz; b1 = mxz; k = side == 4 ? mxx : mnx; }
}

// Box::hit = hit_hittables over its sides (hittable.rs:229-231): closest, ties to the later side.
// No bounding-box pre-test, like the reference (Q8): a per-box slab pre-test and per-side
// candidate tests both measured slower (a lane that skips a test saves the wave nothing unless
// every lane does).
template <bool RCP = false, bool LRCP = false, class R>
__device__ __forceinline__ bool box_t(const rt_prim& p, const RayT<R>& r, R t_min, R t_max, R& t, int& side)
{
    bool any = false;
    // f64: the six sides divide by three directions; one correctly rounded reciprocal y per
    // direction and a Markstein step per side (RN(q / d) bit for bit when y = RN(1 / d): see
    // div_rcp) instead of six divisions. The range guard is taken once per box (a ray with a
    // direction component outside [2^-900, 2^900], e.g. an exact 0, divides as the reference).
    constexpr bool LOCAL_RCP = LRCP && !RCP && std::is_same<R, double>::value;
    auto in_range = [](R d) { const R m = r_fabs(d); return m >= (R)0x1.0p-900 && m <= (R)0x1.0p+900; };
    if (LOCAL_RCP && in_range(r.dx) && in_range(r.dy) && in_range(r.dz)) {
        R y = (R)0;   // of the side pair's direction (sides 2a, 2a+1 share axis a)
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            int axis;
            R a0, a1, b0, b1, k, ts;
            box_side(p, s, axis, a0, a1, b0, b1, k);
            if ((s & 1) == 0) y = (R)1 / (s == 0 ? r.dz : s == 2 ? r.dy : r.dx);
            if (rect_t_y(axis, a0, a1, b0, b1, k, r, y, t_min, t_max, ts)) {
                t_max = ts;
                t = ts;
                side = s;
                any = true;
            }
        }
        return any;
    }
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        int axis;
        R a0, a1, b0, b1, k, ts;
        box_side(p, s, axis, a0, a1, b0, b1, k);
        if (rect_t<RCP>(axis, a0, a1, b0, b1, k, r, t_min, t_max, ts)) {
            t_max = ts;
            t = ts;
            side = s;
            any = true;
        }
    }
    return any;
}

// The centre of a Sphere, or of a MovingSphere at the ray's time: center_0 +
// ((time - time_0) / (time_1 - time_0)) * (center_1 - center_0) (hittable.rs:556-558).
// Both kinds go through one code path with no select: the upload stores a Sphere as a
// MovingSphere of velocity 0 (abi.cpp), whose c0 + 0 * s is c0 bit for bit (s finite), so
// a wave whose lanes hold both kinds runs one test and loads no kind.
template <class R>
__device__ __forceinline__ void sphere_center(const rt_prim& p, const RayT<R>& r, bool general, double& cx, double& cy,
                                              double& cz, bool is_static = false)
{
    if (is_static) {   // FEAT_STATIC: a Sphere, whose c0 + 0 * s is c0 bit for bit
        cx = p.p[0];
        cy = p.p[1];
        cz = p.p[2];
        return;
    }
    double s = (double)r.time;
    // general: the variant has FEAT_SHUTTER (no reference scene does: their moving spheres
    // all have the [0, 1] shutter); without it the flag is not loaded at all
    if (general && !p.a) s = ((double)r.time - p.p[8]) / (p.p[9] - p.p[8]);   // a MovingSphere with a general shutter
    cx = p.p[0] + p.p[5] * s;
    cy = p.p[1] + p.p[6] * s;
    cz = p.p[2] + p.p[7] * s;
}

// Sphere, MovingSphere, rects, Box: t-only (hittable.rs:211-231).
template <class C, class R = typename C::Real>
__device__ __forceinline__ bool simple_t(const rt_prim& p, const RayT<R>& r, R t_min, R t_max, R& t, int& side,
                                         Count& cnt, bool gs)
{
    if (C::COUNT) cnt.prims++;
    if (!(C::F & FEAT_RECT) || p.kind <= RT_PRIM_MOVING_SPHERE) {
        double cx, cy, cz;
        sphere_center(p, r, gs, cx, cy, cz, (C::F & FEAT_STATIC) != 0);
        return sphere_t<C::F == FEAT_SET_SPHERES || (RT_F32_SMALL_ALL && C::F32)>(cx, cy, cz, p.p[3], r, t_min, t_max, t);
    } else {
        const R q0 = (R)p.p[0], q1 = (R)p.p[1], q2 = (R)p.p[2], q3 = (R)p.p[3], q4 = (R)p.p[4];
        switch (p.kind) {
        case RT_PRIM_XY_RECT: return rect_t<RectRcp<C>()>(0, q0, q1, q2, q3, q4, r, t_min, t_max, t);
        case RT_PRIM_XZ_RECT: return rect_t<RectRcp<C>()>(1, q0, q1, q2, q3, q4, r, t_min, t_max, t);
        case RT_PRIM_YZ_RECT: return rect_t<RectRcp<C>()>(2, q0, q1, q2, q3, q4, r, t_min, t_max, t);
        case RT_PRIM_BOX: return box_t<RectRcp<C>(), BoxRcp<C>()>(p, r, t_min, t_max, t, side);
        default: return false;
        }
    }
}

template <class C, class R = typename C::Real>
__device__ __forceinline__ void simple_finish(const rt_prim& p, const RayT<R>& r, R t, int side, HitT<R>& h, bool gs)
{
    if constexpr ((C::F & FEAT_RECT) != 0) {
        if (p.kind >= RT_PRIM_XY_RECT && p.kind <= RT_PRIM_YZ_RECT) {
            rect_finish<C>(p.kind - RT_PRIM_XY_RECT, (R)p.p[0], (R)p.p[1], (R)p.p[2], (R)p.p[3], r, t, p.mat, h);
            return;
        }
        if (p.kind == RT_PRIM_BOX) {
            int axis;
            R a0, a1, b0, b1, k;
            box_side(p, side, axis, a0, a1, b0, b1, k);
            rect_finish<C>(axis, a0, a1, b0, b1, r, t, p.mat, h);
            return;
        }
    }
    double cx, cy, cz;
    sphere_center(p, r, gs, cx, cy, cz, (C::F & FEAT_STATIC) != 0);
    sphere_finish<C>((R)cx, (R)cy, (R)cz, (R)p.p[4], r, t, p.mat, h);
}

// ---------------------------------------------------------------------------
// BVH traversal
// ---------------------------------------------------------------------------
constexpr int RT_DONE = (int)0x80000000;

// A node as four 16-B loads (ds_read_b128 from LDS, global_load_dwordx4 from L1/L2).
struct Node {
    float lo0[3], hi0[3], lo1[3], hi1[3];
    int child[2];
};
__device__ __forceinline__ Node load_node(const rt_bvh_node* base, int i)
{
    const uint4* q = reinterpret_cast<const uint4*>(base + i);
    const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    Node n;
    n.lo0[0] = __uint_as_float(a.x); n.lo0[1] = __uint_as_float(a.y); n.lo0[2] = __uint_as_float(a.z);
    n.hi0[0] = __uint_as_float(a.w); n.hi0[1] = __uint_as_float(b.x); n.hi0[2] = __uint_as_float(b.y);
    n.lo1[0] = __uint_as_float(b.z); n.lo1[1] = __uint_as_float(b.w); n.lo1[2] = __uint_as_float(c.x);
    n.hi1[0] = __uint_as_float(c.y); n.hi1[1] = __uint_as_float(c.z); n.hi1[2] = __uint_as_float(c.w);
    n.child[0] = (int)d.x;
    n.child[1] = (int)d.y;
    return n;
}

// A node from LDS by byte address (four ds_read_b128 through an address-space-3 pointer: a
// generic pointer that may be LDS or global would be read with flat loads)
__device__ __forceinline__ Node load_node_lds(uint32_t addr);

// The TLAS node as staged in LDS by the variants whose whole TLAS is there and whose slab
// tests are f32 (OctNodes): per axis both children's lower planes, upper planes and the lower
// ones again, so a ray reads its near and far planes with one 16-B (2 x 8-B) read at an
// offset its direction sign selects (RayT::onx..onz); children as byte offsets of LdsNode
// (leaf codes unchanged). 80 B instead of rt_bvh_node's 64.
struct LdsNode {
    float ax[3][6];   // [axis][lo0 lo1 hi0 hi1 lo0 lo1]
    int32_t child[2];
};
static_assert(sizeof(LdsNode) == 80, "LdsNode layout");
template <class C>
constexpr bool OctNodes() { return C::NALL && C::S32; }
// LDS byte address of a __shared__ object (the low 32 bits of its flat address), and an LDS
// pointer from one: OctNodes node references are such addresses, so a node read needs no add
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)p; }
template <class T>
__device__ __forceinline__ const __attribute__((address_space(3))) T* lds_ptr(uint32_t a)
{
    return (const __attribute__((address_space(3))) T*)(uintptr_t)a;
}
template <class C>
constexpr int lds_node_bytes()
{
    return OctNodes<C>() ? (int)sizeof(LdsNode) : (int)sizeof(rt_bvh_node);
}
__device__ __forceinline__ Node load_node_lds(uint32_t addr)
{
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
    const auto q = lds_ptr<u4v>(addr);
    const u4v a = q[0], b = q[1], c = q[2], d = q[3];
    Node n;
    n.lo0[0] = __uint_as_float(a.x); n.lo0[1] = __uint_as_float(a.y); n.lo0[2] = __uint_as_float(a.z);
    n.hi0[0] = __uint_as_float(a.w); n.hi0[1] = __uint_as_float(b.x); n.hi0[2] = __uint_as_float(b.y);
    n.lo1[0] = __uint_as_float(b.z); n.lo1[1] = __uint_as_float(b.w); n.lo1[2] = __uint_as_float(c.x);
    n.hi1[0] = __uint_as_float(c.y); n.hi1[1] = __uint_as_float(c.z); n.hi1[2] = __uint_as_float(c.w);
    n.child[0] = (int)d.x;
    n.child[1] = (int)d.y;
    return n;
}

// The material / texture table a shading step reads: staged in LDS by the block prologue
// (north_star: "stages the top BVH levels and material table in LDS") when the variant
// has rects or media and the tables are small (Cornell 4-6 materials, final scene 10), else
// global memory (the random scene's 485 materials would cost the spheres variant blocks per
// CU). The flag is per launch, so the choice is wave-uniform.
template <class C>
constexpr bool StageShade() { return C::F != FEAT_SET_SPHERES; }
// The block's dynamic LDS: [TLAS nodes][BLAS nodes][stack: entries x block lanes][materials][textures], one
// layout for the kernel's offsets and the launcher's allocation (launch_one)
struct LdsLayout {
    size_t blas, stack, shade, total;   // byte offsets of the BLAS nodes, the stack and the material table; bytes
};
__host__ __device__ constexpr LdsLayout lds_layout(int n_nodes, int node_bytes, int n_blas, int stack_entries,
                                                   int entry_bytes, int n_materials, int n_textures, int lanes)
{
    const size_t blas = (size_t)n_nodes * (size_t)node_bytes;
    const size_t stack = blas + (size_t)n_blas * sizeof(rt_bvh_node);
    const size_t shade = stack + (size_t)stack_entries * (size_t)lanes * (size_t)entry_bytes;
    return LdsLayout{blas, stack, shade, shade + (size_t)n_materials * 64 + (size_t)n_textures * 96};
}
// the variants that stage BLAS nodes (SceneDev.n_lds_blas; the host sets it only for them)
#ifndef RT_STAGE_BLAS
#define RT_STAGE_BLAS 1
#endif
template <class C>
constexpr bool StageBlas() { return RT_STAGE_BLAS && (C::F & FEAT_INST_BLAS) != 0; }
template <class C>
__device__ __forceinline__ LdsLayout lds_layout_of(const SceneDev& S)
{
    return lds_layout(S.n_lds_nodes, lds_node_bytes<C>(), StageBlas<C>() ? S.n_lds_blas : 0, C::LDS ? S.stack_entries : 0,
                      Stack16Cfg<C>() ? 2 : 4, StageShade<C>() ? S.n_lds_materials : 0,
                      StageShade<C>() ? S.n_lds_textures : 0, BlockThreads<C>());
}

// Closest hit in a BVH (nodes + leaf ranges of slots j, whose records are leaf_prims[j]).
// `leaf(slot, t_max, best)` tests one primitive; on a closer hit it fills best (t and sub
// ids) and returns true; best.prim is then the slot.
template <class C, bool NL = false, class LeafFn, class R = typename C::Real>
__device__ __forceinline__ bool traverse(const SceneDev& S, int root, const RayT<R>& r, R t_min, R t_max,
                                         HitRefT<R>& best, StackT<C>& stack, int sp0, Count& cnt, LeafFn&& leaf)
{
    // NL: this is the TLAS, whose first S.n_lds_nodes nodes (BFS order) were copied into
    // LDS at block start; deeper nodes are read from L1/L2
    const rt_bvh_node* lds_nodes =
        reinterpret_cast<const rt_bvh_node*>(rt_lds);   // at LDS address 0: node offsets are addresses
    bool any = false;
    // the walk's bottom entry is RT_DONE (the host reserves it: SceneDev.stack_entries,
    // blas_base), so a pop needs no empty-stack test: popping it ends the walk
    constexpr int DONE = Stack16Cfg<C>() ? -32768 : RT_DONE;   // the walk's bottom entry
    // the stack pointer as an address, pre-scaled by the entry stride: a push or pop is one
    // add (not an add plus a shift-add of the index)
    constexpr int SSTR = C::LDS ? BlockThreads<C>() : 1;
    auto* sptr = &stack[sp0];
    using SE = typename std::remove_reference<decltype(*sptr)>::type;
    *sptr = (SE)DONE;
    sptr += SSTR;
    auto push = [&](int v) { *sptr = (SE)v; sptr += SSTR; };
    auto pop = [&]() -> int { sptr -= SSTR; return (int)*sptr; };
    int cur = root;
    float tmin_f = 0.0f, tmax_f = 0.0f;
    if constexpr (C::S32) {
        tmin_f = f32_down(t_min);
        tmax_f = f32_up(t_max);
    }
    // TLAS entirely in LDS, f32 slabs (OctNodes): the node is the 80-B LdsNode layout and
    // node references are byte offsets; per axis one 16-B read at the offset the ray's
    // direction sign selects gives both children's near planes, then their far planes, so
    // the slab test needs no min/max pair per axis: t_near = max(near planes), t_far =
    // min(far planes). One address add per axis, the child pair at a fixed offset.
    constexpr bool OCT = NL && OctNodes<C>();
    float ninf = -__builtin_inff();
    if constexpr (OCT) asm("s_mov_b32 %0, 0xff800000" : "=s"(ninf));
    const char* const lb = reinterpret_cast<const char*>(lds_nodes);
    uint32_t blas_lds_base = 0;   // LDS byte address of the staged BLAS nodes (nested walks)
    if constexpr (!NL && StageBlas<C>()) blas_lds_base = lds_addr(lb) + (uint32_t)lds_layout_of<C>(S).blas;
    (void)blas_lds_base;
    if constexpr (OCT) cur = cur >= 0 ? (int)(lds_addr(lb) + (uint32_t)cur * (uint32_t)sizeof(LdsNode)) : cur;
    // one node visit: test both children, continue with the nearer, push the farther
    auto visit = [&](int node) -> int {
        if (C::COUNT) cnt.nodes++;
        if constexpr (OCT) {
            const uint32_t nb = (uint32_t)node;   // LDS address of the node
            typedef float f2v __attribute__((ext_vector_type(2)));
            typedef int i2v __attribute__((ext_vector_type(2)));
            auto pairs = [&](uint32_t off, f2v& n, f2v& f) {
                const auto q = lds_ptr<f2v>(nb + off);   // one ds_read2_b64
                n = q[0];
                f = q[1];
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
                // min(fz, t_max) as v_med3(fz, t_max, -inf): fminf would re-quiet the loop-carried
                // t_max (a v_max_f32 t, t) at every visit; the plane products are never NaN.
                // (-inf from an SGPR: with the constant the compiler folds med3 back to fminf.)
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
        }
        Node nd;
        if constexpr (!NL && StageBlas<C>()) {
            // a nested (BLAS) walk: its staged top levels from LDS (ds_read_b128 through an LDS
            // pointer), the rest from L1/L2
            const uint32_t j = (uint32_t)(node - S.n_tlas_nodes);
            if (j < (uint32_t)S.n_lds_blas) nd = load_node_lds(blas_lds_base + j * (uint32_t)sizeof(rt_bvh_node));
            else nd = load_node(S.nodes, node);
        } else {
            nd = (NL && (C::NALL || node < S.n_lds_nodes)) ? load_node(lds_nodes, node) : load_node(S.nodes, node);
        }
        bool h0, h1, near0;
        if constexpr (C::S32) {
            float tn0, tn1;
            h0 = slab32(nd.lo0, nd.hi0, r, tmin_f, tmax_f, tn0);
            h1 = slab32(nd.lo1, nd.hi1, r, tmin_f, tmax_f, tn1);
            near0 = tn0 <= tn1;
        } else {
            R tn0, tn1;
            h0 = slab(nd.lo0, nd.hi0, r, t_min, t_max, tn0);
            h1 = slab(nd.lo1, nd.hi1, r, t_min, t_max, tn1);
            near0 = tn0 <= tn1;
        }
        if (h0 && h1) {
            push(near0 ? nd.child[1] : nd.child[0]);
            return near0 ? nd.child[0] : nd.child[1];
        }
        if (h0) return nd.child[0];
        if (h1) return nd.child[1];
        return pop();
    };
    auto do_leaf = [&](int code) {
        code = ~code;
        const int first = code >> 5, count = code & 31;
        for (int i = 0; i < count; ++i) {
            if (C::COUNT && first_active_lane()) cnt.wave_leaves++;
            const int slot = first + i;
            if (leaf(slot, t_max, best)) {
                best.prim = slot;
                t_max = best.t;
                any = true;
                if constexpr (C::S32) tmax_f = f32_up(t_max);
            }
        }
    };
    uint64_t t0 = 0;
    while (cur != DONE) {
        if (C::COUNT && NL) t0 = __builtin_amdgcn_s_memtime();
        while (cur >= 0) {
            if (C::COUNT && first_active_lane()) cnt.wave_nodes++;
            cur = visit(cur);
        }
        if (NL) RT_STAMP(cnt.t_nodes, t0);   // the TLAS walk only: a nested walk is part of its leaf
        if (cur == DONE) break;
        do_leaf(cur);
        cur = pop();
        if (NL) RT_STAMP(cnt.t_leaves, t0);
    }
    return any;
}

// ---------------------------------------------------------------------------
// Translate / RotateY instances (hittable.rs:232-244, 386-415), outermost op first
// ---------------------------------------------------------------------------
template <class R>
__device__ __forceinline__ void instance_ray(const rt_instance& in, RayT<R>& r)
{
    const int n = in.n_ops;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (i < n) {
            if (in.op_kind[i] == RT_OP_TRANSLATE) {  // moved_ray = (o - offset, d, time)
                r.ox = r.ox - (R)in.op[i][0];
                r.oy = r.oy - (R)in.op[i][1];
                r.oz = r.oz - (R)in.op[i][2];
            } else {                                  // rotated_ray
                const R s = (R)in.op[i][0], c = (R)in.op[i][1];
                const R ox = c * r.ox - s * r.oz, oz = s * r.ox + c * r.oz;
                const R dx = c * r.dx - s * r.dz, dz = s * r.dx + c * r.dz;
                r.ox = ox; r.oz = oz; r.dx = dx; r.dz = dz;
            }
        }
    }
}

template <class C, class R = typename C::Real>
__device__ bool medium_t(const SceneDev& S, const rt_prim& m, const RayT<R>& r, R t_min, R t_max, R& t,
                         StackT<C>& stack, int sp0, const Keyed& key, Count& cnt);
template <class R>
__device__ __forceinline__ void medium_finish(const rt_prim& m, const RayT<R>& r, R t, HitT<R>& h);

// t-only: the closest hit of the instance's child; sub = BLAS prim (or the child prim),
// side = winning box side.
template <class C, class R = typename C::Real>
__device__ bool instance_t(const SceneDev& S, const rt_instance& in, const RayT<R>& ray, R t_min, R t_max,
                           HitRefT<R>& ref, StackT<C>& stack, int sp0, const Keyed& key, Count& cnt)
{
    RayT<R> r = ray;
    instance_ray(in, r);
    if (in.child_kind == RT_CHILD_PRIM) {
        if constexpr ((C::F & FEAT_INST_MEDIUM) != 0) {
            const rt_prim& cp = S.prims[in.child];
            if (cp.kind == RT_PRIM_MEDIUM) {   // the medium in object space (its boundary walks at sp0)
                finish_ray<C>(r, S.has_spheres != 0);
                if (!medium_t<InstMedC<C>>(S, cp, r, t_min, t_max, ref.t, stack, sp0, key, cnt)) return false;
                ref.sub = in.child;
                ref.side = 0;
                return true;
            }
        }
        // one primitive: no node-slab terms
        finish_ray<C, false>(r, S.has_spheres != 0);
        int side = 0;
        if (!simple_t<InstC<C>>(S.prims[in.child], r, t_min, t_max, ref.t, side, cnt, (C::F & FEAT_SHUTTER) != 0)) return false;
        ref.sub = in.child;
        ref.side = side;
        return true;
    }
    // an instance over a BVH: a nested walk (its state on top of the TLAS walk's is what
    // set the Cornell variants' register count, 157 vs 125 VGPRs: 3 vs 4 waves per SIMD)
    if constexpr ((C::F & FEAT_INST_BLAS) == 0) return false;
    finish_ray<C>(r, S.has_spheres != 0);
    HitRefT<R> inner;
    const rt_prim* const blas_prims = S.leaf_prims + in.pad;   // the BLAS's leaf codes count from its first slot
    if (!traverse<C>(S, in.child, r, t_min, t_max, inner, stack, sp0, cnt,
                     [&](int slot, R tmax, HitRefT<R>& b) {
                         return simple_t<InstC<C>>(blas_prims[slot], r, t_min, tmax, b.t, b.side, cnt, (C::F & FEAT_SHUTTER) != 0);
                     }))
        return false;
    ref.t = inner.t;
    ref.sub = in.pad + inner.prim;   // absolute leaf slot (instance_finish)
    ref.side = inner.side;
    return true;
}

// The ray direction after ops 0..i (only RotateY changes it; y never changes): recomputed
// per op on the way back instead of kept in arrays through the child's finisher, which
// held 8 f64 registers live and pushed the instance variants into scratch spills.
template <class R>
__device__ __forceinline__ void dir_after(const rt_instance& in, const RayT<R>& ray, int i, R& dx, R& dz)
{
    dx = ray.dx;
    dz = ray.dz;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (j <= i && j < in.n_ops && in.op_kind[j] != RT_OP_TRANSLATE) {
            const R s = (R)in.op[j][0], c = (R)in.op[j][1];
            const R x = c * dx - s * dz, z = s * dx + c * dz;
            dx = x;
            dz = z;
        }
    }
}

template <class C, class R = typename C::Real>
__device__ void instance_finish(const SceneDev& S, const rt_instance& in, const RayT<R>& ray, const HitRefT<R>& ref,
                                HitT<R>& h)
{
    RayT<R> r = ray;
    instance_ray(in, r);
    // ref.sub: the child prim (RT_CHILD_PRIM) or the BLAS leaf slot
    bool done = false;
    if constexpr ((C::F & FEAT_INST_MEDIUM) != 0) {
        if (in.child_kind == RT_CHILD_PRIM && S.prims[ref.sub].kind == RT_PRIM_MEDIUM) {
            medium_finish(S.prims[ref.sub], r, ref.t, h);   // hittable.rs:452-463 in object space
            done = true;
        }
    }
    if (!done)
        simple_finish<InstC<C>>((C::F & FEAT_INST_BLAS) == 0 || in.child_kind == RT_CHILD_PRIM ? S.prims[ref.sub]
                                                                                               : S.leaf_prims[ref.sub],
                                r, ref.t, ref.side, h, (C::F & FEAT_SHUTTER) != 0);
    const int n = in.n_ops;
#pragma unroll
    for (int i = 3; i >= 0; --i) {
        if (i < n) {
            R dx, dz;
            dir_after(in, ray, i, dx, dz);
            if (in.op_kind[i] == RT_OP_TRANSLATE) {  // rec.point += offset; set_face_normal(moved_ray, normal)
                h.px = h.px + (R)in.op[i][0];
                h.py = h.py + (R)in.op[i][1];
                h.pz = h.pz + (R)in.op[i][2];
                set_face_normal(h, dx, ray.dy, dz, h.nx, h.ny, h.nz);
            } else {                                  // rotate back; set_face_normal(rotated_ray, normal)
                const R s = (R)in.op[i][0], c = (R)in.op[i][1];
                const R px = c * h.px + s * h.pz, pz = -s * h.px + c * h.pz;
                const R nx = c * h.nx + s * h.nz, nz = -s * h.nx + c * h.nz;
                h.px = px; h.pz = pz;
                set_face_normal(h, dx, ray.dy, dz, nx, h.ny, nz);
            }
        }
    }
}

// t of a medium boundary (a simple prim or an instance).
template <class C, class R = typename C::Real>
__device__ __forceinline__ bool boundary_t(const SceneDev& S, int prim, const RayT<R>& r, R t_min, R t_max, R& t,
                                           StackT<C>& stack, int sp0, const Keyed& key, Count& cnt)
{
    const rt_prim& p = S.prims[prim];
    if constexpr ((BoundC<C>::F & FEAT_INST) != 0) {
        if (p.kind == RT_PRIM_INSTANCE) {
            HitRefT<R> ref;
            if (!instance_t<BoundC<C>>(S, S.instances[p.a], r, t_min, t_max, ref, stack, sp0, key, cnt)) return false;
            t = ref.t;
            return true;
        }
    }
    int side = 0;
    return simple_t<BoundC<C>>(p, r, t_min, t_max, t, side, cnt, (C::F & FEAT_SHUTTER) != 0);
}

// ConstantMedium (hittable.rs:417-473), keyed draw instead of the in-hit thread_rng().
template <class C, class R>
__device__ bool medium_t(const SceneDev& S, const rt_prim& m, const RayT<R>& r, R t_min, R t_max, R& t,
                         StackT<C>& stack, int sp0, const Keyed& key, Count& cnt)
{
    R t1, t2;
    if constexpr ((BoundC<C>::F & (FEAT_INST | FEAT_RECT)) == 0) {
        // every medium boundary of this variant is a sphere: both queries from one quadratic
        const rt_prim& p = S.prims[m.a];
        if (C::COUNT) cnt.prims += 2;
        double cx, cy, cz;
        sphere_center(p, r, (C::F & FEAT_SHUTTER) != 0, cx, cy, cz, (BoundC<C>::F & FEAT_STATIC) != 0);
        if (!sphere_t2(cx, cy, cz, p.p[3], r, t1, t2)) return false;
    } else {
        if (!boundary_t<C>(S, m.a, r, (R)-RT_INF, (R)RT_INF, t1, stack, sp0, key, cnt)) return false;
        // the second boundary hit after t1 + 0.0001 (hittable.rs:433); in f32 the step must
        // also clear t1's own rounding (a fog sphere of r = 5000 has ulp(t1) = 4.9e-4 > 1e-4)
        R t1_next = t1 + (R)0.0001;
        if constexpr (C::F32) t1_next = t1 + fmaxf(0.0001f, __builtin_fabsf(t1) * 0x1.0p-19f);
        if (!boundary_t<C>(S, m.a, r, t1_next, (R)RT_INF, t2, stack, sp0, key, cnt)) return false;
    }
    if (t1 < t_min) t1 = t_min;
    if (t2 > t_max) t2 = t_max;
    if (t1 >= t2) return false;
    if (t1 < (R)0) t1 = (R)0;
    const R ray_length = r_sqrt(r.a);
    const R distance_inside = (t2 - t1) * ray_length;
    const uint64_t bits = rt_keyed_u64(key.seed, key.pixel, key.sample, key.bounce, RT_STREAM_MEDIUM + (uint32_t)m.b);
    R xi;
    if constexpr (C::F32) xi = (float)(bits >> 40) * 0x1.0p-24f;   // [0, 1) in 2^-24 steps
    else xi = rt_unit53(bits);
    const R hit_distance = (R)m.p[0] * r_log(xi);
    if (hit_distance > distance_inside) return false;
    t = t1 + hit_distance / ray_length;
    return true;
}

// hittable.rs:452-463
template <class R>
__device__ __forceinline__ void medium_finish(const rt_prim& m, const RayT<R>& r, R t, HitT<R>& h)
{
    h.t = t;
    h.px = r.ox + r.dx * t;
    h.py = r.oy + r.dy * t;
    h.pz = r.oz + r.dz * t;
    h.nx = (R)1; h.ny = (R)0; h.nz = (R)0;
    h.front = 1;
    h.mat = m.mat;
    h.uvkind = 0;
}

// The HitRecord of the closest hit (t, leaf slot, sub-primitive, box side) of a world-space ray:
// the arithmetic of the winning primitive's hit (hittable.rs:254-384, 417-473) and of the
// instance chain back to world space (hittable.rs:232-244, 386-415). Traversal keeps only the
// reference; the record is built once per cast (trace_world).
template <class C, class R = typename C::Real>
__device__ __forceinline__ void finish_hit(const SceneDev& S, const RayT<R>& r, const HitRefT<R>& best, HitT<R>& h)
{
    const rt_prim& p = S.leaf_prims[best.prim];
    bool done = false;
    if constexpr ((C::F & FEAT_INST) != 0) {
        if (p.kind == RT_PRIM_INSTANCE) {
            instance_finish<C>(S, S.instances[p.a], r, best, h);
            done = true;
        }
    }
    if constexpr ((C::F & FEAT_MEDIUM) != 0) {
        if (!done && p.kind == RT_PRIM_MEDIUM) {
            medium_finish(p, r, best.t, h);
            done = true;
        }
    }
    if (!done) simple_finish<C>(p, r, best.t, best.side, h, (C::F & FEAT_SHUTTER) != 0);
}

// hit_hittables(world, ray, 0.001, inf) (hittable.rs:43-55) over the TLAS, then the
// The variants that test SceneDev.pre_leaf before the walk: the spheres ones (random scene:
// C2 19.17 -> 17.70 ms); the final scene gains nothing (its fog medium's test inlined twice
// spills) and the Cornell variant would drop to 3 waves per SIMD.
template <class C>
constexpr bool PreLeaf() { return C::F == FEAT_SET_SPHERES; }
// the variants whose instances can hold a BLAS (a nested walk) defer their first instance test
template <class C>
constexpr bool DeferInst() { return RT_DEFER_INST && (C::F & FEAT_INST_BLAS) != 0; }

// The variants that walk a one-leaf top level (the Cornell scenes: S.tlas_root is a leaf code) as
// a plain loop over its slots: no stack, no node loop, a loop count the same in every lane (scalar
// control instead of exec-masked loops). Measured: C3 800x800x200 45.71 -> 41.88 ms, Cornell smoke
// 57.80 -> 52.50, same images; making the kind and instance index wave-uniform on top (scalar
// dispatch) was slower (42.51 / 52.80; profiles/r04q_ab_*.log, r04r_ab_*.log). Not in the variants
// with nested BLAS walks (the final and all-features ones keep their register allocation); the
// spheres variants take the pre-leaf path.
#ifndef RT_UNIFORM_LEAF
#define RT_UNIFORM_LEAF 1
#endif
template <class C>
constexpr bool UniformLeaf() { return RT_UNIFORM_LEAF && (C::F & FEAT_INST_BLAS) == 0 && !PreLeaf<C>(); }

// HitRecord of the closest primitive.
template <class C, class R = typename C::Real>
__device__ bool trace_world(const SceneDev& S, const RayT<R>& r, HitT<R>& h, StackT<C>& stack, const Keyed& key,
                            Count& cnt)
{
    const R t_min = (R)0.001;
    HitRefT<R> best;
    best.sub = 0;
    best.side = 0;
    // DeferInst: the first instance a lane's walk reaches is tested after the walk (pend), so
    // the lanes of a wave that have one walk its BLAS together, once, instead of each at its
    // own step of the top-level walk while the others wait; its t_max is then the walk's final
    // closest hit, which prunes it further. Closest hit does not depend on the order of the
    // tests (the instance's t is the ray's t), so the image does not change.
    int pend = -1;
    (void)pend;
    auto leaf = [&](int slot, R tmax, HitRefT<R>& b) {
        const rt_prim& p = S.leaf_prims[slot];
        if constexpr ((C::F & FEAT_INST) != 0)
            if (p.kind == RT_PRIM_INSTANCE) {
                if constexpr (DeferInst<C>()) {
                    if (pend < 0 && p.b != 0) {   // (b: its child is a BVH, upload)
                        pend = slot;
                        return false;
                    }
                }
                uint64_t ti = 0;
                if (C::COUNT) ti = __builtin_amdgcn_s_memtime();
                const bool hit = instance_t<C>(S, S.instances[p.a], r, t_min, tmax, b, stack, S.blas_base, key, cnt);
                RT_STAMP(cnt.t_inst, ti);
                return hit;
            }
        if constexpr ((C::F & FEAT_MEDIUM) != 0)
            if (p.kind == RT_PRIM_MEDIUM) {
                uint64_t tm = 0;
                if (C::COUNT) tm = __builtin_amdgcn_s_memtime();
                const bool hit = medium_t<C>(S, p, r, t_min, tmax, b.t, stack, S.blas_base, key, cnt);
                RT_STAMP(cnt.t_med, tm);
                return hit;
            }
        return simple_t<C>(p, r, t_min, tmax, b.t, b.side, cnt, (C::F & FEAT_SHUTTER) != 0);
    };
    uint64_t tp = 0;
    if (C::COUNT) tp = __builtin_amdgcn_s_memtime();
    bool hit;
    if constexpr (PreLeaf<C>()) {
        R t_max = (R)RT_INF;
        hit = false;
        int root = S.tlas_root;
        if (S.pre_leaf != 0) {   // wave-uniform: the huge root-child leaf first (SceneDev.pre_leaf)
            root = S.pre_root;
            bool in_box;
            if constexpr (C::S32) {
                float tn;
                in_box = slab32(S.pre_lo, S.pre_hi, r, f32_down(t_min), f32_up(t_max), tn);
            } else {
                R tn;
                in_box = slab(S.pre_lo, S.pre_hi, r, t_min, t_max, tn);
            }
            if (in_box) {
                const int code = ~S.pre_leaf;
                for (int slot = code >> 5, end = (code >> 5) + (code & 31); slot < end; ++slot) {
                    if (leaf(slot, t_max, best)) {
                        best.prim = slot;
                        t_max = best.t;
                        hit = true;
                    }
                }
            }
        }
        if (S.pre_leaf != 0) root = S.pre_root;
        RT_STAMP(cnt.t_pre, tp);
        hit |= traverse<C, true>(S, root, r, t_min, t_max, best, stack, 0, cnt, leaf);
    } else {
        RT_STAMP(cnt.t_pre, tp);
        if (UniformLeaf<C>() && S.tlas_root < 0 && S.tlas_root != RT_DONE) {   // (wave-uniform)
            const int code = ~S.tlas_root;
            R t_max = (R)RT_INF;
            hit = false;
            uint64_t tl = 0;
            if (C::COUNT) tl = __builtin_amdgcn_s_memtime();
            for (int slot = code >> 5, end = (code >> 5) + (code & 31); slot < end; ++slot) {
                if (C::COUNT && first_active_lane()) cnt.wave_leaves++;
                if (leaf(slot, t_max, best)) {   // traverse's do_leaf, in slot order
                    best.prim = slot;
                    t_max = best.t;
                    hit = true;
                }
            }
            RT_STAMP(cnt.t_leaves, tl);
        } else {
            hit = traverse<C, true>(S, S.tlas_root, r, t_min, (R)RT_INF, best, stack, 0, cnt, leaf);
        }
    }
    if (C::COUNT) tp = __builtin_amdgcn_s_memtime();   // the walk stamped its own phases
    if constexpr (DeferInst<C>()) {
        if (pend >= 0) {
            const rt_prim& p = S.leaf_prims[pend];
            HitRefT<R> b;
            b.sub = 0;
            b.side = 0;
            // the top-level walk is done: its stack is free, the BLAS walk starts at entry 0
            if (instance_t<C>(S, S.instances[p.a], r, t_min, hit ? best.t : (R)RT_INF, b, stack, 0, key, cnt)) {
                best = b;
                best.prim = pend;
                hit = true;
            }
            RT_STAMP(cnt.t_defer, tp);
        }
        if (C::COUNT) tp = __builtin_amdgcn_s_memtime();   // lanes without one
    }
    if (!hit) return false;
    finish_hit<C>(S, r, best, h);
    RT_STAMP(cnt.t_rec, tp);
    return true;
}

// ---------------------------------------------------------------------------
// appearance: texture.rs:30-75, perlin.rs:32-108, material.rs:15-94
// ---------------------------------------------------------------------------
template <class R>
__device__ R perlin_noise(const double* ranvec, const int32_t* perm, R px, R py, R pz)
{
    const R fx = r_floor(px), fy = r_floor(py), fz = r_floor(pz);
    R u = px - fx, v = py - fy, w = pz - fz;
    u = u * u * ((R)3 - (R)2 * u);
    v = v * v * ((R)3 - (R)2 * v);
    w = w * w * ((R)3 - (R)2 * w);
    const int32_t i = r_sat_i32(fx), j = r_sat_i32(fy), k = r_sat_i32(fz);
    const R uu = u * u * ((R)3 - (R)2 * u);
    const R vv = v * v * ((R)3 - (R)2 * v);
    const R ww = w * w * ((R)3 - (R)2 * w);
    R accum = (R)0;
    // (the corner and octave loops unrolled: rolled measured slower, C4 143.3 vs 136.9 ms,
    // r03b_ab_c4.log)
#pragma unroll
    for (int di = 0; di < 2; ++di)
#pragma unroll
        for (int dj = 0; dj < 2; ++dj)
#pragma unroll
            for (int dk = 0; dk < 2; ++dk) {
                const uint32_t xi = ((uint32_t)i + (uint32_t)di) & 255u;
                const uint32_t yi = ((uint32_t)j + (uint32_t)dj) & 255u;
                const uint32_t zi = ((uint32_t)k + (uint32_t)dk) & 255u;
                const uint32_t idx = (uint32_t)(perm[xi] ^ perm[256 + yi] ^ perm[512 + zi]) & 255u;
                const R cx = (R)ranvec[3 * idx], cy = (R)ranvec[3 * idx + 1], cz = (R)ranvec[3 * idx + 2];
                const R fi = (R)di, fj = (R)dj, fk = (R)dk;
                const R wx = u - fi, wy = v - fj, wz = w - fk;
                accum += (fi * uu + ((R)1 - fi) * ((R)1 - uu)) * (fj * vv + ((R)1 - fj) * ((R)1 - vv)) *
                         (fk * ww + ((R)1 - fk) * ((R)1 - ww)) * (cx * wx + cy * wy + cz * wz);
            }
    return accum;
}

template <class R>
__device__ R perlin_turb(const double* ranvec, const int32_t* perm, R px, R py, R pz)
{
    R accum = (R)0, weight = (R)1;
    for (int i = 0; i < 7; ++i) {
        accum += weight * perlin_noise(ranvec, perm, px, py, pz);
        weight *= (R)0.5;
        px = px * (R)2;
        py = py * (R)2;
        pz = pz * (R)2;
    }
    return r_fabs(accum);
}

template <class R>
__device__ __forceinline__ R clampd(R x, R mn, R mx)
{
    if (x < mn) return mn;
    if (x > mx) return mx;
    return x;
}

template <class C, class R>
__device__ void hit_uv(const HitT<R>& h, R& u, R& v)
{
    if (h.uvkind == 1) {  // sphere_uv (math.rs:288-300)
        R ox = h.uv0, oy = h.uv1, oz = h.uv2;
        if constexpr (!UVStore<C>()) {   // the outward normal (set_face_normal negated it on a back face)
            ox = h.front ? h.nx : -h.nx;
            oy = h.front ? h.ny : -h.ny;
            oz = h.front ? h.nz : -h.nz;
        }
        const R theta = r_acos(-oy);
        const R phi = r_atan2(-oz, ox) + (R)RT_PI;
        u = phi / ((R)2 * (R)RT_PI);
        v = theta / (R)RT_PI;
    } else if (h.uvkind == 2) {
        u = h.uv0 / h.uv1;
        v = h.uv2 / h.uv3;
    } else {
        u = (R)0;
        v = (R)0;
    }
}

// texture.rs:35-41: sin(10x)*sin(10y)*sin(10z) < 0 from the three signs (rt_sin_sign);
// the full product only when a factor may be tiny enough to underflow it
// f32 mode: the same sign test without the three sinf: sin(10a) < 0 exactly when floor(10a / pi)
// is odd, so the product is negative when the three floors sum to an odd number (the zeros of a
// factor, where the reference's product is 0 and not < 0, are a measure-zero set)
__device__ __forceinline__ bool checker_odd(const HitT<float>& h)
{
    constexpr float k = (float)(10.0 / 3.14159265358979323846);
    const int n = (int)__builtin_floorf(h.px * k) + (int)__builtin_floorf(h.py * k) + (int)__builtin_floorf(h.pz * k);
    return (n & 1) != 0;
}
__device__ __forceinline__ bool checker_odd(const HitT<double>& h)
{
    const double ax = 10.0 * h.px, ay = 10.0 * h.py, az = 10.0 * h.pz;
    const int sx = rt_sin_sign(ax), sy = rt_sin_sign(ay), sz = rt_sin_sign(az);
    if (sx == 2 || sy == 2 || sz == 2) return rt_sin(ax) * rt_sin(ay) * rt_sin(az) < 0.0;
    return sx * sy * sz < 0;
}

template <class C>
__device__ __forceinline__ const rt_texture& texture_of(const SceneDev& S, int i);

template <class C, class R = typename C::Real>
__device__ void tex_value(const SceneDev& S, int ti, const HitT<R>& h, R& cr, R& cg, R& cb)
{
    const rt_texture& t = texture_of<C>(S, ti);
    if constexpr (!(C::F & (FEAT_NOISE | FEAT_IMAGE))) {
        if (t.kind == RT_TEX_CHECKER) {
            const double* c = checker_odd(h) ? t.c1 : t.c0;
            cr = (R)c[0]; cg = (R)c[1]; cb = (R)c[2];
        } else {
            cr = (R)t.c0[0]; cg = (R)t.c0[1]; cb = (R)t.c0[2];
        }
        return;
    }
    switch (t.kind) {
    case RT_TEX_SOLID: cr = (R)t.c0[0]; cg = (R)t.c0[1]; cb = (R)t.c0[2]; return;
    case RT_TEX_CHECKER: {
        if (checker_odd(h)) { cr = (R)t.c1[0]; cg = (R)t.c1[1]; cb = (R)t.c1[2]; }
        else { cr = (R)t.c0[0]; cg = (R)t.c0[1]; cb = (R)t.c0[2]; }
        return;
    }
    case RT_TEX_NOISE: {
        const double* rv = S.perlin_ranvec + (size_t)t.perlin * 768;
        const int32_t* pm = S.perlin_perm + (size_t)t.perlin * 768;
        const R s = (R)1 + r_sin((R)t.scale * h.pz + (R)10 * perlin_turb(rv, pm, h.px, h.py, h.pz));
        const R c = (R)1 * (R)0.5 * s;
        cr = c; cg = c; cb = c;
        return;
    }
    default: {
        if (t.img_w <= 0 || t.img_h <= 0) { cr = (R)0; cg = (R)1; cb = (R)1; return; }
        R u, v;
        hit_uv<C>(h, u, v);
        u = clampd(u, (R)0, (R)1);
        v = (R)1 - clampd(v, (R)0, (R)1);
        uint64_t i = r_sat_u64(u * (R)t.img_w);
        uint64_t j = r_sat_u64(v * (R)t.img_h);
        if (i >= (uint64_t)t.img_w) i = (uint64_t)t.img_w - 1;
        if (j >= (uint64_t)t.img_h) j = (uint64_t)t.img_h - 1;
        const uint8_t* px = S.image + t.img_offset + j * (uint64_t)t.img_bps + i * 3;
        const R color_scale = (R)1 / (R)255;
        cr = color_scale * (R)px[0];
        cg = color_scale * (R)px[1];
        cb = color_scale * (R)px[2];
        return;
    }
    }
}

// The path stream of rt_numerics.h (rt_pstream): one Philox block of (pixel, sample) seeds
// a xoshiro128++ state, from which the path draws in the reference's order.
__device__ __forceinline__ void ds_start(rt_pstream& st, uint64_t seed, uint32_t pixel, uint32_t sample)
{
    rt_pstream_init(&st, seed, pixel, sample);
}
// The f32 mode's path stream: the same counter and key through 7 Philox rounds instead of 10
// (Salmon et al., SC'11: Philox4x32-7 already passes TestU01's BigCrush; the f64 mode keeps the
// 10 rounds of the protocol the oracle restates). 30 % fewer of the per-sample
// seeding's 32x32-bit products, which take ~7 % of the f32 kernel on the random scene.
#ifndef RT_F32_PHILOX_ROUNDS
#define RT_F32_PHILOX_ROUNDS 7
#endif
__device__ __forceinline__ void ds_start_f32(rt_pstream& st, uint64_t seed, uint32_t pixel, uint32_t sample)
{
    rt_u32x4 c;
    c.v[0] = pixel; c.v[1] = sample; c.v[2] = 0; c.v[3] = RT_STREAM_PATH;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < RT_F32_PHILOX_ROUNDS; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.v[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.v[2];
        rt_u32x4 n;
        n.v[0] = (uint32_t)(p1 >> 32) ^ c.v[1] ^ k0;
        n.v[1] = (uint32_t)p1;
        n.v[2] = (uint32_t)(p0 >> 32) ^ c.v[3] ^ k1;
        n.v[3] = (uint32_t)p0;
        c = n;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    st.s0 = c.v[0]; st.s1 = c.v[1]; st.s2 = c.v[2]; st.s3 = c.v[3];
    if ((st.s0 | st.s1 | st.s2 | st.s3) == 0) st.s0 = 1;
}
__device__ __forceinline__ uint64_t ds_u64(rt_pstream& st) { return rt_pstream_u64(&st); }

// The path's draws. f64: rand's Standard / gen_range mappings of 64-bit draws (math.rs:268-280,
// rt_numerics.h); f32 mode: one 32-bit draw each, 24 significant bits.
__device__ __forceinline__ double draw_unit(rt_pstream& st, double) { return rt_unit53(ds_u64(st)); }
__device__ __forceinline__ float draw_unit(rt_pstream& st, float)
{
    return (float)(rt_pstream_u32(&st) >> 8) * 0x1.0p-24f;
}
__device__ __forceinline__ double draw_m11(rt_pstream& st, double scale_m11) { return rt_uniform_sample(ds_u64(st), -1.0, scale_m11); }
__device__ __forceinline__ float draw_m11(rt_pstream& st, float)
{
    return (float)(rt_pstream_u32(&st) >> 8) * 0x1.0p-23f - 1.0f;
}

// math.rs:51-58: random_double_range(-1, 1) x 3 until inside
template <class R>
__device__ __forceinline__ void random_in_unit_sphere(rt_pstream& st, R scale_m11, R& x, R& y, R& z, R& len2)
{
    for (;;) {
        x = draw_m11(st, scale_m11);
        y = draw_m11(st, scale_m11);
        z = draw_m11(st, scale_m11);
        len2 = x * x + y * y + z * z;
        if (len2 < (R)1) return;
    }
}

// ---------------------------------------------------------------------------
// the integrator
// ---------------------------------------------------------------------------

// main.rs:517-520 + Camera::get_ray (camera.rs:58-66) in three steps: camera_begin (the
// pixel jitter draws), the lens draws (random_in_unit_disk: 2 draws per try, the same
// mapping as random_in_unit_sphere's, whose loop the pool schedules share with it) and
// camera_end (the ray and its time draw). camera_ray runs them in a row.
__device__ __forceinline__ void camera_begin(const KParams& P, int x, int y, rt_pstream& st, float& u, float& v)
{   // f32 mode
    u = ((float)x + draw_unit(st, 0.0f)) / (float)P.wm1;
    v = ((float)y + draw_unit(st, 0.0f)) / (float)P.hm1;
}
__device__ __forceinline__ void camera_begin(const KParams& P, int x, int y, rt_pstream& st, double& u, double& v)
{
    u = div_rcp((double)x + rt_unit53(ds_u64(st)), P.wm1, P.inv_wm1);
    v = div_rcp((double)y + rt_unit53(ds_u64(st)), P.hm1, P.inv_hm1);
}
// one try of random_in_unit_disk (3 = false) or random_in_unit_sphere (3 = true): the
// length test of a disk candidate is x*x + y*y + 0*0, the same value as x*x + y*y
template <class R>
__device__ __forceinline__ bool unit_try(rt_pstream& st, R scale_m11, bool three, R& x, R& y, R& z, R& len2)
{
    x = draw_m11(st, scale_m11);
    y = draw_m11(st, scale_m11);
    z = (R)0;
    if (three) z = draw_m11(st, scale_m11);
    len2 = x * x + y * y + z * z;
    return len2 < (R)1;
}
__device__ __forceinline__ void camera_end(const KParams& P, rt_pstream& st, float u, float v, float dxl, float dyl,
                                           RayT<float>& r)
{   // f32 mode
    const rt_camera& c = P.cam;
    const float rdx = dxl * (float)c.lens_radius, rdy = dyl * (float)c.lens_radius;
    const float offx = (float)c.u[0] * rdx + (float)c.v[0] * rdy;
    const float offy = (float)c.u[1] * rdx + (float)c.v[1] * rdy;
    const float offz = (float)c.u[2] * rdx + (float)c.v[2] * rdy;
    r.ox = (float)c.origin[0] + offx;
    r.oy = (float)c.origin[1] + offy;
    r.oz = (float)c.origin[2] + offz;
    // lower_left_corner - origin folded in f64 on the way (one rounding instead of two)
    r.dx = (float)(c.lower_left_corner[0] - c.origin[0]) + (float)c.horizontal[0] * u + (float)c.vertical[0] * v - offx;
    r.dy = (float)(c.lower_left_corner[1] - c.origin[1]) + (float)c.horizontal[1] * u + (float)c.vertical[1] * v - offy;
    r.dz = (float)(c.lower_left_corner[2] - c.origin[2]) + (float)c.horizontal[2] * u + (float)c.vertical[2] * v - offz;
    r.time = (float)c.time0 + draw_unit(st, 0.0f) * (float)(c.time1 - c.time0);
}
__device__ __forceinline__ void camera_end(const KParams& P, rt_pstream& st, double u, double v, double dxl,
                                           double dyl, RayT<double>& r)
{
    const double rdx = dxl * P.cam.lens_radius, rdy = dyl * P.cam.lens_radius;
    const double offx = P.cam.u[0] * rdx + P.cam.v[0] * rdy;
    const double offy = P.cam.u[1] * rdx + P.cam.v[1] * rdy;
    const double offz = P.cam.u[2] * rdx + P.cam.v[2] * rdy;
    r.ox = P.cam.origin[0] + offx;
    r.oy = P.cam.origin[1] + offy;
    r.oz = P.cam.origin[2] + offz;
    r.dx = P.cam.lower_left_corner[0] + P.cam.horizontal[0] * u + P.cam.vertical[0] * v - P.cam.origin[0] - offx;
    r.dy = P.cam.lower_left_corner[1] + P.cam.horizontal[1] * u + P.cam.vertical[1] * v - P.cam.origin[1] - offy;
    r.dz = P.cam.lower_left_corner[2] + P.cam.horizontal[2] * u + P.cam.vertical[2] * v - P.cam.origin[2] - offz;
    r.time = rt_uniform_sample(ds_u64(st), P.cam.time0, P.scale_time);
}
template <class R>
__device__ __forceinline__ void camera_ray(const KParams& P, int x, int y, rt_pstream& st, RayT<R>& r)
{
    R u, v, dxl, dyl, dzl, l2;
    camera_begin(P, x, y, st, u, v);
    while (!unit_try(st, (R)P.scale_m11, false, dxl, dyl, dzl, l2)) {
    }
    camera_end(P, st, u, v, dxl, dyl, r);
}

template <class C>
__device__ __forceinline__ int lds_stack_offset(const SceneDev& S)   // in ints, after the TLAS nodes
{
    return (int)(lds_layout_of<C>(S).stack / 4);
}
template <class C>
__device__ __forceinline__ int lds_shade_offset(const SceneDev& S)   // in ints
{
    return (int)(lds_layout_of<C>(S).shade / 4);
}
template <class C>
__device__ __forceinline__ const rt_material& material_of(const SceneDev& S, int i)
{
    if constexpr (StageShade<C>()) {
        if (S.n_lds_materials > 0)
            return reinterpret_cast<const rt_material*>(rt_lds + lds_shade_offset<C>(S))[i];
    }
    return S.materials[i];
}
template <class C>
__device__ __forceinline__ const rt_texture& texture_of(const SceneDev& S, int i)
{
    if constexpr (StageShade<C>()) {
        if (S.n_lds_materials > 0)
            return reinterpret_cast<const rt_texture*>(rt_lds + lds_shade_offset<C>(S) + S.n_lds_materials * 16)[i];
    }
    return S.textures[i];
}
// block prologue: TLAS nodes, then the material and texture tables (every thread takes part)
template <class C>
__device__ __forceinline__ void stage_lds(const SceneDev& S)
{
    bool any = false;
    const int off = 0;   // the TLAS nodes first (traverse)
    if (S.n_lds_nodes > 0) {
        if constexpr (OctNodes<C>()) {   // one node per thread, rt_bvh_node -> LdsNode
            LdsNode* dst = reinterpret_cast<LdsNode*>(rt_lds + off);
            for (int i = threadIdx.x; i < S.n_lds_nodes; i += BlockThreads<C>()) {
                const rt_bvh_node n = S.nodes[i];
                LdsNode o;
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    o.ax[a][0] = n.lo0[a]; o.ax[a][1] = n.lo1[a];
                    o.ax[a][2] = n.hi0[a]; o.ax[a][3] = n.hi1[a];
                    o.ax[a][4] = n.lo0[a]; o.ax[a][5] = n.lo1[a];
                }
#pragma unroll
                for (int c = 0; c < 2; ++c)   // node references: LDS addresses (leaf codes stay < 0)
                    o.child[c] = n.child[c] >= 0 ? (int)(lds_addr(dst) + (uint32_t)n.child[c] * (uint32_t)sizeof(LdsNode))
                                                 : n.child[c];
                dst[i] = o;
            }
        } else {
            uint4* dst = reinterpret_cast<uint4*>(rt_lds + off);
            const uint4* src = reinterpret_cast<const uint4*>(S.nodes);
            for (int i = threadIdx.x; i < S.n_lds_nodes * 4; i += BlockThreads<C>()) dst[i] = src[i];
        }
        any = true;
    }
    if constexpr (StageBlas<C>()) {
        if (S.n_lds_blas > 0) {   // the BLAS's BFS prefix, nodes[n_tlas_nodes, ...) (abi.cpp)
            uint4* db = reinterpret_cast<uint4*>(reinterpret_cast<char*>(rt_lds) + lds_layout_of<C>(S).blas);
            const uint4* sb = reinterpret_cast<const uint4*>(S.nodes + S.n_tlas_nodes);
            for (int i = threadIdx.x; i < S.n_lds_blas * 4; i += BlockThreads<C>()) db[i] = sb[i];
            any = true;
        }
    }
    if constexpr (StageShade<C>()) {
        if (S.n_lds_materials > 0) {
            uint4* dm = reinterpret_cast<uint4*>(rt_lds + lds_shade_offset<C>(S));
            const uint4* sm = reinterpret_cast<const uint4*>(S.materials);
            for (int i = threadIdx.x; i < S.n_lds_materials * 4; i += BlockThreads<C>()) dm[i] = sm[i];
            uint4* dt = dm + S.n_lds_materials * 4;
            const uint4* stx = reinterpret_cast<const uint4*>(S.textures);
            for (int i = threadIdx.x; i < S.n_lds_textures * 6; i += BlockThreads<C>()) dt[i] = stx[i];
            any = true;
        }
    }
    if (any) __syncthreads();
}

// One hit of ray_color (main.rs:25-34): emitted + attenuation * (next), with the
// recursion unrolled into the throughput T. A path carries at most one emission (a
// DiffuseLight ends it), so adding T*e straight into the chunk sum gives the same bits
// as the reference's per-sample sum. In three steps: shade_begin (emission; false if the
// path ends there), the material's draws (random_in_unit_sphere unless Dielectric), and
// shade_end (the scattered ray; false if Metal absorbs it). shade() runs them in a row; the
// pool schedules run the draws in one rejection loop with the camera's.
template <class C, class R = typename C::Real>
__device__ __forceinline__ bool shade_begin(const SceneDev& S, const HitT<R>& h, R Tr, R Tg, R Tb, double& sum_r,
                                            double& sum_g, double& sum_b)
{
    if (!S.has_lights) return true;   // wave-uniform: no material of the scene emits (no read needed)
    const rt_material& m = material_of<C>(S, h.mat);
    if (m.kind == RT_MAT_DIFFUSE_LIGHT) {  // material.rs:25-34 (emits on both faces, never scatters)
        R er, eg, eb;
        tex_value<C>(S, m.tex, h, er, eg, eb);
        sum_r = sum_r + (double)(Tr * er);   // the chunk sums stay f64 in the f32 mode too
        sum_g = sum_g + (double)(Tg * eg);
        sum_b = sum_b + (double)(Tb * eb);
        return false;
    }
    return true;
}
// whether the material draws a random_in_unit_sphere candidate (Lambertian, Metal, Isotropic)
template <class C>
__device__ __forceinline__ bool shade_draws(const SceneDev& S, int mat)
{
    return material_of<C>(S, mat).kind != RT_MAT_DIELECTRIC;
}
// (qx, qy, qz, l2): the material's random_in_unit_sphere draw (0, 0, 0, 1 for Dielectric)
template <class C, bool FIN = true, class R = typename C::Real>
__device__ __forceinline__ bool shade_end(const SceneDev& S, const HitT<R>& h, RayT<R>& r, rt_pstream& st, R& Tr,
                                          R& Tg, R& Tb, R qx, R qy, R qz, R l2)
{
    const rt_material& m = material_of<C>(S, h.mat);
    const int kind = m.kind;
    // The materials share their expensive steps, so a wave holding several materials runs
    // each once: one unit-sphere loop (Lambertian, Metal, Isotropic), one 1/sqrt (of the
    // candidate for Lambertian, of the ray direction for Metal and Dielectric), one texture
    // lookup (Lambertian, Isotropic).
    const R inv = (R)1 / r_sqrt(kind == RT_MAT_LAMBERTIAN ? l2 : r.a);
    R sdx, sdy, sdz, ar = (R)1, ag = (R)1, ab = (R)1;
    bool scattered = true;
    if (kind == RT_MAT_LAMBERTIAN) {  // material.rs:36-48
        sdx = h.nx + qx * inv;
        sdy = h.ny + qy * inv;
        sdz = h.nz + qz * inv;
        if (r_fabs(sdx) < (R)1e-8 && r_fabs(sdy) < (R)1e-8 && r_fabs(sdz) < (R)1e-8) {
            sdx = h.nx; sdy = h.ny; sdz = h.nz;
        }
    } else if (kind == RT_MAT_METAL || kind == RT_MAT_DIELECTRIC) {
        const R ux = r.dx * inv, uy = r.dy * inv, uz = r.dz * inv;  // normalize(r_in.direction)
        if (kind == RT_MAT_METAL) {  // material.rs:50-60
            const R fuzz = (R)m.fuzz;
            const R k2 = (R)2 * (ux * h.nx + uy * h.ny + uz * h.nz);
            sdx = (ux - h.nx * k2) + qx * fuzz;
            sdy = (uy - h.ny * k2) + qy * fuzz;
            sdz = (uz - h.nz * k2) + qz * fuzz;
            scattered = sdx * h.nx + sdy * h.ny + sdz * h.nz > (R)0;
            ar = (R)m.albedo[0]; ag = (R)m.albedo[1]; ab = (R)m.albedo[2];
        } else {  // material.rs:62-82, 89-94
            const R ir = (R)m.ir;
            const R ratio = h.front ? ((R)1 / ir) : ir;
            const R cos_theta = r_fmin((-ux) * h.nx + (-uy) * h.ny + (-uz) * h.nz, (R)1);
            const R sin_theta = r_sqrt((R)1 - cos_theta * cos_theta);
            const bool cannot_refract = ratio * sin_theta > (R)1;
            bool reflect = cannot_refract;
            if (!reflect) {  // the draw is skipped on TIR (the || short-circuit of material.rs:72)
                R r0 = ((R)1 - ratio) / ((R)1 + ratio);
                r0 = r0 * r0;
                const R refl = r0 + ((R)1 - r0) * r_pow5((R)1 - cos_theta);
                reflect = refl > draw_unit(st, (R)0);
            }
            if (reflect) {
                const R k2 = (R)2 * (ux * h.nx + uy * h.ny + uz * h.nz);
                sdx = ux - h.nx * k2;
                sdy = uy - h.ny * k2;
                sdz = uz - h.nz * k2;
            } else {  // math.rs:110-117 (cos_theta recomputed there from the same inputs)
                const R px = (ux + h.nx * cos_theta) * ratio;
                const R py = (uy + h.ny * cos_theta) * ratio;
                const R pz = (uz + h.nz * cos_theta) * ratio;
                const R pl = px * px + py * py + pz * pz;
                const R kk = -r_sqrt(r_fabs((R)1 - pl));
                sdx = px + h.nx * kk;
                sdy = py + h.ny * kk;
                sdz = pz + h.nz * kk;
            }
        }
    } else {  // isotropic, material.rs:84-87
        sdx = qx; sdy = qy; sdz = qz;
    }
    if (!scattered) return false;  // emitted (0) only
    if (kind == RT_MAT_LAMBERTIAN || kind == RT_MAT_ISOTROPIC) tex_value<C>(S, m.tex, h, ar, ag, ab);
    Tr = Tr * ar;
    Tg = Tg * ag;
    Tb = Tb * ab;
    r.ox = h.px; r.oy = h.py; r.oz = h.pz;
    if constexpr (C::F32) {
        // f32 mode: the hit point carries ~|p| 2^-24 of rounding, which t_min = 0.001 does not
        // cover at grazing angles on the final scene's |p| ~ 1000 boxes (the next ray would hit
        // its own surface again); move the origin off the surface, to the side the new ray
        // leaves on (Wachter & Binder, Ray Tracing Gems ch. 6). Media (uvkind 0) have no surface.
        // The scale is measured (round 6, C4 geometry at 16 spp, count variant; f64 paths: 3.690
        // casts per sample, 9.75 node visits per cast): |p| 2^-23 4.44 / 11.88, 2^-21 4.33 /
        // 11.85, 2^-19 (rounds 3-5) 4.14 / 11.64, 2^-17 3.93 / 10.85, 2^-15 3.696 / 9.72, 2^-13
        // 3.693 / 9.53 (profiles/r06m_*, r06n_*, r06o_*). Below 2^-15 the f32 paths re-hit their
        // own surfaces and run longer than the reference's; 2^-15 gives its path lengths (and
        // the statistical parity of tests/test_gpu_f32.py), 2^-13 starts to skip geometry.
        if (h.uvkind != 0) {
            const float m = fmaxf(fmaxf(__builtin_fabsf(h.px), __builtin_fabsf(h.py)), __builtin_fabsf(h.pz));
            float eps = m * 0x1.0p-15f + 1e-5f;
            if (sdx * h.nx + sdy * h.ny + sdz * h.nz < 0.0f) eps = -eps;
            r.ox = h.px + h.nx * eps;
            r.oy = h.py + h.ny * eps;
            r.oz = h.pz + h.nz * eps;
        }
    }
    r.dx = sdx; r.dy = sdy; r.dz = sdz;
    if constexpr (FIN) finish_ray<C>(r, S.has_spheres != 0);   // else the caller's trace step does it
    return true;
}
template <class C, bool FIN = true, class R = typename C::Real>
__device__ __forceinline__ bool shade(const SceneDev& S, const KParams& P, const HitT<R>& h, RayT<R>& r,
                                      rt_pstream& st, R& Tr, R& Tg, R& Tb, double& sum_r, double& sum_g,
                                      double& sum_b)
{
    if (!shade_begin<C>(S, h, Tr, Tg, Tb, sum_r, sum_g, sum_b)) return false;
    R qx = (R)0, qy = (R)0, qz = (R)0, l2 = (R)1;
    if (shade_draws<C>(S, h.mat)) random_in_unit_sphere(st, (R)P.scale_m11, qx, qy, qz, l2);
    return shade_end<C, FIN>(S, h, r, st, Tr, Tg, Tb, qx, qy, qz, l2);
}

// image row of the shard's local row k: y = row_begin + k*row_stride, or in bands of 2^s rows
// y = (row_begin + (k >> s)*row_stride) << s | (k & (2^s - 1))
__device__ __forceinline__ int image_row(const KParams& P, int k)
{
    const int s = P.row_block_shift;
    return ((P.row_begin + (k >> s) * P.row_stride) << s) + (k & ((1 << s) - 1));
}
// image pixel (X, Y) of the shard's grid pixel (x, k): a row shard's x and image_row(k); a tile
// shard's grid is its tiles side by side (tile m = the frame's tile at position row_begin +
// m*row_stride of the context's tile order, or of raster order)
__device__ __forceinline__ void image_xy(const KParams& P, int x, int k, int& X, int& Y)
{
    if (P.tile_shard) {   // wave-uniform
        unsigned t = (unsigned)P.row_begin + (unsigned)(x >> 3) * (unsigned)P.row_stride;
        if (__builtin_expect(P.tile_order != nullptr, 0)) t = P.tile_order[t];
        // (the division by a runtime value was ~25 VALU instructions in every bounce-loop iteration
        // that starts a sample: 0.7 % of C2's kernel as a world-1 tile shard, profiles/r06d_*)
        const unsigned ty = P.tile_div_magic ? __umulhi(t, P.tile_div_magic) : t / (unsigned)P.img_tiles_x;
        X = (int)(t - ty * (unsigned)P.img_tiles_x) * 8 + (x & 7);
        Y = (int)ty * 8 + k;
    } else {
        X = x;
        Y = image_row(P, k);
    }
}

// lane -> (chunk, pixel): a wave64 owns an 8x8 tile of one chunk
struct LaneWork {
    int x, y, k, chunk, s_begin, s_end;   // x, k: the shard's grid; y: image row
    int ix;                               // image column
    uint32_t pixel;
};
__device__ __forceinline__ bool lane_work(const KParams& P, LaneWork& w)
{
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long long n_tiles = (long long)P.tiles_x * P.tiles_y;
    if (wave >= n_tiles * P.n_chunks) return false;
    w.chunk = (int)(wave / n_tiles);
    const int tile = (int)(wave % n_tiles);
    w.x = (tile % P.tiles_x) * 8 + (lane & 7);
    w.k = (tile / P.tiles_x) * 8 + (lane >> 3);
    if (w.x >= P.width || w.k >= P.n_rows) return false;
    int ix;
    image_xy(P, w.x, w.k, ix, w.y);
    w.pixel = (uint32_t)w.y * (uint32_t)P.img_width + (uint32_t)ix;
    w.ix = ix;
    w.s_begin = P.sample_begin + w.chunk * P.spp_chunk;
    w.s_end = min(P.spp, w.s_begin + P.spp_chunk);
    return true;
}

#ifndef RT_MIN_WAVES_F32_SPHERES
#define RT_MIN_WAVES_F32_SPHERES 6   // 76 VGPRs (<= 80 for 6), 512-thread blocks (RT_BLOCK_F32_SPHERES)
#endif
#ifndef RT_MIN_WAVES_SPHERES
#define RT_MIN_WAVES_SPHERES 1
#endif
// the f64 spheres variant with its 16-bit LDS stack (C1, C2, C5): 6 waves per SIMD at 80 VGPRs
// (94 at 5, spill-free) with 768-thread workgroups (RT_BLOCK_SPHERES)
#ifndef RT_MIN_WAVES_SPHERES_S16
#define RT_MIN_WAVES_SPHERES_S16 6
#endif
#ifndef RT_MIN_WAVES_RECTINST
// measured (Cornell 800x800x200): chunk schedule 4 waves 190 vs 202 ms; pool schedule 4: 80.7,
// 3: 81.0; after the reciprocal divisions (more live state, 4 waves spilled to scratch):
// 4: 66.6, 3: 58.6; round 2: without the nested BLAS walk (FEAT_INST_BLAS), the f64-slab
// instantiation the node-free Cornell scenes run needs 125 VGPRs: 4 waves at this bound
#define RT_MIN_WAVES_RECTINST 3
#endif
#ifndef RT_MIN_WAVES_ALL
// measured, pool schedule: final scene 960x540x200 4: 112.0 ms (scratch spills: 0.7 TB of HBM
// writes per launch), 3: 102.8, 2: 131.5; cornell smoke 600x600x200 4: 74.1, 3: 62.3, 2: 79.7
#define RT_MIN_WAVES_ALL 3
#endif
#ifndef RT_MIN_WAVES_MEDIA
#define RT_MIN_WAVES_MEDIA 3
#endif
#ifndef RT_MIN_WAVES_FINAL
// round 3: 4 (127 VGPRs, no spills, once machine LICM no longer pins the cold paths' f64
// constants in VGPRs and the hit record is dead during the walk); round 2 measured 3 best
// (4: 112.0 ms with 0.7 TB of scratch writes per launch, 3: 102.8, 2: 131.5 at 960x540x200)
#define RT_MIN_WAVES_FINAL 4
#endif
// the f32 final-scene variant: 4 like the f64 one (3 waves, 136-142 VGPRs and no spills even with
// the small-sphere test, is slower: C4 1920x1080x100 f32 101.9 ms with 768-thread blocks, 107.0
// with 256, against 89.4 at 4; profiles/r06s_ab_f32final_c4.log)
#ifndef RT_MIN_WAVES_F32_FINAL
#define RT_MIN_WAVES_F32_FINAL RT_MIN_WAVES_FINAL
#endif
// minimum waves per SIMD requested from the register allocator, per feature set
template <class C>
constexpr int min_waves()
{
    return Stack16Cfg<C>() && C::F32 ? RT_MIN_WAVES_F32_SPHERES   // (the f32 mode's spheres variant)
           : C::F32 && C::F == FEAT_SET_FINAL ? RT_MIN_WAVES_F32_FINAL
           : Stack16Cfg<C>() && C::F == FEAT_SET_SPHERES ? RT_MIN_WAVES_SPHERES_S16
           : C::F == FEAT_SET_SPHERES ? RT_MIN_WAVES_SPHERES
           : C::F == FEAT_SET_RECTINST ? RT_MIN_WAVES_RECTINST
           : C::F == FEAT_SET_MEDIA    ? RT_MIN_WAVES_MEDIA
           : C::F == FEAT_SET_FINAL    ? RT_MIN_WAVES_FINAL : RT_MIN_WAVES_ALL;
}

// KParams comes by pointer: read where used (scalar loads) instead of pinning ~70 SGPRs
// for the whole kernel (by value it spilled SGPRs into VGPR lanes).
template <class C>
__global__ void __launch_bounds__(BlockThreads<C>(), min_waves<C>()) trace_chunks(SceneDev S, const KParams* __restrict__ Pp,
                                                                    double* __restrict__ partial,
                                                                    unsigned long long* __restrict__ counters)
{
    const KParams& P = *Pp;
    stage_lds<C>(S);   // every thread of the block takes part, before any early return
    LaneWork w;
    if (!lane_work(P, w)) return;
    StackT<C> stack;
    if constexpr (Stack16Cfg<C>()) stack.base = reinterpret_cast<short*>(rt_lds + lds_stack_offset<C>(S)) + threadIdx.x;
    else if constexpr (C::LDS) stack.init((int)lds_stack_offset<C>(S));
    Count cnt{};
    uint64_t t_cam = 0, t_trace = 0, t_shade = 0, t_prev = 0;
    if (C::COUNT) t_prev = __builtin_amdgcn_s_memtime();
    using R = typename C::Real;
    double sum_r = 0.0, sum_g = 0.0, sum_b = 0.0;
    Keyed key{P.seed, w.pixel, 0, 0};
    rt_pstream st;
    RayT<R> r;
    R Tr = 1, Tg = 1, Tb = 1;
    int depth = 0;
    int s = w.s_begin;
    bool new_sample = true;
    while (s < w.s_end) {
        if (C::COUNT && first_active_lane()) cnt.wave_steps++;
        if (new_sample) {
            new_sample = false;
            if constexpr (C::F32) ds_start_f32(st, P.seed, w.pixel, (uint32_t)s);
            else ds_start(st, P.seed, w.pixel, (uint32_t)s);
            key.sample = (uint32_t)s;
            camera_ray(P, w.ix, w.y, st, r);
            finish_ray<C>(r, S.has_spheres != 0);
            Tr = Tg = Tb = (R)1;
            depth = P.max_depth;
        }
        if (C::COUNT) { const uint64_t t = __builtin_amdgcn_s_memtime(); t_cam += t - t_prev; t_prev = t; }
        bool cont = false;
        if (depth > 0) {  // main.rs:21-23: depth 0 is black
            key.bounce = (uint32_t)(P.max_depth - depth);
            if (C::COUNT) cnt.casts++;
            HitT<R> h;
            const bool hit = trace_world<C>(S, r, h, stack, key, cnt);
            if (C::COUNT) { const uint64_t t = __builtin_amdgcn_s_memtime(); t_trace += t - t_prev; t_prev = t; }
            if (!hit) {  // main.rs:37: background
                sum_r = sum_r + Tr * P.bg[0];
                sum_g = sum_g + Tg * P.bg[1];
                sum_b = sum_b + Tb * P.bg[2];
            } else {
                cont = shade<C>(S, P, h, r, st, Tr, Tg, Tb, sum_r, sum_g, sum_b);
            }
        }
        if (C::COUNT) { const uint64_t t = __builtin_amdgcn_s_memtime(); t_shade += t - t_prev; t_prev = t; }
        if (cont) {
            depth -= 1;
        } else {
            s += 1;
            new_sample = true;
        }
    }
    double* o = partial + (((size_t)w.chunk * P.n_rows + w.k) * P.width + w.x) * 3;
    o[0] = sum_r;
    o[1] = sum_g;
    o[2] = sum_b;
    if (C::COUNT) {
        atomicAdd(&counters[0], (unsigned long long)cnt.casts);
        atomicAdd(&counters[1], (unsigned long long)cnt.nodes);
        atomicAdd(&counters[2], (unsigned long long)cnt.prims);
        atomicAdd(&counters[6], (unsigned long long)cnt.wave_steps);
        atomicAdd(&counters[7], (unsigned long long)cnt.wave_nodes);
        atomicAdd(&counters[10], (unsigned long long)cnt.wave_leaves);
        atomicAdd(&counters[11], (unsigned long long)cnt.cam_lanes);
        atomicAdd(&counters[12], (unsigned long long)cnt.cam_steps);
        atomicAdd(&counters[13], (unsigned long long)cnt.shade_lanes);
        atomicAdd(&counters[14], (unsigned long long)cnt.shade_steps);
        // phase times are per wave (every active lane sees the same clock): one lane adds
        if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1) {
            atomicAdd(&counters[3], (unsigned long long)(t_cam + cnt.t_seed + cnt.t_tries));   // ray generation, all of it
        atomicAdd(&counters[23], (unsigned long long)cnt.t_seed);
        atomicAdd(&counters[24], (unsigned long long)cnt.t_tries);
            atomicAdd(&counters[4], (unsigned long long)t_trace);
            atomicAdd(&counters[5], (unsigned long long)t_shade);
            atomicAdd(&counters[8], (unsigned long long)cnt.t_nodes);
            atomicAdd(&counters[9], (unsigned long long)cnt.t_leaves);
        }
    }
}

// ---------------------------------------------------------------------------
// Sample-pool schedule. Persistent waves take work blocks (one 8x8 tile x one chunk of
// samples) from a global counter; inside the wave, a lane whose path ended takes the
// block's next (pixel, sample) unit at once (ballot + mbcnt), so lanes do not idle until
// the last blocks run out. Each sample's radiance goes to its own slot of a buffer
// ([tile][sample][pixel of the tile], tiled_record); reduce_samples then sums every pixel's samples in sample order,
// so the image does not depend on which lane or wave computed a sample.
// ---------------------------------------------------------------------------
// The hit record's old contents are dead: freeze(poison) for every field, so the
// register allocator need not carry them through the walk that writes the next record.
template <class R>
__device__ __forceinline__ void forget(HitT<R>& h)
{
    h.t = __builtin_nondeterministic_value(h.t);
    h.px = __builtin_nondeterministic_value(h.px);
    h.py = __builtin_nondeterministic_value(h.py);
    h.pz = __builtin_nondeterministic_value(h.pz);
    h.nx = __builtin_nondeterministic_value(h.nx);
    h.ny = __builtin_nondeterministic_value(h.ny);
    h.nz = __builtin_nondeterministic_value(h.nz);
    h.uv0 = __builtin_nondeterministic_value(h.uv0);
    h.uv1 = __builtin_nondeterministic_value(h.uv1);
    h.uv2 = __builtin_nondeterministic_value(h.uv2);
    h.uv3 = __builtin_nondeterministic_value(h.uv3);
    h.front = __builtin_nondeterministic_value(h.front);
    h.mat = __builtin_nondeterministic_value(h.mat);
    h.uvkind = __builtin_nondeterministic_value(h.uvkind);
}

__device__ __forceinline__ unsigned lanes_below(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Per-sample pool, in-kernel reduction (kPoolRing): the whole wave sums one finished block —
// lane p the tile's pixel p — over its samples in order from 0.0, reduce_samples' chunk sum,
// and writes the chunk partial ([chunk][pixel], reduce_chunks' input). The block is one chunk
// of samples (block_samples == spp_chunk, chunk-aligned batches), so the chunk is its group.
#ifndef RING_LOADS
#define RING_LOADS 4
#endif
// lane q of v set to val (the ring state's writes; readlane reads it back as a scalar)
__device__ __forceinline__ int ring_set(int val, int q, int v) { return (int)__lane_id() == q ? val : v; }

template <class C>
__device__ __forceinline__ double* ring_of_wave(const KParams& P)
{
    const unsigned wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (unsigned)(BlockThreads<C>() / 64) + threadIdx.x / 64u);
    return P.ring + (size_t)wave * kRingWaveDoubles;
}
// the ring's header after the records: the block id of each slot (RingSgpr variants)
__device__ __forceinline__ unsigned* ring_block_id(double* ring_wave)
{
    return reinterpret_cast<unsigned*>(ring_wave + (size_t)kPoolRing * kRingSlot * 3);
}
// Where a wave tracks its blocks in flight. The spheres variant: the occupied slots and the
// current slot in SGPRs, the block ids in the ring's header (C2 1200x800x500 73.92 ms against
// 74.45 with the VGPR below; round 4's per-sample buffer 74.52). The others (the final variant's
// SGPRs are at the limit; there the SGPR form took C4 1920x1080x256 to 269.2 ms against 266.9):
// the lanes of one VGPR (profiles/r05o_ab_c{2,4}.log).
template <class C>
constexpr bool RingSgpr() { return C::F == FEAT_SET_SPHERES; }

__device__ __forceinline__ void ring_reduce(const KParams& P, const double* __restrict__ rec,
                                            double* __restrict__ partial, unsigned blk, unsigned n_tiles, unsigned group,
                                            size_t n_px, int lane)
{
    // the block's (sample group, tile), as trace_pool dealt it (KParams.deal_div)
    const unsigned outer = blk / P.deal_div, inner = blk - outer * P.deal_div;
    const unsigned grp = P.tile_major ? inner : outer, tile = P.tile_major ? outer : inner;
    const int s0 = P.sample_begin + (int)(grp * group);
    const int x = (int)(tile % (unsigned)P.tiles_x) * 8 + (lane & 7);
    const int k = (int)(tile / (unsigned)P.tiles_x) * 8 + (lane >> 3);
    const int ns = min(P.spp, s0 + (int)group) - s0;
    // the records were stored by lanes of this wave: order their stores before these loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // one channel at a time, RING_LOADS samples' loads in flight (the wave's path state stays live
    // beside them; one load per round trip left the wave waiting on L2 ~48 times per block)
    constexpr int NB = RING_LOADS;
    const bool own = x < P.width && k < P.n_rows;
    double* o = partial + ((size_t)grp * n_px + (size_t)k * P.width + x) * 3;
#pragma unroll 1
    for (int c = 0; c < 3; ++c) {
        const double* p = rec + (size_t)lane * 3 + c;
        double a = 0.0;
#pragma unroll 1
        for (int j0 = 0; j0 < ns; j0 += NB) {
            double v[NB];
#pragma unroll
            for (int j = 0; j < NB; ++j) v[j] = j0 + j < ns ? p[(size_t)j * 64 * 3] : 0.0;
#pragma unroll
            for (int j = 0; j < NB; ++j)
                if (j0 + j < ns) a = a + v[j];
            p += (size_t)NB * 64 * 3;
        }
        if (own) o[c] = a;
    }
}

// ITEMS (the item pool, default): a unit is a (pixel, chunk) item instead of one sample.
// The lane that takes it traces the chunk's samples in order, summing their radiance in
// registers exactly as trace_chunks does, and writes one partial per (pixel, chunk) when
// the last one ends; a lane whose item ended takes the next item at once, as in the
// per-sample pool, so lanes still do not idle. Output: chunk partials for
// reduce_chunks, 1/chunk of the per-sample buffer's bytes.
template <class C, bool ITEMS, bool RING = false>
__global__ void __launch_bounds__(BlockThreads<C>(), min_waves<C>()) trace_pool(SceneDev S, const KParams* __restrict__ Pp,
                                                                  double* __restrict__ samples,
                                                                  unsigned long long* __restrict__ counters,
                                                                  unsigned* __restrict__ work)
{
    const KParams& P = *Pp;
    stage_lds<C>(S);
    StackT<C> stack;
    if constexpr (Stack16Cfg<C>()) stack.base = reinterpret_cast<short*>(rt_lds + lds_stack_offset<C>(S)) + threadIdx.x;
    else if constexpr (C::LDS) stack.init((int)lds_stack_offset<C>(S));
    Count cnt{};
    uint64_t t_cam = 0, t_trace = 0, t_shade = 0, t_prev = 0, t_start = 0, t_sample = 0;
    if (C::COUNT) t_prev = t_start = __builtin_amdgcn_s_memtime();
    (void)t_trace;
    (void)t_start;
    (void)t_sample;
    const int lane = threadIdx.x & 63;
    const unsigned n_tiles = (unsigned)P.tiles_x * (unsigned)P.tiles_y;
    // a work block = one tile x block_chunks consecutive chunks (items chunk-major; the
    // per-sample pool's units sample-major): lanes stay on one tile longer, and its rays
    // are coherent (C2 item pool, chunks of 4: 108.4 ms with blocks of one chunk, 101.8 with 8)
    // per-sample pool: a block = one tile x block_samples consecutive samples (any count: the
    // per-sample output does not depend on it)
    const unsigned group = ITEMS ? (unsigned)P.block_chunks : (unsigned)P.block_samples;
    const unsigned n_blocks = P.n_work_blocks;   // n_tiles x ceil(samples or chunks / group)
    const size_t n_px = (size_t)P.n_rows * (size_t)P.width;
    // current work block (wave-uniform)
    unsigned blk_units = 0, blk_next = 0, nvalid = 1;
    int tx0 = 0, tk0 = 0, vw = 1, s0 = 0;
    bool exhausted = false;
    // lane state
    bool active = false, new_sample = false;
    int x = 0, k = 0, s = 0, depth = 0;
    int left = 0;      // ITEMS: samples of the lane's item still to trace after the current one
    bool own = false;  // ITEMS: the lane's item has a next sample (taken before any new unit)
    using R = typename C::Real;
    double cr = 0, cg = 0, cb = 0;
    R Tr = 1, Tg = 1, Tb = 1;
    Keyed key{P.seed, 0, 0, 0};
    rt_pstream st;
    RayT<R> r;
    HitT<R> h;             // a hit whose scattered ray the next iteration draws
    bool pending = false;
    bool cam_wait = false;  // RT_TRY_LEFT: camera_begin ran, the disk tries go on (u, v in r.dx, r.dy)
    (void)cam_wait;
    // In-kernel reduction (RING, the per-sample pool with P.ring; kPoolRing): the wave's blocks
    // in flight (RingSgpr: where), wave-uniform — the occupied slots (bit q), the slot units are
    // taken from, each slot's block. A lane's record index in the wave's ring (slot x kRingSlot +
    // sample of the block x 64 + pixel of the tile) rides in the bits of `s` above
    // kRingSampleBits, so a block is finished when it is not the one units are taken from and no
    // active lane holds one of its units.
    constexpr bool ring = RING && !ITEMS;
    // (the two forms are separate `if constexpr` blocks, not else-branches of one another: written
    // as else-branches the spheres variant's kernel compiled to other code, 1.4 % slower on C2)
    int ringv = 0;                       // !RingSgpr: lane q slot q's block, kRingCur, kRingOcc
    unsigned occ = 0, cur_slot = 0;      // RingSgpr (the other form: read from ringv where used)
    for (;;) {
        if constexpr (ring && !RingSgpr<C>()) {   // (final variant) the same, the state in ringv's lanes
            unsigned occv = (unsigned)__builtin_amdgcn_readlane(ringv, kRingOcc);
            if (occv != 0) {
                const unsigned open = blk_next < blk_units ? (unsigned)__builtin_amdgcn_readlane(ringv, kRingCur) : 99u;
#pragma unroll
                for (int q = 0; q < kPoolRing; ++q) {
                    if ((occv >> q & 1u) && (unsigned)q != open &&
                        __ballot(active && ((unsigned)s >> kRingSampleBits) / kRingSlot == (unsigned)q) == 0) {
                        ring_reduce(P, ring_of_wave<C>(P) + (size_t)q * kRingSlot * 3, samples,
                                    (unsigned)__builtin_amdgcn_readlane(ringv, q), n_tiles, group, n_px, lane);
                        occv &= ~(1u << q);
                        ringv = ring_set((int)occv, kRingOcc, ringv);
                    }
                }
            }
        }
        if (ring && RingSgpr<C>()) {   // blocks whose last sample ended: every pixel's samples summed in order
            if (occ != 0) {
                const unsigned open = blk_next < blk_units ? cur_slot : 99u;
#pragma unroll
                for (int q = 0; q < kPoolRing; ++q) {
                    if ((occ >> q & 1u) && (unsigned)q != open &&
                        __ballot(active && ((unsigned)s >> kRingSampleBits) / kRingSlot == (unsigned)q) == 0) {
                        double* rw = ring_of_wave<C>(P);
                        ring_reduce(P, rw + (size_t)q * kRingSlot * 3, samples,
                                    (unsigned)__builtin_amdgcn_readfirstlane(ring_block_id(rw)[q]), n_tiles, group, n_px, lane);
                        occ &= ~(1u << q);
                    }
                }
            }
        }
        if (ITEMS && own) {
            own = false;
            active = true;
            new_sample = true;
            s += 1;
            left -= 1;
        }
        uint64_t need = __ballot(!active);
        while (need != 0 && !exhausted) {
            if (blk_next == blk_units) {
                int free_slot = -1;
                if (ring) {   // a free ring slot first: every one holds an unfinished block -> wait
                    if constexpr (!RingSgpr<C>()) occ = (unsigned)__builtin_amdgcn_readlane(ringv, kRingOcc);
                    if (occ == (1u << kPoolRing) - 1) break;
                    free_slot = __builtin_ctz(~occ);
                }
                unsigned b = 0;
                if (lane == 0) b = atomicAdd(work, 1u);
                b = __builtin_amdgcn_readfirstlane(b);
                if (b >= n_blocks) {
                    exhausted = true;
                    break;
                }
                // group-major (b = grp * n_tiles + tile) or, under a tile order, tile-major
                // (b = tile * n_groups + grp): one division by KParams.deal_div either way
                // group-major (b = grp * n_tiles + tile) or, under a tile order, tile-major
                // (b = tile * n_groups + grp; KParams.deal_div). Two forms of the same mapping: the
                // branch kept the spheres variant's code as it was (a select moved it, C2 +1.1 %),
                // the select the final variant's (the branch added 8 B of spill to its ring kernel)
                unsigned grp, tile;
                if constexpr (C::F == FEAT_SET_SPHERES) {
                    if (__builtin_expect(P.tile_major != 0, 0)) {   // (wave-uniform)
                        tile = b / P.deal_div;
                        grp = b - tile * P.deal_div;
                    } else {
                        grp = b / n_tiles;
                        tile = b - grp * n_tiles;
                    }
                } else {
                    const unsigned outer = b / P.deal_div, inner = b - outer * P.deal_div;
                    grp = P.tile_major ? inner : outer;
                    tile = P.tile_major ? outer : inner;
                }
                tx0 = (int)(tile % (unsigned)P.tiles_x) * 8;
                tk0 = (int)(tile / (unsigned)P.tiles_x) * 8;
                vw = min(8, P.width - tx0);
                nvalid = (unsigned)(vw * min(8, P.n_rows - tk0));
                if constexpr (ITEMS) {
                    const unsigned chunk = grp * group;
                    s0 = P.sample_begin + (int)chunk * P.spp_chunk;
                    blk_units = nvalid * min(group, (unsigned)P.n_chunks - chunk);
                } else {
                    s0 = P.sample_begin + (int)(grp * group);
                    blk_units = nvalid * (unsigned)(min(P.spp, s0 + (int)group) - s0);
                    if (ring) {
                        if constexpr (RingSgpr<C>()) {   // the block id waits in the ring's header
                            if (lane == 0) ring_block_id(ring_of_wave<C>(P))[free_slot] = b;
                            cur_slot = (unsigned)free_slot;
                            occ |= 1u << free_slot;
                        }
                        if constexpr (!RingSgpr<C>()) {
                            ringv = ring_set((int)b, free_slot, ringv);
                            ringv = ring_set(free_slot, kRingCur, ringv);
                            ringv = ring_set((int)(occ | 1u << free_slot), kRingOcc, ringv);
                        }
                    }
                }
                blk_next = 0;
            }
            const unsigned rank = lanes_below(need);
            const unsigned take = min((unsigned)__popcll(need), blk_units - blk_next);
            if (!active && rank < take) {
                const unsigned u = blk_next + rank;
                unsigned si;
                if (nvalid == 64u) {  // a full 8x8 tile (wave-uniform): shifts, not divisions
                    si = u >> 6;
                    x = tx0 + (int)(u & 7u);
                    k = tk0 + (int)((u >> 3) & 7u);
                } else {
                    si = u / nvalid;
                    const unsigned p = u - si * nvalid;
                    x = tx0 + (int)(p % (unsigned)vw);
                    k = tk0 + (int)(p / (unsigned)vw);
                }
                if constexpr (ITEMS) {  // si: the item's chunk within the block; s its first sample
                    s = s0 + (int)si * P.spp_chunk;
                    left = min(P.spp, s + P.spp_chunk) - s - 1;
                    cr = cg = cb = 0.0;
                } else {
                    s = s0 + (int)si;
                    if (ring) {
                        if constexpr (!RingSgpr<C>()) cur_slot = (unsigned)__builtin_amdgcn_readlane(ringv, kRingCur);
                        s |= (int)((cur_slot * kRingSlot + si * 64u + (unsigned)((k & 7) * 8 + (x & 7))) << kRingSampleBits);
                    }
                }
                active = true;
                new_sample = true;
            }
            blk_next += take;
            need = __ballot(!active);
        }
        if (!__any(active)) break;
        if (C::COUNT && first_active_lane()) cnt.wave_steps++;
        if (C::COUNT) {   // lanes the refill left idle: nothing left to take, or (RING) no free slot
            const uint64_t idle = __ballot(!active);
            if (first_active_lane()) {
                if (exhausted) cnt.idle_tail += (uint32_t)__popcll(idle);
                else cnt.idle_ring += (uint32_t)__popcll(idle);
            }
        }
        if (!active) continue;
        // (COUNT) refill and loop overhead since the last iteration's end stamp: lanes refilled this
        // iteration were idle, so their stamp is old — take the wave's latest (max over lanes)
        if (C::COUNT) {
            unsigned long long tw = t_prev;
            for (int off = 32; off > 0; off >>= 1) {
                const unsigned long long o = __shfl_xor(tw, off);
                tw = tw > o ? tw : o;
            }
            t_prev = tw;
            RT_STAMP(cnt.t_refill, t_prev);
        }
        // Ray generation: the camera rays of new samples and the scattered rays of last
        // iteration's hits (pending), whose random_in_unit_disk / random_in_unit_sphere tries
        // run in one rejection loop (the wave used to run the two loops one after the other).
        // Each lane's draws keep their order (its stream is its own), so the bits do not change.
        bool go = true;   // the lane traces this iteration
        bool gen_wait = false;   // RT_TRY_LEFT: the lane's tries go on in the next iteration
        {
            R u = 0, v = 0;
            bool tries = false;
            if (new_sample) {
                if (TryLeft<C>() && cam_wait) {   // camera_begin ran: the jitter waits in r.dx / r.dy
                    u = r.dx;
                    v = r.dy;
                    cam_wait = false;
                } else {
                    if (C::COUNT) {
                        cnt.cam_lanes++;
                        if (first_active_lane()) cnt.cam_steps++;
                    }
                    int ix, y;
                    image_xy(P, x, k, ix, y);
                    if (C::COUNT) t_sample = __builtin_amdgcn_s_memtime();
                    key.pixel = (uint32_t)y * (uint32_t)P.img_width + (uint32_t)ix;
                    const uint32_t sample = ring ? (uint32_t)s & kRingSampleMask : (uint32_t)s;
                    key.sample = sample;
                    if constexpr (C::F32) ds_start_f32(st, P.seed, key.pixel, sample);
                    else ds_start(st, P.seed, key.pixel, sample);
                    camera_begin(P, ix, y, st, u, v);
                    Tr = Tg = Tb = (R)1;
                    if constexpr (!ITEMS) cr = cg = cb = 0.0;  // ITEMS: the chunk's running sum
                    depth = P.max_depth;
                }
                tries = true;
            } else if (pending) {
                tries = shade_draws<C>(S, h.mat);
            }
            RT_STAMP(cnt.t_seed, t_prev);
            R qx = (R)0, qy = (R)0, qz = (R)0, l2 = (R)1;
            const bool three = !new_sample;
            if constexpr (TryLeft<C>()) {
                bool accepted = !tries;
                for (int n = 1;; ++n) {
                    if (!accepted) accepted = unit_try(st, (R)P.scale_m11, three, qx, qy, qz, l2);
                    const uint64_t rejecting = __ballot(!accepted);
                    if (rejecting == 0 || (n >= RT_TRY_MIN && __popcll(rejecting) <= RT_TRY_LEFT)) break;
                }
                gen_wait = !accepted;
            } else {
                while (tries && !unit_try(st, (R)P.scale_m11, three, qx, qy, qz, l2)) {
                }
            }
            RT_STAMP(cnt.t_tries, t_prev);
            if (gen_wait) {   // (RT_TRY_LEFT) no trace this iteration; pending / new_sample stay set
                go = false;
                if (new_sample) {
                    cam_wait = true;
                    r.dx = u;
                    r.dy = v;
                }
            } else if (new_sample) {
                new_sample = false;
                camera_end(P, st, u, v, qx, qy, r);
            } else if (pending) {
                pending = false;
                go = shade_end<C, false>(S, h, r, st, Tr, Tg, Tb, qx, qy, qz, l2);
                if (go) depth -= 1;
            }
        }
        RT_STAMP(t_cam, t_prev);
        if (C::COUNT) {
            cnt.try_wait += gen_wait ? 1u : 0u;
            cnt.no_scatter += (!go && !gen_wait) ? 1u : 0u;
            cnt.depth_cap += (go && depth <= 0) ? 1u : 0u;
        }
        if (go && depth > 0) {  // main.rs:21-23: depth 0 is black
            key.bounce = (uint32_t)(P.max_depth - depth);
            if (C::COUNT) cnt.casts++;
            finish_ray<C>(r, S.has_spheres != 0);
            forget(h);
            RT_STAMP(cnt.t_setup, t_prev);
            const bool hit = trace_world<C>(S, r, h, stack, key, cnt);
            if (C::COUNT) t_prev = __builtin_amdgcn_s_memtime();   // trace_world stamped its phases
            if (!hit) {  // main.rs:37: background
                cr = cr + Tr * P.bg[0];
                cg = cg + Tg * P.bg[1];
                cb = cb + Tb * P.bg[2];
            } else {
                if (C::COUNT) {
                    cnt.shade_lanes++;
                    if (first_active_lane()) cnt.shade_steps++;
                }
                pending = shade_begin<C>(S, h, Tr, Tg, Tb, cr, cg, cb);
            }
            RT_STAMP(t_shade, t_prev);
        }
        if (C::COUNT) t_prev = __builtin_amdgcn_s_memtime();   // lanes that did not trace
        if (C::COUNT && P.tile_cost && !(pending || gen_wait)) {   // the sample ended: its lane-cycles to its tile
            int ix, y;
            image_xy(P, x, k, ix, y);
            atomicAdd(&P.tile_cost[(unsigned)(y >> 3) * (unsigned)P.img_tiles_x + (unsigned)(ix >> 3)],
                      (unsigned long long)(t_prev - t_sample));
        }
        if (pending || gen_wait) {
        } else if (ITEMS && left > 0) {  // the item's next sample: the lane takes it at the loop top
            active = false;
            own = true;
        } else {
            // items: the chunk's partial, [chunk][pixel]; per-sample pool: tiled_record order,
            // or (ring) the record index taken with the unit (in the high bits of s)
            double* o;
            if (ITEMS) {
                o = samples + ((size_t)((unsigned)(s - P.sample_begin) / (unsigned)P.spp_chunk) * n_px +
                               (size_t)k * P.width + x) * 3;
            } else if (ring) {
                o = ring_of_wave<C>(P) + (size_t)((unsigned)s >> kRingSampleBits) * 3;
            } else {
                o = samples + tiled_record(P.tiles_x, P.spp - P.sample_begin, x, k, s - P.sample_begin) * 3;
            }
            if constexpr (C::F32 && !ITEMS && !ring) {
                // the f32 mode's per-sample records are f32 (SampleTiles.f32_records): half the bytes
                float* of = reinterpret_cast<float*>(samples) +
                            tiled_record(P.tiles_x, P.spp - P.sample_begin, x, k, s - P.sample_begin) * 3;
                of[0] = (float)cr;
                of[1] = (float)cg;
                of[2] = (float)cb;
                (void)o;
            } else {
                o[0] = cr;
                o[1] = cg;
                o[2] = cb;
            }
            active = false;
        }
    }
    if (C::COUNT) {
        atomicAdd(&counters[0], (unsigned long long)cnt.casts);
        atomicAdd(&counters[1], (unsigned long long)cnt.nodes);
        atomicAdd(&counters[2], (unsigned long long)cnt.prims);
        atomicAdd(&counters[6], (unsigned long long)cnt.wave_steps);
        atomicAdd(&counters[7], (unsigned long long)cnt.wave_nodes);
        atomicAdd(&counters[10], (unsigned long long)cnt.wave_leaves);
        atomicAdd(&counters[11], (unsigned long long)cnt.cam_lanes);
        atomicAdd(&counters[12], (unsigned long long)cnt.cam_steps);
        atomicAdd(&counters[13], (unsigned long long)cnt.shade_lanes);
        atomicAdd(&counters[14], (unsigned long long)cnt.shade_steps);
        // phase times: each region's first active lane added its intervals, so every lane's
        // share goes in (trace = everything from the ray set-up to the hit record)
        const uint64_t trace = cnt.t_setup + cnt.t_pre + cnt.t_nodes + cnt.t_leaves + cnt.t_defer + cnt.t_rec;
        atomicAdd(&counters[3], (unsigned long long)(t_cam + cnt.t_seed + cnt.t_tries));   // ray generation, all of it
        atomicAdd(&counters[23], (unsigned long long)cnt.t_seed);
        atomicAdd(&counters[24], (unsigned long long)cnt.t_tries);
        atomicAdd(&counters[4], (unsigned long long)trace);
        atomicAdd(&counters[5], (unsigned long long)t_shade);
        atomicAdd(&counters[8], (unsigned long long)cnt.t_nodes);
        atomicAdd(&counters[9], (unsigned long long)cnt.t_leaves);
        atomicAdd(&counters[15], (unsigned long long)cnt.t_setup);
        atomicAdd(&counters[16], (unsigned long long)cnt.t_pre);
        atomicAdd(&counters[17], (unsigned long long)cnt.t_rec);
        atomicAdd(&counters[18], (unsigned long long)cnt.t_med);
        atomicAdd(&counters[19], (unsigned long long)cnt.t_inst);
        atomicAdd(&counters[20], (unsigned long long)cnt.t_refill);
        atomicAdd(&counters[22], (unsigned long long)cnt.t_defer);
        atomicAdd(&counters[27], (unsigned long long)cnt.idle_tail);
        atomicAdd(&counters[28], (unsigned long long)cnt.idle_ring);
        atomicAdd(&counters[29], (unsigned long long)cnt.no_scatter);
        atomicAdd(&counters[30], (unsigned long long)cnt.depth_cap);
        atomicAdd(&counters[31], (unsigned long long)cnt.try_wait);
        if (lane == 0) {   // the wave's lifetime; the longest, and the wave count (the launch's tail: 25, 26)
            const unsigned long long life = __builtin_amdgcn_s_memtime() - t_start;
            atomicAdd(&counters[21], life);
            atomicMax(&counters[25], life);
            atomicAdd(&counters[26], 1ull);
        }
    }
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
struct Launch {
    const SceneDev* S;
    const KParams* P;
    double* out;                   // chunk partials (chunk schedule) or per-sample radiance (pool)
    unsigned long long* counters;
    unsigned* work;                // pool / items: work-block counter
    int pool;                      // 0 chunks, 1 per-sample pool, 2 item pool
    unsigned long long n_blocks;   // 8x8 tiles x chunks
    int* waves_per_simd;           // out (optional): resident blocks per CU = waves per SIMD (4-wave blocks)
    unsigned max_waves = 0;        // per-sample pool with the in-kernel reduction: waves its ring holds
};

// Resident blocks per CU of a kernel (registers, LDS); waves per SIMD reported to the caller.
template <class K>
static int blocks_per_cu(const Launch& L, K kernel, size_t lds, int bt)
{
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, bt, lds) != hipSuccess || per_cu <= 0) per_cu = 1;
    if (L.waves_per_simd) *L.waves_per_simd = per_cu * (bt / 256);   // 4 SIMDs per CU
    return per_cu;
}

// Persistent grid for the pool schedule: as many blocks as fit on the device at once.
template <class K>
static unsigned resident_blocks(const Launch& L, K kernel, size_t lds, int bt)
{
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    }
    return (unsigned)(cus * blocks_per_cu(L, kernel, lds, bt));
}

template <uint32_t F, bool S32, bool LDS, bool COUNT, bool F32>
static void launch_one(const Launch& L, hipStream_t stream, bool nall)
{
    const SceneDev& S = *L.S;
    const bool s16 = RT_STACK16 && LDS && nall && S32 && F == FEAT_SET_SPHERES;   // Stack16Cfg
    const int node_bytes = nall && S32 ? (int)sizeof(LdsNode) : (int)sizeof(rt_bvh_node);   // lds_node_bytes
    const bool stage = F != FEAT_SET_SPHERES;                   // StageShade
    const bool blas = RT_STAGE_BLAS && (F & FEAT_INST_BLAS) != 0;   // StageBlas
    const int bt = block_threads_of(F, F32, RT_STACK16 && LDS && nall && S32), wpb = bt / 64;   // BlockThreads
    const size_t lds = lds_layout(S.n_lds_nodes, node_bytes, blas ? S.n_lds_blas : 0, LDS ? S.stack_entries : 0,
                                  s16 ? 2 : 4, stage ? S.n_lds_materials : 0, stage ? S.n_lds_textures : 0, bt).total;
    if (L.pool) {
        auto go = [&](auto kernel) {
            unsigned nb = std::min<unsigned long long>(resident_blocks(L, kernel, lds, bt), (L.n_blocks + wpb - 1) / wpb);
            if (L.max_waves) nb = std::max(1u, std::min(nb, L.max_waves / (unsigned)wpb));
            hipLaunchKernelGGL(kernel, dim3(nb), dim3(bt), lds, stream, S, L.P, L.out, L.counters, L.work);
        };
        if (L.pool == 2) {
            if (nall) go(trace_pool<Cfg<F, S32, LDS, true, COUNT, F32>, true>);
            else go(trace_pool<Cfg<F, S32, LDS, false, COUNT, F32>, true>);
        } else if (L.max_waves) {   // the per-sample pool reducing in the kernel (KParams.ring)
            if (nall) go(trace_pool<Cfg<F, S32, LDS, true, COUNT, F32>, false, true>);
            else go(trace_pool<Cfg<F, S32, LDS, false, COUNT, F32>, false, true>);
        } else {
            if (nall) go(trace_pool<Cfg<F, S32, LDS, true, COUNT, F32>, false>);
            else go(trace_pool<Cfg<F, S32, LDS, false, COUNT, F32>, false>);
        }
        return;
    }
    const unsigned nb = (unsigned)((L.n_blocks + wpb - 1) / wpb);
    auto go = [&](auto kernel) {
        if (L.waves_per_simd) (void)blocks_per_cu(L, kernel, lds, bt);
        hipLaunchKernelGGL(kernel, dim3(nb), dim3(bt), lds, stream, S, L.P, L.out, L.counters);
    };
    if (nall) go(trace_chunks<Cfg<F, S32, LDS, true, COUNT, F32>>);
    else go(trace_chunks<Cfg<F, S32, LDS, false, COUNT, F32>>);
}

// Variant table: feature set x slab precision x loop form. The launcher takes the
// smallest feature set covering the scene.
template <uint32_t F, bool COUNT>
static void launch_f(const Launch& L, int slab32, int lds, hipStream_t stream)
{
    const SceneDev& S = *L.S;
    bool nall = S.n_lds_nodes > 0 && S.n_lds_nodes == S.n_tlas_nodes;
    // the whole-TLAS spheres instantiation keeps 16-bit stack entries (Stack16Cfg): a scene
    // whose node addresses or leaf codes do not fit takes the partial-TLAS instantiation
    constexpr bool S16F = F == FEAT_SET_SPHERES;   // Stack16Cfg's feature set
    if (RT_STACK16 && S16F && slab32 && lds && !S.stack16_ok) nall = false;
    // stack16_ok (abi.cpp) assumes the node records start at LDS address 0, i.e. that rt_lds is
    // the kernels' only __shared__ object: a static __shared__ variable would move the dynamic
    // base up, and 16-bit stack entries would truncate node addresses past 32 KB. Checked on the
    // compiled kernels: any static LDS in them sends the scene to the 32-bit-stack instantiation.
    if (RT_STACK16 && S16F && slab32 && lds && nall) {
        static int static_lds = -1;
        if (static_lds < 0) {
            static_lds = 0;
            hipFuncAttributes a;
            const void* ks[4] = {(const void*)trace_pool<Cfg<F, true, true, true, COUNT, false>, false>,
                                 (const void*)trace_pool<Cfg<F, true, true, true, COUNT, false>, true>,
                                 (const void*)trace_pool<Cfg<F, true, true, true, COUNT, false>, false, true>,
                                 (const void*)trace_chunks<Cfg<F, true, true, true, COUNT, false>>};
            for (const void* k : ks)
                if (hipFuncGetAttributes(&a, k) != hipSuccess || a.sharedSizeBytes != 0) static_lds = 1;
        }
        if (static_lds) nall = false;
    }
    if (slab32) {
        if (lds) launch_one<F, true, true, COUNT, false>(L, stream, nall);
        else launch_one<F, true, false, COUNT, false>(L, stream, nall);
    } else {
        if (lds) launch_one<F, false, true, COUNT, false>(L, stream, nall);
        else launch_one<F, false, false, COUNT, false>(L, stream, nall);
    }
}

// One feature set's kernels, timed or counting (trace_v_*.hip instantiate one pair each,
// one translation unit per pair).
template <uint32_t F, bool COUNT>
hipError_t launch_variant(const Launch& L, const LaunchOpts& o, hipStream_t stream)
{
    launch_f<F, COUNT>(L, o.slab32, o.lds_stack, stream);
    return hipGetLastError();
}

// The f32 fast mode's kernels of one feature set (trace_f32_*.hip): f32 slab tests always
// (an f32 path gains nothing from f64 boxes), no count variant.
// The whole-TLAS spheres instantiation keeps 16-bit stack entries (Stack16Cfg), as launch_f's: a
// scene whose node addresses or leaf codes do not fit takes the partial-TLAS instantiation.
inline bool f32_nall(const SceneDev& S, uint32_t F, bool lds)
{
    const bool nall = S.n_lds_nodes > 0 && S.n_lds_nodes == S.n_tlas_nodes;
    return nall && !(RT_STACK16 && F == FEAT_SET_SPHERES && lds && !S.stack16_ok);
}
template <uint32_t F>
hipError_t launch_variant_f32(const Launch& L, const LaunchOpts& o, hipStream_t stream)
{
    const bool nall = f32_nall(*L.S, F, o.lds_stack);
    if (o.lds_stack) launch_one<F, true, true, false, true>(L, stream, nall);
    else launch_one<F, true, false, false, true>(L, stream, nall);
    return hipGetLastError();
}

// The f32 mode's count_work variant (final scene and spheres: the f32-vs-f64 path-length and
// step-cost comparison of DESIGN.md §5.6; trace_f32_*_count.hip)
template <uint32_t F>
hipError_t launch_variant_f32_count(const Launch& L, const LaunchOpts& o, hipStream_t stream)
{
    const bool nall = f32_nall(*L.S, F, o.lds_stack);
    if (o.lds_stack) launch_one<F, true, true, true, true>(L, stream, nall);
    else launch_one<F, true, false, true, true>(L, stream, nall);
    return hipGetLastError();
}
#define RT_VARIANT_DECL(F, COUNT) \
    extern template hipError_t launch_variant<F, COUNT>(const Launch&, const LaunchOpts&, hipStream_t);
#define RT_VARIANT_F32_DECL(F) \
    extern template hipError_t launch_variant_f32<F>(const Launch&, const LaunchOpts&, hipStream_t);
RT_VARIANT_DECL(FEAT_SET_SPHERES, false)
RT_VARIANT_DECL(FEAT_SET_SPHERES, true)
RT_VARIANT_DECL(FEAT_SET_RECTINST, false)
RT_VARIANT_DECL(FEAT_SET_RECTINST, true)
RT_VARIANT_DECL(FEAT_SET_MEDIA, false)
RT_VARIANT_DECL(FEAT_SET_MEDIA, true)
RT_VARIANT_DECL(FEAT_SET_FINAL, false)
RT_VARIANT_DECL(FEAT_SET_FINAL, true)
RT_VARIANT_DECL(FEAT_ALL, false)
RT_VARIANT_DECL(FEAT_ALL, true)
RT_VARIANT_F32_DECL(FEAT_SET_SPHERES)
RT_VARIANT_F32_DECL(FEAT_SET_RECTINST)
RT_VARIANT_F32_DECL(FEAT_SET_MEDIA)
RT_VARIANT_F32_DECL(FEAT_SET_FINAL)
RT_VARIANT_F32_DECL(FEAT_ALL)
extern template hipError_t launch_variant_f32_count<FEAT_SET_SPHERES>(const Launch&, const LaunchOpts&, hipStream_t);
extern template hipError_t launch_variant_f32_count<FEAT_SET_FINAL>(const Launch&, const LaunchOpts&, hipStream_t);
#undef RT_VARIANT_DECL
#undef RT_VARIANT_F32_DECL

}  // namespace rtk
