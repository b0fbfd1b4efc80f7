/*
 * rt_numerics.h — deterministic numeric core shared by the HIP megakernel, the
 * C++ host and the CPU oracle.
 *
 * Why this exists: per-pixel parity between
 * the GPU path and the CPU restatement of the reference needs every random draw
 * and every transcendental to produce the SAME BITS on the host (gcc / clang,
 * x86-64 SSE2) and on gfx950. So this header provides, in plain C that also
 * compiles as HIP:
 *
 *   - Philox4x32-10 (Salmon et al., SC'11), the counter RNG that replaces the
 *     reference's unseedable `rand::thread_rng()` (math.rs:268-276). KAT-checked
 *     against Random123's published vectors and ROCm's rocrand host engine. It
 *     drives scene construction directly and seeds one xoshiro128++ path stream per
 *     (pixel, sample) for rendering.
 *   - The `rand` 0.8 float mappings the reference calls:
 *       random_double()            -> `Standard` f64: (u64 >> 11) * 2^-53
 *       random_double_range(a, b)  -> `gen_range(a..=b)`: UniformFloat
 *                                     new_inclusive + sample (52-bit mantissa)
 *     (math.rs:268-276; rand 0.8 src/distributions/{float,uniform}.rs,
 *     restated — the crate is not vendored, version unpinned: Cargo.toml:8).
 *   - sin / log / atan / atan2 / acos written only with IEEE +,-,*,/,sqrt,
 *     rint and bit manipulation (fdlibm / musl algorithms and minimax
 *     coefficients, restated), so host and device agree bit-for-bit where a
 *     libm / ocml pair would differ in the last ulp.
 *
 * The sin / log / atan / acos restatements follow fdlibm (via musl's src/math), whose
 * permission notice is preserved here as it asks:
 *
 *   ====================================================
 *   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
 *
 *   Developed at SunPro, a Sun Microsystems, Inc. business.
 *   Permission to use, copy, modify, and distribute this
 *   software is freely granted, provided that this notice
 *   is preserved.
 *   ====================================================
 *
 * Everything here must be compiled WITHOUT fast-math and WITHOUT FP contraction
 * (-ffp-contract=off): the reference relies on IEEE NaN/inf comparison
 * semantics and parity relies on exact rounding.
 */
#ifndef RT_NUMERICS_H
#define RT_NUMERICS_H

#include <stdint.h>

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#if defined(__HIP__)
#define RT_HD __host__ __device__ static inline
#else
#define RT_HD static inline
#endif

#define RT_PI 3.1415926535897932385 /* math.rs:5 */
#define RT_INF (__builtin_inf())

/* ------------------------------------------------------------------------- */
/* bit helpers                                                                */
/* ------------------------------------------------------------------------- */
RT_HD uint64_t rt_f64_bits(double x) { uint64_t u; __builtin_memcpy(&u, &x, 8); return u; }
RT_HD double rt_bits_f64(uint64_t u) { double x; __builtin_memcpy(&x, &u, 8); return x; }

/* ------------------------------------------------------------------------- */
/* Philox4x32-10                                                              */
/* ------------------------------------------------------------------------- */
typedef struct { uint32_t v[4]; } rt_u32x4;

RT_HD rt_u32x4 rt_philox4x32_10(rt_u32x4 c, uint32_t k0, uint32_t k1)
{
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c.v[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c.v[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        rt_u32x4 n;
        n.v[0] = hi1 ^ c.v[1] ^ k0;
        n.v[1] = lo1;
        n.v[2] = hi0 ^ c.v[3] ^ k1;
        n.v[3] = lo0;
        c = n;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

/* Counter layout of the Philox streams:
 *   c0 = pixel index y*W + x (image coordinates, y = 0 at the bottom)
 *   c1 = sample index
 *   c2 = 0 for the path seed                  | bounce for keyed draws
 *   c3 = RT_STREAM_PATH                       | RT_STREAM_MEDIUM + medium id
 * The scene-construction stream uses c3 = RT_STREAM_SCENE, c0/c1 = block index.
 */
#define RT_STREAM_PATH 0x9A750000u
#define RT_STREAM_SCENE 0x5CE4E000u
#define RT_STREAM_MEDIUM 0x10000u

/* Sequential Philox stream (scene construction): 2 u64 per block, consumed in order. */
typedef struct {
    uint32_t k0, k1;      /* key = seed */
    uint32_t c0, c1, c3;  /* fixed counter words */
    uint32_t blk;         /* next block index (c2) */
    uint32_t have;        /* 1 if spare holds an unread u64 */
    uint64_t spare;
} rt_stream;

RT_HD void rt_stream_init(rt_stream* s, uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c3)
{
    s->k0 = (uint32_t)seed;
    s->k1 = (uint32_t)(seed >> 32);
    s->c0 = c0; s->c1 = c1; s->c3 = c3;
    s->blk = 0; s->have = 0; s->spare = 0;
}

RT_HD uint64_t rt_stream_next_u64(rt_stream* s)
{
    if (s->have) { s->have = 0; return s->spare; }
    rt_u32x4 c; c.v[0] = s->c0; c.v[1] = s->c1; c.v[2] = s->blk; c.v[3] = s->c3;
    rt_u32x4 r = rt_philox4x32_10(c, s->k0, s->k1);
    s->blk += 1;
    s->spare = ((uint64_t)r.v[3] << 32) | r.v[2];
    s->have = 1;
    return ((uint64_t)r.v[1] << 32) | r.v[0];
}

/* Path stream (every draw of one (pixel, sample) path): one
 * Philox4x32-10 block of (pixel, sample, 0, RT_STREAM_PATH) under the render seed is the
 * 128-bit state of a xoshiro128++ generator (Blackman & Vigna, "Scrambled linear
 * pseudorandom number generators", 2019/2021: 32-bit state words, output
 * rotl(s0 + s3, 7) + s0), from which the path draws in the reference's order, one u64
 * per draw = (first output << 32) | second output. The stream is a function of
 * (seed, pixel, sample) only, like the counter streams it replaces, at two xoshiro steps
 * (add / shift / xor / rotate) per draw instead of half a Philox block (ten rounds of
 * 32x32->64 products): the draws of the unit-sphere and unit-disk rejection loops are
 * cheap enough to run at the pace of a wave's slowest lane. The all-zero state (the
 * generator's fixed point, probability 2^-128) is replaced by s0 = 1. */
typedef struct { uint32_t s0, s1, s2, s3; } rt_pstream;

RT_HD void rt_pstream_init(rt_pstream* p, uint64_t seed, uint32_t pixel, uint32_t sample)
{
    rt_u32x4 c; c.v[0] = pixel; c.v[1] = sample; c.v[2] = 0; c.v[3] = RT_STREAM_PATH;
    rt_u32x4 r = rt_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    p->s0 = r.v[0]; p->s1 = r.v[1]; p->s2 = r.v[2]; p->s3 = r.v[3];
    if ((p->s0 | p->s1 | p->s2 | p->s3) == 0) p->s0 = 1;
}

RT_HD uint32_t rt_rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

/* xoshiro128++ next() */
RT_HD uint32_t rt_pstream_u32(rt_pstream* p)
{
    const uint32_t result = rt_rotl32(p->s0 + p->s3, 7) + p->s0;
    const uint32_t t = p->s1 << 9;
    p->s2 ^= p->s0;
    p->s3 ^= p->s1;
    p->s1 ^= p->s2;
    p->s0 ^= p->s3;
    p->s2 ^= t;
    p->s3 = rt_rotl32(p->s3, 11);
    return result;
}

RT_HD uint64_t rt_pstream_u64(rt_pstream* p)
{
    const uint64_t hi = rt_pstream_u32(p);
    return (hi << 32) | rt_pstream_u32(p);
}

/* One keyed u64 (medium draws; counter = pixel, sample, bounce, stream). */
RT_HD uint64_t rt_keyed_u64(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3)
{
    rt_u32x4 c; c.v[0] = c0; c.v[1] = c1; c.v[2] = c2; c.v[3] = c3;
    rt_u32x4 r = rt_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    return ((uint64_t)r.v[1] << 32) | r.v[0];
}

/* rand 0.8 `Standard` for f64: 53 high bits times 2^-53, in [0, 1). */
RT_HD double rt_unit53(uint64_t x) { return (double)(x >> 11) * 0x1.0p-53; }

/* rand 0.8 UniformFloat<f64>::new_inclusive(low, high): scale such that
 * max_rand * scale + low <= high, max_rand = 1 - 2^-52. */
RT_HD double rt_uniform_incl_scale(double low, double high)
{
    const double max_rand = 1.0 - 0x1.0p-52;
    double scale = (high - low) / max_rand;
    while (scale * max_rand + low > high)
        scale = rt_bits_f64(rt_f64_bits(scale) - 1);
    return scale;
}

/* UniformFloat::sample: value1_2 from 52 mantissa bits, minus 1, times scale, plus low. */
RT_HD double rt_uniform_sample(uint64_t x, double low, double scale)
{
    double v12 = rt_bits_f64((x >> 12) | 0x3FF0000000000000ull);
    double v01 = v12 - 1.0;
    return v01 * scale + low;
}

/* Rust `f as usize` / `f as i32`: saturating, NaN -> 0. */
RT_HD uint64_t rt_sat_u64(double x)
{
    if (!(x > 0.0)) return 0;
    if (x >= 18446744073709551616.0) return ~(uint64_t)0;
    return (uint64_t)x;
}
RT_HD int32_t rt_sat_i32(double x)
{
    if (x != x) return 0;
    if (x <= -2147483648.0) return (int32_t)0x80000000u;
    if (x >= 2147483647.0) return 2147483647;
    return (int32_t)x;
}

/* ------------------------------------------------------------------------- */
/* sin (fdlibm/musl: Cody-Waite reduction by pi/2 + minimax kernels)          */
/* ------------------------------------------------------------------------- */
RT_HD double rt__ksin(double x, double y, int iy)
{
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x;
    double w = z * z;
    double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    double v = z * x;
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

RT_HD double rt__kcos(double x, double y)
{
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double w = z * z;
    double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    double hz = 0.5 * z;
    w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}

/* x = n*pi/2 + (y0 + y1); deterministic for all finite x (accurate to
 * |x| < 2^20*pi/2 — far beyond any argument the path produces). */
RT_HD int rt__rem_pio2(double x, double* y0, double* y1)
{
    const double invpio2 = 6.36619772367581382433e-01,
                 pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11,
                 pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21,
                 pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32;
    double fn = __builtin_rint(x * invpio2);
    double r = x - fn * pio2_1;
    double w = fn * pio2_1t;
    double y = r - w;
    int ex = (int)((rt_f64_bits(x) >> 52) & 0x7ff);
    int ey = (int)((rt_f64_bits(y) >> 52) & 0x7ff);
    if (ex - ey > 16) {
        double t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        y = r - w;
        ey = (int)((rt_f64_bits(y) >> 52) & 0x7ff);
        if (ex - ey > 49) {
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            y = r - w;
        }
    }
    *y0 = y;
    *y1 = (r - y) - w;
    /* n mod 4 (fn is integral; fmod-free for |fn| < 2^53) */
    double q = fn - 4.0 * __builtin_floor(fn * 0.25);
    return (int)q;
}

RT_HD double rt_sin(double x)
{
    uint32_t ix = (uint32_t)(rt_f64_bits(x) >> 32) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) {              /* |x| ~< pi/4 */
        if (ix < 0x3e500000u) return x;   /* |x| < 2^-26 */
        return rt__ksin(x, 0.0, 0);
    }
    if (ix >= 0x7ff00000u) return x - x;  /* inf or NaN -> NaN */
    double y0, y1;
    int n = rt__rem_pio2(x, &y0, &y1);
    switch (n & 3) {
    case 0: return rt__ksin(y0, y1, 1);
    case 1: return rt__kcos(y0, y1);
    case 2: return -rt__ksin(y0, y1, 1);
    default: return -rt__kcos(y0, y1);
    }
}

/* Sign of rt_sin(x) without the polynomial: +1 / -1, 0 for a zero, NaN or infinite
 * result, 2 when |sin x| may be below 2^-340 (the caller then evaluates rt_sin). For
 * |y0| <= pi/4 the kernels keep the sign of y0 (|ksin - y0| < |y0|) and kcos > 0.7, so a
 * product of three such factors is nonzero with this sign unless a factor is tiny. */
RT_HD int rt_sin_sign(double x)
{
    /* Fast path, no argument reduction: for |x| < 2^16, q = x * (1/pi) is within 5e-12 of
     * x/pi, so when its fractional part lies 1e-9 or more away from an integer,
     * floor(x/pi) = floor(q) and sin x has the sign (-1)^floor(q), with |sin x| > 3e-9,
     * far above rt_sin's error: the same sign rt_sin gives. Otherwise (near a multiple
     * of pi, large, inf or NaN) the reduction below decides. */
    if (__builtin_fabs(x) < 65536.0) {
        const double q = x * 0.31830988618379067154;
        const double k = __builtin_floor(q);
        const double f = q - k;
        if (f > 1e-9 && f < 1.0 - 1e-9) return (((int64_t)k) & 1) ? -1 : 1;
    }
    const double tiny = 0x1.0p-339;
    uint32_t ix = (uint32_t)(rt_f64_bits(x) >> 32) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) {
        if (x == 0.0) return 0;
        if (__builtin_fabs(x) < tiny) return 2;
        return x < 0.0 ? -1 : 1;
    }
    if (ix >= 0x7ff00000u) return 0;
    double y0, y1;
    int n = rt__rem_pio2(x, &y0, &y1);
    switch (n & 3) {
    case 0: return __builtin_fabs(y0) < tiny ? 2 : (y0 < 0.0 ? -1 : 1);
    case 1: return 1;
    case 2: return __builtin_fabs(y0) < tiny ? 2 : (y0 < 0.0 ? 1 : -1);
    default: return -1;
    }
}

RT_HD double rt_cos(double x)
{
    uint32_t ix = (uint32_t)(rt_f64_bits(x) >> 32) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) {
        if (ix < 0x3e46a09eu) return 1.0;
        return rt__kcos(x, 0.0);
    }
    if (ix >= 0x7ff00000u) return x - x;
    double y0, y1;
    int n = rt__rem_pio2(x, &y0, &y1);
    switch (n & 3) {
    case 0: return rt__kcos(y0, y1);
    case 1: return -rt__ksin(y0, y1, 1);
    case 2: return -rt__kcos(y0, y1);
    default: return rt__ksin(y0, y1, 1);
    }
}

/* ------------------------------------------------------------------------- */
/* log (fdlibm/musl)                                                          */
/* ------------------------------------------------------------------------- */
RT_HD double rt_log(double x)
{
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                 Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                 Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    uint64_t u = rt_f64_bits(x);
    uint32_t hx = (uint32_t)(u >> 32);
    int k = 0;
    if (hx < 0x00100000u || (hx >> 31)) {
        if ((u << 1) == 0) return -RT_INF;              /* log(+-0) = -inf */
        if (hx >> 31) return __builtin_nan("");         /* log(<0) = NaN */
        k -= 54;                                        /* subnormal: scale up */
        x *= 0x1.0p54;
        u = rt_f64_bits(x);
        hx = (uint32_t)(u >> 32);
    } else if (hx >= 0x7ff00000u) {
        return x;                                       /* inf or NaN */
    } else if (hx == 0x3ff00000u && (uint32_t)u == 0) {
        return 0.0;
    }
    hx += 0x3ff00000u - 0x3fe6a09eu;
    k += (int)(hx >> 20) - 0x3ff;
    hx = (hx & 0x000fffffu) + 0x3fe6a09eu;
    u = ((uint64_t)hx << 32) | (u & 0xffffffffull);
    x = rt_bits_f64(u);
    double f = x - 1.0;
    double hfsq = 0.5 * f * f;
    double s = f / (2.0 + f);
    double z = s * s;
    double w = z * z;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    double R = t2 + t1;
    double dk = (double)k;
    return s * (hfsq + R) + dk * ln2_lo - hfsq + f + dk * ln2_hi;
}

/* ------------------------------------------------------------------------- */
/* atan / atan2 / acos (fdlibm/musl)                                          */
/* ------------------------------------------------------------------------- */
RT_HD double rt_atan(double x)
{
    const double atanhi0 = 4.63647609000806093515e-01, atanhi1 = 7.85398163397448278999e-01,
                 atanhi2 = 9.82793723247329054082e-01, atanhi3 = 1.57079632679489655800e+00;
    const double atanlo0 = 2.26987774529616870924e-17, atanlo1 = 3.06161699786838301793e-17,
                 atanlo2 = 1.39033110312309984516e-17, atanlo3 = 6.12323399573676603587e-17;
    const double a0 = 3.33333333333329318027e-01, a1 = -1.99999999998764832476e-01,
                 a2 = 1.42857142725034663711e-01, a3 = -1.11111104054623557880e-01,
                 a4 = 9.09088713343650656196e-02, a5 = -7.69187620504482999495e-02,
                 a6 = 6.66107313738753120669e-02, a7 = -5.83357013379057348645e-02,
                 a8 = 4.97687799461593236017e-02, a9 = -3.65315727442169155270e-02,
                 a10 = 1.62858201153657823623e-02;
    uint32_t ix = (uint32_t)(rt_f64_bits(x) >> 32);
    uint32_t sign = ix >> 31;
    ix &= 0x7fffffffu;
    int id;
    double hi = 0.0, lo = 0.0;
    if (ix >= 0x44100000u) {                  /* |x| >= 2^66 */
        if (x != x) return x;
        return sign ? -atanhi3 : atanhi3;
    }
    if (ix < 0x3fdc0000u) {                   /* |x| < 0.4375 */
        if (ix < 0x3e400000u) return x;       /* |x| < 2^-27 */
        id = -1;
    } else {
        x = __builtin_fabs(x);
        if (ix < 0x3ff30000u) {
            if (ix < 0x3fe60000u) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); hi = atanhi0; lo = atanlo0; }
            else                  { id = 1; x = (x - 1.0) / (x + 1.0);       hi = atanhi1; lo = atanlo1; }
        } else {
            if (ix < 0x40038000u) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); hi = atanhi2; lo = atanlo2; }
            else                  { id = 3; x = -1.0 / x;                     hi = atanhi3; lo = atanlo3; }
        }
    }
    double z = x * x;
    double w = z * z;
    double s1 = z * (a0 + w * (a2 + w * (a4 + w * (a6 + w * (a8 + w * a10)))));
    double s2 = w * (a1 + w * (a3 + w * (a5 + w * (a7 + w * a9))));
    if (id < 0) return x - x * (s1 + s2);
    z = hi - (x * (s1 + s2) - lo - x);
    return sign ? -z : z;
}

RT_HD double rt_atan2(double y, double x)
{
    const double pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
    if (x != x || y != y) return x + y;
    uint64_t ux = rt_f64_bits(x), uy = rt_f64_bits(y);
    uint32_t ix = (uint32_t)(ux >> 32), lx = (uint32_t)ux;
    uint32_t iy = (uint32_t)(uy >> 32), ly = (uint32_t)uy;
    if (((ix - 0x3ff00000u) | lx) == 0) return rt_atan(y);   /* x == 1.0 */
    uint32_t m = ((iy >> 31) & 1) | ((ix >> 30) & 2);
    ix &= 0x7fffffffu;
    iy &= 0x7fffffffu;
    if ((iy | ly) == 0) {
        switch (m) {
        case 0: case 1: return y;
        case 2: return pi;
        default: return -pi;
        }
    }
    if ((ix | lx) == 0) return (m & 1) ? -pi / 2 : pi / 2;
    if (ix == 0x7ff00000u) {
        if (iy == 0x7ff00000u) {
            switch (m) {
            case 0: return pi / 4;
            case 1: return -pi / 4;
            case 2: return 3 * pi / 4;
            default: return -3 * pi / 4;
            }
        } else {
            switch (m) {
            case 0: return 0.0;
            case 1: return -0.0;
            case 2: return pi;
            default: return -pi;
            }
        }
    }
    if (ix + (64u << 20) < iy || iy == 0x7ff00000u) return (m & 1) ? -pi / 2 : pi / 2;
    double z;
    if ((m & 2) && iy + (64u << 20) < ix) z = 0.0;
    else z = rt_atan(__builtin_fabs(y / x));
    switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}

RT_HD double rt__acos_R(double z)
{
    const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                 pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                 pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
                 qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                 qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    return p / q;
}

RT_HD double rt_acos(double x)
{
    const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
    uint64_t u = rt_f64_bits(x);
    uint32_t hx = (uint32_t)(u >> 32);
    uint32_t ix = hx & 0x7fffffffu;
    if (ix >= 0x3ff00000u) {
        if (((ix - 0x3ff00000u) | (uint32_t)u) == 0) {
            if (hx >> 31) return 2 * pio2_hi;
            return 0.0;
        }
        return __builtin_nan("");            /* |x| > 1 or NaN */
    }
    if (ix < 0x3fe00000u) {                  /* |x| < 0.5 */
        if (ix <= 0x3c600000u) return pio2_hi;
        return pio2_hi - (x - (pio2_lo - x * rt__acos_R(x * x)));
    }
    if (hx >> 31) {                          /* x < -0.5 */
        double z = (1.0 + x) * 0.5;
        double s = __builtin_sqrt(z);
        double w = rt__acos_R(z) * s - pio2_lo;
        return 2 * (pio2_hi - (s + w));
    }
    double z = (1.0 - x) * 0.5;              /* x > 0.5 */
    double s = __builtin_sqrt(z);
    double df = rt_bits_f64(rt_f64_bits(s) & 0xffffffff00000000ull);
    double c = (z - df * df) / (s + df);
    double w = rt__acos_R(z) * s + c;
    return 2 * (df + w);
}

/* (1 - cos)^5 of Schlick's approximation (material.rs:93, `powf(5.0)`):
 * evaluated as (x^2)^2 * x — within 2 ulp of a correctly rounded pow. */
RT_HD double rt_pow5(double x)
{
    double x2 = x * x;
    return (x2 * x2) * x;
}

#endif /* RT_NUMERICS_H */
