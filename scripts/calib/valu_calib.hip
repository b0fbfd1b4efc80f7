// valu_calib.hip — VALU issue-rate calibration for the roofline.
//
// Each kernel runs one VALU instruction class in a loop: 8 independent accumulators per
// lane (no dependency stalls at >= 2 waves per SIMD), the loop body unrolled 8x, so the
// class's wave-instructions dominate everything else the kernel issues. Launched with many
// waves on every SIMD, a kernel is issue-bound on that class, and
//     cycles per wave-instruction = 1024 SIMDs x kernel cycles / SQ_INSTS_VALU
// calibrates the counters the trace kernel's roofline reads (scripts/valu_roofline.py).
// Kernel cycles come from rocprofv3's GRBM_GUI_ACTIVE / 8 (8 XCDs) in the PMC pass, and
// are cross-checked here with hipEvent time x the in-kernel clock (s_memtime over
// s_memrealtime, 100 MHz).
//
// Modes: "sat" (grid = 8 blocks x 256 threads per CU, every SIMD holds 8 waves),
//        "one" (1 block of 256 threads per CU: one wave per SIMD, the single-wave issue cost),
//        "lat" (one dependent accumulator, one wave per SIMD: dependent-issue latency).
// Output: one JSON line per (class, mode) on stdout.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            std::exit(2);                                                               \
        }                                                                               \
    } while (0)

enum Op { F64_FMA, F64_ADD, F64_MUL, F64_RCP, F64_SQRT, F32_FMA, F32_ADD, F32_RCP, I32_ADD, I32_MUL, B32_XOR,
          CNDMASK, MOV_B32, CNDMASK_VCC, CMP_F64, CMP_F32, MAX_F64, MIN_F32, LSHL_B64, CVT_F64_U32, BFE_U32,
          PK_FMA_F32, MAX3_F32, MED3_F32, AND_B32, OR_B32, LSHL_B32, LSHR_B32, ALIGNBIT, BITOP3, MOV_B64,
          CMP_I32, LDEXP_F64, DIV_SCALE_F64, DIV_FMAS_F64, DIV_FIXUP_F64, MAD_U64_U32, LSHL_ADD_U64, LSHR_B64,
          MBCNT_LO, MUL_HI_U32, CVT_F32_F64, CMP_CLASS_F64, SUB_U32, FMAC_F64, MUL_F32, RSQ_F64, CNDMASK_E32, MIX,
          KMIX_C2, KMIX_C4, KMIX_C3, N_OPS };
static const char* kNames[N_OPS] = {"f64_fma", "f64_add", "f64_mul", "f64_rcp", "f64_sqrt", "f32_fma", "f32_add",
                                    "f32_rcp", "i32_add", "i32_mul", "b32_xor", "cndmask", "mov_b32", "cndmask_vcc",
                                    "cmp_f64", "cmp_f32", "max_f64", "min_f32", "lshl_b64", "cvt_f64_u32",
                                    "bfe_u32", "pk_fma_f32", "max3_f32", "med3_f32", "and_b32", "or_b32", "lshl_b32",
                                    "lshr_b32", "alignbit_b32", "bitop3_b32", "mov_b64", "cmp_i32", "ldexp_f64",
                                    "div_scale_f64", "div_fmas_f64", "div_fixup_f64", "mad_u64_u32", "lshl_add_u64",
                                    "lshr_b64", "mbcnt_lo", "mul_hi_u32", "cvt_f32_f64", "cmp_class_f64", "sub_u32",
                                    "fmac_f64", "mul_f32", "rsq_f64", "cndmask_e32", "mix", "kmix_c2",
                                    "kmix_c4", "kmix_c3"};

// KMIX_*: a trace kernel's own VALU mix replayed (scripts/calib/gen_kmix.py writes the op
// sequences from its PMC class shares and ISA): each accumulator runs the whole sequence
template <int... OPS>
struct Seq {
};
#include "kmix_seq.h"
#ifndef KMIX_C3_SEQ   // until gen_kmix.py has a C3 entry (kmix_seq.json then lists kmix_c3; pmc_r02.py reports only those)
#define KMIX_C3_SEQ F64_FMA
#endif

// Each class as one exact instruction (inline asm): the compiler may not fold repeated
// adds, pack f32 pairs into v_pk_* or strength-reduce, so the loop issues exactly
// 8 x NACC wave-instructions of the class per iteration (plus two scalar loop ops).
#define CALIB_ARGS                                                                                             \
    double(&d)[8], float(&f)[8], unsigned(&u)[8], unsigned long long(&cm)[8], unsigned(&cm2)[8], double db,     \
        double dc, float fb, float fc, unsigned ub, unsigned long long mask
#define CALIB_PASS d, f, u, cm, cm2, db, dc, fb, fc, ub, mask

template <int OP>
__device__ __forceinline__ void one(int i, CALIB_ARGS)
{
    {
        if constexpr (OP == F64_FMA) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(db), "v"(dc));
        if constexpr (OP == F64_ADD) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(db));
        if constexpr (OP == F64_MUL) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(db));
        if constexpr (OP == F64_RCP) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[i]));
        if constexpr (OP == F64_SQRT) asm volatile("v_sqrt_f64 %0, %0" : "+v"(d[i]));
        if constexpr (OP == F32_FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[i]) : "v"(fb), "v"(fc));
        if constexpr (OP == F32_ADD) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fb));
        if constexpr (OP == F32_RCP) asm volatile("v_rcp_f32 %0, %0" : "+v"(f[i]));
        if constexpr (OP == I32_ADD) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(ub));
        if constexpr (OP == I32_MUL) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(ub));
        if constexpr (OP == B32_XOR) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[i]) : "v"(ub));
        if constexpr (OP == CNDMASK) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[i]) : "v"(ub), "s"(mask));
        if constexpr (OP == MOV_B32) asm volatile("v_mov_b32 %0, %1" : "=v"(u[i]) : "v"(u[(i + 1) & 7]));
        // a compare into vcc and the select reading it: the pair the compiler emits (a select
        // reading a vcc that nothing wrote issued at ~22 cycles in r02b: not what kernels do)
        if constexpr (OP == CNDMASK_VCC)
            asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(ub) : "vcc");
        if constexpr (OP == CMP_F64) asm volatile("v_cmp_gt_f64 %0, %1, %2" : "=s"(cm[i]) : "v"(d[i]), "v"(db));
        if constexpr (OP == CMP_F32) asm volatile("v_cmp_gt_f32 %0, %1, %2" : "=s"(cm[i]) : "v"(f[i]), "v"(fb));
        if constexpr (OP == MAX_F64) asm volatile("v_max_f64 %0, %0, %1" : "+v"(d[i]) : "v"(db));
        if constexpr (OP == MIN_F32) asm volatile("v_min_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fb));
        if constexpr (OP == LSHL_B64) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(d[i]));
        if constexpr (OP == CVT_F64_U32) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[i]) : "v"(u[i]));
        if constexpr (OP == BFE_U32) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(u[i]));
        // packed f32 FMA, both halves of src1 / src2 from one register each (op_sel_hi): the
        // slab-plane product of two BVH children per instruction
        if constexpr (OP == PK_FMA_F32)
            asm volatile("v_pk_fma_f32 %0, %0, %1, %1 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "+v"(d[i]) : "v"(db));
        if constexpr (OP == MAX3_F32) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(f[i]) : "v"(fb), "v"(fc));
        if constexpr (OP == MED3_F32) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(f[i]) : "v"(fb), "v"(fc));
        if constexpr (OP == AND_B32) asm volatile("v_and_b32 %0, %0, %1" : "+v"(u[i]) : "v"(ub));
        if constexpr (OP == OR_B32) asm volatile("v_or_b32 %0, %0, %1" : "+v"(u[i]) : "v"(ub));
        if constexpr (OP == LSHL_B32) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(u[i]));
        if constexpr (OP == LSHR_B32) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(u[i]));
        if constexpr (OP == ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(u[i]) : "v"(ub));
        if constexpr (OP == BITOP3) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(u[i]) : "v"(ub));
        if constexpr (OP == MOV_B64) asm volatile("v_mov_b64 %0, %1" : "=v"(d[i]) : "v"(d[(i + 1) & 7]));
        if constexpr (OP == CMP_I32) asm volatile("v_cmp_lt_i32 %0, %1, %2" : "=s"(cm[i]) : "v"(u[i]), "v"(ub));
        if constexpr (OP == LDEXP_F64) asm volatile("v_ldexp_f64 %0, %0, 1" : "+v"(d[i]));
        if constexpr (OP == DIV_SCALE_F64) asm volatile("v_div_scale_f64 %0, vcc, %0, %1, %0" : "+v"(d[i]) : "v"(db) : "vcc");
        if constexpr (OP == DIV_FMAS_F64) asm volatile("v_div_fmas_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(db), "v"(dc));
        if constexpr (OP == DIV_FIXUP_F64) asm volatile("v_div_fixup_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(db), "v"(dc));
        if constexpr (OP == MAD_U64_U32) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(d[i]), "=s"(cm[i]) : "v"(u[i]), "v"(ub));
        if constexpr (OP == LSHL_ADD_U64) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(d[i]) : "v"(db));
        if constexpr (OP == LSHR_B64) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(d[i]));
        if constexpr (OP == MBCNT_LO) asm volatile("v_mbcnt_lo_u32_b32 %0, %1, %0" : "+v"(u[i]) : "v"(ub));
        if constexpr (OP == MUL_HI_U32) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[i]) : "v"(ub));
        if constexpr (OP == CVT_F32_F64) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[i]) : "v"(d[i]));
        if constexpr (OP == CMP_CLASS_F64) asm volatile("v_cmp_class_f64 %0, %1, %2" : "=s"(cm[i]) : "v"(d[i]), "v"(ub));
        if constexpr (OP == SUB_U32) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(u[i]) : "v"(ub));
        if constexpr (OP == FMAC_F64) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(d[i]) : "v"(db), "v"(dc));
        if constexpr (OP == MUL_F32) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fb));
        if constexpr (OP == RSQ_F64) asm volatile("v_rsq_f64 %0, %0" : "+v"(d[i]));
        // a select reading vcc that a compare outside the unrolled body wrote (the compiler's
        // v_cmp ... ; v_cndmask_b32_e32 pairs reuse vcc like this)
        if constexpr (OP == CNDMASK_E32) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(ub));
        // MIX: a fixed sequence of known composition (validates that per-class costs add up):
        // 1 f64 fma, 1 f64 add, 2 f32 fma, 1 i32 add, 1 xor, 1 mov, 1 cndmask, 1 max3 per accumulator
        if constexpr (OP == MIX)
            asm volatile("v_fma_f64 %0, %0, %4, %5\n\tv_add_f64 %0, %0, %4\n\tv_fma_f32 %1, %1, %6, %7\n\t"
                         "v_fma_f32 %1, %1, %6, %7\n\tv_add_u32 %2, %2, %8\n\tv_xor_b32 %2, %2, %8\n\t"
                         "v_mov_b32 %3, %2\n\tv_cndmask_b32_e64 %2, %2, %8, %9\n\tv_max3_f32 %1, %1, %6, %7"
                         : "+v"(d[i]), "+v"(f[i]), "+v"(u[i]), "=v"(cm2[i])
                         : "v"(db), "v"(dc), "v"(fb), "v"(fc), "v"(ub), "s"(mask));
    }
}

template <int OP, int NACC>
__device__ __forceinline__ void each_acc(CALIB_ARGS)
{
#pragma unroll
    for (int i = 0; i < NACC; ++i) one<OP>(i, CALIB_PASS);
}

// a sequence op by op, each over the accumulators (consecutive instructions independent: a
// dependent chain across inline-asm statements gets a hazard s_nop after each one)
template <int NACC, int... OPS>
__device__ __forceinline__ void seq_all(Seq<OPS...>, CALIB_ARGS)
{
    (each_acc<OPS, NACC>(CALIB_PASS), ...);
}

template <int OP, int NACC>
__device__ __forceinline__ void body(CALIB_ARGS)
{
    if constexpr (OP == KMIX_C2) seq_all<NACC>(Seq<KMIX_C2_SEQ>{}, CALIB_PASS);
    else if constexpr (OP == KMIX_C4) seq_all<NACC>(Seq<KMIX_C4_SEQ>{}, CALIB_PASS);
    else if constexpr (OP == KMIX_C3) seq_all<NACC>(Seq<KMIX_C3_SEQ>{}, CALIB_PASS);
    else each_acc<OP, NACC>(CALIB_PASS);
}

template <int OP, int NACC>
__global__ void __launch_bounds__(256) calib(const double* __restrict__ in, double* __restrict__ out, int iters,
                                             unsigned long long* __restrict__ clk)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    double d[8];
    float f[8];
    unsigned u[8];
    unsigned long long cm[8];
    unsigned cm2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        cm[i] = 0;
        cm2[i] = 0;
        d[i] = in[(t + i) & 1023];
        f[i] = (float)d[i];
        u[i] = (unsigned)t * 2654435761u + i;
    }
    const double db = in[1024], dc = in[1025];
    const float fb = (float)db, fc = (float)dc;
    const unsigned ub = (unsigned)in[1026];
    const unsigned long long mask = __builtin_amdgcn_read_exec() & 0x5555555555555555ull;
    unsigned long long c0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        c0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int k = 0; k < iters; ++k) {
#pragma unroll
        for (int j = 0; j < 8; ++j) body<OP, NACC>(d, f, u, cm, cm2, db, dc, fb, fc, ub, mask);
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - c0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += d[i] + (double)f[i] + (double)u[i] + (double)(cm[i] & 1u) + (double)cm2[i];
    out[t] = acc;
}

template <int OP>
static void run(const char* mode, int cus, double* din, double* dout, unsigned long long* dclk, int iters)
{
    const bool lat = !std::strcmp(mode, "lat");
    const int blocks = !std::strcmp(mode, "sat") ? cus * 8 : cus;
    auto kern = lat ? calib<OP, 1> : calib<OP, 8>;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, din, dout, 2, dclk);  // warm-up
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, din, dout, iters, dclk);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long clk[2];
    CHECK(hipMemcpy(clk, dclk, sizeof clk, hipMemcpyDeviceToHost));
    const double ghz = clk[1] ? (double)clk[0] / (double)clk[1] * 0.1 : 0.0;  // memrealtime = 100 MHz
    const int nacc = lat ? 1 : 8;
    const double waves = (double)blocks * 4.0;
    const double inst = waves * (double)iters * 8.0 * nacc;  // class wave-instructions
    const double simds = cus * 4.0;
    const double cyc = ms * 1e-3 * ghz * 1e9;
    std::printf("{\"op\": \"%s\", \"mode\": \"%s\", \"blocks\": %d, \"iters\": %d, \"ms\": %.4f, \"clock_ghz\": %.4f, "
                "\"class_insts\": %.6g, \"cycles_per_inst_per_simd\": %.4f}\n",
                kNames[OP], mode, blocks, iters, ms, ghz, inst, simds * cyc / inst);
    std::fflush(stdout);
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

template <int OP>
static void run_modes(const std::vector<std::string>& modes, int cus, double* din, double* dout,
                      unsigned long long* dclk, int iters)
{
    for (const auto& m : modes) run<OP>(m.c_str(), cus, din, dout, dclk, m == "sat" ? iters : iters * 2);
}

template <int OP, class W>
static void dispatch(const W& want, const std::vector<std::string>& modes, int cus, double* din, double* dout,
                     unsigned long long* dclk, int iters)
{
    if constexpr (OP < N_OPS) {
        if (want(OP)) run_modes<OP>(modes, cus, din, dout, dclk, iters);
        dispatch<OP + 1>(want, modes, cus, din, dout, dclk, iters);
    }
}

int main(int argc, char** argv)
{
    // usage: valu_calib [ops,comma,separated|all] [modes: sat,one,lat] [iters]
    const std::string ops = argc > 1 ? argv[1] : "all";
    std::vector<std::string> modes;
    {
        std::string m = argc > 2 ? argv[2] : "sat,one,lat";
        size_t p = 0;
        while (p <= m.size()) {
            size_t q = m.find(',', p);
            if (q == std::string::npos) q = m.size();
            modes.push_back(m.substr(p, q - p));
            p = q + 1;
        }
    }
    const int iters = argc > 3 ? std::atoi(argv[3]) : 4000;
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<double> h(1028);
    for (int i = 0; i < 1024; ++i) h[i] = 1.0 + i * 1e-3;
    h[1024] = 0.999999;
    h[1025] = 1e-7;
    h[1026] = 3;
    h[1027] = 5;
    double *din, *dout;
    unsigned long long* dclk;
    CHECK(hipMalloc(&din, h.size() * sizeof(double)));
    CHECK(hipMalloc(&dout, (size_t)cus * 8 * 256 * sizeof(double)));
    CHECK(hipMalloc(&dclk, 2 * sizeof(unsigned long long)));
    CHECK(hipMemcpy(din, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
    auto want = [&](int op) { return ops == "all" || ("," + ops + ",").find("," + std::string(kNames[op]) + ",") != std::string::npos; };
    dispatch<0>(want, modes, cus, din, dout, dclk, iters);
    CHECK(hipFree(din));
    CHECK(hipFree(dout));
    CHECK(hipFree(dclk));
    return 0;
}
