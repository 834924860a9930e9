// valu_rates.hip -- issue cost of the VALU instruction forms the path kernel is made of, on gfx950.
// Each test runs a long unrolled stream of one instruction form on 8 independent register chains
// per lane, every SIMD holding `waves` waves; cycles per wave-instruction per SIMD are computed
// from the kernel time and the shader clock read with s_memtime (one tick = one shader cycle).
//   hipcc --offload-arch=gfx950 -O3 -o scripts/valu_rates scripts/valu_rates.hip
//   ./scripts/valu_rates            (one JSON line per test)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
constexpr int kInner = 32;     // 8 instructions x kInner per loop iteration
constexpr int kIters = 256;

// one test = one asm body applied to 8 chains; a0..a7 (and b, c operands) are VGPRs
#define TEST(NAME, BODY)                                                                          \
    __global__ __launch_bounds__(256) void NAME(float* out, int iters, unsigned long long* clk) { \
        float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
              a6 = a0 + 6, a7 = a0 + 7, b = a0 * 0.5f, c = a0 * 0.25f;                           \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                               \
        for (int it = 0; it < iters; it++) {                                                      \
            _Pragma("unroll") for (int k = 0; k < kInner; k++) {                                  \
                asm volatile(BODY : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),   \
                             "+v"(a6), "+v"(a7) : "v"(b), "v"(c) : "vcc", "s0", "s1", "s2");      \
            }                                                                                     \
        }                                                                                         \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                               \
        if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;                                \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;             \
    }

#define B8(F) F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7)
#define S(x) #x
// instruction forms (operands: %0..%7 = chains, %8 = b, %9 = c)
#define ADD_F32(i) "v_add_f32 %" S(i) ", %" S(i) ", %8\n"
#define FMA_F32(i) "v_fma_f32 %" S(i) ", %" S(i) ", %8, %9\n"
#define ADD_U32_LIT(i) "v_add_u32 %" S(i) ", 0xc3dc28f5, %" S(i) "\n"
#define SUB_F32_LIT(i) "v_sub_f32 %" S(i) ", 0x42480000, %" S(i) "\n"
#define MIN3_U32(i) "v_min3_u32 %" S(i) ", %" S(i) ", %8, %9\n"
#define MIN_U32(i) "v_min_u32 %" S(i) ", %" S(i) ", %8\n"
#define CNDMASK_VCC(i) "v_cndmask_b32 %" S(i) ", %" S(i) ", %8, vcc\n"
#define CMP_CND(i) "v_cmp_lt_f32 vcc, %" S(i) ", %8\n v_cndmask_b32 %" S(i) ", %" S(i) ", %9, vcc\n"
#define CMP64(i) "v_cmp_lt_u32 s[0:1], %" S(i) ", %8\n"
#define SQRT_F32(i) "v_sqrt_f32 %" S(i) ", %" S(i) "\n"
#define RCP_F32(i) "v_rcp_f32 %" S(i) ", %" S(i) "\n"
#define ADD3_U32(i) "v_add3_u32 %" S(i) ", %" S(i) ", %8, %9\n"
#define LSHR(i) "v_lshrrev_b32 %" S(i) ", 31, %" S(i) "\n"
#define SUBSAT(i) "v_sub_u32 %" S(i) ", %" S(i) ", 1 clamp\n"
#define MOV(i) "v_mov_b32 %" S(i) ", %8\n"
#define MUL_F32(i) "v_mul_f32 %" S(i) ", %" S(i) ", %8\n"
#define MIN_F32(i) "v_min_f32 %" S(i) ", %" S(i) ", %8\n"
#define MAX_F32(i) "v_max_f32 %" S(i) ", %" S(i) ", %8\n"
#define MIN3_F32(i) "v_min3_f32 %" S(i) ", %" S(i) ", %8, %9\n"
#define MED3_F32(i) "v_med3_f32 %" S(i) ", %" S(i) ", %8, %9\n"
#define AND_B32(i) "v_and_b32 %" S(i) ", %" S(i) ", %8\n"
#define OR_B32(i) "v_or_b32 %" S(i) ", %" S(i) ", %8\n"
#define XOR_B32(i) "v_xor_b32 %" S(i) ", %" S(i) ", %8\n"
#define BFI_B32(i) "v_bfi_b32 %" S(i) ", %" S(i) ", %8, %9\n"
#define ASHR(i) "v_ashrrev_i32 %" S(i) ", 31, %" S(i) "\n"
#define SUBCO(i) "v_sub_co_u32 %" S(i) ", vcc, %" S(i) ", %8\n"
#define CND_E64(i) "v_cndmask_b32 %" S(i) ", %" S(i) ", %8, s[0:1]\n"
#define CMP_E64F(i) "v_cmp_gt_f32 s[0:1], %" S(i) ", %8\n"
#define CVT_F32_U32(i) "v_cvt_f32_u32 %" S(i) ", %" S(i) "\n"
#define MUL_HI(i) "v_mul_hi_u32 %" S(i) ", %" S(i) ", %8\n"
#define MUL_LO(i) "v_mul_lo_u32 %" S(i) ", %" S(i) ", %8\n"
#define ADD_F32_S(i) "v_add_f32 %" S(i) ", s2, %" S(i) "\n"
#define MAX_I32(i) "v_max_i32 %" S(i) ", %" S(i) ", %8\n"
#define ADD_U32(i) "v_add_u32 %" S(i) ", %" S(i) ", %8\n"
#define LSHL_ADD(i) "v_lshl_add_u32 %" S(i) ", %" S(i) ", 2, %8\n"
#define CMPX(i) "v_cmp_lt_f32 vcc, %" S(i) ", %8\n"
#define NOP1(i) "s_nop 1\n"

TEST(t_add_f32, B8(ADD_F32))
TEST(t_mul_f32, B8(MUL_F32))
TEST(t_fma_f32, B8(FMA_F32))
TEST(t_add_u32_lit, B8(ADD_U32_LIT))
TEST(t_sub_f32_lit, B8(SUB_F32_LIT))
TEST(t_min3_u32, B8(MIN3_U32))
TEST(t_min_u32, B8(MIN_U32))
TEST(t_cndmask_vcc, B8(CNDMASK_VCC))
TEST(t_cmp_cndmask, B8(CMP_CND))
TEST(t_cmp_e64, B8(CMP64))
TEST(t_sqrt_f32, B8(SQRT_F32))
TEST(t_rcp_f32, B8(RCP_F32))
TEST(t_add3_u32, B8(ADD3_U32))
TEST(t_lshr, B8(LSHR))
TEST(t_sub_sat, B8(SUBSAT))
TEST(t_mov, B8(MOV))
TEST(t_nop1, B8(NOP1))
TEST(t_min_f32, B8(MIN_F32))
TEST(t_max_f32, B8(MAX_F32))
TEST(t_min3_f32, B8(MIN3_F32))
TEST(t_med3_f32, B8(MED3_F32))
TEST(t_and_b32, B8(AND_B32))
TEST(t_or_b32, B8(OR_B32))
TEST(t_xor_b32, B8(XOR_B32))
TEST(t_bfi_b32, B8(BFI_B32))
TEST(t_ashr, B8(ASHR))
TEST(t_subco, B8(SUBCO))
TEST(t_cnd_e64, B8(CND_E64))
TEST(t_cmp_e64f, B8(CMP_E64F))
TEST(t_cvt_f32_u32, B8(CVT_F32_U32))
TEST(t_mul_hi, B8(MUL_HI))
TEST(t_mul_lo, B8(MUL_LO))
TEST(t_add_f32_s, B8(ADD_F32_S))
TEST(t_max_i32, B8(MAX_I32))
TEST(t_add_u32, B8(ADD_U32))
TEST(t_lshl_add, B8(LSHL_ADD))
TEST(t_cmp_vcc, B8(CMPX))

// f64 chains need register pairs: a separate kernel
__global__ __launch_bounds__(256) void t_fma_f64(float* out, int iters, unsigned long long* clk) {
    double d0 = threadIdx.x, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, b = d0 * 0.5, c = d0 * 0.25;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < kInner * 2; k++)
            asm volatile("v_fma_f64 %0, %0, %4, %5\n v_fma_f64 %1, %1, %4, %5\n v_fma_f64 %2, %2, %4, %5\n v_fma_f64 %3, %3, %4, %5\n"
                         : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(b), "v"(c));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (float)(d0 + d1 + d2 + d3);
}

// f32 -> f64 -> op -> f32 chains (register pairs)
#define F64KERNEL(NAME, BODY)                                                                       \
    __global__ __launch_bounds__(256) void NAME(float* out, int iters, unsigned long long* clk) {   \
        float a0 = threadIdx.x + 1, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;                          \
        double d0 = a0, d1 = a1, d2 = a2, d3 = a3;                                                  \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                 \
        for (int it = 0; it < iters; it++) {                                                        \
            _Pragma("unroll") for (int k = 0; k < kInner * 2; k++)                                  \
                asm volatile(BODY : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(d0), "+v"(d1),      \
                             "+v"(d2), "+v"(d3));                                                   \
        }                                                                                           \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                 \
        if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;                                  \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + (float)(d0 + d1 + d2 + d3);      \
    }
F64KERNEL(t_cvt_f64_f32, "v_cvt_f64_f32 %4, %0\n v_cvt_f64_f32 %5, %1\n v_cvt_f64_f32 %6, %2\n v_cvt_f64_f32 %7, %3\n")
F64KERNEL(t_cvt_f32_f64, "v_cvt_f32_f64 %0, %4\n v_cvt_f32_f64 %1, %5\n v_cvt_f32_f64 %2, %6\n v_cvt_f32_f64 %3, %7\n")
F64KERNEL(t_sqrt_f64, "v_sqrt_f64 %4, %4\n v_sqrt_f64 %5, %5\n v_sqrt_f64 %6, %6\n v_sqrt_f64 %7, %7\n")
F64KERNEL(t_rsq_f64, "v_rsq_f64 %4, %4\n v_rsq_f64 %5, %5\n v_rsq_f64 %6, %6\n v_rsq_f64 %7, %7\n")
F64KERNEL(t_rcp_f64, "v_rcp_f64 %4, %4\n v_rcp_f64 %5, %5\n v_rcp_f64 %6, %6\n v_rcp_f64 %7, %7\n")
F64KERNEL(t_mul_f64, "v_mul_f64 %4, %4, %5\n v_mul_f64 %5, %5, %6\n v_mul_f64 %6, %6, %7\n v_mul_f64 %7, %7, %4\n")
F64KERNEL(t_add_f64, "v_add_f64 %4, %4, %5\n v_add_f64 %5, %5, %6\n v_add_f64 %6, %6, %7\n v_add_f64 %7, %7, %4\n")
F64KERNEL(t_rsq_f32, "v_rsq_f32 %0, %0\n v_rsq_f32 %1, %1\n v_rsq_f32 %2, %2\n v_rsq_f32 %3, %3\n")
F64KERNEL(t_rndne_f64, "v_rndne_f64 %4, %4\n v_rndne_f64 %5, %5\n v_rndne_f64 %6, %6\n v_rndne_f64 %7, %7\n")
F64KERNEL(t_cvt_i32_f64, "v_cvt_i32_f64 %0, %4\n v_cvt_i32_f64 %1, %5\n v_cvt_i32_f64 %2, %6\n v_cvt_i32_f64 %3, %7\n")

typedef void (*kfn)(float*, int, unsigned long long*);
struct T { const char* name; kfn f; int instr_per_inner; };

int main(int argc, char** argv) {
    const T tests[] = {
        {"v_add_f32", t_add_f32, 8}, {"v_mul_f32", t_mul_f32, 8}, {"v_fma_f32", t_fma_f32, 8},
        {"v_add_u32 literal", t_add_u32_lit, 8}, {"v_sub_f32 literal", t_sub_f32_lit, 8},
        {"v_min3_u32", t_min3_u32, 8}, {"v_min_u32", t_min_u32, 8},
        {"v_cndmask vcc", t_cndmask_vcc, 8}, {"v_cmp_lt_f32 vcc + v_cndmask", t_cmp_cndmask, 16},
        {"v_cmp_lt_u32 e64 sgpr", t_cmp_e64, 8}, {"v_sqrt_f32", t_sqrt_f32, 8},
        {"v_rcp_f32", t_rcp_f32, 8}, {"v_add3_u32", t_add3_u32, 8}, {"v_lshrrev_b32", t_lshr, 8},
        {"v_sub_u32 clamp", t_sub_sat, 8}, {"v_mov_b32", t_mov, 8}, {"s_nop 1", t_nop1, 8},
        {"v_fma_f64", t_fma_f64, 8},
        {"v_min_f32", t_min_f32, 8}, {"v_max_f32", t_max_f32, 8}, {"v_min3_f32", t_min3_f32, 8},
        {"v_med3_f32", t_med3_f32, 8}, {"v_and_b32", t_and_b32, 8}, {"v_or_b32", t_or_b32, 8},
        {"v_xor_b32", t_xor_b32, 8}, {"v_bfi_b32", t_bfi_b32, 8}, {"v_ashrrev_i32", t_ashr, 8},
        {"v_sub_co_u32 vcc", t_subco, 8}, {"v_cndmask e64 s[0:1]", t_cnd_e64, 8},
        {"v_cmp_gt_f32 e64 s[0:1]", t_cmp_e64f, 8}, {"v_cvt_f32_u32", t_cvt_f32_u32, 8},
        {"v_mul_hi_u32", t_mul_hi, 8}, {"v_mul_lo_u32", t_mul_lo, 8}, {"v_add_f32 sgpr", t_add_f32_s, 8},
        {"v_max_i32", t_max_i32, 8}, {"v_add_u32", t_add_u32, 8}, {"v_lshl_add_u32", t_lshl_add, 8},
        {"v_cmp_lt_f32 vcc", t_cmp_vcc, 8},
        {"v_cvt_f64_f32", t_cvt_f64_f32, 8}, {"v_cvt_f32_f64", t_cvt_f32_f64, 8},
        {"v_sqrt_f64", t_sqrt_f64, 8}, {"v_rsq_f64", t_rsq_f64, 8}, {"v_rcp_f64", t_rcp_f64, 8},
        {"v_mul_f64", t_mul_f64, 8}, {"v_add_f64", t_add_f64, 8}, {"v_rsq_f32", t_rsq_f32, 8},
        {"v_rndne_f64", t_rndne_f64, 8}, {"v_cvt_i32_f64", t_cvt_i32_f64, 8}};
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, sizeof(float) * 256 * 8192);
    hipMalloc(&clk, sizeof(unsigned long long));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int waves : {1, 4, 8}) {
        // 256-thread blocks = 1 wave per SIMD each; waves/SIMD = blocks per CU
        const int blocks = cus * waves;
        for (const T& t : tests) {
            t.f<<<blocks, 256>>>(out, 4, clk);                      // warm
            hipDeviceSynchronize();
            hipEventRecord(e0);
            t.f<<<blocks, 256>>>(out, kIters, clk);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long cyc = 0;
            hipMemcpy(&cyc, clk, sizeof cyc, hipMemcpyDeviceToHost);
            const double winstr = (double)kIters * kInner * t.instr_per_inner;   // per wave
            // one wave's own loop: cycles per instruction of ITS stream; per SIMD with `waves`
            // waves sharing it: cycles per wave-instruction = cyc / (winstr * waves)
            // cycles per wave-instruction per SIMD from the kernel time at 2.2 GHz (the clock the
            // 1-wave runs read with s_memtime); relative costs are what matter
            printf("{\"test\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_wave_instr_per_simd\": %.3f, "
                   "\"wave0_cyc_per_instr\": %.3f, \"ms\": %.4f, \"clock_ghz_wave0\": %.3f}\n",
                   t.name, waves, ms * 1e6 * 2.2 / (winstr * waves), (double)cyc / winstr, ms, cyc / (ms * 1e6));
        }
    }
    return 0;
}
