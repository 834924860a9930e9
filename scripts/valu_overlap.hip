// valu_overlap.hip -- do gfx950's transcendental (v_sqrt/v_rcp_f32) and fp64 instructions issue
// beside full-rate fp32 work, or do they take VALU issue cycles from it?  Each test runs a long
// unrolled stream on independent register chains with 8 waves per SIMD: a pure fp32-FMA stream, a
// pure v_sqrt_f32 / v_fma_f64 stream, and the two interleaved on separate chains.  If the mixed
// stream costs about the sum of its parts, the instructions share one issue port; if about the
// larger part, they overlap.  (Round 6: the sin/cos planes removed every fp64 instruction of the
// cornell kernel, 4.3 % of its VALU instructions, and its time did not move.)
//   hipcc --offload-arch=gfx950 -O3 -o scripts/valu_overlap scripts/valu_overlap.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kInner = 32;
constexpr int kIters = 256;
#define S(x) #x
#define FMA(i) "v_fma_f32 %" S(i) ", %" S(i) ", %16, %17\n"
#define SQRT(i) "v_sqrt_f32 %" S(i) ", %" S(i) "\n"
#define FMA8 FMA(0) FMA(1) FMA(2) FMA(3) FMA(4) FMA(5) FMA(6) FMA(7)
#define SQRT8 SQRT(8) SQRT(9) SQRT(10) SQRT(11) SQRT(12) SQRT(13) SQRT(14) SQRT(15)
#define SQRT2 SQRT(8) SQRT(9)
#define MIX_FS FMA(0) SQRT(8) FMA(1) SQRT(9) FMA(2) SQRT(10) FMA(3) SQRT(11) FMA(4) SQRT(12) FMA(5) SQRT(13) FMA(6) SQRT(14) FMA(7) SQRT(15)
#define MIX_F4S FMA(0) FMA(1) FMA(2) FMA(3) SQRT(8) FMA(4) FMA(5) FMA(6) FMA(7) SQRT(9)

#define TEST(NAME, BODY)                                                                           \
    __global__ __launch_bounds__(256) void NAME(float* out, int iters) {                           \
        float a[16];                                                                               \
        _Pragma("unroll") for (int k = 0; k < 16; k++) a[k] = threadIdx.x + k + 1.f;             \
        const float b = 0.999f, c = 1e-3f;                                                         \
        for (int it = 0; it < iters; it++) {                                                       \
            _Pragma("unroll") for (int k = 0; k < kInner; k++)                                     \
                asm volatile(BODY : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]),    \
                             "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]),           \
                             "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]),      \
                             "+v"(a[15]) : "v"(b), "v"(c));                                        \
        }                                                                                          \
        float s = 0.f;                                                                             \
        _Pragma("unroll") for (int k = 0; k < 16; k++) s += a[k];                                  \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                                   \
    }
TEST(t_fma8, FMA8)
TEST(t_sqrt8, SQRT8)
TEST(t_sqrt2, SQRT2)
TEST(t_fma8_sqrt8, MIX_FS)
TEST(t_fma8_sqrt2, MIX_F4S)

// fp64 FMAs on 4 register pairs, alone and interleaved with 8 fp32 FMAs
#define D64(NAME, BODY)                                                                            \
    __global__ __launch_bounds__(256) void NAME(float* out, int iters) {                           \
        float a0 = threadIdx.x + 1.f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,          \
              a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                               \
        double d0 = a0, d1 = a1, d2 = a2, d3 = a3;                                                 \
        const float b = 0.999f, c = 1e-3f;                                                         \
        const double db = 0.999, dc = 1e-3;                                                        \
        for (int it = 0; it < iters; it++) {                                                       \
            _Pragma("unroll") for (int k = 0; k < kInner; k++)                                     \
                asm volatile(BODY : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),   \
                             "+v"(a6), "+v"(a7), "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3)            \
                             : "v"(b), "v"(c), "v"(db), "v"(dc));                                  \
        }                                                                                          \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 +              \
                                              (float)(d0 + d1 + d2 + d3);                          \
    }
#define F(i) "v_fma_f32 %" S(i) ", %" S(i) ", %12, %13\n"
#define D(i) "v_fma_f64 %" S(i) ", %" S(i) ", %14, %15\n"
D64(t_f64x4, D(8) D(9) D(10) D(11))
D64(t_fma8_f64x4, F(0) D(8) F(1) F(2) D(9) F(3) F(4) D(10) F(5) F(6) D(11) F(7))

typedef void (*kfn)(float*, int);
struct T { const char* name; kfn f; int n32, ntrans, n64; };

int main() {
    const T tests[] = {{"fma8", t_fma8, 8, 0, 0}, {"sqrt8", t_sqrt8, 0, 8, 0}, {"sqrt2", t_sqrt2, 0, 2, 0},
                       {"fma8+sqrt8", t_fma8_sqrt8, 8, 8, 0}, {"fma8+sqrt2", t_fma8_sqrt2, 8, 2, 0},
                       {"f64x4", t_f64x4, 0, 0, 4}, {"fma8+f64x4", t_fma8_f64x4, 8, 0, 4}};
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, sizeof(float) * 256 * 8192);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int waves = 8, blocks = cus * waves;             // 256-thread blocks: 1 wave per SIMD each
    for (const T& t : tests) {
        t.f<<<blocks, 256>>>(out, 4);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        t.f<<<blocks, 256>>>(out, kIters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        // SIMD cycles per inner step (all `waves` waves' instructions of one step), 2.4 GHz
        const double cyc = ms * 1e-3 * 2.4e9 / ((double)kIters * kInner * waves);
        printf("{\"test\": \"%s\", \"fp32\": %d, \"trans\": %d, \"fp64\": %d, \"simd_cycles_per_step\": %.2f, \"ms\": %.4f}\n",
               t.name, t.n32, t.ntrans, t.n64, cyc, ms);
    }
    return 0;
}
