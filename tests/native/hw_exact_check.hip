// Exhaustive GPU check of hardware shortcuts against the correctly rounded results the render
// path needs (all 2^31 non-negative float bit patterns; denormals and specials included):
//   sqrt: v_sqrt_f32 alone                      vs bdpt_sqrt_rn_core (v_sqrt + residual fix)
//   sqrt: bdpt_sqrt_rn_core                     vs (float)sqrt((double)x) on x = +0, x >= 2^-96
//   rcp : v_rcp_f32 + one fma Newton step       vs (float)(1.0 / (double)x)  (double division is
//         correctly rounded and 53 >= 2*24+2, so its rounding to float is the exact 1.f/x);
//         for both signs (x and -x in one thread)
// Prints per check the number of mismatches and the smallest / largest mismatching input.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off hw_exact_check.hip && ./a.out
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../gpu_bidirectional_raytracer_amd/csrc/bdpt_math.h"

struct stats {
    unsigned long long bad;
    unsigned lo, hi;
};

__global__ void check(unsigned base, stats* st) {
    const unsigned long long idx = (unsigned long long)base + blockIdx.x * 256ull + threadIdx.x;
    if (idx >= 0x80000000ull) return;
    const unsigned bits = (unsigned)idx;
    const float x = __uint_as_float(bits);
    // sqrt
    {
        const float a = __builtin_amdgcn_sqrtf(x), b = bdpt_sqrt_rn_core(x);
        if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) {
            atomicAdd(&st[0].bad, 1ull);
            atomicMin(&st[0].lo, bits);
            atomicMax(&st[0].hi, bits);
        }
    }
    // the kernel's sqrt core (bdpt_sqrt_rn_core, sign-bit correction) vs the correctly rounded
    // sqrt, on its domain: x = +0 and x >= 2^-96 (double sqrt is correctly rounded, 53 >= 2*24+2)
    if (bits == 0u || x >= 0x1p-96f) {
        const float a = bdpt_sqrt_rn_core(x), ref = (float)sqrt((double)x);
        if (__float_as_uint(a) != __float_as_uint(ref) && !(a != a && ref != ref)) {
            atomicAdd(&st[3].bad, 1ull);
            atomicMin(&st[3].lo, bits);
            atomicMax(&st[3].hi, bits);
        }
    }
    // reciprocal, x and -x
    for (int sgn = 0; sgn < 2; sgn++) {
        const float x = __uint_as_float(bits | (sgn ? 0x80000000u : 0u));
        const float r = __builtin_amdgcn_rcpf(x);
        const float e = __builtin_fmaf(-x, r, 1.0f);
        const float y = __builtin_fmaf(e, r, r);
        const float ref = (float)(1.0 / (double)x);
        if (__float_as_uint(y) != __float_as_uint(ref) && !(y != y && ref != ref)) {
            // [2^-125, 2^125): neither x, 1/x nor the Newton residual is denormal or overflows
            const int k = (fabsf(x) >= 0x1p-125f && fabsf(x) < 0x1p125f) ? 1 : 2;
            atomicAdd(&st[k].bad, 1ull);
            atomicMin(&st[k].lo, bits);
            atomicMax(&st[k].hi, bits);
        }
    }
}

int main() {
    stats h[4] = {{0, 0xffffffffu, 0}, {0, 0xffffffffu, 0}, {0, 0xffffffffu, 0}, {0, 0xffffffffu, 0}};
    stats* d;
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    const unsigned chunk = 1u << 28;
    for (unsigned long long b = 0; b < 0x80000000ull; b += chunk)
        hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, (unsigned)b, d);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[4] = {"sqrt (v_sqrt_f32 alone)", "rcp + 1 Newton fma, x in [2^-125, 2^125)",
                            "rcp + 1 Newton fma, other x", "sqrt core, x = +0 or x >= 2^-96"};
    for (int k = 0; k < 4; k++) {
        float lo = __builtin_bit_cast(float, h[k].lo), hi = __builtin_bit_cast(float, h[k].hi);
        printf("{\"check\": \"%s\", \"mismatches\": %llu, \"min_bad\": \"%g\", \"max_bad\": \"%g\"}\n", names[k],
               h[k].bad, h[k].bad ? lo : 0.f, h[k].bad ? hi : 0.f);
    }
    (void)hipFree(d);
    return 0;
}
