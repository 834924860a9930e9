// Probe: direction of v_sqrt_f32's error vs the correctly rounded sqrt over all non-negative
// floats >= 2^-96 (the range where bdpt_sqrt_rn_core is exact).  Prints counts of
// v_sqrt == cr, == cr - 1 ulp, == cr + 1 ulp, other.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../gpu_bidirectional_raytracer_amd/csrc/bdpt_math.h"
__global__ void probe(unsigned base, unsigned long long* c) {
    const unsigned long long idx = (unsigned long long)base + blockIdx.x * 256ull + threadIdx.x;
    if (idx >= 0x7f800000ull) return;
    const unsigned bits = (unsigned)idx;
    const float x = __uint_as_float(bits);
    {   // negative inputs (-0 excluded): the core sequence must return a NaN (so r > eps fails)
        const float xn = __uint_as_float(bits | 0x80000000u);
        if (bits != 0 && !(bdpt_sqrt_rn_core(xn) != bdpt_sqrt_rn_core(xn))) atomicAdd(&c[4], 1ull);
        if (bits != 0 && !(__builtin_amdgcn_sqrtf(xn) != __builtin_amdgcn_sqrtf(xn))) atomicAdd(&c[5], 1ull);
    }
    if (!(x >= 0x1p-96f)) return;
    const float a = __builtin_amdgcn_sqrtf(x);
    const float ref = (float)sqrt((double)x);
    const int d = (int)__float_as_uint(a) - (int)__float_as_uint(ref);
    const int k = d == 0 ? 0 : d == -1 ? 1 : d == 1 ? 2 : 3;
    atomicAdd(&c[k], 1ull);
}
int main() {
    unsigned long long h[6] = {0, 0, 0, 0, 0, 0}, *d;
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    const unsigned chunk = 1u << 28;
    for (unsigned long long b = 0; b < 0x80000000ull; b += chunk)
        hipLaunchKernelGGL(probe, dim3(chunk / 256), dim3(256), 0, 0, (unsigned)b, d);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("{\"exact\": %llu, \"low_by_1ulp\": %llu, \"high_by_1ulp\": %llu, \"other\": %llu, "
           "\"neg_core_not_nan\": %llu, \"neg_vsqrt_not_nan\": %llu}\n", h[0], h[1], h[2], h[3], h[4], h[5]);
    return 0;
}
