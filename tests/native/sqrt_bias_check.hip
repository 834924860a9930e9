// Distribution of v_sqrt_f32's error against the correctly rounded sqrt over all non-negative
// floats in [2^-96, 2^128): how often it is 1 ulp low, 1 ulp high, or further off.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../gpu_bidirectional_raytracer_amd/csrc/bdpt_math.h"

__global__ void k(unsigned base, unsigned long long* c) {
    const unsigned long long idx = (unsigned long long)base + blockIdx.x * 256ull + threadIdx.x;
    if (idx >= 0x7f800000ull) return;
    const float x = __uint_as_float((unsigned)idx);
    if (!(x >= 0x1p-96f)) return;
    const int a = (int)__float_as_uint(__builtin_amdgcn_sqrtf(x));
    const int b = (int)__float_as_uint(bdpt_sqrt_rn_core(x));
    const int d = a - b;
    atomicAdd(&c[d == 0 ? 0 : d == -1 ? 1 : d == 1 ? 2 : 3], 1ull);
}

int main() {
    unsigned long long* c;
    unsigned long long h[4] = {0, 0, 0, 0};
    if (hipMalloc(&c, sizeof(h)) != hipSuccess) return 2;
    (void)hipMemcpy(c, h, sizeof(h), hipMemcpyHostToDevice);
    for (unsigned long long b = 0; b < 0x7f800000ull; b += 1ull << 28)
        hipLaunchKernelGGL(k, dim3((1u << 28) / 256), dim3(256), 0, 0, (unsigned)b, c);
    (void)hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    printf("{\"exact\": %llu, \"low_1ulp\": %llu, \"high_1ulp\": %llu, \"other\": %llu}\n", h[0], h[1], h[2], h[3]);
    (void)hipFree(c);
    return 0;
}
