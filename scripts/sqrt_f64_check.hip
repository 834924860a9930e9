// Exhaustive: (float) v_sqrt_f64((double) x) -- the hardware fp64 square root, unrefined, rounded
// once to fp32 -- against the path kernel's bdpt_sqrt_rn_core and against (float)sqrt((double)x)
// (the library's correctly rounded fp64 sqrt), on all 2^32 inputs; mismatches per input class.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/sqrt_f64_check scripts/sqrt_f64_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../gpu_bidirectional_raytracer_amd/csrc/bdpt_math.h"
__device__ __forceinline__ float sqrt_via_f64(float x) {
    double d = (double)x, r;
    asm("v_sqrt_f64 %0, %1" : "=v"(r) : "v"(d));
    return (float)r;
}
__global__ void chk(unsigned long long base, unsigned long long* c, unsigned* ex) {
    const unsigned long long idx = base + blockIdx.x * 256ull + threadIdx.x;
    const unsigned bits = (unsigned)idx;
    const float x = __uint_as_float(bits);
    const float a = sqrt_via_f64(x), core = bdpt_sqrt_rn_core(x);
    const float ref = (float)sqrt((double)x);
    const bool an = a != a;
    // classes: 0 = +0, 1 = -0, 2 = negative, 3 = (0, 2^-96), 4 = [2^-96, inf], 5 = NaN
    const int cls = (bits == 0u) ? 0 : (bits == 0x80000000u) ? 1 : (x != x) ? 5 : (bits >> 31) ? 2 : (x < 0x1p-96f) ? 3 : 4;
    if (!(an && ref != ref) && __float_as_uint(a) != __float_as_uint(ref)) { atomicAdd(&c[cls], 1ull); atomicMax(&ex[cls], bits); }
    if (cls == 4 && __float_as_uint(a) != __float_as_uint(core)) atomicAdd(&c[6], 1ull);
}
int main() {
    unsigned long long h[7] = {0}, *d; unsigned e[7] = {0}, *de;
    if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMalloc(&de, sizeof(e)) != hipSuccess) return 2;
    (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    (void)hipMemcpy(de, e, sizeof(e), hipMemcpyHostToDevice);
    const unsigned chunk = 1u << 28;
    for (unsigned long long b = 0; b < 0x100000000ull; b += chunk)
        hipLaunchKernelGGL(chk, dim3(chunk / 256), dim3(256), 0, 0, b, d, de);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipMemcpy(e, de, sizeof(e), hipMemcpyDeviceToHost);
    printf("{\"vs_cr_plus0\": %llu, \"vs_cr_minus0\": %llu, \"vs_cr_negative\": %llu, \"vs_cr_below_2^-96\": %llu, "
           "\"vs_cr_normal\": %llu, \"vs_cr_nan\": %llu, \"vs_core_normal\": %llu, \"example_bits\": [%u, %u, %u, %u, %u]}\n",
           h[0], h[1], h[2], h[3], h[4], h[5], h[6], e[0], e[1], e[2], e[3], e[4]);
    return 0;
}
