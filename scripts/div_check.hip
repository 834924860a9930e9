// Exhaustive over every pair of fp32 significands: the quotient a / b formed as
//   y = RN(1/b) (v_rcp_f32 + one Newton fma, exact: tests/native/hw_exact_check.hip),
//   q = RN(a * y), r = fma(-q, b, a), q' = fma(r, y, q)
// against the correctly rounded a / b (the library division), for a, b in [1, 2): correct
// rounding of a quotient of normal numbers depends on the significands only, so this covers
// every a, b whose quotient and intermediate products stay normal.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/div_check scripts/div_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ float rcp_inrange(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, r, 1.f), r, r);
}
__global__ void chk(unsigned mb0, unsigned long long* bad, unsigned* ex) {
    // one thread per (a significand); loops over 64 b significands
    const unsigned ma = blockIdx.x * 256u + threadIdx.x;           // 0 .. 2^23-1
    const float a = __uint_as_float(0x3F800000u | ma);
    unsigned n = 0;
    for (unsigned k = 0; k < 64; k++) {
        const float b = __uint_as_float(0x3F800000u | (mb0 + k));
        const float ref = a / b;
        const float y = rcp_inrange(b);
        const float q = a * y;
        const float r = __builtin_fmaf(-q, b, a);
        const float q2 = __builtin_fmaf(r, y, q);
        if (__float_as_uint(q2) != __float_as_uint(ref)) { n++; ex[0] = ma; ex[1] = mb0 + k; }
    }
    if (n) atomicAdd(bad, (unsigned long long)n);
}
int main() {
    unsigned long long* d; unsigned* de;
    if (hipMalloc(&d, 8) != hipSuccess || hipMalloc(&de, 8) != hipSuccess) return 2;
    (void)hipMemset(d, 0, 8); (void)hipMemset(de, 0, 8);
    const unsigned nb = 1u << 23;
    for (unsigned mb0 = 0; mb0 < nb; mb0 += 64) {
        hipLaunchKernelGGL(chk, dim3((1u << 23) / 256), dim3(256), 0, 0, mb0, d, de);
        if ((mb0 & ((1u << 20) - 1)) == 0) {
            (void)hipDeviceSynchronize();
            unsigned long long h = 0; (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
            fprintf(stderr, "progress b_sig=%u/%u mismatches=%llu\n", mb0, nb, h);
        }
    }
    (void)hipDeviceSynchronize();
    unsigned long long h = 0; unsigned e[2] = {0, 0};
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(e, de, 8, hipMemcpyDeviceToHost);
    printf("{\"pairs\": %llu, \"mismatches\": %llu, \"example_a_sig\": %u, \"example_b_sig\": %u}\n",
           (unsigned long long)nb * nb, h, e[0], e[1]);
    return 0;
}
