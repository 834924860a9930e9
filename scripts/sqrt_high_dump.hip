// Probe: dump every non-negative float x >= 2^-96 where v_sqrt_f32(x) is 1 ulp ABOVE the correctly
// rounded sqrt (to characterise them); prints a histogram by exponent and the first 64 inputs
// as hex along with the residual sign pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void probe(unsigned base, unsigned* cnt, unsigned* out, unsigned cap) {
    const unsigned long long idx = (unsigned long long)base + blockIdx.x * 256ull + threadIdx.x;
    if (idx >= 0x7f800000ull) return;
    const unsigned bits = (unsigned)idx;
    const float x = __uint_as_float(bits);
    if (!(x >= 0x1p-96f)) return;
    const float a = __builtin_amdgcn_sqrtf(x);
    const float ref = (float)sqrt((double)x);
    if ((int)__float_as_uint(a) - (int)__float_as_uint(ref) == 1) {
        const unsigned k = atomicAdd(cnt, 1u);
        if (k < cap) out[k] = bits;
    }
}
int main() {
    const unsigned cap = 1u << 20;
    unsigned *dc, *dout;
    if (hipMalloc(&dc, 4) != hipSuccess || hipMalloc(&dout, cap * 4) != hipSuccess) return 2;
    (void)hipMemset(dc, 0, 4);
    const unsigned chunk = 1u << 28;
    for (unsigned long long b = 0; b < 0x80000000ull; b += chunk)
        hipLaunchKernelGGL(probe, dim3(chunk / 256), dim3(256), 0, 0, (unsigned)b, dc, dout, cap);
    unsigned n = 0;
    (void)hipMemcpy(&n, dc, 4, hipMemcpyDeviceToHost);
    std::vector<unsigned> v(n < cap ? n : cap);
    (void)hipMemcpy(v.data(), dout, v.size() * 4, hipMemcpyDeviceToHost);
    FILE* f = fopen("gpurun_out/sqrt_high.bin", "wb");
    if (f) { fwrite(v.data(), 4, v.size(), f); fclose(f); }
    printf("high cases: %u\n", n);
    return 0;
}
