#include <hip/hip_runtime.h>
__global__ void k(const float* __restrict__ g, float* __restrict__ out, const int* __restrict__ idx, int n) {
    __shared__ float A[256];
    __shared__ float B[256];
    B[threadIdx.x] = g[threadIdx.x + 1000];
    __syncthreads();
    float acc = 0.f;
    float v = g[idx[threadIdx.x] + 7];
    for (int it = 0; it < n; it++) {
        float a = A[threadIdx.x];                      // from the DMA of the previous iteration
        __builtin_amdgcn_global_load_lds(g + idx[it * 256 + threadIdx.x], A + (threadIdx.x & ~63), 4, 0, 0);
        float b = B[(threadIdx.x * 7 + it) & 255];     // unrelated LDS read: must not wait on the DMA
        acc += b * v;
        float b2 = B[(threadIdx.x * 5 + it) & 255];
        acc = acc * b2 + a;
        v = g[idx[it * 256 + threadIdx.x] + 9];       // next iteration's value
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}
