// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the path kernel's access patterns
// (MI355X_MICROARCH.md "HBM": FETCH_SIZE reports 1/2 of the bytes of a 16-B/lane streaming read
// on gfx950; other widths must be calibrated on a known byte count).  Each kernel moves a known
// number of bytes through a 1 GiB buffer (4x the Infinity Cache, so nothing is served on-die
// from an earlier kernel):
//   stream16  16 B/lane coalesced loads                     (the guide's reference pattern)
//   gather20  20 B per lane at the start of its own 128-B line  (d_Rand[j..j+4] prefetch)
//   aos12     12 B/lane AoS loads, lanes contiguous         (colors read)
//   store4    4 B/lane coalesced stores                     (counter / pixels write)
//   store12   12 B/lane AoS stores                          (colors write)
// Prints one JSON line per kernel with its byte counts; scripts/pmc_traffic.py divides the
// counters of each kernel by these.  Build: hipcc --offload-arch=gfx950 -O3 pmc_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void stream16(const float4* __restrict__ a, float* __restrict__ sink, long n) {
    float acc = 0.f;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 123.456f) sink[0] = acc;
}

__global__ void gather20(const float* __restrict__ a, float* __restrict__ sink, long lines) {
    float acc = 0.f;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < lines; i += (long)gridDim.x * blockDim.x) {
        const float* p = a + i * 32;          // 128-B line i
        acc += p[0] + p[1] + p[2] + p[3] + p[4];
    }
    if (acc == 123.456f) sink[0] = acc;
}

struct v3 { float x, y, z; };

__global__ void aos12(const v3* __restrict__ a, float* __restrict__ sink, long n) {
    float acc = 0.f;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const v3 v = a[i];
        acc += v.x + v.y + v.z;
    }
    if (acc == 123.456f) sink[0] = acc;
}

__global__ void store4(unsigned* __restrict__ a, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        a[i] = (unsigned)i;
}

__global__ void store12(v3* __restrict__ a, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        v3 v;
        v.x = (float)i; v.y = 1.f; v.z = 2.f;
        a[i] = v;
    }
}

int main() {
    const size_t bytes = 1ull << 30;
    void* buf = nullptr;
    float* sink = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0, bytes));
    CK(hipDeviceSynchronize());
    const dim3 grid(256 * 8), block(256);
    const long n16 = (long)(bytes / 16), lines = (long)(bytes / 128), n12 = (long)(bytes / 12), n4 = (long)(bytes / 4);
    // each kernel twice (rocprofv3 averages dispatches); a 1 GiB memset in between evicts
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(stream16, grid, block, 0, 0, (const float4*)buf, sink, n16);
        CK(hipMemset(buf, rep, bytes));
        hipLaunchKernelGGL(gather20, grid, block, 0, 0, (const float*)buf, sink, lines);
        CK(hipMemset(buf, rep, bytes));
        hipLaunchKernelGGL(aos12, grid, block, 0, 0, (const v3*)buf, sink, n12);
        CK(hipMemset(buf, rep, bytes));
        hipLaunchKernelGGL(store4, grid, block, 0, 0, (unsigned*)buf, n4);
        hipLaunchKernelGGL(store12, grid, block, 0, 0, (v3*)buf, n12);
        CK(hipDeviceSynchronize());
    }
    printf("{\"kernel\": \"stream16\", \"read_bytes\": %zu}\n", (size_t)n16 * 16);
    printf("{\"kernel\": \"gather20\", \"read_bytes\": %zu, \"line_bytes\": %zu}\n", (size_t)lines * 20, (size_t)lines * 128);
    printf("{\"kernel\": \"aos12\", \"read_bytes\": %zu}\n", (size_t)n12 * 12);
    printf("{\"kernel\": \"store4\", \"write_bytes\": %zu}\n", (size_t)n4 * 4);
    printf("{\"kernel\": \"store12\", \"write_bytes\": %zu}\n", (size_t)n12 * 12);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
