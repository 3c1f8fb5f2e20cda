// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the family
// kernels use.  MI355X_MICROARCH.md ("HBM"): FETCH_SIZE is half the bytes of a 16-B-per-lane
// streaming read; other widths are uncalibrated.  Each kernel here moves a known byte count
// (1 GiB, past the 256 MiB Infinity Cache) with one access width; profiles/calib_fetch.sh runs
// it under the FETCH_SIZE and WRITE_SIZE passes and divides.
//   hipcc --offload-arch=gfx950 -O3 -o profiles/_build/calib_fetch profiles/calib_fetch.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr size_t kBytes = size_t(1) << 30;

template <class T>
__global__ void rd(const T *__restrict__ src, size_t n, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = src[i];
        const uint32_t *w = reinterpret_cast<const uint32_t *>(&v);
#pragma unroll
        for (int k = 0; k < (int)(sizeof(T) / 4); k++) acc ^= w[k];
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;  // (keeps the loads; never true for zeros)
}

template <class T>
__global__ void wr(T *__restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T v;
        uint32_t *w = reinterpret_cast<uint32_t *>(&v);
#pragma unroll
        for (int k = 0; k < (int)(sizeof(T) / 4); k++) w[k] = (uint32_t)i + k;
        dst[i] = v;
    }
}

// one byte per lane (k_join's part OR records, the tag rows' partial columns)
__global__ void rd8(const uint8_t *__restrict__ src, size_t n, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc = acc * 0x01000193u + src[i];  // (all 32 bits live: the loads stay)
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}
__global__ void wr8(uint8_t *__restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = (uint8_t)i;
}

#define CHECK(x)                                                                 \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main() {
    void *a = nullptr;
    uint32_t *sink = nullptr;
    CHECK(hipMalloc(&a, kBytes));
    CHECK(hipMalloc(&sink, 4096 * sizeof(uint32_t)));
    CHECK(hipMemset(a, 0, kBytes));
    const dim3 grid(4096), block(256);
    // two rounds: the second round's dispatches are the ones to read (the first warms the TLB)
    for (int round = 0; round < 2; round++) {
        hipLaunchKernelGGL(rd<uint4>, grid, block, 0, 0, (const uint4 *)a, kBytes / 16, sink);
        hipLaunchKernelGGL(rd<uint2>, grid, block, 0, 0, (const uint2 *)a, kBytes / 8, sink);
        hipLaunchKernelGGL(rd<uint32_t>, grid, block, 0, 0, (const uint32_t *)a, kBytes / 4, sink);
        hipLaunchKernelGGL(rd8, grid, block, 0, 0, (const uint8_t *)a, kBytes, sink);
        hipLaunchKernelGGL(wr<uint4>, grid, block, 0, 0, (uint4 *)a, kBytes / 16);
        hipLaunchKernelGGL(wr<uint2>, grid, block, 0, 0, (uint2 *)a, kBytes / 8);
        hipLaunchKernelGGL(wr<uint32_t>, grid, block, 0, 0, (uint32_t *)a, kBytes / 4);
        hipLaunchKernelGGL(wr8, grid, block, 0, 0, (uint8_t *)a, kBytes);
        CHECK(hipDeviceSynchronize());
    }
    CHECK(hipGetLastError());
    printf("bytes per dispatch %zu\n", kBytes);
    CHECK(hipFree(a));
    CHECK(hipFree(sink));
    return 0;
}
