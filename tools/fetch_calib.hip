// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// shapes of the fdx kernels (MI355X_MICROARCH.md: FETCH_SIZE reads half of a wide coalesced
// streaming read; other widths "uncalibrated: calibrate on a known byte count").
//
// Kernels (one dispatch each, buffers far larger than the 256 MiB Infinity Cache):
//   stream16  coalesced 16 B/lane reads of 2 GiB           (known: 2 GiB)
//   stream8   coalesced 8 B/lane reads of 2 GiB            (known: 2 GiB)
//   stream4   coalesced 4 B/lane reads of 2 GiB            (known: 2 GiB)
//   gather8   64M random 8 B reads from a 2 GiB table      (>= 512 MiB; a line each)
//   gather16  64M random 16 B reads from a 2 GiB table
//   gather24  64M random 24 B reads (3 x 8 B, one record)
//   scatter24 64M random 24 B writes (3 x 8 B records) into a 2 GiB table
//   write16   coalesced 16 B/lane writes of 2 GiB          (known: 2 GiB)
// Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes) and
// `--kernel-trace --stats`; tools/fetch_calib_report.py turns the CSVs into
// profiles/r02_fetch_calibration.json.  Indices: a fixed LCG, so every pass reads the same lines.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                      \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

__global__ void stream16(const uint4 *__restrict__ a, size_t n, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}
__global__ void stream8(const uint2 *__restrict__ a, size_t n, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint2 v = a[i];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}
__global__ void stream4(const uint32_t *__restrict__ a, size_t n, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= a[i];
    if (acc == 0x9e3779b9u) sink[0] = acc;
}
__device__ __forceinline__ uint64_t lcg(uint64_t i) { return (i * 6364136223846793005ull + 1442695040888963407ull) >> 17; }

template <int W>  // W 8-byte words per record, records of W*8 bytes at random record slots
__global__ void gather(const uint64_t *__restrict__ t, size_t n_rec, size_t m, uint32_t *__restrict__ sink) {
    uint64_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = lcg(i) % n_rec;
#pragma unroll
        for (int w = 0; w < W; ++w) acc ^= t[r * W + w];
    }
    if (acc == 0x9e3779b97f4a7c15ull) sink[0] = (uint32_t)acc;
}
__global__ void scatter24(uint64_t *__restrict__ t, size_t n_rec, size_t m) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = lcg(i) % n_rec;
        t[r * 3] = i;
        t[r * 3 + 1] = i + 1;
        t[r * 3 + 2] = i + 2;
    }
}
__global__ void write16(uint4 *__restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

int main() {
    const size_t bytes = size_t(2) << 30;  // 2 GiB per buffer
    const size_t m = size_t(64) << 20;     // 64M random accesses
    void *a, *b;
    uint32_t *sink;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(a, 1, bytes));
    CHECK(hipMemset(b, 2, bytes));
    CHECK(hipDeviceSynchronize());
    const dim3 grid(256 * 8), block(256);
    for (int rep = 0; rep < 2; ++rep) {  // 2nd repetition = the measured one (1st warms up)
        hipLaunchKernelGGL(stream16, grid, block, 0, 0, (const uint4 *)a, bytes / 16, sink);
        hipLaunchKernelGGL(stream8, grid, block, 0, 0, (const uint2 *)b, bytes / 8, sink);
        hipLaunchKernelGGL(stream4, grid, block, 0, 0, (const uint32_t *)a, bytes / 4, sink);
        hipLaunchKernelGGL(gather<1>, grid, block, 0, 0, (const uint64_t *)b, bytes / 8, m, sink);
        hipLaunchKernelGGL(gather<2>, grid, block, 0, 0, (const uint64_t *)a, bytes / 16, m, sink);
        hipLaunchKernelGGL(gather<3>, grid, block, 0, 0, (const uint64_t *)b, bytes / 24, m, sink);
        hipLaunchKernelGGL(scatter24, grid, block, 0, 0, (uint64_t *)a, bytes / 24, m);
        hipLaunchKernelGGL(write16, grid, block, 0, 0, (uint4 *)b, bytes / 16);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
    }
    printf("fetch_calib done: bytes=%zu accesses=%zu\n", bytes, m);
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(sink));
    return 0;
}
