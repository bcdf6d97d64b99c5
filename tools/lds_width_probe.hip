// lds_width_probe.hip -- LDS read throughput by instruction width and address pattern, in the
// forest walk's launch shape (one 1,024-thread block per CU, a 128 KiB table in LDS).  Question
// it answers (round 5, forest item): does a random-address ds_read_b64 / ds_read_b128 cost the
// CU the same as a random ds_read_b32 (then wider node packets cut the walk's LDS instructions
// per tree level), or twice / four times as much (then they do not)?
//
// Modes (independent reads, K in flight per lane, no dependency between steps):
//   rand<W>   every lane a hashed random W-byte-aligned address: natural bank conflicts
//   perm<W>   random rows, but the 32 lanes of a lane group on distinct banks
//   bcast<W>  every lane of a wave the same random address
//   seq<W>    lane-consecutive addresses (conflict-free, one row)
// and dependent walks (K chains per lane, the next address from the loaded value):
//   dep<W>    one W-byte read per step
// Prints wave-instructions per CU per clock (wall clock at the measured shader clock).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
            return 1;                                                           \
        }                                                                       \
    } while (0)

constexpr int kBytes = 128 * 1024;
constexpr uint32_t kMask = kBytes - 1;

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <int W>
struct Vec;
template <>
struct Vec<4> {
    typedef uint32_t T;
    static __device__ uint32_t fold(T v) { return v; }
};
template <>
struct Vec<8> {
    typedef uint2 T;
    static __device__ uint32_t fold(T v) { return v.x ^ v.y; }
};
template <>
struct Vec<16> {
    typedef uint4 T;
    static __device__ uint32_t fold(T v) { return v.x ^ v.y ^ v.z ^ v.w; }
};

// MODE 0 rand, 1 perm, 2 bcast, 3 seq, 4 dep
template <int MODE, int W, int K>
__global__ void __launch_bounds__(1024) probe(const uint32_t *__restrict__ table, int steps,
                                              uint32_t *__restrict__ sink) {
    typedef typename Vec<W>::T T;
    __shared__ __align__(16) uint32_t s[kBytes / 4];
    for (int i = threadIdx.x; i < kBytes / 4; i += blockDim.x) s[i] = table[i];
    __syncthreads();
    const char *lds = reinterpret_cast<const char *>(s);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = hash(threadIdx.x * 977u + k * 131u + blockIdx.x) & kMask & ~(W - 1u);
    uint32_t rb[K], lo;  // perm / bcast: a random row base per (wave, chain), the lane's slot in it
#pragma unroll
    for (int k = 0; k < K; ++k) rb[k] = hash(wave * 7919u + k * 104729u + blockIdx.x * 31u);
    lo = W == 4 ? (lane & 31u) * 4u + (lane >> 5) * 128u : (lane * W) & 255u;
    uint32_t acc = 0;
    for (int st = 0; st < steps; ++st) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint32_t addr;
            if constexpr (MODE == 0) {
                addr = (a[k] + st * 0x9E3779B1u * W) & kMask & ~(W - 1u);
            } else if constexpr (MODE == 1) {
                addr = ((rb[k] + st * 0x9E3779B1u * 256u) & kMask & ~255u) + lo;
            } else if constexpr (MODE == 2) {
                addr = (rb[k] + st * 0x9E3779B1u * W) & kMask & ~(W - 1u);
            } else if constexpr (MODE == 3) {
                addr = ((st * K + k) * 64u * W + lane * W) & kMask;
            } else {
                addr = a[k];
            }
            const T v = *reinterpret_cast<const T *>(lds + addr);
            if constexpr (MODE == 4) {
                a[k] = (Vec<W>::fold(v) + lane * 4u) & kMask & ~(W - 1u);
            } else {
                acc += Vec<W>::fold(v);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) acc += a[k];
    if (acc == 0x12345678u) sink[0] = acc;
}

static double g_clock_ghz = 2.4;

template <int MODE, int W, int K>
static int run(const char *name, const uint32_t *table_d, int steps, int n_cu, uint32_t *sink) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((probe<MODE, W, K>), dim3(n_cu), dim3(1024), 0, 0, table_d, 16, sink);  // warm
    float ms[2];
    const int st[2] = {steps / 4, steps};
    for (int i = 0; i < 2; ++i) {
        CHECK(hipEventRecord(a, 0));
        hipLaunchKernelGGL((probe<MODE, W, K>), dim3(n_cu), dim3(1024), 0, 0, table_d, st[i], sink);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventElapsedTime(&ms[i], a, b));
    }
    // the difference of two step counts removes the table load and launch
    const double wave_reads = 16.0 * K * (st[1] - st[0]);
    const double cyc = (ms[1] - ms[0]) * 1e-3 * g_clock_ghz * 1e9;
    printf("%-6s W=%2d K=%2d  %.3f cycles per wave-read per CU  (%.2f B/clk/CU; %.3f / %.3f ms)\n", name, W, K,
           cyc / wave_reads, wave_reads * 64 * W / cyc, ms[0], ms[1]);
    return 0;
}

int main(int argc, char **argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 4000;
    if (argc > 2) g_clock_ghz = atof(argv[2]);
    int dev = 0, n_cu = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<uint32_t> t(kBytes / 4);
    srand(7);
    for (auto &x : t) x = (uint32_t)rand() * 2654435761u;
    uint32_t *table_d, *sink;
    CHECK(hipMalloc(&table_d, kBytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemcpy(table_d, t.data(), kBytes, hipMemcpyHostToDevice));
    printf("lds_width_probe: %d CUs, 1 block of 1024 threads per CU, %d steps, clock %.2f GHz assumed\n", n_cu,
           steps, g_clock_ghz);
#define RUNW(M, NAME, K)                                 \
    run<M, 4, K>(NAME, table_d, steps, n_cu, sink);      \
    run<M, 8, K>(NAME, table_d, steps, n_cu, sink);      \
    run<M, 16, K>(NAME, table_d, steps, n_cu, sink);
    RUNW(3, "seq", 8)
    RUNW(1, "perm", 8)
    RUNW(0, "rand", 8)
    RUNW(0, "rand", 4)
    RUNW(2, "bcast", 8)
    RUNW(4, "dep", 4)
    RUNW(4, "dep", 8)
    CHECK(hipFree(table_d));
    CHECK(hipFree(sink));
    return 0;
}
