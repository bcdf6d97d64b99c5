// lds_probe.hip -- what the forest walk's LDS access pattern can sustain on one MI355X CU,
// measured the way k_forest_rank runs: one 1,024-thread block per CU (4 waves per SIMD),
// a 64 KiB table in LDS, every lane walking K independent pointer chains.
//
//   chase<K>    K dependent chains per lane: idx = T[idx] (random cycle over the table) --
//               the node reads of a tree walk, latency + throughput
//   chase2<K>   each step two dependent reads: x = T[idx]; idx = T[x ^ lane-offset] -- the
//               rank step's (node read -> feature read) pair
//   rankstep<K> chase2 with k_forest_rank v1's step arithmetic between the reads (x - node,
//               v_med3 step, addresses): the forest step without the tree
//   indep       independent random reads (32 in flight per lane), no dependency: throughput
//   seq         independent conflict-free reads (lane-consecutive words): the array's peak
// Prints reads per cycle per CU (clock from s_memtime) for each; argv[1] = steps per chain.
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

constexpr int kWords = 16 * 1024;  // 64 KiB (a power of two: index masks, no division)

template <int MODE, int K>
__global__ void __launch_bounds__(1024) probe(const uint32_t *__restrict__ table, int steps,
                                              uint32_t *__restrict__ sink, unsigned long long *__restrict__ cycles) {
    __shared__ uint32_t T[kWords];
    for (int i = threadIdx.x; i < kWords; i += blockDim.x) T[i] = table[i];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    uint32_t idx[K];
#pragma unroll
    for (int k = 0; k < K; ++k) idx[k] = (threadIdx.x * 7919u + k * 104729u + blockIdx.x) & (kWords - 1);
    uint32_t acc = 0;
    for (int s = 0; s < steps; ++s) {
        if constexpr (MODE == 0) {  // dependent chase
#pragma unroll
            for (int k = 0; k < K; ++k) idx[k] = T[idx[k]];
        } else if constexpr (MODE == 1) {  // two dependent reads per step
            uint32_t x[K];
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = T[idx[k]];
#pragma unroll
            for (int k = 0; k < K; ++k) idx[k] = T[(x[k] + (threadIdx.x & 63) * 16) & (kWords - 1)];
        } else if constexpr (MODE == 4) {  // the rank step itself: node read -> rank read -> 4 VALU
            // (x - nd, med3 step, address, plane address), the k_forest_rank v1 arithmetic
            uint32_t x[K];
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = T[(((idx[k] >> 2) & 0xF000u) | ((threadIdx.x & 1023u) * 4u)) >> 2 & (kWords - 1)];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int32_t d = (int32_t)(x[k] - idx[k]);
                uint32_t st;
                asm("v_med3_i32 %0, %1, 1, %2" : "=v"(st) : "v"(d), "v"(idx[k] & 0xFFFu));
                idx[k] = T[(idx[k] + st * 977u) & (kWords - 1)];
            }
        } else if constexpr (MODE == 2) {  // independent random
#pragma unroll
            for (int k = 0; k < K; ++k) acc += T[(idx[k] + s * 2654435761u) & (kWords - 1)];
        } else {  // independent conflict-free
#pragma unroll
            for (int k = 0; k < K; ++k) acc += T[((s * K + k) * 64 + (threadIdx.x & 63)) & (kWords - 1)];
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int k = 0; k < K; ++k) acc += idx[k];
    if (acc == 0x12345678u) sink[0] = acc;
    if (threadIdx.x == 0) cycles[blockIdx.x] = t1 - t0;
}

template <int MODE, int K>
static int run(const char *name, const uint32_t *table_d, int steps, int n_cu, uint32_t *sink,
               unsigned long long *cyc_d, int reads_per_step) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((probe<MODE, K>), dim3(n_cu), dim3(1024), 0, 0, table_d, steps, sink, cyc_d);  // warm
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((probe<MODE, K>), dim3(n_cu), dim3(1024), 0, 0, table_d, steps, sink, cyc_d);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    std::vector<unsigned long long> cyc(n_cu);
    CHECK(hipMemcpy(cyc.data(), cyc_d, 8 * n_cu, hipMemcpyDeviceToHost));
    double mean = 0;
    for (auto c : cyc) mean += (double)c;
    mean /= n_cu;
    // wave-level reads per CU: 16 waves x K chains x steps x reads_per_step
    const double wave_reads = 16.0 * K * steps * reads_per_step;
    printf("%-10s K=%2d  %.4f wave-reads/cycle/CU  (%.1f cycles per wave-read; %.0f cycles)  %.4g wave-reads/s chip"
           " (%.3f ms, incl. the 64 KiB table load)\n", name, K, wave_reads / mean, mean / wave_reads, mean,
           wave_reads * n_cu / (ms * 1e-3), ms);
    return 0;
}

int main(int argc, char **argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 2000;
    int dev = 0, n_cu = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    // a random single cycle over the table (Sattolo), so chains never collapse
    std::vector<uint32_t> t(kWords);
    for (int i = 0; i < kWords; ++i) t[i] = i;
    srand(7);
    for (int i = kWords - 1; i > 0; --i) {
        const int j = rand() % i;
        std::swap(t[i], t[j]);
    }
    uint32_t *table_d, *sink;
    unsigned long long *cyc_d;
    CHECK(hipMalloc(&table_d, 4 * kWords));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMalloc(&cyc_d, 8 * n_cu));
    CHECK(hipMemcpy(table_d, t.data(), 4 * kWords, hipMemcpyHostToDevice));
    printf("lds_probe: %d CUs, 1 block of 1024 threads per CU, %d steps per chain\n", n_cu, steps);
    run<0, 6>("chase", table_d, steps, n_cu, sink, cyc_d, 1);
    run<0, 12>("chase", table_d, steps, n_cu, sink, cyc_d, 1);
    run<1, 6>("chase2", table_d, steps, n_cu, sink, cyc_d, 2);
    run<1, 12>("chase2", table_d, steps, n_cu, sink, cyc_d, 2);
    run<4, 6>("rankstep", table_d, steps, n_cu, sink, cyc_d, 2);
    run<4, 12>("rankstep", table_d, steps, n_cu, sink, cyc_d, 2);
    run<2, 8>("indep", table_d, steps, n_cu, sink, cyc_d, 1);
    run<2, 32>("indep", table_d, steps, n_cu, sink, cyc_d, 1);
    run<3, 8>("seq", table_d, steps, n_cu, sink, cyc_d, 1);
    run<3, 32>("seq", table_d, steps, n_cu, sink, cyc_d, 1);
    CHECK(hipFree(table_d));
    CHECK(hipFree(sink));
    CHECK(hipFree(cyc_d));
    return 0;
}
