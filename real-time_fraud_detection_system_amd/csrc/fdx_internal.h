// Internal helpers shared by the fdx HIP translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "fdx.h"

namespace fdx {

constexpr int kWave = 64;  // CDNA wavefront width

void set_error(const char *fmt, ...);

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

#define FDX_REQUIRE(cond, ...)                     \
    do {                                           \
        if (!(cond)) {                             \
            ::fdx::set_error(__VA_ARGS__);         \
            return FDX_E_INVALID;                  \
        }                                          \
    } while (0)

#define FDX_HIP(call)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess) {                                                           \
            ::fdx::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),       \
                             __FILE__, __LINE__);                                         \
            return FDX_E_HIP;                                                             \
        }                                                                                 \
    } while (0)

// Checks the launch that was just enqueued.
#define FDX_LAUNCHED(name)                                                                \
    do {                                                                                  \
        hipError_t e_ = hipGetLastError();                                                \
        if (e_ != hipSuccess) {                                                           \
            ::fdx::set_error("launch of %s failed: %s", name, hipGetErrorString(e_));      \
            return FDX_E_HIP;                                                             \
        }                                                                                 \
    } while (0)

// Integer min / max for device code.  HIP's min<int64_t>(a, b) with either argument not already
// int64_t converts both to double (v_cvt + v_ldexp + v_min_f64 + v_cvt back): slow, and a VGPR
// result where the operands were wave-uniform -- a buffer descriptor built from one made every
// buffer store of k_customer_walk a readfirstlane loop.
__device__ __forceinline__ int64_t imin64(int64_t a, int64_t b) { return a < b ? a : b; }
__device__ __forceinline__ int64_t imax64(int64_t a, int64_t b) { return a > b ? a : b; }

// Terminal count record word (fdx_terminal_windows_packed): NB | FRAUD << 32.
__device__ __forceinline__ int64_t term_word(int32_t nb, int32_t fraud) {
    return (int64_t)(((uint64_t)(uint32_t)fraud << 32) | (uint32_t)nb);
}
__device__ __forceinline__ int32_t term_nb(int64_t w) { return (int32_t)(uint32_t)((uint64_t)w & 0xFFFFFFFFu); }
// RISK = FRAUD / NB with fillna(0) of 0/0 (feature_transformation.ipynb:1512-1517)
__device__ __forceinline__ double term_risk(int64_t w) {
    const uint32_t nb = (uint32_t)((uint64_t)w & 0xFFFFFFFFu), fr = (uint32_t)((uint64_t)w >> 32);
    return nb > 0 ? (double)fr / (double)nb : 0.0;
}

// COMPACT count records (fdx_terminal_windows_grouped_compact, W = 3): 16 bytes per row,
// lo = NB_0 | NB_1 << 21 | NB_2 << 42, hi = FRAUD_0 | FRAUD_1 << 21 | FRAUD_2 << 42 (one
// aligned 16-byte access instead of a 24-byte record over two).  A row whose window count
// does not fit 21 bits has bit 63 of lo set and the low 63 bits = the word offset, from the
// start of the record array, of its full 3-word record (the array's overflow area).
constexpr int kCompactBits = 21;
constexpr int64_t kCompactMax = (1LL << kCompactBits) - 1;
__device__ __forceinline__ void compact_load(const int64_t *rec, int64_t q, int64_t (&tw)[3]) {
    const longlong2 p = *reinterpret_cast<const longlong2 *>(rec + 2 * q);
    if (p.x < 0) {
        const int64_t *wide = rec + (p.x & INT64_MAX);
        tw[0] = wide[0];
        tw[1] = wide[1];
        tw[2] = wide[2];
    } else {
#pragma unroll
        for (int w = 0; w < 3; ++w)
            tw[w] = term_word((int32_t)((p.x >> (kCompactBits * w)) & kCompactMax),
                              (int32_t)((p.y >> (kCompactBits * w)) & kCompactMax));
    }
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t round_up(size_t a, size_t m) { return (a + m - 1) / m * m; }

// Grid for a grid-stride streaming kernel: enough blocks to fill 256 CUs several times,
// capped so launch overhead and tail stay small (cdna_hip_programming.md Guideline 11).
inline unsigned stream_grid(int64_t n, int block, int64_t cap = 256 * 8) {
    int64_t g = ceil_div(n, block);
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (unsigned)g;
}

}  // namespace fdx
