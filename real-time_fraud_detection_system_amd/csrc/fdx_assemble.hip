// fdx_assemble.hip -- K3's first half: the scoring rows.  Flags (is_weekend / is_night or the
// Spark forms), the customer averages (SUM / NB) and terminal risks (FRAUD / NB), StandardScaler
// (z = (x - mean) / scale in float64, then float32 as sklearn's _validate_X_predict), and each
// value replaced by its rank among the forest's float32 thresholds of that feature, so that the
// walk (fdx_forest.hip) compares integers: x32 <= thr64  <=>  rank(x32) <= k  exactly.
// Replaces loaded_scaler.transform (pyspark/scripts/fraud_detection.py:190; shared_functions.py
// :114-120) and the feature assembly of feature_transformation.ipynb:2890-2905 / the UDF frame of
// fraud_detection.py:183-189; optionally writes the featurized table itself
// (fdx_forest_prepare_grouped_rows).
#include "fdx_forest_internal.h"

namespace fdx {
namespace {

// lower_bound(U_f, v) - U_f, branch-free (Khuong & Morin); NaN -> 0xFFFF
__device__ __forceinline__ uint32_t rank_of(float v, const float *__restrict__ u, int32_t n) {
    if (v != v) return 0xFFFFu;
    if (n <= 0) return 0u;
    const float *b = u;
    while (n > 1) {
        const int32_t h = n >> 1;
        b = (b[h] < v) ? b + h : b;
        n -= h;
    }
    return (uint32_t)(b - u) + (uint32_t)(*b < v);
}

// ranks of a whole row: per feature, a branch-free lower_bound over the segment samples
// in LDS (all features advance together), then the count of values < v inside the one
// segment it lands in, read from global memory as seg/4 independent float4 loads.
// r = #{u in U_f : u < v}:  c = #{samples < v};  c == 0 -> 0, else seg*(c-1) + #{u < v in
// segment c-1} (every value of later segments is >= the next sample >= v; padding is +inf).
// Only the features in `need` are searched; out[f] of the others is left as the caller set it.
__device__ __forceinline__ void rank_row(const float (&v)[16], int nf, const RankTab &rt, const float *s_smp,
                                         uint32_t (&out)[16], uint32_t need = 0xFFFFu) {
    int32_t lo[16], n[16];
    int32_t nmax = 0;
#pragma unroll
    for (int f = 0; f < 16; ++f) {
        lo[f] = rt.soff[f];
        n[f] = (f < nf && ((need >> f) & 1u)) ? rt.scnt[f] : 0;
        nmax = max(nmax, n[f]);
    }
    while (nmax > 1) {
        nmax = 0;
#pragma unroll
        for (int f = 0; f < 16; ++f) {
            if (n[f] > 1) {
                const int32_t h = n[f] >> 1;
                lo[f] = (s_smp[lo[f] + h] < v[f]) ? lo[f] + h : lo[f];
                n[f] -= h;
            }
            nmax = max(nmax, n[f]);
        }
    }
#pragma unroll
    for (int f = 0; f < 16; ++f) {
        if (!((need >> f) & 1u)) continue;
        uint32_t r = 0u;
        if (f < nf && n[f] > 0) {
            const int32_t c = lo[f] - rt.soff[f] + (s_smp[lo[f]] < v[f] ? 1 : 0);
            if (c > 0) {
                const float4 *sg = reinterpret_cast<const float4 *>(rt.useg + rt.uoff[f] + (int64_t)(c - 1) * rt.seg);
                uint32_t k = 0;
                auto seg_count = [&](auto nq) {  // the segment's loads all in flight: one round trip
                    constexpr int NQ = decltype(nq)::value;
                    float4 w[NQ];
#pragma unroll
                    for (int q = 0; q < NQ; ++q) w[q] = sg[q];
#pragma unroll
                    for (int q = 0; q < NQ; ++q)
                        k += (uint32_t)(w[q].x < v[f]) + (uint32_t)(w[q].y < v[f]) + (uint32_t)(w[q].z < v[f]) +
                             (uint32_t)(w[q].w < v[f]);
                };
                if (rt.seg == 16) {  // (uniform)
                    seg_count(std::integral_constant<int, 4>{});
                } else if (rt.seg == 32) {
                    seg_count(std::integral_constant<int, 8>{});
                } else if (rt.seg == 64) {  // (forests with ~300k thresholds: the deployed RF, rank layout v2)
                    seg_count(std::integral_constant<int, 16>{});
                } else {
                    for (int q = 0; q < rt.seg / 4; ++q) {
                        const float4 w = sg[q];
                        k += (uint32_t)(w.x < v[f]) + (uint32_t)(w.y < v[f]) + (uint32_t)(w.z < v[f]) +
                             (uint32_t)(w.w < v[f]);
                    }
                }
                r = (uint32_t)(c - 1) * (uint32_t)rt.seg + k;
            }
        }
        out[f] = (f < nf && v[f] != v[f]) ? 0xFFFFu : r;
    }
}

// rank_row over a compile-time feature list (the continuous features of the reference's
// 15-column layout): the search loop runs a fixed, uniform number of rounds over only them.
template <int NS>
__device__ __forceinline__ void rank_fixed(const float (&v)[16], const int (&fs)[NS], const RankTab &rt,
                                           const float *s_smp, uint32_t (&out)[16]) {
    int32_t lo[NS], n[NS];
    int32_t nmax = 0;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        lo[i] = rt.soff[fs[i]];
        n[i] = rt.scnt[fs[i]];
        nmax = max(nmax, n[i]);
    }
    while (nmax > 1) {  // uniform: the trip count depends on the table sizes only
        nmax = 0;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            if (n[i] > 1) {
                const int32_t h = n[i] >> 1;
                lo[i] = (s_smp[lo[i] + h] < v[fs[i]]) ? lo[i] + h : lo[i];
                n[i] -= h;
            }
            nmax = max(nmax, n[i]);
        }
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const int f = fs[i];
        uint32_t r = 0u;
        if (n[i] > 0) {
            const int32_t c = lo[i] - rt.soff[f] + (s_smp[lo[i]] < v[f] ? 1 : 0);
            if (c > 0) {
                const float4 *sg = reinterpret_cast<const float4 *>(rt.useg + rt.uoff[f] + (int64_t)(c - 1) * rt.seg);
                uint32_t k = 0;
                for (int q = 0; q < rt.seg / 4; ++q) {
                    const float4 w = sg[q];
                    k += (uint32_t)(w.x < v[f]) + (uint32_t)(w.y < v[f]) + (uint32_t)(w.z < v[f]) +
                         (uint32_t)(w.w < v[f]);
                }
                r = (uint32_t)(c - 1) * (uint32_t)rt.seg + k;
            }
        }
        out[f] = v[f] != v[f] ? 0xFFFFu : r;
    }
}


// every thread of the block: stage the sample table into LDS (prepare kernels, RANK mode)
__device__ __forceinline__ void stage_samples(float *s_smp, const RankTab &rt) {
    for (int i = threadIdx.x; i < rt.n_smp; i += blockDim.x) s_smp[i] = rt.smp[i];
    __syncthreads();
}

// Row writers of the prepare kernels: float32 rows [n][FS], or rank rows [n][16] u16.
template <int FS, bool RANK>
__device__ __forceinline__ void store_row(void *z, int64_t r, const float (&v)[FS], int nf, const RankTab &rt,
                                          const float *s_smp) {
    if constexpr (RANK) {
        static_assert(FS == 16, "rank rows have 16 slots");
        uint32_t q[16];
        rank_row(v, nf, rt, s_smp, q);
        uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<uint16_t *>(z) + r * 16);
        dst[0] = make_uint4(q[0] | q[1] << 16, q[2] | q[3] << 16, q[4] | q[5] << 16, q[6] | q[7] << 16);
        dst[1] = make_uint4(q[8] | q[9] << 16, q[10] | q[11] << 16, q[12] | q[13] << 16, q[14] | q[15] << 16);
    } else {
        float4 *dst = reinterpret_cast<float4 *>(reinterpret_cast<float *>(z) + r * FS);
#pragma unroll
        for (int q = 0; q < FS / 4; ++q) dst[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
}

template <int FS, bool RANK>
__device__ __forceinline__ void store_col(void *z, int64_t r, int col, float v, const RankTab &rt) {
    if constexpr (RANK)
        reinterpret_cast<uint16_t *>(z)[r * 16 + col] = (uint16_t)rank_of(v, rt.u + rt.off[col], rt.cnt[col]);
    else
        reinterpret_cast<float *>(z)[r * FS + col] = v;
}

// z32[r][f] = (float)((x - mean[f]) / scale[f]) (or its rank); slots >= nf are 0.
template <int FS, bool RANK>
__global__ void __launch_bounds__(256) k_prepare(const double *__restrict__ X, int64_t n, int64_t rs,
                                                 int64_t cs, int32_t nf, const double *__restrict__ mean,
                                                 const double *__restrict__ scale, void *__restrict__ z,
                                                 int32_t *__restrict__ nan_flag, RankTab rt) {
    __shared__ float s_smp[RANK ? kMaxRankSamples : 1];
    if (RANK) stage_samples(s_smp, rt);
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        float v[FS];
        bool nan = false;
#pragma unroll
        for (int f = 0; f < FS; ++f) {
            if (f < nf) {
                double x = X[r * rs + (int64_t)f * cs];
                if (mean) x = x - mean[f];
                if (scale) x = x / scale[f];
                v[f] = (float)x;
                nan |= x != x;
            } else {
                v[f] = 0.0f;
            }
        }
        if (nan) *nan_flag = 1;  // routes the traversal through the NaN-aware step
        store_row<FS, RANK>(z, r, v, nf, rt, s_smp);
    }
}

// Rank layout v2 rows: 32 u16 slots per row (64 B), slot s = the clamped rank of its
// feature (build_rank_layout), 0xFFFF for a NaN feature; unused slots 0.  One 512-thread block
// per CU (the v2 sample table, up to kMaxRankSamplesV2 floats, + the threads' slot rows in LDS;
// the lockstep search of 15 features takes ~210 VGPRs: 1,024 threads spilled 208); every feature's
// rank at once (rank_row: the searches advance together, each 16-float segment read in one round
// trip), then the slots through the thread's LDS row.  (One feature after the other over 64-float
// segments: 7.7 ms for 20M deployed-model rows, r06k.)
constexpr int kPrepV2Block = 512;
__global__ void __launch_bounds__(kPrepV2Block) k_prepare_v2(const double *__restrict__ X, int64_t n, int64_t rs,
                                                             int64_t cs, int32_t nf, const double *__restrict__ mean,
                                                             const double *__restrict__ scale, uint16_t *__restrict__ z,
                                                             int32_t *__restrict__ nan_flag, RankTab rt) {
    __shared__ float s_smp[kMaxRankSamplesV2];
    __shared__ __align__(16) uint16_t s_row[kPrepV2Block][32];  // the thread's slot row (64 B)
    __shared__ int32_t s_sf[32], s_sb[32];                       // slot -> feature, slot base
    for (int i = threadIdx.x; i < rt.n_smp; i += blockDim.x) s_smp[i] = rt.smp[i];
    if (threadIdx.x < 32) {
        s_sf[threadIdx.x] = (int)threadIdx.x < rt.n_slots ? rt.slot_feat[threadIdx.x] : -1;
        s_sb[threadIdx.x] = rt.slot_base[threadIdx.x];
    }
    __syncthreads();
    uint16_t *mine = s_row[threadIdx.x];
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        bool any_nan = false;
        float v[16];
#pragma unroll
        for (int f = 0; f < 16; ++f) {
            v[f] = 0.0f;
            if (f < nf) {
                double x = X[r * rs + (int64_t)f * cs];
                if (mean) x = x - mean[f];
                if (scale) x = x / scale[f];
                v[f] = (float)x;
                any_nan |= v[f] != v[f];
            }
        }
        uint32_t rk[16];
        rank_row(v, nf, rt, s_smp, rk, (1u << nf) - 1u);
#pragma unroll
        for (int q = 0; q < 4; ++q) reinterpret_cast<uint4 *>(mine)[q] = make_uint4(0, 0, 0, 0);
        // slots in feature order (build_rank_layout): feature f's slots follow one another
        int s = 0;
#pragma unroll
        for (int f = 0; f < 16; ++f) {
            if (f < nf) {
                const bool isn = v[f] != v[f];
                for (; s < 32 && s_sf[s] == f; ++s) {  // (uniform)
                    const int64_t c = (int64_t)rk[f] - s_sb[s];
                    mine[s] = isn ? (uint16_t)0xFFFFu : (uint16_t)(c < 0 ? 0 : (c > 32767 ? 32767 : c));
                }
            }
        }
        if (any_nan) *nan_flag = 1;
        uint4 *dst = reinterpret_cast<uint4 *>(z + r * 32);
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[q] = reinterpret_cast<const uint4 *>(mine)[q];
    }
}

// out = (X - mean) / scale elementwise in float64 (StandardScaler.transform), any strides.
__global__ void __launch_bounds__(256) k_scale(const double *__restrict__ X, int64_t n, int32_t nf,
                                               int64_t rs, int64_t cs, const double *__restrict__ mean,
                                               const double *__restrict__ scale, double *__restrict__ out,
                                               int64_t ors, int64_t ocs) {
    const int64_t total = n * nf;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / nf;
        const int f = (int)(e - r * nf);
        double x = X[r * rs + (int64_t)f * cs];
        if (mean) x = x - mean[f];
        if (scale) x = x / scale[f];
        out[r * ors + (int64_t)f * ocs] = x;
    }
}

// The weekend / night flags of a nanosecond timestamp, with the floor divisions of pandas'
// dt accessors (feature_transformation.ipynb's is_weekend / is_night; fraud_detection.py's
// dayofweek / hour for FDX_FLAGS_SPARK).  floor(t / 1 day) = floor(floor(t / 1 s) / 86,400 s) and
// the hour likewise, so one 64-bit division to whole seconds, then 32-bit day / hour / weekday
// arithmetic while the seconds fit (1901-2038), the 64-bit form otherwise: the same values.
__device__ __forceinline__ void day_flags(int64_t t, int32_t flags_mode, bool &we, bool &ni) {
    int64_t sec = t / 1000000000LL;
    if (sec * 1000000000LL != t && t < 0) --sec;
    int32_t hour, wd;
    if (sec >= INT32_MIN && sec <= INT32_MAX) {
        const int32_t s32 = (int32_t)sec;
        int32_t day = s32 / 86400;
        if (day * 86400 != s32 && s32 < 0) --day;
        hour = (s32 - day * 86400) / 3600;
        wd = (day + 3) % 7;
    } else {
        int64_t day = sec / 86400;
        if (day * 86400 != sec && sec < 0) --day;
        hour = (int32_t)((sec - day * 86400) / 3600);
        wd = (int32_t)((day + 3) % 7);
    }
    if (wd < 0) wd += 7;
    we = flags_mode == FDX_FLAGS_NOTEBOOK ? wd >= 5 : (((wd + 1) % 7) + 1) >= 5;
    ni = flags_mode == FDX_FLAGS_NOTEBOOK ? hour <= 6 : hour >= 20;
}

__device__ __forceinline__ float zval(double x, const double *mean, const double *scale, int f) {
    if (mean) x = x - mean[f];
    if (scale) x = x / scale[f];
    return (float)x;
}

// Fused assemble + scale: the scoring pipeline writes the forest's float32 feature rows
// directly (no float64 feature matrix round trip).  Columns follow input_features.
template <int FS, bool RANK>
__global__ void __launch_bounds__(256) k_zfill_time(const double *__restrict__ amount,
                                                   const uint8_t *__restrict__ weekend,
                                                   const uint8_t *__restrict__ night, int64_t n,
                                                   const double *__restrict__ mean,
                                                   const double *__restrict__ scale, void *__restrict__ z,
                                                   int32_t *__restrict__ nan_flag, RankTab rt) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const float a = zval(amount[r], mean, scale, 0);
        store_col<FS, RANK>(z, r, 0, a, rt);
        store_col<FS, RANK>(z, r, 1, zval((double)weekend[r], mean, scale, 1), rt);
        store_col<FS, RANK>(z, r, 2, zval((double)night[r], mean, scale, 2), rt);
        if (RANK) store_col<FS, RANK>(z, r, 15, 0.0f, rt);  // unused slot: defined bytes
        if (a != a) *nan_flag = 1;
    }
}

template <int FS, bool RANK>
__global__ void __launch_bounds__(256) k_zfill_group(const int32_t *__restrict__ perm,
                                                    const int32_t *__restrict__ nb,
                                                    const double *__restrict__ val, int64_t n, int32_t W,
                                                    int32_t col0, const double *__restrict__ mean,
                                                    const double *__restrict__ scale, void *__restrict__ z,
                                                    int32_t *__restrict__ nan_flag, RankTab rt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = perm[i];
        bool nan = false;
        for (int w = 0; w < W; ++w) {
            store_col<FS, RANK>(z, o, col0 + 2 * w, zval((double)nb[(int64_t)w * n + i], mean, scale, col0 + 2 * w),
                                rt);
            const float v = zval(val[(int64_t)w * n + i], mean, scale, col0 + 2 * w + 1);
            store_col<FS, RANK>(z, o, col0 + 2 * w + 1, v, rt);
            nan |= v != v;
        }
        if (nan) *nan_flag = 1;
    }
}

// same, from the multi-GPU count records (fdx_terminal_windows_packed), row j -> perm[j]
template <int FS, bool RANK>
__global__ void __launch_bounds__(256) k_zfill_reply(const int64_t *__restrict__ reply,
                                                    const int32_t *__restrict__ perm, int64_t n, int32_t W,
                                                    int32_t col0, const double *__restrict__ mean,
                                                    const double *__restrict__ scale, void *__restrict__ z,
                                                    int32_t *__restrict__ nan_flag, RankTab rt) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t *r = reply + j * W;
        const int64_t o = perm[j];
        bool nan = false;
        for (int w = 0; w < W; ++w) {
            store_col<FS, RANK>(z, o, col0 + 2 * w, zval((double)term_nb(r[w]), mean, scale, col0 + 2 * w), rt);
            const float v = zval(term_risk(r[w]), mean, scale, col0 + 2 * w + 1);
            store_col<FS, RANK>(z, o, col0 + 2 * w + 1, v, rt);
            nan |= v != v;
        }
        if (nan) *nan_flag = 1;
    }
}

// Scoring rows in CUSTOMER-grouped order, written whole (64-byte coalesced rows): row i
// holds the transaction r = cust_perm[i]; amount / time flags / customer windows are
// already in this order, the terminal half is one count record read from
// term_rec[term_inv[r]] (term_inv: row -> send position; NULL = records already by row).
template <int FS, bool RANK>
__global__ void __launch_bounds__(256) k_zfill_grouped(
    const int64_t *__restrict__ cts, const double *__restrict__ camt, const int32_t *__restrict__ cnb,
    const double *__restrict__ cval, const int32_t *__restrict__ cust_perm, const int32_t *__restrict__ term_inv,
    const int64_t *__restrict__ term_rec, int64_t n, int32_t W, int32_t flags_mode, int32_t val_is_sum,
    const double *__restrict__ mean, const double *__restrict__ scale, void *__restrict__ z,
    int32_t *__restrict__ nan_flag, RankTab rt) {
    const int nf = 3 + 4 * W;
    __shared__ float s_smp[RANK ? kMaxRankSamples : 1];
    __shared__ uint16_t s_itab[RANK ? 16 * kIntTab : 1];
    if (RANK) {
        for (int e = threadIdx.x; e < 16 * kIntTab; e += blockDim.x) s_itab[e] = rt.itab[e];
        stage_samples(s_smp, rt);  // (its __syncthreads covers s_itab too)
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        float v[FS];
#pragma unroll
        for (int f = 0; f < FS; ++f) v[f] = 0.0f;
        const int32_t r = cust_perm ? cust_perm[i] : (int32_t)i;
        if (r < 0) {  // padding slot of the interleaved layout: never written back
            if constexpr (RANK) {
                uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<uint16_t *>(z) + i * 16);
                dst[0] = make_uint4(0, 0, 0, 0);
                dst[1] = make_uint4(0, 0, 0, 0);
            } else {
                float4 *dst = reinterpret_cast<float4 *>(reinterpret_cast<float *>(z) + i * FS);
#pragma unroll
                for (int qd = 0; qd < FS / 4; ++qd) dst[qd] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            continue;
        }
        bool we, ni;
        day_flags(cts[i], flags_mode, we, ni);
        if constexpr (RANK) {
            // flags and window counts: integer rank table; amount, averages and risks: search
            uint32_t q[16];
            uint32_t need = 1u | (0xFFFFu << nf);
            auto count = [&](int f, int32_t c) {
                if (c >= 0 && c < kIntTab) {
                    q[f] = s_itab[f * kIntTab + c];
                } else {
                    v[f] = zval((double)c, mean, scale, f);
                    need |= 1u << f;
                }
            };
            q[1] = s_itab[1 * kIntTab + (we ? 1 : 0)];
            q[2] = s_itab[2 * kIntTab + (ni ? 1 : 0)];
            q[15] = 0u;
            v[0] = zval(camt[i], mean, scale, 0);
            bool nan = v[0] != v[0];
            const int64_t q_ = term_inv ? term_inv[r] : r;
            const int64_t *rec = term_rec + q_ * W;
            int64_t ctw[3] = {0, 0, 0};
            if (val_is_sum & 4) compact_load(term_rec, q_, ctw);  // (W = 3, checked by the host)
#pragma unroll
            for (int w = 0; w < FDX_MAX_WINDOWS; ++w) {
                if (w < W) {
                    const int32_t c = cnb[(int64_t)w * n + i];
                    const double cv = cval[(int64_t)w * n + i];
                    count(3 + 2 * w, c);
                    v[4 + 2 * w] = zval((val_is_sum & 1) ? cv / (double)c : cv, mean, scale, 4 + 2 * w);
                    const int64_t tw = (val_is_sum & 4) ? ctw[w < 3 ? w : 0] : rec[w];
                    const int32_t tnb = term_nb(tw), tfr = (int32_t)((uint64_t)tw >> 32);
                    count(3 + 2 * W + 2 * w, tnb);
                    const int fr_ = 4 + 2 * W + 2 * w;
                    if (rt.rat && tnb >= 0 && tnb < kRatN && tfr >= 0 && tfr <= tnb) {
                        q[fr_] = rt.rat[((int64_t)fr_ * kRatN + tnb) * kRatN + tfr];
                    } else {
                        v[fr_] = zval(term_risk(tw), mean, scale, fr_);
                        need |= 1u << fr_;
                        nan |= v[fr_] != v[fr_];
                    }
                    need |= 1u << (4 + 2 * w);
                    nan |= v[4 + 2 * w] != v[4 + 2 * w];
                }
            }
            if (nan) *nan_flag = 1;
            if (W == 3 && !rt.rat) {  // the reference's layout, risks searched too
                constexpr int kFix[7] = {0, 4, 6, 8, 10, 12, 14};
                rank_fixed<7>(v, kFix, rt, s_smp, q);
                need &= ~((1u << 0) | (1u << 4) | (1u << 6) | (1u << 8) | (1u << 10) | (1u << 12) | (1u << 14));
                need &= (1u << nf) - 1u;
                if (__any(need != 0)) rank_row(v, nf, rt, s_smp, q, need);  // table overflows (rare)
            } else if (W == 3) {  // the reference's layout: amount + 3 averages searched in fixed rounds
                constexpr int kFix[4] = {0, 4, 6, 8};
                rank_fixed<4>(v, kFix, rt, s_smp, q);
                need &= ~((1u << 0) | (1u << 4) | (1u << 6) | (1u << 8));
                need &= (1u << nf) - 1u;
                if (__any(need != 0)) rank_row(v, nf, rt, s_smp, q, need);  // table overflows (rare)
            } else {
                rank_row(v, nf, rt, s_smp, q, need & 0xFFFFu);
            }
            uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<uint16_t *>(z) + i * 16);
            dst[0] = make_uint4(q[0] | q[1] << 16, q[2] | q[3] << 16, q[4] | q[5] << 16, q[6] | q[7] << 16);
            dst[1] = make_uint4(q[8] | q[9] << 16, q[10] | q[11] << 16, q[12] | q[13] << 16, q[14] | q[15] << 16);
            continue;
        }
        v[0] = zval(camt[i], mean, scale, 0);
        v[1] = zval((double)we, mean, scale, 1);
        v[2] = zval((double)ni, mean, scale, 2);
        bool nan = v[0] != v[0];
        const int64_t q = term_inv ? term_inv[r] : r;
        const int64_t *rec = term_rec + q * W;
        int64_t ctw[3] = {0, 0, 0};
        if (val_is_sum & 4) compact_load(term_rec, q, ctw);  // (W = 3, checked by the host)
#pragma unroll
        for (int w = 0; w < FDX_MAX_WINDOWS; ++w) {
            if (w < W) {
                const int32_t c = cnb[(int64_t)w * n + i];
                const double cv = cval[(int64_t)w * n + i];
                v[3 + 2 * w] = zval((double)c, mean, scale, 3 + 2 * w);
                v[4 + 2 * w] = zval((val_is_sum & 1) ? cv / (double)c : cv, mean, scale, 4 + 2 * w);
                const int64_t tw = (val_is_sum & 4) ? ctw[w < 3 ? w : 0] : rec[w];
                v[3 + 2 * W + 2 * w] = zval((double)term_nb(tw), mean, scale, 3 + 2 * W + 2 * w);
                v[4 + 2 * W + 2 * w] = zval(term_risk(tw), mean, scale, 4 + 2 * W + 2 * w);
                nan |= (v[4 + 2 * w] != v[4 + 2 * w]) | (v[4 + 2 * W + 2 * w] != v[4 + 2 * W + 2 * w]);
            }
        }
        if (nan) *nan_flag = 1;
        store_row<FS, RANK>(z, i, v, nf, rt, s_smp);
    }
}

// k_zfill_grouped for the reference's layout (W = 3, rank rows, ratio table, the four searched
// features' S-trees), restructured for memory-level parallelism.  The general kernel is bound by
// dependent round trips per row at 3 waves/SIMD (cust_perm -> term record -> ratio table;
// amount/average -> one search segment per feature, each behind its own branch).  Here the
// next row's loads (scoring-order columns + its term record, whose row index is fetched two
// rows ahead) are in flight while the current row is ranked, and the current row's four
// segment reads and three ratio-table reads are issued together, unconditionally (clamped
// addresses; the host pads useg by one segment).
// Search of the four continuous features (amount, the three averages): the descent of an
// S-tree in LDS -- every kW3Gap-th threshold in 8-key nodes, two ds_read_b128 per level, 4
// levels for <= 6,560 samples (the r03 form: an Eytzinger descent over every 16th threshold, 11
// dependent ds_read_b32 levels, then 64-byte segments read by lane quads) -- then one 16-byte
// read of the kW3Gap thresholds the sample count leaves.  One 1,024-thread block per CU (the
// trees take ~100 KiB of LDS).  Results are bit-identical to k_zfill_grouped<16, true> (same
// arithmetic, same fallbacks).
constexpr int kW3Block = 1024;

// [a < x] as the sign bit of a - x: the S-tree / segment keys are finite or +inf and never -0.0
// (build_search_trees and the segment table store +0.0 for -0.0: the same comparisons), f32
// denormals are kept (a - x == 0 only for a == x), and a NaN x never reaches it (nan_free; the
// caller ranks a NaN as 0xFFFF) -- so this is exactly the IEEE compare, without a v_cmp -> v_cndmask pair per key
// (each pair took an s_nop for the VCC hazard: 8 per S-tree level, r05 ISA)
__device__ __forceinline__ uint32_t lt_bit(float a, float x) { return __float_as_uint(a - x) >> 31; }
// The value a search descends with: a NaN replaced by 0.  a - NaN is that NaN, so with its sign
// bit set (x86 0/0, inf - inf) lt_bit would be 1 for every key, +inf padding included: the descent
// would count past the feature's samples and the segment load would read past its thresholds.
// The rank of a NaN is 0xFFFF whatever the search finds.
__device__ __forceinline__ float nan_free(float x) { return x == x ? x : 0.0f; }

// k_prepare<16, true> with the four kW3Search features ranked by their S-trees (the descent of
// k_zfill_grouped_w3 below) instead of the binary search over every 16th threshold: those four
// hold 17k-20k thresholds each in the bench model (11 dependent search rounds; 2.1 of the 9.4 ms
// of configs[2]'s prepare, profiles/r05be_prepare_ab.txt), the S-tree takes 4 levels.  The other
// features keep rank_row's search.  1,024-thread blocks: the S-trees (<= 112 KiB) + the samples
// (32 KiB) in LDS.  Same ranks as k_prepare bit for bit (same thresholds, same compares).
constexpr int kPrepStBlock = 1024;
__global__ void __launch_bounds__(kPrepStBlock) k_prepare_st(const double *__restrict__ X, int64_t n, int64_t rs,
                                                              int64_t cs, int32_t nf, const double *__restrict__ mean,
                                                              const double *__restrict__ scale, void *__restrict__ z,
                                                              int32_t *__restrict__ nan_flag, RankTab rt) {
    __shared__ float s_smp[kMaxRankSamples];
    __shared__ __align__(16) float s_t[kW3TreeFloats];
    __shared__ uint16_t s_itab[16 * kIntTab];
    for (int e = threadIdx.x; e < rt.n_etab / 4; e += blockDim.x)
        reinterpret_cast<float4 *>(s_t)[e] = reinterpret_cast<const float4 *>(rt.etab)[e];
    for (int e = threadIdx.x; e < 16 * kIntTab; e += blockDim.x) s_itab[e] = rt.itab[e];
    stage_samples(s_smp, rt);  // (its barrier covers the S-trees and the integer table too)
    const int e_lmax = max(max(rt.elev[0], rt.elev[1]), max(rt.elev[2], rt.elev[3]));
    uint32_t others = (1u << nf) - 1u;
#pragma unroll
    for (int s = 0; s < 4; ++s) others &= ~(1u << kW3Search[s]);
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        float v[16];
        uint32_t q[16];
        uint32_t need = others;
        bool nan = false;
        double xp = -1.0;  // the previous column's raw value
#pragma unroll
        for (int f = 0; f < 16; ++f) {
            q[f] = 0u;
            if (f < nf) {
                const double x0 = X[r * rs + (int64_t)f * cs];
                double x = x0;
                if (mean) x = x - mean[f];
                if (scale) x = x / scale[f];
                v[f] = (float)x;
                nan |= x != x;
                // Exact shortcuts for the searched features, bit-identical to the search (the host
                // built both tables with the same float64 scaling, float32 cast and lower_bound):
                // a small non-negative integer (the flags and window counts of the reference's
                // layout) -> RankTab::itab in LDS; a value that IS fr / nb for small integers with nb
                // the previous column (the terminal risks after their counts) -> RankTab::rat (L2)
                if ((others >> f) & 1u) {
                    const bool pint = xp >= 0.0 && xp < (double)kRatN && xp == (double)(int32_t)xp;
                    const int32_t nb = pint ? (int32_t)xp : 0;
                    const int32_t fr = (int32_t)__builtin_rint(x0 * (double)nb);
                    if (x0 >= 0.0 && x0 < (double)kIntTab && x0 == (double)(int32_t)x0) {
                        q[f] = s_itab[f * kIntTab + (int32_t)x0];
                        need &= ~(1u << f);
                    } else if (pint && nb > 0 && fr >= 0 && fr <= nb && (double)fr / (double)nb == x0) {
                        q[f] = rt.rat[((int64_t)f * kRatN + nb) * kRatN + fr];
                        need &= ~(1u << f);
                    }
                }
                xp = x0;
            } else {
                v[f] = 0.0f;
            }
        }
        if (nan) *nan_flag = 1;
        rank_row(v, nf, rt, s_smp, q, need);
        int32_t ek[4] = {0, 0, 0, 0}, cnt[4] = {0, 0, 0, 0};
        float xs[4];  // the searched values, a NaN as 0 (see nan_free)
#pragma unroll
        for (int s = 0; s < 4; ++s) xs[s] = nan_free(v[kW3Search[s]]);
        for (int l = 0; l < e_lmax; ++l) {  // uniform trip count
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if (l < rt.elev[s]) {
                    const float4 *nd = reinterpret_cast<const float4 *>(s_t) + 2 * (rt.eoff[s] + ek[s]);
                    const float4 a = nd[0], b = nd[1];
                    const float x = xs[s];
                    const int32_t c = (int32_t)(lt_bit(a.x, x) + lt_bit(a.y, x) + lt_bit(a.z, x) + lt_bit(a.w, x) +
                                                lt_bit(b.x, x) + lt_bit(b.y, x) + lt_bit(b.z, x) + lt_bit(b.w, x));
                    cnt[s] = cnt[s] * 9 + c;
                    ek[s] = ek[s] * 9 + 1 + c;
                }
            }
        }
        float4 sg[4];
#pragma unroll
        for (int s = 0; s < 4; ++s)  // (unconditional: the host pads useg by one segment)
            sg[s] = *reinterpret_cast<const float4 *>(rt.useg + rt.uoff[kW3Search[s]] +
                                                      (int64_t)max(cnt[s] - 1, 0) * kW3Gap);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int f = kW3Search[s];
            const float x = xs[s];
            const uint32_t kc = lt_bit(sg[s].x, x) + lt_bit(sg[s].y, x) + lt_bit(sg[s].z, x) + lt_bit(sg[s].w, x);
            const uint32_t rk = cnt[s] > 0 ? (uint32_t)(cnt[s] - 1) * kW3Gap + kc : 0u;
            q[f] = v[f] != v[f] ? 0xFFFFu : rk;
        }
        uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<uint16_t *>(z) + r * 16);
        dst[0] = make_uint4(q[0] | q[1] << 16, q[2] | q[3] << 16, q[4] | q[5] << 16, q[6] | q[7] << 16);
        dst[1] = make_uint4(q[8] | q[9] << 16, q[10] | q[11] << 16, q[12] | q[13] << 16, q[14] | q[15] << 16);
    }
}

struct PrepRow {
    int64_t t;
    double a;
    int32_t c[3];
    double cv[3];
    int64_t tw[3];  // the terminal count words: the wide record, or the compact one decoded (decode_tw)
    longlong2 raw;  // the compact record as loaded (decoded when the row is consumed)
    int32_t r;
};

// The feature table is stored behind the row's segment / ratio loads (r04: right after the row's
// loads or after the rank row measured slower), by nontemporal stores, and the row loop runs its
// first iteration peeled.
// EMIT: the featurized table besides the rank rows (fdx_forest_prepare_grouped_rows): 0 = none,
// FDX_ROWS_INPUT_ORDER / FDX_ROWS_SLOT_ORDER = the fdx_feature_row record of each slot's row at its
// input row / at its slot, stored as soon as the row's values are loaded (the record's registers
// die before the rank search; kept to the end, 15 VGPRs spilled)
// Loads of the NEXT row are issued at the top of each iteration and consumed one iteration
// later; nothing in that load phase may wait on a load (a wait covers every older load, the
// prefetch included: with the compact record's overflow branch and a runtime term_inv select
// in it, the r03 kernel waited twice per row on HBM round trips -- vmcnt(0) -- before doing the
// current row).  So the record is loaded raw and decoded when consumed (COMPACT), and the
// term_inv indirection (TINV, the multi-GPU reply records) runs one more iteration ahead.
template <bool COMPACT>
__device__ __forceinline__ void decode_tw(const int64_t *rec, PrepRow &L) {
    if constexpr (COMPACT) {
        if (L.raw.x < 0) {  // a count past 2^21 - 1: its full record in the overflow area (rare)
            const int64_t *wide = rec + (L.raw.x & INT64_MAX);
#pragma unroll
            for (int w = 0; w < 3; ++w) L.tw[w] = wide[w];
            // waited for inside the branch: a wait after it (taken or not) would cover every
            // load and store in flight, the next row's loads and the previous row's stores
#pragma unroll
            for (int w = 0; w < 3; ++w) asm volatile("" ::"v"(L.tw[w]));
        } else {
#pragma unroll
            for (int w = 0; w < 3; ++w)
                L.tw[w] = term_word((int32_t)((L.raw.x >> (kCompactBits * w)) & kCompactMax),
                                    (int32_t)((L.raw.y >> (kCompactBits * w)) & kCompactMax));
        }
    }
}

template <int EMIT, bool COMPACT, bool TINV>
__global__ void __launch_bounds__(kW3Block) k_zfill_grouped_w3(
    const int64_t *__restrict__ cts, const double *__restrict__ camt, const int32_t *__restrict__ cnb,
    const double *__restrict__ cval, const int32_t *__restrict__ cust_perm, const int32_t *__restrict__ term_inv,
    const int64_t *__restrict__ term_rec, int64_t n, int32_t flags_mode, int32_t val_is_sum,
    const double *__restrict__ mean, const double *__restrict__ scale, void *__restrict__ z,
    int32_t *__restrict__ nan_flag, RankTab rt, char *__restrict__ feat, int64_t fcap) {
    constexpr int W = 3, nf = 15;
    static_assert(sizeof(fdx_feature_row) == 80, "5 x 16-byte stores per feature record");
    __shared__ __align__(16) float s_t[kW3TreeFloats];  // the S-trees (RankTab::etab)
    __shared__ uint16_t s_itab[16 * kIntTab];
    // the scaler in LDS (identity where absent: x - 0.0 and x / 1.0 are exact): as kernel-argument
    // scalars its 30 doubles stayed live in SGPRs across the row loop, which spilled 129 SGPRs
    // into VGPR lanes (a v_readlane per use in the loop; r05 ISA)
    __shared__ double s_ms[32];
    __shared__ int32_t s_oc[32];  // rt.off / rt.cnt of the 16 slots: the rare full-search fallback
    if (threadIdx.x < 16) {
        s_ms[threadIdx.x] = mean && (int)threadIdx.x < nf ? mean[threadIdx.x] : 0.0;
        s_ms[16 + threadIdx.x] = scale && (int)threadIdx.x < nf ? scale[threadIdx.x] : 1.0;
        s_oc[threadIdx.x] = rt.off[threadIdx.x];
        s_oc[16 + threadIdx.x] = rt.cnt[threadIdx.x];
    }
    auto zs = [&](double x, int f) -> float { return (float)((x - s_ms[f]) / s_ms[16 + f]); };
    for (int e = threadIdx.x; e < 16 * kIntTab; e += blockDim.x) s_itab[e] = rt.itab[e];
    for (int e = threadIdx.x; e < rt.n_etab / 4; e += blockDim.x)
        reinterpret_cast<float4 *>(s_t)[e] = reinterpret_cast<const float4 *>(rt.etab)[e];
    __syncthreads();
    const int e_lmax = max(max(rt.elev[0], rt.elev[1]), max(rt.elev[2], rt.elev[3]));
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    auto row_of = [&](int64_t j) -> int32_t { return j < n ? (cust_perm ? cust_perm[j] : (int32_t)j) : -1; };
    auto rec_of = [&](int32_t r) -> int64_t { return TINV ? (r >= 0 ? (int64_t)term_inv[r] : -1) : (int64_t)r; };
    // issues every load of slot j (row r, record q) and waits on none of them
    auto load = [&](int64_t j, int32_t r, int64_t q, PrepRow &L) {
        L.r = r;
        const bool ok = j < n && r >= 0;
        const int64_t jj = ok ? j : 0, qq = ok ? q : 0;  // defined values: every lane runs the row arithmetic
        L.t = cts[jj];
        L.a = camt[jj];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            L.c[w] = cnb[(int64_t)w * n + jj];
            L.cv[w] = cval[(int64_t)w * n + jj];
        }
        if constexpr (COMPACT) {
            L.raw = *reinterpret_cast<const longlong2 *>(term_rec + 2 * qq);
        } else {
#pragma unroll
            for (int w = 0; w < W; ++w) L.tw[w] = term_rec[qq * W + w];
        }
    };
    auto settle = [&](int64_t j, PrepRow &L) {  // the consume side: dummies for dead lanes, decode
        if (!(j < n && L.r >= 0)) {
            L.t = 0;
            L.a = 0.0;
            L.raw = make_longlong2(0, 0);
#pragma unroll
            for (int w = 0; w < W; ++w) {
                L.c[w] = 1;
                L.cv[w] = 0.0;
                L.tw[w] = 0;
            }
        }
        decode_tw<COMPACT>(term_rec, L);
    };
    // wave-uniform loop (stride and the wave's first slot are multiples of 64): every lane of a
    // wave runs each iteration, so the quads of k_seg_count_quad stay whole; lanes past n and
    // padding slots compute on defined dummies and store the zero row / nothing
    const int lane = threadIdx.x & (kWave - 1);
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    PrepRow cur;
    {
        const int32_t r0 = row_of(i);
        load(i, r0, rec_of(r0), cur);
    }
    int32_t r1 = row_of(i + stride), r2 = row_of(i + 2 * stride);  // slots one and two ahead
    int64_t q1 = rec_of(r1);
    // one row per call; the loop below runs it with its first iteration peeled, so
    // that the loop header is reached only in the steady state: entered straight from the
    // prologue, whose last memory operations are the first row's loads, the header's merged wait
    // state forced s_waitcnt vmcnt(0) there -- every iteration then waited for the previous row's
    // stores to complete
    auto row_iter = [&]() {
        settle(i, cur);
        PrepRow nxt;
        load(i + stride, r1, q1, nxt);  // next row's loads in flight during this row
        q1 = rec_of(r2);                // (r2 arrived during the previous row)
        r1 = r2;
        r2 = row_of(i + 3 * stride);
        const bool live = i < n && cur.r >= 0;
        bool we, ni;
        day_flags(cur.t, flags_mode, we, ni);
        float v[16];
        uint32_t q[16];
#pragma unroll
        for (int f = 0; f < 16; ++f) {
            v[f] = 0.0f;
            q[f] = 0u;
        }
        uint32_t need = 0u;
        auto count = [&](int f, int32_t c) {
            if (c >= 0 && c < kIntTab) {
                q[f] = s_itab[f * kIntTab + c];
            } else {
                v[f] = zs((double)c, f);
                need |= 1u << f;
            }
        };
        q[1] = s_itab[1 * kIntTab + (we ? 1 : 0)];
        q[2] = s_itab[2 * kIntTab + (ni ? 1 : 0)];
        v[0] = zs(cur.a, 0);
        bool nan = v[0] != v[0];
        auto fst = [](auto *p, auto v) {  // feature-table store: nontemporal, the step never reads it
            __builtin_nontemporal_store(v, p);
        };
        auto emit = [&]() {
            // the featurized row: a record at its input row (one random 80-byte write), or the
            // columns at its slot (consecutive lanes, consecutive elements: every store of a wave
            // is whole lines; an 80-byte record per slot, 5 strided 16-byte stores, measured
            // +0.62 ms at config 2; padding slots: row -1, zero features)
            // (slot order: every lane stores, i < round_up(n, 64) <= fcap -- no branch, so that
            // no wait behind it has to assume the stores were skipped)
            if (EMIT == FDX_ROWS_SLOT_ORDER || (i < n && live && (uint64_t)cur.r < (uint64_t)fcap)) {
                auto u32 = [](double d, int h) { return (uint32_t)((uint64_t)__double_as_longlong(d) >> (32 * h)); };
                uint32_t c[W], tn[W];
                double avg[W], rk[W];
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    c[w] = live ? (uint32_t)cur.c[w] : 0u;
                    avg[w] = !live ? 0.0 : (val_is_sum & 1) ? cur.cv[w] / (double)cur.c[w] : cur.cv[w];
                    tn[w] = live ? (uint32_t)term_nb(cur.tw[w]) : 0u;
                    rk[w] = live ? term_risk(cur.tw[w]) : 0.0;
                }
                const uint32_t fl = live ? ((uint32_t)we | (uint32_t)ni << 8) : 0u;
                if constexpr (EMIT == FDX_ROWS_SLOT_ORDER) {
#pragma unroll
                    for (int w = 0; w < W; ++w) {
                        fst(reinterpret_cast<uint32_t *>(feat + FDX_FEATURE_COL(w, fcap)) + i, c[w]);
                        fst(reinterpret_cast<uint32_t *>(feat + FDX_FEATURE_COL(3 + w, fcap)) + i, tn[w]);
                        fst(reinterpret_cast<double *>(feat + FDX_FEATURE_COL(6 + w, fcap)) + i, avg[w]);
                        fst(reinterpret_cast<double *>(feat + FDX_FEATURE_COL(9 + w, fcap)) + i, rk[w]);
                    }
                    fst(reinterpret_cast<int32_t *>(feat + FDX_FEATURE_COL(12, fcap)) + i, live ? cur.r : -1);
                    fst(reinterpret_cast<uint16_t *>(feat + FDX_FEATURE_COL(13, fcap)) + i, (uint16_t)fl);
                } else {
                    uint4 *dst = reinterpret_cast<uint4 *>(feat) + (int64_t)cur.r * 5;
                    dst[0] = make_uint4(c[0], c[1], c[2], tn[0]);
                    dst[1] = make_uint4(tn[1], tn[2], u32(avg[0], 0), u32(avg[0], 1));
                    dst[2] = make_uint4(u32(avg[1], 0), u32(avg[1], 1), u32(avg[2], 0), u32(avg[2], 1));
                    dst[3] = make_uint4(u32(rk[0], 0), u32(rk[0], 1), u32(rk[1], 0), u32(rk[1], 1));
                    dst[4] = make_uint4(u32(rk[2], 0), u32(rk[2], 1), fl, (uint32_t)cur.r);
                }
            }
        };
        uint16_t rq[W];
        bool rat_ok[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int32_t c = cur.c[w];
            count(3 + 2 * w, c);
            v[4 + 2 * w] = zs((val_is_sum & 1) ? cur.cv[w] / (double)c : cur.cv[w], 4 + 2 * w);
            nan |= v[4 + 2 * w] != v[4 + 2 * w];
            const int64_t tw = cur.tw[w];
            const int32_t tnb = term_nb(tw), tfr = (int32_t)((uint64_t)tw >> 32);
            count(3 + 2 * W + 2 * w, tnb);
            const int fr_ = 4 + 2 * W + 2 * w;
            rat_ok[w] = tnb >= 0 && tnb < kRatN && tfr >= 0 && tfr <= tnb;
            // unconditional read (index clamped to 0 when the table does not apply)
            rq[w] = rt.rat[rat_ok[w] ? ((int64_t)fr_ * kRatN + tnb) * kRatN + tfr : 0];
        }
        // the 4 continuous features: S-tree descents (cs = #samples < v: the digits c of the
        // levels in base 9), then the kW3Gap thresholds of the segment the count leaves
        int32_t ek[4] = {0, 0, 0, 0}, cs[4] = {0, 0, 0, 0};
        float xs[4];  // the searched values, a NaN as 0 (see nan_free)
#pragma unroll
        for (int s = 0; s < 4; ++s) xs[s] = nan_free(v[kW3Search[s]]);
        for (int l = 0; l < e_lmax; ++l) {  // uniform trip count
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if (l < rt.elev[s]) {
                    const float4 *nd = reinterpret_cast<const float4 *>(s_t) + 2 * (rt.eoff[s] + ek[s]);
                    const float4 a = nd[0], b = nd[1];
                    const float x = xs[s];
                    const int32_t c = (int32_t)(lt_bit(a.x, x) + lt_bit(a.y, x) + lt_bit(a.z, x) + lt_bit(a.w, x) +
                                                lt_bit(b.x, x) + lt_bit(b.y, x) + lt_bit(b.z, x) + lt_bit(b.w, x));
                    cs[s] = cs[s] * 9 + c;
                    ek[s] = ek[s] * 9 + 1 + c;
                }
            }
        }
        uint32_t kc[4];
        {
            float4 sg[4];
#pragma unroll
            for (int s = 0; s < 4; ++s)
                sg[s] = *reinterpret_cast<const float4 *>(rt.useg + rt.uoff[kW3Search[s]] +
                                                          (int64_t)max(cs[s] - 1, 0) * kW3Gap);
            // (stores issued behind the segment and ratio loads: waiting for those loads does
            // not wait for the stores -- vmcnt counts stores, in issue order)
            if constexpr (EMIT != 0) emit();
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float x = xs[s];
                kc[s] = lt_bit(sg[s].x, x) + lt_bit(sg[s].y, x) + lt_bit(sg[s].z, x) + lt_bit(sg[s].w, x);
            }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int f = kW3Search[s];
            const uint32_t r = cs[s] > 0 ? (uint32_t)(cs[s] - 1) * kW3Gap + kc[s] : 0u;
            q[f] = v[f] != v[f] ? 0xFFFFu : r;
        }
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int fr_ = 4 + 2 * W + 2 * w;
            if (rat_ok[w]) {
                q[fr_] = rq[w];
            } else {
                v[fr_] = zs(term_risk(cur.tw[w]), fr_);
                need |= 1u << fr_;
                nan |= v[fr_] != v[fr_];
            }
        }
        if (live && nan) *nan_flag = 1;
        need &= (1u << nf) - 1u;
        if (live && need) {  // table overflows (rare): a full lower_bound over U_f in HBM
#pragma unroll
            for (int f = 0; f < 16; ++f)
                if ((need >> f) & 1u) q[f] = rank_of(v[f], rt.u + s_oc[f], s_oc[16 + f]);
        }
        q[15] = 0u;
        if (i < n) {  // padding slot of the interleaved layout: the zero row
            uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<uint16_t *>(z) + i * 16);
            dst[0] = live ? make_uint4(q[0] | q[1] << 16, q[2] | q[3] << 16, q[4] | q[5] << 16, q[6] | q[7] << 16)
                          : make_uint4(0, 0, 0, 0);
            dst[1] = live ? make_uint4(q[8] | q[9] << 16, q[10] | q[11] << 16, q[12] | q[13] << 16, q[14] | q[15] << 16)
                          : make_uint4(0, 0, 0, 0);
        }
        cur = nxt;
    };
    if (i - lane < n) {  // (the first iteration peeled)
        row_iter();
        i += stride;
    }
    for (; i - lane < n; i += stride) row_iter();
}


// The featurized table alone (W = 3), for scoring rows that k_zfill_grouped_w3 does not build
// (the wide layout, or a forest whose searched features outgrow the S-trees' LDS budget: the
// rank rows then come from k_zfill_grouped).  Same columns, same arithmetic as k_zfill_grouped_w3's
// emit: slot order writes every slot i < round_up(n, 64) (padding slots: row -1, zeros), input
// order one fdx_feature_row at each live slot's row.
template <int EMIT, bool COMPACT>
__global__ void __launch_bounds__(256) k_feature_rows(
    const int64_t *__restrict__ cts, const int32_t *__restrict__ cnb, const double *__restrict__ cval,
    const int32_t *__restrict__ cust_perm, const int32_t *__restrict__ term_inv, const int64_t *__restrict__ term_rec,
    int64_t n, int32_t flags_mode, int32_t val_is_sum, char *__restrict__ feat, int64_t fcap) {
    constexpr int W = 3;
    const int64_t end = EMIT == FDX_ROWS_SLOT_ORDER ? (n + 63) / 64 * 64 : n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < end; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = i < n ? (cust_perm ? cust_perm[i] : (int32_t)i) : -1;
        const bool live = r >= 0;
        if (EMIT == FDX_ROWS_INPUT_ORDER && !(live && (uint64_t)r < (uint64_t)fcap)) continue;
        uint32_t c[W] = {0u, 0u, 0u}, tn[W] = {0u, 0u, 0u}, fl = 0u;
        double avg[W] = {0.0, 0.0, 0.0}, rk[W] = {0.0, 0.0, 0.0};
        if (live) {
            bool we, ni;
            day_flags(cts[i], flags_mode, we, ni);
            fl = (uint32_t)we | (uint32_t)ni << 8;
            const int64_t q = term_inv ? (int64_t)term_inv[r] : (int64_t)r;
            int64_t tw[3];
            if constexpr (COMPACT) {
                compact_load(term_rec, q, tw);
            } else {
#pragma unroll
                for (int w = 0; w < W; ++w) tw[w] = term_rec[q * W + w];
            }
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const int32_t cw = cnb[(int64_t)w * n + i];
                const double cv = cval[(int64_t)w * n + i];
                c[w] = (uint32_t)cw;
                avg[w] = (val_is_sum & 1) ? cv / (double)cw : cv;
                tn[w] = (uint32_t)term_nb(tw[w]);
                rk[w] = term_risk(tw[w]);
            }
        }
        if constexpr (EMIT == FDX_ROWS_SLOT_ORDER) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                reinterpret_cast<uint32_t *>(feat + FDX_FEATURE_COL(w, fcap))[i] = c[w];
                reinterpret_cast<uint32_t *>(feat + FDX_FEATURE_COL(3 + w, fcap))[i] = tn[w];
                reinterpret_cast<double *>(feat + FDX_FEATURE_COL(6 + w, fcap))[i] = avg[w];
                reinterpret_cast<double *>(feat + FDX_FEATURE_COL(9 + w, fcap))[i] = rk[w];
            }
            reinterpret_cast<int32_t *>(feat + FDX_FEATURE_COL(12, fcap))[i] = live ? r : -1;
            reinterpret_cast<uint16_t *>(feat + FDX_FEATURE_COL(13, fcap))[i] = (uint16_t)fl;
        } else {
            fdx_feature_row *o = reinterpret_cast<fdx_feature_row *>(feat) + r;
            fdx_feature_row v;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                v.cust_nb[w] = (int32_t)c[w];
                v.term_nb[w] = (int32_t)tn[w];
                v.cust_avg[w] = avg[w];
                v.term_risk[w] = rk[w];
            }
            v.weekend = (uint8_t)(fl & 1u);
            v.night = (uint8_t)(fl >> 8);
            v.pad[0] = v.pad[1] = 0;
            v.row = r;
            *o = v;
        }
    }
}

}  // namespace

// compute units of the current device (grid of the one-block-per-CU kernels)
static int device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 256;
    return cus > 0 ? cus : 256;
}

RankTab rank_tab(const fdx_forest_s *F) {
    RankTab rt;
    rt.u = F->rthr_d;
    rt.useg = F->rseg_d;
    rt.smp = F->rsmp_d;
    for (int f = 0; f < 32; ++f) {
        rt.off[f] = F->rthr_off[f];
        rt.cnt[f] = F->rthr_cnt[f];
        rt.uoff[f] = F->ruoff[f];
        rt.soff[f] = F->rsoff[f];
        rt.scnt[f] = F->rscnt[f];
        rt.slot_feat[f] = F->rslot_feat[f];
        rt.slot_base[f] = F->rslot_base[f];
    }
    rt.n_slots = F->rn_slots;
    rt.seg = F->rseg;
    rt.n_smp = F->rnsmp;
    rt.itab = F->ritab_d;
    rt.rat = F->rrat_d;
    rt.etab = F->rnetab > 0 ? F->retab_d : nullptr;
    rt.n_etab = F->rnetab;
    for (int s = 0; s < 4; ++s) {
        rt.eoff[s] = F->reoff[s];
        rt.elev[s] = F->relev[s];
    }
    return rt;
}


}  // namespace fdx

using namespace fdx;

// Launch a prepare kernel in the row format of the forest's current variant: rank rows
// (rank layout), float32 rows of 16 or 32 slots (wide layout).
#define FDX_PREP(KERNEL, GRID, ST, ...)                                                                    \
    do {                                                                                                  \
        const RankTab rt_ = rank_tab(F);                                                                  \
        if (rank_mode(F))                                                                                 \
            hipLaunchKernelGGL((KERNEL<16, true>), GRID, dim3(256), 0, ST, __VA_ARGS__, rt_);             \
        else if (F->zstride == 16)                                                                        \
            hipLaunchKernelGGL((KERNEL<16, false>), GRID, dim3(256), 0, ST, __VA_ARGS__, rt_);            \
        else                                                                                              \
            hipLaunchKernelGGL((KERNEL<32, false>), GRID, dim3(256), 0, ST, __VA_ARGS__, rt_);            \
    } while (0)


extern "C" int fdx_forest_prepare(fdx_forest F, const double *X_d, int64_t n, int64_t row_stride,
                                  int64_t col_stride, void *ws, size_t ws_bytes, void *stream) {
    FDX_REQUIRE(F, "null forest");
    FDX_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(X_d, "null pointer");
    float *z;
    double *acc;
    int32_t *flag;
    int rc = forest_ws(F, n, ws, ws_bytes, &z, &acc, &flag);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    FDX_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), st));
    unsigned grid = stream_grid(n, 256);
    if (rank_mode(F) && v2_rows(kVariants[F->variant].p16)) {
        FDX_REQUIRE(F->rnsmp <= kMaxRankSamplesV2, "v2 sample table of %d floats exceeds the LDS budget", F->rnsmp);
        const unsigned g2 = (unsigned)std::min<int64_t>(ceil_div(n, (int64_t)kPrepV2Block), (int64_t)F->n_cu * 4);
        hipLaunchKernelGGL(k_prepare_v2, dim3(g2), dim3(kPrepV2Block), 0, st, X_d, n, row_stride, col_stride,
                           F->n_features, F->mean_d, F->scale_d, reinterpret_cast<uint16_t *>(z), flag, rank_tab(F));
        FDX_LAUNCHED("k_prepare_v2");
        return FDX_OK;
    }
    if (rank_mode(F) && F->rnetab > 0 && F->n_features == 15) {  // the S-trees of the four searched features
        const RankTab rt = rank_tab(F);
        const unsigned g = (unsigned)std::min<int64_t>(ceil_div(n, (int64_t)kPrepStBlock), (int64_t)F->n_cu * 2);
        hipLaunchKernelGGL(k_prepare_st, dim3(g), dim3(kPrepStBlock), 0, st, X_d, n, row_stride, col_stride,
                           F->n_features, F->mean_d, F->scale_d, (void *)z, flag, rt);
        FDX_LAUNCHED("k_prepare_st");
        return FDX_OK;
    }
    FDX_PREP(k_prepare, dim3(grid), st, X_d, n, row_stride, col_stride, F->n_features, F->mean_d, F->scale_d,
             (void *)z, flag);
    FDX_LAUNCHED("k_prepare");
    return FDX_OK;
}


extern "C" int fdx_standard_scale(const double *X_d, int64_t n, int32_t n_features, int64_t row_stride,
                                  int64_t col_stride, const double *mean_d, const double *scale_d,
                                  double *out_d, int64_t out_row_stride, int64_t out_col_stride,
                                  void *stream) {
    FDX_REQUIRE(n >= 0 && n_features >= 1, "bad shape");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(X_d && out_d, "null pointer");
    hipLaunchKernelGGL(k_scale, dim3(stream_grid(n * n_features, 256)), dim3(256), 0, as_stream(stream), X_d,
                       n, n_features, row_stride, col_stride, mean_d, scale_d, out_d, out_row_stride,
                       out_col_stride);
    FDX_LAUNCHED("k_scale");
    return FDX_OK;
}

extern "C" int fdx_forest_prepare_features(fdx_forest F, int64_t n, int32_t n_windows, const double *amount_d,
                                           const uint8_t *weekend_d, const uint8_t *night_d,
                                           const int32_t *cust_perm_d, const int32_t *cust_nb_d,
                                           const double *cust_avg_d, const int32_t *term_perm_d,
                                           const int32_t *term_nb_d, const double *term_risk_d, void *ws,
                                           size_t ws_bytes, void *stream) {
    FDX_REQUIRE(F, "null forest");
    FDX_REQUIRE(!(rank_mode(F) && v2_rows(kVariants[F->variant].p16)),
                "the fused scoring rows need the v1 row format (one slot per feature)");
    FDX_REQUIRE(n >= 0 && n_windows >= 1 && n_windows <= FDX_MAX_WINDOWS, "bad argument");
    FDX_REQUIRE(F->n_features == 3 + 4 * n_windows, "forest has %d features, expected %d", F->n_features,
                3 + 4 * n_windows);
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(amount_d && weekend_d && night_d && cust_perm_d && cust_nb_d && cust_avg_d, "null pointer");
    float *z;
    double *acc;
    int32_t *flag;
    int rc = forest_ws(F, n, ws, ws_bytes, &z, &acc, &flag);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    FDX_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), st));
    const unsigned grid = stream_grid(n, 256);
    FDX_PREP(k_zfill_time, dim3(grid), st, amount_d, weekend_d, night_d, n, F->mean_d, F->scale_d, (void *)z, flag);
    FDX_PREP(k_zfill_group, dim3(grid), st, cust_perm_d, cust_nb_d, cust_avg_d, n, n_windows, 3, F->mean_d,
             F->scale_d, (void *)z, flag);
    if (term_perm_d && term_nb_d && term_risk_d)
        FDX_PREP(k_zfill_group, dim3(grid), st, term_perm_d, term_nb_d, term_risk_d, n, n_windows, 3 + 2 * n_windows,
                 F->mean_d, F->scale_d, (void *)z, flag);
    FDX_LAUNCHED("k_zfill");
    return FDX_OK;
}

extern "C" int fdx_forest_prepare_reply(fdx_forest F, const int64_t *reply_d, const int32_t *perm_d, int64_t n,
                                        int32_t n_windows, int32_t col0, void *ws, size_t ws_bytes,
                                        void *stream) {
    FDX_REQUIRE(F, "null forest");
    FDX_REQUIRE(!(rank_mode(F) && v2_rows(kVariants[F->variant].p16)),
                "the fused scoring rows need the v1 row format (one slot per feature)");
    FDX_REQUIRE(n >= 0 && n_windows >= 1 && n_windows <= FDX_MAX_WINDOWS, "bad argument");
    FDX_REQUIRE(col0 >= 0 && col0 + 2 * n_windows <= F->n_features, "columns out of range");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(reply_d && perm_d, "null pointer");
    float *z;
    double *acc;
    int32_t *flag;
    int rc = forest_ws(F, n, ws, ws_bytes, &z, &acc, &flag);
    if (rc) return rc;
    const unsigned grid = stream_grid(n, 256);
    FDX_PREP(k_zfill_reply, dim3(grid), as_stream(stream), reply_d, perm_d, n, n_windows, col0, F->mean_d,
             F->scale_d, (void *)z, flag);
    FDX_LAUNCHED("k_zfill_reply");
    return FDX_OK;
}

extern "C" int fdx_forest_clear_flag(fdx_forest F, int64_t n, void *ws, size_t ws_bytes, void *stream) {
    FDX_REQUIRE(F, "null forest");
    FDX_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return FDX_OK;
    float *z;
    double *acc;
    int32_t *flag;
    int rc = forest_ws(F, n, ws, ws_bytes, &z, &acc, &flag);
    if (rc) return rc;
    FDX_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), as_stream(stream)));
    return FDX_OK;
}

extern "C" int fdx_forest_prepare_grouped(fdx_forest F, int64_t n, int32_t n_windows, int32_t flags_mode,
                                          int32_t cust_val_is_sum, const int64_t *cust_ts_d, const double *cust_amount_d,
                                          const int32_t *cust_nb_d, const double *cust_avg_d,
                                          const int32_t *cust_perm_d, const int32_t *term_inv_d,
                                          const int64_t *term_rec_d, void *ws, size_t ws_bytes, void *stream) {
    return fdx_forest_prepare_grouped_rows(F, n, n_windows, flags_mode, cust_val_is_sum, cust_ts_d, cust_amount_d,
                                           cust_nb_d, cust_avg_d, cust_perm_d, term_inv_d, term_rec_d, nullptr, 0, 0,
                                           ws, ws_bytes, stream);
}

extern "C" int fdx_forest_prepare_grouped_rows(fdx_forest F, int64_t n, int32_t n_windows, int32_t flags_mode,
                                               int32_t cust_val_is_sum, const int64_t *cust_ts_d,
                                               const double *cust_amount_d, const int32_t *cust_nb_d,
                                               const double *cust_avg_d, const int32_t *cust_perm_d,
                                               const int32_t *term_inv_d, const int64_t *term_rec_d, void *rows_out_d,
                                               int64_t out_cap, int32_t rows_order, void *ws, size_t ws_bytes,
                                               void *stream) {
    FDX_REQUIRE(F, "null forest");
    FDX_REQUIRE(!rows_out_d || rows_order == FDX_ROWS_INPUT_ORDER || rows_order == FDX_ROWS_SLOT_ORDER,
                "rows_order must be FDX_ROWS_INPUT_ORDER or FDX_ROWS_SLOT_ORDER");
    FDX_REQUIRE(!rows_out_d || rows_order != FDX_ROWS_SLOT_ORDER || (out_cap >= n && out_cap % 64 == 0),
                "slot-order feature table: out_cap %lld must be >= n = %lld and a multiple of 64",
                (long long)out_cap, (long long)n);
    FDX_REQUIRE(!rows_out_d || ((uintptr_t)rows_out_d & 15) == 0, "feature output must be 16-byte aligned");
    FDX_REQUIRE(!(rank_mode(F) && v2_rows(kVariants[F->variant].p16)),
                "the fused scoring rows need the v1 row format (one slot per feature)");
    FDX_REQUIRE(n >= 0 && n_windows >= 1 && n_windows <= FDX_MAX_WINDOWS, "bad argument");
    FDX_REQUIRE(flags_mode == FDX_FLAGS_NOTEBOOK || flags_mode == FDX_FLAGS_SPARK, "bad flags mode");
    FDX_REQUIRE(F->n_features == 3 + 4 * n_windows, "forest has %d features, expected %d", F->n_features,
                3 + 4 * n_windows);
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(cust_ts_d && cust_amount_d && cust_nb_d && cust_avg_d && term_rec_d, "null pointer");
    FDX_REQUIRE((cust_val_is_sum & ~13) == 0,
                "cust_val_is_sum: FDX_PREP_VAL_IS_SUM | FDX_PREP_TERM_COMPACT | FDX_PREP_FLAG_CLEARED only");
    FDX_REQUIRE(!(cust_val_is_sum & 4) || (n_windows == 3 && ((uintptr_t)term_rec_d & 15) == 0),
                "compact terminal records: W = 3 and a 16-byte aligned record array");
    float *z;
    double *acc;
    int32_t *flag;
    int rc = forest_ws(F, n, ws, ws_bytes, &z, &acc, &flag);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    if (!(cust_val_is_sum & FDX_PREP_FLAG_CLEARED)) FDX_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), st));
    cust_val_is_sum &= ~FDX_PREP_FLAG_CLEARED;
    const unsigned grid = stream_grid(n, 256);
    const RankTab rt = rank_tab(F);
    if (rank_mode(F) && n_windows == 3 && rt.rat && rt.etab) {
#define FDX_ZFILL_W3(E, C, T)                                                                                     \
    hipLaunchKernelGGL((k_zfill_grouped_w3<E, C, T>), dim3(grid_w3), dim3(kW3Block), 0, st, cust_ts_d, cust_amount_d, \
                       cust_nb_d, cust_avg_d, cust_perm_d, term_inv_d, term_rec_d, n, flags_mode, cust_val_is_sum,   \
                       F->mean_d, F->scale_d, (void *)z, flag, rt, reinterpret_cast<char *>(rows_out_d), out_cap)
#define FDX_ZFILL_W3_E(E)                                                                                         \
    do {                                                                                                          \
        if (cust_val_is_sum & 4) {                                                                                \
            if (term_inv_d) FDX_ZFILL_W3(E, true, true); else FDX_ZFILL_W3(E, true, false);                       \
        } else {                                                                                                  \
            if (term_inv_d) FDX_ZFILL_W3(E, false, true); else FDX_ZFILL_W3(E, false, false);                     \
        }                                                                                                         \
    } while (0)
        const unsigned grid_w3 = stream_grid(n, kW3Block, device_cus());
        if (!rows_out_d)
            FDX_ZFILL_W3_E(0);
        else if (rows_order == FDX_ROWS_SLOT_ORDER)
            FDX_ZFILL_W3_E(FDX_ROWS_SLOT_ORDER);
        else
            FDX_ZFILL_W3_E(FDX_ROWS_INPUT_ORDER);
#undef FDX_ZFILL_W3_E
#undef FDX_ZFILL_W3
        FDX_LAUNCHED("k_zfill_grouped_w3");
        return FDX_OK;
    }
    // (the wide layout, or a forest whose searched features outgrow the S-trees' LDS budget)
    FDX_REQUIRE(!rows_out_d || n_windows == 3, "the featurized table has 3 windows (n_windows = %d)", n_windows);
    FDX_PREP(k_zfill_grouped, dim3(grid), st, cust_ts_d, cust_amount_d, cust_nb_d, cust_avg_d, cust_perm_d,
             term_inv_d, term_rec_d, n, n_windows, flags_mode, cust_val_is_sum, F->mean_d, F->scale_d, (void *)z, flag);
    FDX_LAUNCHED("k_zfill_grouped");
    if (rows_out_d) {
        char *feat = reinterpret_cast<char *>(rows_out_d);
        const int32_t vs = cust_val_is_sum & 1;
#define FDX_ROWS_K(E, C)                                                                                          \
    hipLaunchKernelGGL((k_feature_rows<E, C>), dim3(stream_grid(n, 256)), dim3(256), 0, st, cust_ts_d, cust_nb_d,  \
                       cust_avg_d, cust_perm_d, term_inv_d, term_rec_d, n, flags_mode, vs, feat, out_cap)
        const bool compact = (cust_val_is_sum & 4) != 0;
        if (rows_order == FDX_ROWS_SLOT_ORDER) {
            if (compact) FDX_ROWS_K(FDX_ROWS_SLOT_ORDER, true); else FDX_ROWS_K(FDX_ROWS_SLOT_ORDER, false);
        } else {
            if (compact) FDX_ROWS_K(FDX_ROWS_INPUT_ORDER, true); else FDX_ROWS_K(FDX_ROWS_INPUT_ORDER, false);
        }
#undef FDX_ROWS_K
        FDX_LAUNCHED("k_feature_rows");
    }
    return FDX_OK;
}
