// fdx_forest.hip -- K3: StandardScaler + tree-ensemble predict_proba on gfx950.
//
// Replaces loaded_scaler.transform + model.predict_proba(...)[:, 1]
// (pyspark/scripts/fraud_detection.py:190-193; shared_functions.py:304-333) for sklearn
// DecisionTreeClassifier / RandomForestClassifier (2 classes, 1 output).
//
// Exactness recipe (bit-identical to sklearn 1.6/1.7 Tree._apply_dense + forest
// accumulation):
//   z64 = (x - mean) / scale                (float64, StandardScaler.transform)
//   z32 = (float)z64                        (_validate_X_predict casts to float32, RNE)
//   go left  <=>  isnan(z32) ? missing_go_to_left : (double)z32 <= thr64
//           <=>  isnan(z32) ? missing_go_to_left : z32 <= thr32_down
//   where thr32_down is the largest float <= thr64 (round toward -inf at load time)
//   proba = (((0 + v_t0) + v_t1) + ...) / n_trees  in float64, trees in index order.
//
// Node format (8 bytes, trees re-laid out in pre-order so the left child is p+1):
//   internal: hi = 0x80000000 | missing_left<<30 | feature<<24 | 8*(right - p)   lo = thr32_down
//   leaf    : the float64 class-1 value itself (sign bit 0, so hi bit 31 = 0)
// A leaf is a fixed point of the step (its step is masked to 0 by the sign of hi), so every
// walk runs exactly depth(tree group) steps with no per-step leaf test.
//
// Kernel structure: trees are cut into chunks that fit the LDS budget; one launch per
// chunk streams every row once: the block stages the chunk's nodes into LDS, each thread
// stages its row's 16 scaled features into its own LDS column and walks G trees at once
// (G independent dependency chains per lane hide the LDS latency).  The running float64
// sum of a row crosses chunk launches through a workspace vector, preserving tree order.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <new>
#include <type_traits>
#include <vector>

#include "fdx_internal.h"

struct fdx_forest_s {
    int32_t n_trees = 0, n_features = 0, zstride = 16;
    int64_t n_nodes = 0;
    uint64_t *nodes_d = nullptr;   // packed nodes, all trees
    int32_t *orig_d = nullptr;     // sklearn node id of each packed node
    int32_t *root_d = nullptr;     // packed position of each tree root
    int32_t *depth_d = nullptr;    // max leaf depth of each tree (steps to reach any leaf)
    double *mean_d = nullptr, *scale_d = nullptr;
    struct Chunk {
        int32_t t0, t1;
        int64_t node_base, nodes;
        bool in_lds;
    };
    std::vector<Chunk> chunks;
    int32_t *chunk_t_d = nullptr;     // [n_trees+1] first tree of each chunk (all-chunks-at-once launch)
    int64_t *chunk_base_d = nullptr;  // [n_trees+1] first node of each chunk
    int variant = 0;        // index into kVariants
    std::vector<int64_t> node_offsets;  // host copy (chunking)
    // rank layout (4-byte nodes over per-feature threshold ranks, see "Rank layout" below)
    bool rank_ok = false;
    std::vector<int64_t> rank_offsets;  // [n_trees+1] first rank-layout node of each tree
    int64_t rank_nodes = 0;
    uint32_t *rnodes_d = nullptr;
    int32_t *rorig_d = nullptr, *rroot_d = nullptr, *rdepth_d = nullptr;
    double *rlval_d = nullptr;
    uint8_t *rml_d = nullptr;
    float *rthr_d = nullptr;
    int32_t rthr_off[32] = {}, rthr_cnt[32] = {};
    float *rseg_d = nullptr, *rsmp_d = nullptr;  // two-level rank search tables
    uint16_t *ritab_d = nullptr;                  // [16][kIntTab] ranks of small integer values
    uint16_t *rrat_d = nullptr;                   // [16][kRatN][kRatN] ranks of small ratios fr / nb
    float *retab_d = nullptr;                     // Eytzinger sample tables (RankTab::etab)
    int32_t reoff[4] = {}, relev[4] = {}, rnetab = 0;
    int32_t ruoff[32] = {}, rsoff[32] = {}, rscnt[32] = {}, rseg = 16, rnsmp = 0;
    // rank layout v2 (32 threshold-rank slots, see build_rank_layout)
    bool rank_v2 = false;
    bool rank_identity = false;  // v2 with slot s = feature s (<= 16 slots): v1 rank rows, compact planes
    // host copies of the packed forest and scaler (set_variant rebuilds the rank layout in the
    // other node format when a variant needs it)
    std::vector<uint64_t> h_packed;
    std::vector<int32_t> h_orig, h_depth;
    std::vector<double> h_mean, h_scale;
    int32_t rn_slots = 0, rslot_feat[32] = {}, rslot_base[32] = {};
    int32_t n_cu = 256;  // compute units of the forest's device: one rank-kernel block per CU
};

namespace fdx {
namespace {

constexpr uint32_t kInternal = 0x80000000u;

__device__ __forceinline__ double leaf_value(uint64_t nd) { return __longlong_as_double((long long)nd); }

// ---------------------------------------------------------------------- rank layout
// The traversal is VALU-issue bound (r01 PMC: ~0.85 VALU wave-instructions / clk / CU in
// k_forest_chunk), so the default layout is the one with the fewest instructions per step.
// Per feature f, U_f = sorted unique float32 thresholds (thr32_down) of the forest.  A row
// value x is replaced by its rank r_f(x) = #{u in U_f : u < x} (lower_bound), and a node
// with threshold U_f[k] by k:  x <= U_f[k]  <=>  r_f(x) <= k  (exact, U_f sorted unique).
// 4-byte node:  [31] 0  [30:16] k  [15:12] feature  [11:0] right offset (left child = p+1)
// Row values in LDS are x = r << 16 in a [16][1024] u32 plane array at LDS offset 0, so
//   feature address = (node & 0xF000) | lane_base                 (v_and_or_b32)
//   d = x - node (as int32; both < 2^31):  d <= 0 iff r <= k (go left); when r > k,
//       d >= 65536 - (node & 0xFFFF) > 4095 >= right offset   (features 0..14)
//   step = med3(d, 1, node & 0xFFF)   -> 1 (left) or the right offset
//   next address = addr + 4 * step                             (sub, and, med3, lshl_add)
// Feature slot 15 holds the sentinel 0x4000 << 16 for every row: a LEAF (0x7FFFF000) has
// d < 0 and right offset 0, so med3 = 0 (fixed point); a JUMP node (0x0000F000 | j) has
// d > 4095, so med3 = j: it forwards to p + j (the packer inserts jumps after leaves wherever
// a right offset would exceed 4095).  No lane-mask instruction, so no VCC hazard stalls.
// Leaf values (float64) and sklearn node ids live in global arrays indexed by rank-layout
// position; NaN row values are 0xFFFF (u16) / 0xFFFFFFFF (LDS), resolved by
// missing_go_to_left from a global byte array in the NaN-aware walk.  Ranks travel through
// HBM as 16 x u16 = 32 B per row (half the float32 row).
constexpr uint32_t kRankLeaf = 0x7FFFF000u;
constexpr uint32_t kRankJump = 0x0000F000u;
constexpr uint32_t kRankSentinel = 0x4000u << 16;
constexpr int kRankMaxOffset = 4095;
constexpr int kRankMaxRank = 32766;  // rank values stay <= 0x7FFF so x < 2^31
constexpr int kRankPlaneRows = 1024;
constexpr int kRankXWords = 16 * kRankPlaneRows;  // 64 KiB of row planes

struct RankTab {
    const float *u;  // concatenated U_f
    int32_t off[32], cnt[32];
    // two-level search tables (rank_row): U_f padded with +inf to whole segments of `seg`
    // floats at 16-float-aligned offsets (useg + uoff[f]), and the first float of every
    // segment (smp + soff[f], scnt[f] segments) -- staged into LDS by the prepare kernels
    const float *useg, *smp;
    int32_t uoff[32], soff[32], scnt[32];
    int32_t seg, n_smp;
    // rank layout v2: slot s holds min(max(rank(feature slot_feat[s]) - slot_base[s], 0), 32767)
    int32_t n_slots, slot_feat[32], slot_base[32];
    // itab[f * kIntTab + c] = rank of the scaled integer c (c < kIntTab) in feature f: the
    // flags and window counts are small integers, so the prepare looks their ranks up
    const uint16_t *itab;
    // rat[(f * kRatN + nb) * kRatN + fr] = rank of the scaled ratio fr / nb (0 when nb == 0,
    // the reference's fillna(0)) for nb < kRatN: the terminal risks are such ratios
    const uint16_t *rat;
    // Eytzinger form of the segment samples of the reference layout's searched features
    // (kW3Search: amount + the three averages), for k_zfill_grouped_w3: feature kW3Search[s]'s
    // samples padded with +inf to 2^elev[s] - 1 entries, BFS order, entry k (1-based) at
    // etab[eoff[s] + k].  A lane's descent reads level d from a window of 2^d consecutive words,
    // so the first levels are bank-conflict free (the sorted table's binary search puts every
    // probe of a level on one bank: stride n / 2^d).  NULL when the tables exceed the LDS budget.
    const float *etab;
    int32_t eoff[4], elev[4], n_etab;
};
constexpr int kW3Search[4] = {0, 4, 6, 8};  // TX_AMOUNT, CUSTOMER_ID_AVG_AMOUNT_{1,7,30}DAY_WINDOW
constexpr int kMaxRankSamples = 8192;  // LDS sample table of the prepare kernels (32 KiB)
constexpr int kIntTab = 256;           // integer rank table entries per feature (8 KiB in LDS)
constexpr int kRatN = 128;             // ratio rank table: nb, fr < kRatN (32 KiB per feature, global)

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
                for (int q = 0; q < rt.seg / 4; ++q) {
                    const float4 w = sg[q];
                    k += (uint32_t)(w.x < v[f]) + (uint32_t)(w.y < v[f]) + (uint32_t)(w.z < v[f]) +
                         (uint32_t)(w.w < v[f]);
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

// ranks of the features in `need` by a full lower_bound over U_f in global memory (the rare
// fallback of k_zfill_grouped_w3: values outside its integer / ratio rank tables)
__device__ __forceinline__ void rank_row_global(const float (&v)[16], const RankTab &rt, uint32_t (&out)[16],
                                             uint32_t need) {
#pragma unroll
    for (int f = 0; f < 16; ++f)
        if ((need >> f) & 1u) out[f] = rank_of(v[f], rt.u + rt.off[f], rt.cnt[f]);
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

// rank of v in feature f (lower_bound over U_f), two-level search as rank_row, one feature
__device__ __forceinline__ uint32_t rank_one(float v, int f, const RankTab &rt, const float *s_smp) {
    int32_t lo = rt.soff[f], n = rt.scnt[f];
    if (n <= 0) return 0u;
    while (n > 1) {
        const int32_t h = n >> 1;
        lo = (s_smp[lo + h] < v) ? lo + h : lo;
        n -= h;
    }
    const int32_t c = lo - rt.soff[f] + (s_smp[lo] < v ? 1 : 0);
    if (c <= 0) return 0u;
    const float4 *sg = reinterpret_cast<const float4 *>(rt.useg + rt.uoff[f] + (int64_t)(c - 1) * rt.seg);
    uint32_t k = 0;
    for (int q = 0; q < rt.seg / 4; ++q) {
        const float4 w = sg[q];
        k += (uint32_t)(w.x < v) + (uint32_t)(w.y < v) + (uint32_t)(w.z < v) + (uint32_t)(w.w < v);
    }
    return (uint32_t)(c - 1) * (uint32_t)rt.seg + k;
}

// Rank layout v2 rows: 32 u16 slots per row (64 B), slot s = the clamped rank of its
// feature (build_rank_layout), 0xFFFF for a NaN feature; unused slots 0.
__global__ void __launch_bounds__(256) k_prepare_v2(const double *__restrict__ X, int64_t n, int64_t rs, int64_t cs,
                                                    int32_t nf, const double *__restrict__ mean,
                                                    const double *__restrict__ scale, uint16_t *__restrict__ z,
                                                    int32_t *__restrict__ nan_flag, RankTab rt) {
    __shared__ float s_smp[kMaxRankSamples];
    __shared__ __align__(16) uint16_t s_row[256][32];
    stage_samples(s_smp, rt);
    uint16_t *mine = s_row[threadIdx.x];
    for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = r0 + threadIdx.x;
        if (r < n) {
            bool any_nan = false;
            for (int s = 0; s < 32; ++s) mine[s] = 0;
            for (int f = 0; f < nf; ++f) {
                double x = X[r * rs + (int64_t)f * cs];
                if (mean) x = x - mean[f];
                if (scale) x = x / scale[f];
                const float v = (float)x;
                const bool isn = v != v;
                any_nan |= isn;
                const uint32_t rk = isn ? 0u : rank_one(v, f, rt, s_smp);
                for (int s = 0; s < rt.n_slots; ++s) {
                    if (rt.slot_feat[s] != f) continue;
                    const int64_t c = (int64_t)rk - rt.slot_base[s];
                    mine[s] = isn ? (uint16_t)0xFFFFu : (uint16_t)(c < 0 ? 0 : (c > 32767 ? 32767 : c));
                }
            }
            if (any_nan) *nan_flag = 1;
            const uint4 *src = reinterpret_cast<const uint4 *>(mine);
            uint4 *dst = reinterpret_cast<uint4 *>(z + r * 32);
#pragma unroll
            for (int q = 0; q < 4; ++q) dst[q] = src[q];
        }
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
    constexpr int64_t kDay = 86400LL * 1000000000LL, kHour = 3600LL * 1000000000LL;
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
        const int64_t t = cts[i];
        int64_t day = t / kDay;
        if (t % kDay != 0 && t < 0) --day;
        const int64_t hour = (t - day * kDay) / kHour;
        int64_t wd = (day + 3) % 7;
        if (wd < 0) wd += 7;
        const bool we = flags_mode == FDX_FLAGS_NOTEBOOK ? wd >= 5 : (((wd + 1) % 7) + 1) >= 5;
        const bool ni = flags_mode == FDX_FLAGS_NOTEBOOK ? hour <= 6 : hour >= 20;
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

// k_zfill_grouped for the reference's layout (W = 3, rank rows, ratio table, 16-float search
// segments), restructured for memory-level parallelism.  The general kernel is bound by
// dependent round trips per row at 3 waves/SIMD (cust_perm -> term record -> ratio table;
// amount/average -> one search segment per feature, each behind its own branch).  Here the
// next row's loads (scoring-order columns + its term record, whose row index is fetched two
// rows ahead) are in flight while the current row is ranked, and the current row's four
// segment reads and three ratio-table reads are issued together, unconditionally (clamped
// addresses; the host pads useg by one segment), so a row costs about one round trip.
// Results are bit-identical to k_zfill_grouped<16, true> (same arithmetic, same fallbacks).
// A/B switch (compile time): k_zfill_grouped_w3's segment counts by lane quads (1) or per lane (0)
#ifndef FDX_ZFILL_QUAD
#define FDX_ZFILL_QUAD 1
#endif
constexpr bool kZfillQuad = FDX_ZFILL_QUAD != 0;

// lane K of each quad of lanes, to all 4 (DPP quad_perm broadcast; every lane of the wave active)
template <int K>
__device__ __forceinline__ int32_t quad_bcast(int32_t x) {
    return __builtin_amdgcn_update_dpp(0, x, K * 0x55, 0xF, 0xF, false);
}
// the sum over each quad of lanes, in all 4 (DPP quad_perm [1,0,3,2] then [2,3,0,1])
__device__ __forceinline__ uint32_t quad_sum(uint32_t c) {
    c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)c, 0xB1, 0xF, 0xF, false);
    c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)c, 0x4E, 0xF, 0xF, false);
    return c;
}

struct PrepRow {
    int64_t t;
    double a;
    int32_t c[3];
    double cv[3];
    int64_t tw[3];
    int32_t r;
};

// A/B switch (compile time): minimum waves per SIMD the compiler must fit k_zfill_grouped_w3's
// registers to (0: the compiler's choice, 156 VGPRs / 3 waves; 4: 128 VGPRs, assembly 1.02-1.09 -> 0.985 ms
// alone, profiles/r03af_zfill_waves_ab.txt)
#ifndef FDX_ZFILL_WAVES
#define FDX_ZFILL_WAVES 4
#endif
// EMIT: the featurized table besides the rank rows (fdx_forest_prepare_grouped_rows): 0 = none,
// FDX_ROWS_INPUT_ORDER / FDX_ROWS_SLOT_ORDER = the fdx_feature_row record of each slot's row at its
// input row / at its slot, stored as soon as the row's values are loaded (the record's registers
// die before the rank search; kept to the end, 15 VGPRs spilled)
template <int EMIT>
__global__ void __launch_bounds__(256, FDX_ZFILL_WAVES) k_zfill_grouped_w3(
    const int64_t *__restrict__ cts, const double *__restrict__ camt, const int32_t *__restrict__ cnb,
    const double *__restrict__ cval, const int32_t *__restrict__ cust_perm, const int32_t *__restrict__ term_inv,
    const int64_t *__restrict__ term_rec, int64_t n, int32_t flags_mode, int32_t val_is_sum,
    const double *__restrict__ mean, const double *__restrict__ scale, void *__restrict__ z,
    int32_t *__restrict__ nan_flag, RankTab rt, char *__restrict__ feat, int64_t fcap) {
    constexpr int64_t kDay = 86400LL * 1000000000LL, kHour = 3600LL * 1000000000LL;
    constexpr int W = 3, nf = 15;
    static_assert(sizeof(fdx_feature_row) == 80, "5 x 16-byte stores per feature record");
    __shared__ float s_e[kMaxRankSamples];  // Eytzinger sample tables (RankTab::etab)
    __shared__ uint16_t s_itab[16 * kIntTab];
    for (int e = threadIdx.x; e < 16 * kIntTab; e += blockDim.x) s_itab[e] = rt.itab[e];
    for (int e = threadIdx.x; e < rt.n_etab; e += blockDim.x) s_e[e] = rt.etab[e];
    __syncthreads();
    const int e_lmax = max(max(rt.elev[0], rt.elev[1]), max(rt.elev[2], rt.elev[3]));
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const bool rec16 = ((uintptr_t)term_rec & 15) == 0;  // uniform
    auto row_of = [&](int64_t j) -> int32_t { return j < n ? (cust_perm ? cust_perm[j] : (int32_t)j) : -1; };
    auto load = [&](int64_t j, int32_t r, PrepRow &L) {
        L.r = r;
        if (j >= n || r < 0) {  // defined values: every lane runs the row arithmetic (quad rounds)
            L.t = 0;
            L.a = 0.0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                L.c[w] = 1;
                L.cv[w] = 0.0;
                L.tw[w] = 0;
            }
            return;
        }
        L.t = cts[j];
        L.a = camt[j];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            L.c[w] = cnb[(int64_t)w * n + j];
            L.cv[w] = cval[(int64_t)w * n + j];
        }
        const int64_t q_ = term_inv ? term_inv[r] : r;
        const int64_t *src = term_rec + q_ * W;
        if (val_is_sum & 4) {
            compact_load(term_rec, q_, L.tw);
        } else if (rec16) {  // the 24-byte record in two loads (16-byte aligned pair first or second)
            if ((q_ & 1) == 0) {
                const longlong2 p = *reinterpret_cast<const longlong2 *>(src);
                L.tw[0] = p.x;
                L.tw[1] = p.y;
                L.tw[2] = src[2];
            } else {
                const longlong2 p = *reinterpret_cast<const longlong2 *>(src + 1);
                L.tw[0] = src[0];
                L.tw[1] = p.x;
                L.tw[2] = p.y;
            }
        } else {
#pragma unroll
            for (int w = 0; w < W; ++w) L.tw[w] = src[w];
        }
    };
    // wave-uniform loop (stride and the wave's first slot are multiples of 64): every lane of a
    // wave runs each iteration, so the quads of k_seg_count_quad stay whole; lanes past n and
    // padding slots compute on defined dummies and store the zero row / nothing
    const int lane = threadIdx.x & (kWave - 1);
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    PrepRow cur;
    load(i, row_of(i), cur);
    int32_t r_next = row_of(i + stride);
    for (; i - lane < n; i += stride) {
        PrepRow nxt;
        load(i + stride, r_next, nxt);  // next row's loads in flight during this row
        r_next = row_of(i + 2 * stride);
        const bool live = i < n && cur.r >= 0;
        const int64_t t = cur.t;
        int64_t day = t / kDay;
        if (t % kDay != 0 && t < 0) --day;
        const int64_t hour = (t - day * kDay) / kHour;
        int64_t wd = (day + 3) % 7;
        if (wd < 0) wd += 7;
        const bool we = flags_mode == FDX_FLAGS_NOTEBOOK ? wd >= 5 : (((wd + 1) % 7) + 1) >= 5;
        const bool ni = flags_mode == FDX_FLAGS_NOTEBOOK ? hour <= 6 : hour >= 20;
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
                v[f] = zval((double)c, mean, scale, f);
                need |= 1u << f;
            }
        };
        q[1] = s_itab[1 * kIntTab + (we ? 1 : 0)];
        q[2] = s_itab[2 * kIntTab + (ni ? 1 : 0)];
        v[0] = zval(cur.a, mean, scale, 0);
        bool nan = v[0] != v[0];
        if constexpr (EMIT != 0) {
            // the featurized row: a record at its input row (one random 80-byte write), or the
            // columns at its slot (consecutive lanes, consecutive elements: every store of a wave
            // is whole lines; an 80-byte record per slot, 5 strided 16-byte stores, measured
            // +0.62 ms at config 2; padding slots: row -1, zero features)
            if (i < n && (EMIT == FDX_ROWS_SLOT_ORDER || (live && (uint64_t)cur.r < (uint64_t)fcap))) {
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
                        reinterpret_cast<uint32_t *>(feat + FDX_FEATURE_COL(w, fcap))[i] = c[w];
                        reinterpret_cast<uint32_t *>(feat + FDX_FEATURE_COL(3 + w, fcap))[i] = tn[w];
                        reinterpret_cast<double *>(feat + FDX_FEATURE_COL(6 + w, fcap))[i] = avg[w];
                        reinterpret_cast<double *>(feat + FDX_FEATURE_COL(9 + w, fcap))[i] = rk[w];
                    }
                    reinterpret_cast<int32_t *>(feat + FDX_FEATURE_COL(12, fcap))[i] = live ? cur.r : -1;
                    reinterpret_cast<uint16_t *>(feat + FDX_FEATURE_COL(13, fcap))[i] = (uint16_t)fl;
                } else {
                    uint4 *dst = reinterpret_cast<uint4 *>(feat) + (int64_t)cur.r * 5;
                    dst[0] = make_uint4(c[0], c[1], c[2], tn[0]);
                    dst[1] = make_uint4(tn[1], tn[2], u32(avg[0], 0), u32(avg[0], 1));
                    dst[2] = make_uint4(u32(avg[1], 0), u32(avg[1], 1), u32(avg[2], 0), u32(avg[2], 1));
                    dst[3] = make_uint4(u32(rk[0], 0), u32(rk[0], 1), u32(rk[1], 0), u32(rk[1], 1));
                    dst[4] = make_uint4(u32(rk[2], 0), u32(rk[2], 1), fl, (uint32_t)cur.r);
                }
            }
        }
        uint16_t rq[W];
        bool rat_ok[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int32_t c = cur.c[w];
            count(3 + 2 * w, c);
            v[4 + 2 * w] = zval((val_is_sum & 1) ? cur.cv[w] / (double)c : cur.cv[w], mean, scale, 4 + 2 * w);
            nan |= v[4 + 2 * w] != v[4 + 2 * w];
            const int64_t tw = cur.tw[w];
            const int32_t tnb = term_nb(tw), tfr = (int32_t)((uint64_t)tw >> 32);
            count(3 + 2 * W + 2 * w, tnb);
            const int fr_ = 4 + 2 * W + 2 * w;
            rat_ok[w] = tnb >= 0 && tnb < kRatN && tfr >= 0 && tfr <= tnb;
            // unconditional read (index clamped to 0 when the table does not apply)
            rq[w] = rt.rat[rat_ok[w] ? ((int64_t)fr_ * kRatN + tnb) * kRatN + tfr : 0];
        }
        // two-level search of the 4 continuous features: the Eytzinger descent over the LDS
        // samples (cs = #samples < v: k - 2^L after L levels), then all 4 segments at once
        int32_t ek[4] = {1, 1, 1, 1};
        for (int l = 0; l < e_lmax; ++l) {  // uniform trip count
#pragma unroll
            for (int s = 0; s < 4; ++s)
                if (l < rt.elev[s]) ek[s] = 2 * ek[s] + (s_e[rt.eoff[s] + ek[s]] < v[kW3Search[s]] ? 1 : 0);
        }
        int32_t cs[4];
        uint32_t kc[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) cs[s] = ek[s] - (1 << rt.elev[s]);
        if constexpr (kZfillQuad) {
            // a quad of lanes per segment: round K loads lane K's 64-byte segment as 4 x 16 B
            // (lane j of the quad: bytes 16j..16j+15), so each load instruction touches 16 lines
            // instead of 64 -- the address unit serves a gather line by line -- and the quad sums
            // its 4 partial counts (DPP); lane K keeps round K's count
            const int qj = lane & 3;
            int32_t sidx[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) sidx[s] = max(cs[s] - 1, 0);
            auto round = [&](auto kk) {
                constexpr int K = decltype(kk)::value;
                float4 w4[4];
                float vk[4];
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int f = kW3Search[s];
                    const int32_t si = quad_bcast<K>(sidx[s]);
                    vk[s] = __int_as_float(quad_bcast<K>(__float_as_int(v[f])));
                    w4[s] = reinterpret_cast<const float4 *>(rt.useg + rt.uoff[f] + (int64_t)si * 16)[qj];
                }
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    uint32_t c = (uint32_t)(w4[s].x < vk[s]) + (uint32_t)(w4[s].y < vk[s]) +
                                 (uint32_t)(w4[s].z < vk[s]) + (uint32_t)(w4[s].w < vk[s]);
                    c = quad_sum(c);
                    kc[s] = qj == K ? c : kc[s];
                }
            };
            round(std::integral_constant<int, 0>{});
            round(std::integral_constant<int, 1>{});
            round(std::integral_constant<int, 2>{});
            round(std::integral_constant<int, 3>{});
        } else {
            float4 sg[4][4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int f = kW3Search[s];
                const float4 *p = reinterpret_cast<const float4 *>(rt.useg + rt.uoff[f] + (int64_t)max(cs[s] - 1, 0) * 16);
#pragma unroll
                for (int k = 0; k < 4; ++k) sg[s][k] = p[k];
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int f = kW3Search[s];
                uint32_t k = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    k += (uint32_t)(sg[s][e].x < v[f]) + (uint32_t)(sg[s][e].y < v[f]) +
                         (uint32_t)(sg[s][e].z < v[f]) + (uint32_t)(sg[s][e].w < v[f]);
                kc[s] = k;
            }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int f = kW3Search[s];
            const uint32_t r = cs[s] > 0 ? (uint32_t)(cs[s] - 1) * 16u + kc[s] : 0u;
            q[f] = v[f] != v[f] ? 0xFFFFu : r;
        }
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int fr_ = 4 + 2 * W + 2 * w;
            if (rat_ok[w]) {
                q[fr_] = rq[w];
            } else {
                v[fr_] = zval(term_risk(cur.tw[w]), mean, scale, fr_);
                need |= 1u << fr_;
                nan |= v[fr_] != v[fr_];
            }
        }
        if (live && nan) *nan_flag = 1;
        need &= (1u << nf) - 1u;
        if (live && need) rank_row_global(v, rt, q, need);  // table overflows (rare): full lower_bound in HBM
        q[15] = 0u;
        if (i < n) {  // padding slot of the interleaved layout: the zero row
            uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<uint16_t *>(z) + i * 16);
            dst[0] = live ? make_uint4(q[0] | q[1] << 16, q[2] | q[3] << 16, q[4] | q[5] << 16, q[6] | q[7] << 16)
                          : make_uint4(0, 0, 0, 0);
            dst[1] = live ? make_uint4(q[8] | q[9] << 16, q[10] | q[11] << 16, q[12] | q[13] << 16, q[14] | q[15] << 16)
                          : make_uint4(0, 0, 0, 0);
        }
        cur = nxt;
    }
}

template <bool LDS>
__device__ __forceinline__ uint64_t node_at(const uint64_t *s_nodes, const char *gbase, uint32_t byte_off) {
    if (LDS) return *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(s_nodes) + byte_off);
    return *reinterpret_cast<const uint64_t *>(gbase + byte_off);
}

// Kernel variants.  rank = 0: k_forest_chunk over the wide layout (float32 rows, 8-byte
// nodes) -- forests the rank layout cannot hold or with more than 15 features; rank = 1:
// k_forest_rank over the rank layout (4-byte nodes, u16 rank rows), block size BLOCK, one row
// per lane, G trees walked at once per lane (G independent LDS dependency chains), the
// software-pipelined walk with waits grouped by PIPE chains.  p16 = the rank node / plane
// format: 0 = v1 (u32 planes), 2 = v2 (32 threshold slots over u16 planes), 3 = v2 nodes over
// 16 u16 planes (forests whose every feature fits one slot).
struct Variant {
    int block, rows, group, rank, p16, pipe;
};
constexpr Variant kVariants[] = {
    {512, 1, 4, 0, 0, 0},    // 0: wide layout
    {1024, 1, 10, 1, 0, 2},  // 1: rank layout v1, 10 chains per lane (the default: r03 sweep, 7.63 vs
                             //    8.43 ms for 6 chains at config 2; 12 chains spill, 11.7 ms)
    {1024, 1, 6, 1, 2, 2},   // 2: rank layout v2 (forests v1 cannot hold: the deployed model)
    {1024, 1, 6, 1, 3, 2},   // 3: v2 nodes over 16 u16 planes (a third more nodes per LDS chunk)
    {1024, 1, 10, 1, 2, 2},  // 4: v2, 10 chains
    {1024, 1, 8, 1, 3, 2},   // 5: compact v2, 8 chains
    {1024, 1, 10, 1, 3, 2},  // 6: compact v2, 10 chains
};
// (Round 3 also measured v1 with 6 / 8 / 9 chains, compact v2 with 10 chains and register
// ranks -- the lane's rank row in 8 VGPRs, one ds_read per step: 16.3 vs 7.6 ms -- and removed
// them; DESIGN.md §4 keeps their numbers.)
constexpr int kDefaultRankVariant = 1;
constexpr int kDefaultRankV2Variant = 2;
constexpr int kDefaultRankCompactVariant = 3;
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
constexpr int kLdsTotal = 160 * 1024 - 2048;  // leave room for the static bookkeeping

constexpr int lds_node_bytes(int fs, int block, int rows) { return kLdsTotal - fs * block * rows * 4; }

// One launch = one chunk of trees [t0, t1) over rows [r0, r1).  Each lane walks G trees
// for each of its R rows at once (R*G independent chains).  A step is branch-free (leaves
// are fixed points); all feature reads of a step are issued together, then all node reads,
// so a lane keeps R*G LDS reads in flight; a walk group runs at most max(depth) steps and
// stops as soon as every chain of the wave is at a leaf (the loop is uniform across the
// wave).  NaN routing (missing_go_to_left) costs 3 extra VALU per step: it is compiled in
// a second loop that runs only when the prepare step saw a NaN feature (*nan_flag != 0).
template <bool NAN_AWARE, bool LDS, int XSTRIDE, int K>
__device__ __forceinline__ void walk_step(const uint64_t *s_nodes, const char *gbase, const float *const (&xcol)[K],
                                          uint32_t (&p)[K], uint64_t (&nd)[K]) {
    float x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t hi = (uint32_t)(nd[k] >> 32);
        x[k] = xcol[k][((hi >> 24) & 63u) * XSTRIDE];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t hi = (uint32_t)(nd[k] >> 32);
        bool left = x[k] <= __uint_as_float((uint32_t)nd[k]);
        if (NAN_AWARE) left = left | ((x[k] != x[k]) & ((hi >> 30) & 1u));
        const uint32_t step = left ? 8u : (hi & 0xFFFFFFu);
        p[k] += step & (uint32_t)((int32_t)hi >> 31);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) nd[k] = node_at<LDS>(s_nodes, gbase, p[k]);
}

// Walks every chain to its leaf: at most `depth` steps, in blocks of kExitEvery steps with a
// wave-uniform exit test between blocks (all chains of the wave at leaves).  In-distribution
// rows of the bench forest end at ~5 nodes (depth 20), far-out rows run all 20 steps; testing
// every kExitEvery steps keeps the test's cost small in the second case.
#ifndef FDX_EXIT_EVERY
#define FDX_EXIT_EVERY 4
#endif
constexpr int kExitEvery = FDX_EXIT_EVERY;
template <bool NAN_AWARE, bool LDS, int XSTRIDE, int K>
__device__ __forceinline__ void walk_group(const uint64_t *s_nodes, const char *gbase, const float *const (&xcol)[K],
                                           uint32_t (&p)[K], uint64_t (&nd)[K], int depth) {
    int d = 0;
    for (; d + kExitEvery <= depth; d += kExitEvery) {
#pragma unroll
        for (int e = 0; e < kExitEvery; ++e) walk_step<NAN_AWARE, LDS, XSTRIDE, K>(s_nodes, gbase, xcol, p, nd);
        uint32_t internal = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) internal |= (uint32_t)(nd[k] >> 32);
        if (!__any((int32_t)internal < 0)) return;
    }
    for (; d < depth; ++d) walk_step<NAN_AWARE, LDS, XSTRIDE, K>(s_nodes, gbase, xcol, p, nd);
}

template <int FS, bool LDS, int BLOCK, int R, int G>
__global__ void __launch_bounds__(BLOCK) k_forest_chunk(
    const uint64_t *__restrict__ nodes, int64_t node_base, int32_t chunk_nodes,
    const int32_t *__restrict__ root, const int32_t *__restrict__ depth, int32_t t0, int32_t t1,
    const float *__restrict__ z, const int32_t *__restrict__ nan_flag, int64_t r0, int64_t r1,
    double *__restrict__ acc, double *__restrict__ proba, const int32_t *__restrict__ out_perm,
    int32_t *__restrict__ leaf_out, const int32_t *__restrict__ orig, int32_t n_trees, int first, int last) {
    constexpr int kNodeCap = LDS ? lds_node_bytes(FS, BLOCK, R) / 8 : 1;
    constexpr int K = R * G;
    constexpr int kRowsPerBlock = BLOCK * R;
    __shared__ uint64_t s_nodes[kNodeCap];
    __shared__ float s_x[FS][kRowsPerBlock];
    const int tid = threadIdx.x;
    const uint64_t *nb = nodes + node_base;
    const char *gbase = reinterpret_cast<const char *>(nb);
    const bool any_nan = *nan_flag != 0;  // uniform
    if (LDS) {
        for (int i = tid; i < chunk_nodes; i += BLOCK) s_nodes[i] = nb[i];
        __syncthreads();
    }
    // walk k = r*G + g reads the features of row slot r
    const float *xcol[K];
#pragma unroll
    for (int k = 0; k < K; ++k) xcol[k] = &s_x[0][(k / G) * BLOCK + tid];
    for (int64_t base = r0 + (int64_t)blockIdx.x * kRowsPerBlock; base < r1;
         base += (int64_t)gridDim.x * kRowsPerBlock) {
        int64_t row[R];
        bool ok[R];
        double a[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            row[r] = base + r * BLOCK + tid;
            ok[r] = row[r] < r1;
            const float4 *src = reinterpret_cast<const float4 *>(z + (ok[r] ? row[r] : r0) * FS);
#pragma unroll
            for (int q = 0; q < FS / 4; ++q) {
                float4 v = src[q];
                s_x[4 * q + 0][r * BLOCK + tid] = v.x;
                s_x[4 * q + 1][r * BLOCK + tid] = v.y;
                s_x[4 * q + 2][r * BLOCK + tid] = v.z;
                s_x[4 * q + 3][r * BLOCK + tid] = v.w;
            }
            a[r] = (first || !ok[r]) ? 0.0 : acc[row[r]];
        }
        for (int t = t0; t < t1; t += G) {
            uint32_t p[K];
            uint64_t nd[K];
            int dmax = 0;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const bool act = t + g < t1;
                const uint32_t p0 = act ? (uint32_t)(root[t + g] - node_base) * 8u : 0u;
                const uint64_t n0 = act ? node_at<LDS>(s_nodes, gbase, p0) : 0ull;  // inactive: leaf-like 0
                dmax = act ? max(dmax, depth[t + g]) : dmax;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    p[r * G + g] = p0;
                    nd[r * G + g] = n0;
                }
            }
            if (any_nan)
                walk_group<true, LDS, kRowsPerBlock, K>(s_nodes, gbase, xcol, p, nd, dmax);
            else
                walk_group<false, LDS, kRowsPerBlock, K>(s_nodes, gbase, xcol, p, nd, dmax);
#pragma unroll
            for (int r = 0; r < R; ++r) {
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    if (t + g < t1) {
                        a[r] += leaf_value(nd[r * G + g]);
                        if (leaf_out && ok[r]) {
                            const int64_t dst = out_perm ? (int64_t)out_perm[row[r]] : row[r];
                            if (dst >= 0) leaf_out[dst * n_trees + t + g] = orig[node_base + (p[r * G + g] >> 3)];
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!ok[r]) continue;
            if (last) {
                const int64_t dst = out_perm ? (int64_t)out_perm[row[r]] : row[r];
                if (dst >= 0) proba[dst] = a[r] / (double)n_trees;  // < 0: padding slot
            } else {
                acc[row[r]] = a[r];
            }
        }
    }
}

// Rank-layout walk step (see "Rank layout"): 5 VALU + 2 LDS reads per chain.  pa = LDS byte
// address of the chain's node, nd = that node.
constexpr uint32_t kRankNodeB = kRankXWords * 4;  // byte offset of the node region in LDS

__device__ __forceinline__ uint32_t lds32(const char *lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(lds + byte_addr);
}
__device__ __forceinline__ uint32_t lds16(const char *lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint16_t *>(lds + byte_addr);
}
// P16: row planes hold the raw u16 ranks (NaN = 0xFFFF) and the LDS copy of every node is
// S = node ^ 0xFFFF0000, i.e. its high half is -(k+1) mod 2^16.  Then
//   d = (r << 16) + S = ((r - k - 1) << 16) + (node & 0xFFFF)     (one v_lshl_add_u32)
// is < 0 iff r <= k, and >= node & 0xFFFF >= right offset otherwise, so med3(d, 1, off)
// steps exactly as in the 32-bit form (leaf: k = 0x7FFF vs sentinel 0x4000 -> d < 0, off 0;
// jump: k = 0 -> d > 0); |d| < 2^31 because r, k <= 0x7FFF.
// Node / plane formats (template parameter P16): 0 = u32 planes, 4-bit feature, 12-bit right
// offset (rank layout v1); 2 = rank layout v2: u16 planes of 1,024 rows, a 5-bit SLOT field and
// an 11-bit right offset (see build_rank_layout).
template <int P16>
constexpr uint32_t kSlotMask = (P16 == 2 || P16 == 3) ? 0xF800u : 0xF000u;
template <int P16>
constexpr uint32_t kOffMask = (P16 == 2 || P16 == 3) ? 0x7FFu : 0xFFFu;
// 3 = the v2 node format over 16 u16 planes of 1,024 rows (32 KiB): forests whose every feature
// fits one slot (slot = feature, the v1 row format); the node region starts at 32 KiB, so a
// chunk holds a third more nodes than with 64 KiB of planes (fewer chunk launches per batch)
template <int P16>
constexpr uint32_t kNodeB = P16 == 3 ? 32768u : kRankNodeB;

// Compact planes (P16 = 3) are read a DWORD at a time: the lane's u16 rank is the low half
// (lanes 0-31 of the wave) or the high half (lanes 32-63) of the dword it shares with lane
// l +- 32 (the plane swizzle in k_forest_rank), and d = (x << sh) + S with sh = 16 / 0 puts it
// in bits 31:16 either way.  For the high half the other row's rank (<= 0x7FFF) stays in bits
// 15:0, where it adds to S's low half (slot << 11 | offset <= 0x7FFF) without a carry into bit 16:
// d < 0 iff r <= k as before, and d >= S's low half >= offset when r > k, so med3(d, 1, offset)
// steps exactly as with the u16 read (which measured ~27 % slower per tree than the u32 planes'
// ds_read_b32: r04d forest trace, 70 vs 55 us per tree).
template <int P16>
__device__ __forceinline__ uint32_t plane_shift() {
    return P16 == 3 && (threadIdx.x & 32) ? 0u : 16u;
}
template <int P16>
__device__ __forceinline__ uint32_t rank_x(const char *lds, uint32_t addr) {
    return P16 == 3 ? lds32(lds, addr) : (P16 ? lds16(lds, addr) : lds32(lds, addr));
}

template <bool NAN_AWARE, int P16, int K>
__device__ __forceinline__ void rank_step(const char *lds, const uint32_t (&lane_base)[K], uint32_t (&pa)[K],
                                          uint32_t (&nd)[K], const uint8_t *__restrict__ mleft) {
    const uint32_t sh = plane_shift<P16>();
    uint32_t x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        x[k] = rank_x<P16>(lds, (nd[k] & kSlotMask<P16>) | lane_base[k]);
        if (P16 == 3) x[k] = (x[k] >> (16u - sh)) & 0xFFFFu;  // this lane's half
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint32_t st;
        if (NAN_AWARE && x[k] == (P16 ? 0xFFFFu : 0xFFFFFFFFu)) {
            st = mleft[(pa[k] - kNodeB<P16>) >> 2] != 0 ? 1u : (nd[k] & kOffMask<P16>);
        } else {
            const int32_t d = P16 ? (int32_t)((x[k] << 16) + nd[k]) : (int32_t)(x[k] - nd[k]);
            asm("v_med3_i32 %0, %1, 1, %2" : "=v"(st) : "v"(d), "v"(nd[k] & kOffMask<P16>));
        }
        pa[k] += st << 2;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) nd[k] = lds32(lds, pa[k]);
}

template <bool NAN_AWARE, int P16, int K>
__device__ __forceinline__ void rank_walk(const char *lds, const uint32_t (&lane_base)[K], uint32_t (&pa)[K],
                                          uint32_t (&nd)[K], int depth, const uint8_t *__restrict__ mleft) {
    int d = 0;
    for (; d + kExitEvery <= depth; d += kExitEvery) {
#pragma unroll
        for (int e = 0; e < kExitEvery; ++e) rank_step<NAN_AWARE, P16, K>(lds, lane_base, pa, nd, mleft);
        uint32_t moving = 0;  // leaves (and only leaves) have right offset 0
#pragma unroll
        for (int k = 0; k < K; ++k) moving |= nd[k] & kOffMask<P16>;
        if (!__any(moving != 0)) return;
    }
    for (; d < depth; ++d) rank_step<NAN_AWARE, P16, K>(lds, lane_base, pa, nd, mleft);
}

// Walk trees [t, t+GG) for the R rows of this lane (chain k = r*GG + g); pa = final leaves.
// Software-pipelined form of rank_walk (no NaN rows): the source order -- per chain, its
// step arithmetic then at once its node read; then per chain, its feature read -- is pinned
// with sched_barrier, so every chain has its next LDS read in flight while the others
// compute (the default schedule clusters all K reads of a phase behind all K updates, and
// a wave's outstanding reads drain to zero twice per step).
// PW > 1: chains in groups of PW, the node reads of a group issued in reverse chain order
// and its feature reads in forward order, so the first use in each group waits for the
// group's last-issued read and one s_waitcnt covers the whole group (LDS reads of a wave
// return in order): fewer issue slots per step.
// `pre` steps run before the first exit test (the caller's estimate of the steps the wave will
// need: extra steps at leaves are fixed points); returns the steps run (wave-uniform).
template <int P16, int K, int PW>
__device__ __forceinline__ int rank_walk_pipe(const char *lds, const uint32_t (&lane_base)[K], uint32_t (&pa)[K],
                                              uint32_t (&nd)[K], int depth, int pre = 0) {
    auto fetch_x = [&](int k) -> uint32_t { return rank_x<P16>(lds, (nd[k] & kSlotMask<P16>) | lane_base[k]); };
    const uint32_t sh = plane_shift<P16>();
    uint32_t x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = fetch_x(k);
    auto step = [&]() {
#pragma unroll
        for (int g = 0; g < K; g += PW) {
#pragma unroll
            for (int j = PW - 1; j >= 0; --j) {
                const int k = g + j;
                if (k < K) {
                    const int32_t d = P16 ? (int32_t)((x[k] << (P16 == 3 ? sh : 16u)) + nd[k]) : (int32_t)(x[k] - nd[k]);
                    uint32_t st, pn;  // pa += med3(d, 1, off) << 2, kept as 2 VALU on the byte address
                    // (a separate output: a read-write operand made the compiler copy pa first)
                    asm("v_med3_i32 %1, %2, 1, %3\n\tv_lshl_add_u32 %0, %1, 2, %4"
                        : "=v"(pn), "=&v"(st) : "v"(d), "v"(nd[k] & kOffMask<P16>), "v"(pa[k]));
                    pa[k] = pn;
                    nd[k] = lds32(lds, pa[k]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x[k] = fetch_x(k);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    int d = 0;
    for (; d + kExitEvery <= pre; d += kExitEvery) {  // whole unrolled intervals, no test
#pragma unroll
        for (int e = 0; e < kExitEvery; ++e) step();
    }
    for (; d + kExitEvery <= depth; d += kExitEvery) {
#pragma unroll
        for (int e = 0; e < kExitEvery; ++e) step();
        uint32_t moving = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) moving |= nd[k] & kOffMask<P16>;
        if (!__any(moving != 0)) return d + kExitEvery;
    }
    for (; d < depth; ++d) step();
    return d;
}

template <int R, int GG, int P16, int PIPE>
__device__ __forceinline__ void rank_trees(const char *lds, const uint32_t (&lrow)[R], int t,
                                           const int32_t *__restrict__ root, const int32_t *__restrict__ depth,
                                           int64_t node_base, bool any_nan, const uint8_t *__restrict__ ml,
                                           uint32_t (&pa)[R * GG]) {
    constexpr int K = R * GG;
    uint32_t lane_base[K], nd[K];
    int dmax = 0;
#pragma unroll
    for (int g = 0; g < GG; ++g) {
        const uint32_t p0 = kNodeB<P16> + (uint32_t)(root[t + g] - node_base) * 4u;
        const uint32_t n0 = lds32(lds, p0);
        dmax = max(dmax, depth[t + g]);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            pa[r * GG + g] = p0;
            nd[r * GG + g] = n0;
            lane_base[r * GG + g] = lrow[r];
        }
    }
    if (any_nan)
        rank_walk<true, P16, K>(lds, lane_base, pa, nd, dmax, ml);
    else
        rank_walk_pipe<P16, K, PIPE>(lds, lane_base, pa, nd, dmax);
}

// rank_trees with the roots read once per launch (rp = root byte addresses, rn = root nodes,
// dmax = the deepest of the trees): no scalar loads of root / depth per tile
template <int R, int GG, int P16, int PIPE>
__device__ __forceinline__ int rank_trees_from(const char *lds, const uint32_t (&lrow)[R], const uint32_t (&rp)[GG],
                                               const uint32_t (&rn)[GG], int dmax, bool any_nan,
                                               const uint8_t *__restrict__ ml, uint32_t (&pa)[R * GG], int pre) {
    constexpr int K = R * GG;
    uint32_t lane_base[K], nd[K];
#pragma unroll
    for (int g = 0; g < GG; ++g)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            pa[r * GG + g] = rp[g];
            nd[r * GG + g] = rn[g];
            lane_base[r * GG + g] = lrow[r];
        }
    if (any_nan) {
        rank_walk<true, P16, K>(lds, lane_base, pa, nd, dmax, ml);
        return 0;
    }
    return rank_walk_pipe<P16, K, PIPE>(lds, lane_base, pa, nd, dmax, pre);
}

template <int K>
__device__ __forceinline__ void rank_leaf_values(const uint32_t (&pa)[K], int64_t node_base,
                                                 const double *__restrict__ lval, double (&v)[K],
                                                 uint32_t nodeb = kRankNodeB) {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = lval[node_base + ((pa[k] - nodeb) >> 2)];
}

// a[r] += v[r*GG + g] in tree order
template <int R, int GG>
__device__ __forceinline__ void rank_accumulate(double (&a)[R], const double (&v)[R * GG]) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int g = 0; g < GG; ++g) a[r] += v[r * GG + g];
}

template <int R, int GG>
__device__ __forceinline__ void rank_leaf_ids(const uint32_t (&pa)[R * GG], int64_t node_base, int t,
                                              const int64_t (&row)[R], const bool (&ok)[R],
                                              const int32_t *__restrict__ out_perm, int32_t *__restrict__ leaf_out,
                                              const int32_t *__restrict__ orig, int32_t n_trees,
                                              uint32_t nodeb = kRankNodeB) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!ok[r]) continue;
        const int64_t dst = out_perm ? (int64_t)out_perm[row[r]] : row[r];
        if (dst < 0) continue;
#pragma unroll
        for (int g = 0; g < GG; ++g)
            leaf_out[dst * n_trees + t + g] = orig[node_base + ((pa[r * GG + g] - nodeb) >> 2)];
    }
}

// concurrent-chunk mode: tree t's value of row r at tv[t * tv_n + r] (lanes = consecutive rows)
template <int R, int GG>
__device__ __forceinline__ void rank_tree_values(const double (&v)[R * GG], int t, const int64_t (&row)[R],
                                                 const bool (&ok)[R], double *__restrict__ tv, int64_t tv_n) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!ok[r]) continue;
#pragma unroll
        for (int g = 0; g < GG; ++g) tv[(int64_t)(t + g) * tv_n + row[r]] = v[r * GG + g];
    }
}

// proba[row] = (sum of the row's tree values in tree order) / n_trees: the same float64
// additions, in the same order, as the chunk-sequential launches' running sum.
__global__ void __launch_bounds__(256) k_tree_sum(const double *__restrict__ tv, int64_t n, int32_t n_trees,
                                                  const int32_t *__restrict__ out_perm, double *__restrict__ proba) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        double a = 0.0;
        for (int t = 0; t < n_trees; ++t) a += tv[(int64_t)t * n + r];
        const int64_t dst = out_perm ? (int64_t)out_perm[r] : r;
        if (dst >= 0) proba[dst] = a / (double)n_trees;
    }
}

// One launch = trees [t0, t1) of one LDS chunk over rows [r0, r1), rank layout; one block
// per CU (the LDS holds one block), grid-striding over row tiles of BLOCK*R rows.  Each lane
// walks G trees for each of its R rows at once (K = R*G chains); a chunk's last t1-t0 mod G
// trees run as a narrower tail group.  Latency hiding: the next tile's rank rows and running
// sums are loaded into registers while the current tile walks (a thread's LDS row slots are
// only ever read by that thread, so no barrier is needed to refill them), and the leaf
// values of a walk group are loaded while the next group walks (accumulation stays in tree
// order).  The float64 running sum crosses launches through acc, as in k_forest_chunk.
template <int BLOCK, int R, int G, int P16, int PIPE>
__global__ void __launch_bounds__(BLOCK, 1) k_forest_rank(
    const uint32_t *__restrict__ nodes, int64_t node_base, int32_t chunk_nodes, const int32_t *__restrict__ root,
    const int32_t *__restrict__ depth, int32_t t0, int32_t t1, const uint16_t *__restrict__ zr,
    const int32_t *__restrict__ nan_flag, int64_t r0, int64_t r1, const double *__restrict__ lval,
    const uint8_t *__restrict__ mleft, double *__restrict__ acc, double *__restrict__ proba,
    const int32_t *__restrict__ out_perm, int32_t *__restrict__ leaf_out, const int32_t *__restrict__ orig,
    int32_t n_trees, int first, int last, const int32_t *__restrict__ chunk_t,
    const int64_t *__restrict__ chunk_base, double *__restrict__ tv, int64_t tv_n) {
    // u32 planes: 1,024 rows x 16 slots; v2: u16, 1,024 rows x 32 slots; compact v2: u16, 16 slots
    constexpr int kPlaneRows = kRankPlaneRows;
    constexpr int kRowU16 = P16 == 2 ? 32 : 16;  // u16 slots per rank row in HBM
    constexpr int kXW = P16 == 3 ? kRankXWords / 2 : kRankXWords;  // row-plane words in LDS
    constexpr uint32_t kNB = kNodeB<P16>;
    if (tv) {  // all chunks at once (blockIdx.y = chunk): per-tree values out, summed by k_tree_sum
        const int c = blockIdx.y;
        t0 = chunk_t[c];
        t1 = chunk_t[c + 1];
        node_base = chunk_base[c];
        chunk_nodes = (int32_t)(chunk_base[c + 1] - node_base);
        first = 1;
        last = 0;
    }
    static_assert(BLOCK * R <= kPlaneRows, "row planes hold 1024 (u32) / 2048 (u16) rows");
    static_assert(BLOCK % 64 == 0, "whole waves (the u16 plane swizzle)");
    constexpr int K = R * G;
    constexpr int kRowsPerBlock = BLOCK * R;
    constexpr int kNodeWords = (kLdsTotal - kXW * 4) / 4;
    __shared__ __align__(16) uint32_t s_mem[kXW + kNodeWords];
    uint32_t *s_x = s_mem;
    const char *lds = reinterpret_cast<const char *>(s_mem);
    const int tid = threadIdx.x;
    {
        const uint32_t *nb = nodes + node_base;
        for (int i = tid; i < chunk_nodes; i += BLOCK) s_mem[kXW + i] = P16 ? nb[i] ^ 0xFFFF0000u : nb[i];
    }
    uint16_t *s_x16 = reinterpret_cast<uint16_t *>(s_mem);
#pragma unroll
    for (int r = 0; r < R; ++r) {  // slot 15: the leaf / jump sentinel (v2 needs none)
        if (P16 == 0) s_x[15 * kRankPlaneRows + r * BLOCK + tid] = kRankSentinel;
    }
    __syncthreads();
    const uint8_t *ml = mleft + node_base;
    const bool any_nan = *nan_flag != 0;  // uniform
    // u16 planes: a dword holds two rows' ranks; the lane of row slot 2i + h within its wave is
    // i + 32h, so the two halves of a dword are read by lanes l and l + 32 -- different LDS lane
    // groups -- and the 32 lanes of a group read 32 different banks whatever features they test
    // (natural order put rows 2i, 2i+1 in one group: a 2-way conflict whenever their features
    // differ).  u32 planes are conflict-free in natural order.
    const int pslot = P16 ? ((tid & ~63) | ((tid & 31) << 1) | ((tid >> 5) & 1)) : tid;
    uint32_t lrow[R];
#pragma unroll
    for (int r = 0; r < R; ++r)  // compact planes: the byte address of the dword holding the lane's u16
        lrow[r] = (uint32_t)(P16 == 3 ? ((r * BLOCK + pslot) & ~1) * 2 : (r * BLOCK + pslot) * (P16 ? 2 : 4));
    const int64_t stride = (int64_t)gridDim.x * kRowsPerBlock;
    int64_t base = r0 + (int64_t)blockIdx.x * kRowsPerBlock;
    uint4 q0[R], q1[R], q2[R], q3[R];
    double pacc[R];
    auto fetch = [&](int64_t b) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t rw = b + r * BLOCK + tid;
            const bool okr = rw < r1;
            const uint4 *src = reinterpret_cast<const uint4 *>(zr + (okr ? rw : r0) * kRowU16);
            q0[r] = src[0];
            q1[r] = src[1];
            if (P16 == 2) {
                q2[r] = src[2];
                q3[r] = src[3];
            }
            pacc[r] = (first || !okr) ? 0.0 : acc[rw];
        }
    };
    if (base < r1) fetch(base);
    // A chunk of at most G trees (every chunk of the bench forest: 5-6 trees of ~3.9k nodes per
    // 94 KiB) is ONE walk group per tile, so the group pipeline below never runs and each tile
    // waited for its leaf-value loads (and, last chunk, its output slots) right after its walk.
    // Here a tile's leaf values are folded into its running sums one tile LATER -- after the next
    // tile's walk -- and its output slots are loaded with its rank rows: no global load is
    // waited on right after it is issued.  Same float64 additions in the same (tree) order.
    auto one_group = [&](auto ntag) {
        constexpr int NT = decltype(ntag)::value;
        double pv[R * NT], ap[R];
        int64_t rowp[R];
        int32_t dstp[R], dst_n[R];
        bool okp[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            ap[r] = 0.0;
            rowp[r] = 0;
            dstp[r] = -1;
            okp[r] = false;
#pragma unroll
            for (int g = 0; g < NT; ++g) pv[r * NT + g] = 0.0;
        }
        uint32_t rp[NT], rn[NT];  // the chunk's roots, read once
        int dmax = 0, pre = 0;
#pragma unroll
        for (int g = 0; g < NT; ++g) {
            rp[g] = kNB + (uint32_t)(root[t0 + g] - node_base) * 4u;
            rn[g] = lds32(lds, rp[g]);
            dmax = max(dmax, depth[t0 + g]);
        }
        auto out_slot = [&](int64_t rw) -> int32_t {  // loaded here, used one tile later
            return rw < r1 ? (last && out_perm ? out_perm[rw] : (int32_t)rw) : -1;
        };
#pragma unroll
        for (int r = 0; r < R; ++r) dst_n[r] = out_slot(base + r * BLOCK + tid);
        auto fold = [&]() {
#pragma unroll
            for (int r = 0; r < R; ++r) {
#pragma unroll
                for (int g = 0; g < NT; ++g) ap[r] += pv[r * NT + g];
                // formed before the store's branch: sunk into it, the wait for pv would land
                // behind the store and cover the store too (vmcnt counts stores)
                asm volatile("" ::"v"(ap[r]));
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (!okp[r]) continue;
                if (last) {
                    if (dstp[r] >= 0) proba[dstp[r]] = ap[r] / (double)n_trees;  // < 0: padding slot
                } else {
                    acc[rowp[r]] = ap[r];
                }
            }
        };
        for (; base < r1; base += stride) {
            int64_t row[R];
            bool ok[R];
            double a[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                row[r] = base + r * BLOCK + tid;
                ok[r] = row[r] < r1;
                if constexpr (P16 == 2) {
                    const uint32_t w16[16] = {q0[r].x, q0[r].y, q0[r].z, q0[r].w, q1[r].x, q1[r].y, q1[r].z, q1[r].w,
                                              q2[r].x, q2[r].y, q2[r].z, q2[r].w, q3[r].x, q3[r].y, q3[r].z, q3[r].w};
#pragma unroll
                    for (int f = 0; f < 32; ++f)
                        s_x16[f * kPlaneRows + r * BLOCK + pslot] = (uint16_t)((w16[f >> 1] >> ((f & 1) * 16)) & 0xFFFFu);
                } else {
                    const uint32_t w8[8] = {q0[r].x, q0[r].y, q0[r].z, q0[r].w, q1[r].x, q1[r].y, q1[r].z, q1[r].w};
#pragma unroll
                    for (int f = 0; f < (P16 == 3 ? 16 : 15); ++f) {
                        const uint32_t u = (w8[f >> 1] >> ((f & 1) * 16)) & 0xFFFFu;
                        if (P16)
                            s_x16[f * kPlaneRows + r * BLOCK + pslot] = (uint16_t)u;
                        else
                            s_x[f * kRankPlaneRows + r * BLOCK + tid] = u == 0xFFFFu ? 0xFFFFFFFFu : u << 16;
                    }
                }
                a[r] = pacc[r];
            }
            int32_t dst[R];
#pragma unroll
            for (int r = 0; r < R; ++r) dst[r] = dst_n[r];
            if (base + stride < r1) {
                fetch(base + stride);
#pragma unroll
                for (int r = 0; r < R; ++r) dst_n[r] = out_slot(base + stride + r * BLOCK + tid);
            }
            uint32_t pt[R * NT];
            // the previous tile's step count, less one exit interval, runs without exit tests
            // (rows of the bench forest walk ~20 of 20 steps: 5 tests per tile otherwise); when
            // the first test already found every chain at a leaf, the prefix shrinks by one more
            // interval, so it follows shorter walks down
            const int ran = rank_trees_from<R, NT, P16, PIPE>(lds, lrow, rp, rn, dmax, any_nan, ml, pt, pre);
            pre = ran - (ran <= pre + kExitEvery ? 2 : 1) * kExitEvery;
            fold();  // the previous tile
            rank_leaf_values<R * NT>(pt, node_base, lval, pv, kNB);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                ap[r] = a[r];
                rowp[r] = row[r];
                dstp[r] = dst[r];
                okp[r] = ok[r];
            }
        }
        fold();
    };
    // (9+ trees: register spills)
    if (!tv && !leaf_out && t1 - t0 <= (G < 8 ? G : 8) && r1 <= INT32_MAX) {
#define FDX_ONE_GROUP(NT) \
    if constexpr (G >= NT) \
        if (t1 - t0 == NT) one_group(std::integral_constant<int, NT>{});
        FDX_ONE_GROUP(1)
        FDX_ONE_GROUP(2)
        FDX_ONE_GROUP(3)
        FDX_ONE_GROUP(4)
        FDX_ONE_GROUP(5)
        FDX_ONE_GROUP(6)
        FDX_ONE_GROUP(7)
        FDX_ONE_GROUP(8)
#undef FDX_ONE_GROUP
        return;
    }
    for (; base < r1; base += stride) {
        int64_t row[R];
        bool ok[R];
        double a[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            row[r] = base + r * BLOCK + tid;
            ok[r] = row[r] < r1;
            if constexpr (P16 == 2) {
                const uint32_t w[16] = {q0[r].x, q0[r].y, q0[r].z, q0[r].w, q1[r].x, q1[r].y, q1[r].z, q1[r].w,
                                        q2[r].x, q2[r].y, q2[r].z, q2[r].w, q3[r].x, q3[r].y, q3[r].z, q3[r].w};
#pragma unroll
                for (int f = 0; f < 32; ++f)
                    s_x16[f * kPlaneRows + r * BLOCK + pslot] = (uint16_t)((w[f >> 1] >> ((f & 1) * 16)) & 0xFFFFu);
            } else {
                const uint32_t w[8] = {q0[r].x, q0[r].y, q0[r].z, q0[r].w, q1[r].x, q1[r].y, q1[r].z, q1[r].w};
#pragma unroll
                for (int f = 0; f < (P16 == 3 ? 16 : 15); ++f) {
                    const uint32_t u = (w[f >> 1] >> ((f & 1) * 16)) & 0xFFFFu;
                    if (P16)
                        s_x16[f * kPlaneRows + r * BLOCK + pslot] = (uint16_t)u;
                    else
                        s_x[f * kRankPlaneRows + r * BLOCK + tid] = u == 0xFFFFu ? 0xFFFFFFFFu : u << 16;
                }
            }
            a[r] = pacc[r];
        }
        if (base + stride < r1) fetch(base + stride);
        double pv[K];
        bool pending = false;
        int t = t0;
        for (; t + G <= t1; t += G) {
            uint32_t pa[K];
            rank_trees<R, G, P16, PIPE>(lds, lrow, t, root, depth, node_base, any_nan, ml, pa);
            if (pending) rank_accumulate<R, G>(a, pv);
            rank_leaf_values<K>(pa, node_base, lval, pv, kNB);
            if (tv) rank_tree_values<R, G>(pv, t, row, ok, tv, tv_n);
            pending = true;
            if (leaf_out) rank_leaf_ids<R, G>(pa, node_base, t, row, ok, out_perm, leaf_out, orig, n_trees, kNB);
        }
        const int nt = t1 - t;
#define FDX_RANK_TAIL(NT)                                                                                  \
    if constexpr (G > NT) {                                                                                \
        if (nt == NT) {                                                                                    \
            uint32_t pt[R * NT];                                                                           \
            double vt[R * NT];                                                                             \
            rank_trees<R, NT, P16, PIPE>(lds, lrow, t, root, depth, node_base, any_nan, ml, pt);           \
            if (pending) rank_accumulate<R, G>(a, pv);                                                     \
            pending = false;                                                                               \
            rank_leaf_values<R * NT>(pt, node_base, lval, vt, kNB);                                        \
            if (tv) rank_tree_values<R, NT>(vt, t, row, ok, tv, tv_n);                                     \
            rank_accumulate<R, NT>(a, vt);                                                                 \
            if (leaf_out) rank_leaf_ids<R, NT>(pt, node_base, t, row, ok, out_perm, leaf_out, orig, n_trees, kNB); \
        }                                                                                                  \
    }
        FDX_RANK_TAIL(1)
        FDX_RANK_TAIL(2)
        FDX_RANK_TAIL(3)
        FDX_RANK_TAIL(4)
        FDX_RANK_TAIL(5)
        FDX_RANK_TAIL(6)
        FDX_RANK_TAIL(7)
        FDX_RANK_TAIL(8)
        FDX_RANK_TAIL(9)
#undef FDX_RANK_TAIL
        if (pending) rank_accumulate<R, G>(a, pv);
        if (tv) continue;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!ok[r]) continue;
            if (last) {
                const int64_t dst = out_perm ? (int64_t)out_perm[row[r]] : row[r];
                if (dst >= 0) proba[dst] = a[r] / (double)n_trees;  // < 0: padding slot
            } else {
                acc[row[r]] = a[r];
            }
        }
    }
}

float round_down_f32(double t) {
    float f = (float)t;
    if ((double)f > t) f = std::nextafter(f, -INFINITY);
    return f;
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace
}  // namespace fdx

using namespace fdx;

namespace fdx {
namespace {
// Host-side validation + pre-order re-layout + 8-byte node packing (see header comment).
int pack_forest(const fdx_forest_desc *d, std::vector<uint64_t> &packed, std::vector<int32_t> &orig,
                std::vector<int32_t> &root, std::vector<int32_t> &depth) {
    FDX_REQUIRE(d, "null pointer");
    FDX_REQUIRE(d->n_trees >= 1, "n_trees must be >= 1");
    FDX_REQUIRE(d->n_features >= 1 && d->n_features <= FDX_MAX_FEATURES, "n_features must be in [1, %d]",
                FDX_MAX_FEATURES);
    FDX_REQUIRE(d->node_offsets && d->children_left && d->children_right && d->feature && d->threshold &&
                    d->value1,
                "null tree array");
    const int64_t total = d->node_offsets[d->n_trees];
    FDX_REQUIRE(d->node_offsets[0] == 0 && total > 0 && total < (int64_t(1) << 31), "bad node_offsets");
    packed.assign((size_t)total, 0);
    orig.assign((size_t)total, 0);
    depth.assign((size_t)d->n_trees, 0);
    root.assign((size_t)d->n_trees, 0);
    std::vector<int64_t> stack;
    for (int32_t t = 0; t < d->n_trees; ++t) {
        const int64_t b = d->node_offsets[t], e = d->node_offsets[t + 1];
        FDX_REQUIRE(e > b, "tree %d is empty", t);
        const int64_t cnt = e - b;
        // pre-order re-layout (identity for sklearn's depth-first builder)
        std::vector<int64_t> pos((size_t)cnt, -1);
        int64_t next = b;
        stack.clear();
        stack.push_back(0);
        std::vector<int64_t> order;
        order.reserve((size_t)cnt);
        while (!stack.empty()) {
            int64_t i = stack.back();
            stack.pop_back();
            FDX_REQUIRE(i >= 0 && i < cnt && pos[(size_t)i] < 0, "tree %d: malformed children", t);
            pos[(size_t)i] = next++;
            order.push_back(i);
            int64_t l = d->children_left[b + i], r = d->children_right[b + i];
            if (l != -1) {
                FDX_REQUIRE(r != -1, "tree %d node %lld has one child", t, (long long)i);
                stack.push_back(r);
                stack.push_back(l);
            }
        }
        FDX_REQUIRE(next == e, "tree %d: %lld unreachable nodes", t, (long long)(e - next));
        root[(size_t)t] = (int32_t)b;
        {   // max leaf depth = number of steps a walk of this tree takes
            std::vector<int32_t> dep((size_t)cnt, 0);
            int32_t dm = 0;
            for (int64_t i : order) {  // pre-order: parents before children
                const int64_t l = d->children_left[b + i];
                if (l != -1) {
                    dep[(size_t)l] = dep[(size_t)i] + 1;
                    dep[(size_t)d->children_right[b + i]] = dep[(size_t)i] + 1;
                } else if (dep[(size_t)i] > dm) {
                    dm = dep[(size_t)i];
                }
            }
            depth[(size_t)t] = dm;
        }
        for (int64_t i : order) {
            const int64_t p = pos[(size_t)i];
            orig[(size_t)p] = (int32_t)i;
            const int64_t l = d->children_left[b + i];
            if (l == -1) {
                double v = d->value1[b + i];
                FDX_REQUIRE(!(v != v), "tree %d leaf %lld value is NaN", t, (long long)i);
                if (v == 0.0) v = 0.0;  // normalise -0.0
                uint64_t bits;
                memcpy(&bits, &v, 8);
                if (bits >> 63) {
                    set_error("tree %d leaf %lld: negative leaf values are not supported", t, (long long)i);
                    return FDX_E_UNSUPPORTED;
                }
                packed[(size_t)p] = bits;
            } else {
                const int64_t rp = pos[(size_t)d->children_right[b + i]];
                FDX_REQUIRE(pos[(size_t)l] == p + 1, "tree %d: pre-order violated", t);
                const int64_t rel = rp - p;
                FDX_REQUIRE(rel > 0 && rel < (int64_t(1) << 21), "tree %d: subtree too large", t);
                const int64_t f = d->feature[b + i];
                FDX_REQUIRE(f >= 0 && f < d->n_features, "tree %d node %lld: feature %lld out of range", t,
                            (long long)i, (long long)f);
                const uint32_t ml = d->missing_go_to_left ? (d->missing_go_to_left[b + i] != 0) : 0u;
                const float thr = round_down_f32(d->threshold[b + i]);
                uint32_t lo;
                memcpy(&lo, &thr, 4);
                const uint32_t hi = kInternal | (ml << 30) | ((uint32_t)f << 24) | (uint32_t)(rel * 8);
                packed[(size_t)p] = ((uint64_t)hi << 32) | lo;
            }
        }
    }
    return FDX_OK;
}

// Rank layout (see the device-side comment "Rank layout") built from the wide packing.
struct RankLayout {
    std::vector<uint32_t> nodes;
    std::vector<int32_t> orig, root, depth;
    std::vector<double> lval;
    std::vector<uint8_t> ml;
    std::vector<int64_t> offsets;
    std::vector<float> thr;
    int32_t thr_off[33] = {};
    // v2: threshold-rank slots (a feature with more than kSlotSpan thresholds spans several)
    bool v2 = false;
    int32_t n_slots = 0, slot_feat[32] = {}, slot_base[32] = {};
};

// Returns FDX_OK, or FDX_E_UNSUPPORTED (with the reason in fdx_last_error) when the forest
// does not fit the layout (> 15 features, > 32767 distinct thresholds of one feature, a
// tree larger than the LDS node budget).  `max_tree_nodes` = LDS node budget per chunk.
//
// v2 (rank layout v2, forests v1 cannot hold -- e.g. the reference's deployed
// RandomForestClassifier(random_state=0): 100 unlimited-depth trees with up to 96k distinct
// thresholds on one feature): 32 u16 SLOTS instead of 16 features.  Feature f with |U_f|
// thresholds owns ceil(|U_f| / kSlotSpan) consecutive slots; slot j of f holds the clamped
// rank  r_j = min(max(r - j*kSlotSpan, 0), kSlotSpan)  and a node testing U_f[k] tests slot
// j = k / kSlotSpan with k' = k - j*kSlotSpan:  r <= k  <=>  r_j <= k'  (r below the slot's
// range gives r_j = 0 <= k', above it r_j = kSlotSpan > k').  Node: [30:16] k' | [15:11]
// slot | [10:0] right offset; leaf 0x7FFF0000 (k' = 0x7FFF >= every r_j: a fixed point of
// the u16-plane step); jump 0xFFFF0000 | offset (k' = -1 in the step's 16-bit arithmetic:
// always right).  No sentinel slot.
constexpr int64_t kSlotSpan = 32767;
int build_rank_layout(const fdx_forest_desc *d, const std::vector<uint64_t> &packed,
                      const std::vector<int32_t> &worig, const std::vector<int32_t> &wdepth, int64_t max_tree_nodes,
                      RankLayout &L, bool v2 = false) {
    if (!v2 && d->n_features > 15) {
        set_error("rank layout: %d features > 15", d->n_features);
        return FDX_E_UNSUPPORTED;
    }
    const int nfeat = v2 ? 32 : 16;
    const uint32_t kOff = v2 ? 0x7FFu : 0xFFFu;
    const int64_t max_off = v2 ? 2047 : kRankMaxOffset;
    const uint32_t leaf_word = v2 ? 0x7FFF0000u : kRankLeaf, jump_word = v2 ? 0xFFFF0000u : kRankJump;
    L.v2 = v2;
    // U_f: sorted unique float32 thresholds per feature
    std::vector<std::vector<float>> U(64);
    for (uint64_t nd : packed)
        if (nd >> 63) {
            const uint32_t hi = (uint32_t)(nd >> 32), lo = (uint32_t)nd;
            float t;
            memcpy(&t, &lo, 4);
            U[(hi >> 24) & 63].push_back(t);
        }
    L.thr.clear();
    int32_t slot_first[32] = {};
    L.n_slots = 0;
    for (int f = 0; f < nfeat; ++f) {
        auto &u = U[f];
        std::sort(u.begin(), u.end());
        u.erase(std::unique(u.begin(), u.end(), [](float a, float b) { return a == b; }), u.end());
        if (!v2 && (int64_t)u.size() > kRankMaxRank + 1) {
            set_error("rank layout: feature %d has %zu distinct thresholds > %d", f, u.size(), kRankMaxRank + 1);
            return FDX_E_UNSUPPORTED;
        }
        L.thr_off[f] = (int32_t)L.thr.size();
        L.thr.insert(L.thr.end(), u.begin(), u.end());
        if (v2 && f < d->n_features) {
            const int ns = (int)std::max<int64_t>(1, ceil_div((int64_t)u.size(), kSlotSpan));
            if (L.n_slots + ns > 32) {
                set_error("rank layout v2: more than 32 threshold slots needed");
                return FDX_E_UNSUPPORTED;
            }
            slot_first[f] = L.n_slots;
            for (int j = 0; j < ns; ++j) {
                L.slot_feat[L.n_slots] = f;
                L.slot_base[L.n_slots] = (int32_t)(j * kSlotSpan);
                ++L.n_slots;
            }
        }
    }
    L.thr_off[nfeat] = (int32_t)L.thr.size();
    L.nodes.clear(); L.orig.clear(); L.lval.clear(); L.ml.clear(); L.root.clear(); L.depth.clear();
    L.offsets.assign(1, 0);
    struct Pend { int64_t owner; };
    std::vector<Pend> pend;
    int margin = 0;
    bool ok = true;
    auto push = [&](uint32_t node, int32_t o, double v, uint8_t m) {
        L.nodes.push_back(node); L.orig.push_back(o); L.lval.push_back(v); L.ml.push_back(m);
    };
    auto set_off = [&](int64_t pos, int64_t off) {
        if (off < 1 || off > max_off) ok = false;
        L.nodes[(size_t)pos] = (L.nodes[(size_t)pos] & ~kOff) | (uint32_t)(off & kOff);
    };
    // pre-order emission; after every leaf, pending right pointers that are about to run out
    // of range are forwarded through a jump node placed right there (the slot after a leaf
    // is only ever reached through a right pointer, so nothing else moves semantically)
    std::function<void(int64_t)> emit = [&](int64_t w) {
        const uint64_t nd = packed[(size_t)w];
        const int64_t pos = (int64_t)L.nodes.size();
        if (!(nd >> 63)) {
            double v;
            memcpy(&v, &nd, 8);
            push(leaf_word, worig[(size_t)w], v, 0);
            for (auto &p : pend)
                if ((int64_t)L.nodes.size() - p.owner + margin > max_off) {
                    const int64_t j = (int64_t)L.nodes.size();
                    push(jump_word, -1, 0.0, 0);
                    set_off(p.owner, j - p.owner);
                    p.owner = j;
                }
            return;
        }
        const uint32_t hi = (uint32_t)(nd >> 32), lo = (uint32_t)nd;
        const int f = (int)((hi >> 24) & 63);
        float t;
        memcpy(&t, &lo, 4);
        const auto &u = U[f];
        const int64_t k = std::lower_bound(u.begin(), u.end(), t) - u.begin();
        uint32_t word;
        if (v2) {
            const int64_t j = k / kSlotSpan;
            word = ((uint32_t)(k - j * kSlotSpan) << 16) | ((uint32_t)(slot_first[f] + j) << 11);
        } else {
            word = ((uint32_t)k << 16) | ((uint32_t)f << 12);
        }
        push(word, worig[(size_t)w], 0.0, (uint8_t)((hi >> 30) & 1));
        pend.push_back({pos});
        const size_t pi = pend.size() - 1;
        emit(w + 1);
        set_off(pend[pi].owner, (int64_t)L.nodes.size() - pend[pi].owner);
        pend.pop_back();
        emit(w + (int64_t)((hi & 0xFFFFFFu) >> 3));
    };
    for (int32_t tr = 0; tr < d->n_trees; ++tr) {
        const int64_t tb = (int64_t)L.nodes.size();
        margin = 2 * wdepth[(size_t)tr] + 16;
        if (margin > max_off / 2) {
            set_error("rank layout: tree %d is too deep (%d)", tr, wdepth[(size_t)tr]);
            return FDX_E_UNSUPPORTED;
        }
        emit(d->node_offsets[tr]);
        if (!ok) {
            set_error("rank layout: tree %d: right offset out of range", tr);
            return FDX_E_UNSUPPORTED;
        }
        const int64_t te = (int64_t)L.nodes.size();
        if (te - tb > max_tree_nodes) {
            set_error("rank layout: tree %d has %lld nodes > LDS budget %lld", tr, (long long)(te - tb),
                      (long long)max_tree_nodes);
            return FDX_E_UNSUPPORTED;
        }
        // steps to reach a leaf (jumps count): children always follow their parent
        std::vector<int32_t> st((size_t)(te - tb), 0);
        int32_t dm = 0;
        for (int64_t p = tb; p < te; ++p) {
            const uint32_t nd = L.nodes[(size_t)p];
            const int64_t off = nd & kOff, s = st[(size_t)(p - tb)];
            if (off == 0) {
                dm = std::max<int32_t>(dm, (int32_t)s);
                continue;
            }
            const bool jump = v2 ? (nd >> 16) == 0xFFFFu : ((nd >> 12) & 15) == 15;
            if (!jump) st[(size_t)(p + 1 - tb)] = (int32_t)s + 1;
            st[(size_t)(p + off - tb)] = (int32_t)s + 1;
        }
        L.root.push_back((int32_t)tb);
        L.depth.push_back(dm);
        L.offsets.push_back(te);
    }
    if (L.nodes.size() >= (size_t(1) << 31)) {
        set_error("rank layout: too many nodes");
        return FDX_E_UNSUPPORTED;
    }
    return FDX_OK;
}
}  // namespace
}  // namespace fdx

namespace fdx {
namespace {
int install_rank_layout(fdx_forest_s *F, bool v2, hipStream_t st);
// node format a variant runs on: 1 = rank layout v1, 2 = v2
int variant_format(const Variant &v) { return v.p16 == 2 || v.p16 == 3 ? 2 : 1; }
int forest_format(const fdx_forest_s *F) { return F->rank_v2 ? 2 : 1; }
int variant_group(const fdx_forest_s *F) { return F->zstride == 16 ? kVariants[F->variant].group : 4; }

constexpr int64_t kRankNodeCap = (kLdsTotal - kRankXWords * 4) / 4 - 1;  // - the parking leaf
constexpr int64_t kRankNodeCapCompact = (kLdsTotal - kRankXWords * 2) / 4 - 1;  // 32 KiB of planes

bool rank_mode(const fdx_forest_s *F) { return kVariants[F->variant].rank != 0; }

// Cut the trees into chunks whose nodes fit the variant's LDS budget; whole groups of G trees
// where more than G fit (a partial group idles walk slots); oversized trees run from global
// (wide layout only: a rank-layout forest has every tree within the budget by construction).
void build_chunks(fdx_forest_s *F) {
    const Variant v = F->zstride == 16 ? kVariants[F->variant] : kVariants[0];
    const int64_t cap_nodes = v.rank ? (v.p16 == 3 ? kRankNodeCapCompact : kRankNodeCap)
                                     : lds_node_bytes(F->zstride, v.block, v.rows) / 8;
    const int G = variant_group(F);
    const auto &off = v.rank ? F->rank_offsets : F->node_offsets;
    F->chunks.clear();
    for (int32_t t = 0; t < F->n_trees;) {
        fdx_forest_s::Chunk c;
        c.t0 = t;
        c.node_base = off[t];
        if (off[t + 1] - off[t] > cap_nodes) {
            c.t1 = t + 1;
            c.in_lds = false;
        } else {
            int32_t u = t + 1;
            while (u < F->n_trees && off[u + 1] - c.node_base <= cap_nodes) ++u;
            if (!v.rank && u - t > G && (u - t) % G) u -= (u - t) % G;  // rank kernel: narrower tail group
            c.t1 = u;
            c.in_lds = true;
        }
        c.nodes = off[c.t1] - c.node_base;
        F->chunks.push_back(c);
        t = c.t1;
    }
}
// Chunk table for the all-chunks-at-once launch (device copy; synchronous, off the hot path).
int upload_chunks(fdx_forest_s *F) {
    if (!F->chunk_t_d) return FDX_OK;
    std::vector<int32_t> ct(F->chunks.size() + 1);
    std::vector<int64_t> cb(F->chunks.size() + 1);
    for (size_t c = 0; c < F->chunks.size(); ++c) {
        ct[c] = F->chunks[c].t0;
        cb[c] = F->chunks[c].node_base;
    }
    ct.back() = F->n_trees;
    cb.back() = F->chunks.empty() ? 0 : F->chunks.back().node_base + F->chunks.back().nodes;
    FDX_HIP(hipMemcpy(F->chunk_t_d, ct.data(), sizeof(int32_t) * ct.size(), hipMemcpyHostToDevice));
    FDX_HIP(hipMemcpy(F->chunk_base_d, cb.data(), sizeof(int64_t) * cb.size(), hipMemcpyHostToDevice));
    return FDX_OK;
}
}  // namespace
}  // namespace fdx

extern "C" int fdx_forest_set_variant(fdx_forest F, int32_t variant) {
    FDX_REQUIRE(F, "null forest");
    FDX_REQUIRE(variant >= 0 && variant < kNumVariants, "variant must be in [0, %d)", kNumVariants);
    FDX_REQUIRE(variant == 0 || F->zstride == 16, "variants > 0 need <= 15 features");
    const Variant &v = kVariants[variant];
    if (v.rank && !F->rank_ok) {
        set_error("variant %d needs the rank layout, which this forest does not fit", variant);
        return FDX_E_UNSUPPORTED;
    }
    const int prev = F->variant, had = forest_format(F);
    // every failure below leaves the forest exactly as it was: the previous node format (the
    // rank layout is rebuilt in it when it was switched), the previous variant and its chunks
    auto refuse = [&](const char *why, int a) {
        if (forest_format(F) != had) install_rank_layout(F, had == 2, nullptr);
        F->variant = prev;
        build_chunks(F);
        upload_chunks(F);
        set_error(why, variant, a);
        return FDX_E_UNSUPPORTED;
    };
    if (v.rank && variant_format(v) != had) {  // the variant runs on the other node format
        if (install_rank_layout(F, variant_format(v) == 2, nullptr))
            return refuse("variant %d needs rank layout v%d, which this forest does not fit", variant_format(v));
    }
    if (v.rank && v.p16 == 3 && !F->rank_identity)
        return refuse("variant %d needs one threshold slot per feature (<= %d slots)", 16);
    F->variant = variant;
    build_chunks(F);
    bool rank_fits = true;  // a rank kernel walks LDS-resident chunks only
    for (const auto &c : F->chunks) rank_fits = rank_fits && c.in_lds;
    if (v.rank && !rank_fits) return refuse("variant %d: a tree does not fit its LDS node budget", 0);
    return upload_chunks(F);
}

extern "C" int fdx_forest_get_variant(fdx_forest F, int32_t *variant) {
    FDX_REQUIRE(F && variant, "null pointer");
    *variant = F->variant;
    return FDX_OK;
}

extern "C" int fdx_forest_pack(const fdx_forest_desc *d, uint64_t *nodes_out, int32_t *orig_out,
                               int32_t *root_out) {
    std::vector<uint64_t> packed;
    std::vector<int32_t> orig, root, depth;
    int rc = pack_forest(d, packed, orig, root, depth);
    if (rc) return rc;
    FDX_REQUIRE(nodes_out && orig_out && root_out, "null output");
    memcpy(nodes_out, packed.data(), packed.size() * 8);
    memcpy(orig_out, orig.data(), orig.size() * 4);
    memcpy(root_out, root.data(), root.size() * 4);
    return FDX_OK;
}

static int rank_layout_host(const fdx_forest_desc *d, RankLayout &RL, int version = 1) {
    std::vector<uint64_t> packed;
    std::vector<int32_t> orig, root, depth;
    int rc = pack_forest(d, packed, orig, root, depth);
    if (rc) return rc;
    return build_rank_layout(d, packed, orig, depth, kRankNodeCap, RL, version == 2);
}

extern "C" int fdx_forest_rank_layout_size2(const fdx_forest_desc *d, int32_t version, int64_t *n_nodes,
                                            int32_t *n_thresholds, int32_t *n_slots) {
    FDX_REQUIRE(n_nodes && n_thresholds && n_slots, "null output");
    FDX_REQUIRE(version == 1 || version == 2, "version must be 1 or 2");
    RankLayout RL;
    int rc = rank_layout_host(d, RL, version);
    if (rc) return rc;
    *n_nodes = (int64_t)RL.nodes.size();
    *n_thresholds = (int32_t)RL.thr.size();
    *n_slots = version == 2 ? RL.n_slots : 16;
    return FDX_OK;
}

extern "C" int fdx_forest_pack_rank2(const fdx_forest_desc *d, int32_t version, uint32_t *nodes_out,
                                     int32_t *orig_out, double *leaf_value_out, uint8_t *missing_left_out,
                                     int32_t *root_out, int32_t *depth_out, float *thr_out, int32_t *thr_off_out,
                                     int32_t *slot_feat_out, int32_t *slot_base_out) {
    FDX_REQUIRE(version == 1 || version == 2, "version must be 1 or 2");
    FDX_REQUIRE(nodes_out && orig_out && leaf_value_out && missing_left_out && root_out && depth_out && thr_off_out &&
                    slot_feat_out && slot_base_out,
                "null output");
    RankLayout RL;
    int rc = rank_layout_host(d, RL, version);
    if (rc) return rc;
    const size_t n = RL.nodes.size();
    memcpy(nodes_out, RL.nodes.data(), 4 * n);
    memcpy(orig_out, RL.orig.data(), 4 * n);
    memcpy(leaf_value_out, RL.lval.data(), 8 * n);
    memcpy(missing_left_out, RL.ml.data(), n);
    memcpy(root_out, RL.root.data(), 4 * RL.root.size());
    memcpy(depth_out, RL.depth.data(), 4 * RL.depth.size());
    if (!RL.thr.empty()) {
        FDX_REQUIRE(thr_out, "null output");
        memcpy(thr_out, RL.thr.data(), 4 * RL.thr.size());
    }
    memcpy(thr_off_out, RL.thr_off, sizeof(RL.thr_off));
    memcpy(slot_feat_out, RL.slot_feat, sizeof(RL.slot_feat));
    memcpy(slot_base_out, RL.slot_base, sizeof(RL.slot_base));
    return FDX_OK;
}

extern "C" int fdx_forest_layout(fdx_forest F, int32_t *layout, int32_t *n_slots) {
    FDX_REQUIRE(F && layout && n_slots, "null pointer");
    *layout = !F->rank_ok ? 0 : (F->rank_v2 ? (F->rank_identity ? 3 : 2) : 1);
    *n_slots = F->rank_v2 ? F->rn_slots : (F->rank_ok ? 16 : 0);
    return FDX_OK;
}

extern "C" int fdx_forest_rank_layout_size(const fdx_forest_desc *d, int64_t *n_nodes, int32_t *n_thresholds) {
    FDX_REQUIRE(n_nodes && n_thresholds, "null output");
    RankLayout RL;
    int rc = rank_layout_host(d, RL);
    if (rc) return rc;
    *n_nodes = (int64_t)RL.nodes.size();
    *n_thresholds = (int32_t)RL.thr.size();
    return FDX_OK;
}

extern "C" int fdx_forest_pack_rank(const fdx_forest_desc *d, uint32_t *nodes_out, int32_t *orig_out,
                                    double *leaf_value_out, uint8_t *missing_left_out, int32_t *root_out,
                                    int32_t *depth_out, float *thr_out, int32_t *thr_off_out) {
    FDX_REQUIRE(nodes_out && orig_out && leaf_value_out && missing_left_out && root_out && depth_out && thr_off_out,
                "null output");
    RankLayout RL;
    int rc = rank_layout_host(d, RL);
    if (rc) return rc;
    const size_t n = RL.nodes.size();
    memcpy(nodes_out, RL.nodes.data(), 4 * n);
    memcpy(orig_out, RL.orig.data(), 4 * n);
    memcpy(leaf_value_out, RL.lval.data(), 8 * n);
    memcpy(missing_left_out, RL.ml.data(), n);
    memcpy(root_out, RL.root.data(), 4 * RL.root.size());
    memcpy(depth_out, RL.depth.data(), 4 * RL.depth.size());
    if (!RL.thr.empty()) {
        FDX_REQUIRE(thr_out, "null output");
        memcpy(thr_out, RL.thr.data(), 4 * RL.thr.size());
    }
    memcpy(thr_off_out, RL.thr_off, 17 * sizeof(int32_t));
    return FDX_OK;
}

namespace fdx {
namespace {
void free_rank_buffers(fdx_forest_s *F) {
    void **bufs[] = {(void **)&F->rnodes_d, (void **)&F->rorig_d, (void **)&F->rlval_d, (void **)&F->rml_d,
                     (void **)&F->rroot_d, (void **)&F->rdepth_d, (void **)&F->rthr_d, (void **)&F->rseg_d,
                     (void **)&F->ritab_d, (void **)&F->rrat_d, (void **)&F->rsmp_d, (void **)&F->retab_d};
    for (void **b : bufs) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
}

// Build the rank layout (v2 nodes when `v2`, else v1) from the host copy of the packed forest
// and upload it with its search tables; synchronous (creation / set_variant, off the hot path).
// On FDX_E_UNSUPPORTED the forest has no rank layout (rank_ok = false).
int install_rank_layout(fdx_forest_s *F, bool v2, hipStream_t st) {
    free_rank_buffers(F);
    F->rank_ok = F->rank_v2 = F->rank_identity = false;
    fdx_forest_desc d{};
    d.n_trees = F->n_trees;
    d.n_features = F->n_features;
    d.node_offsets = F->node_offsets.data();
    RankLayout RL;
    if (v2 && F->zstride != 16) return FDX_E_UNSUPPORTED;
    int rc = build_rank_layout(&d, F->h_packed, F->h_orig, F->h_depth, kRankNodeCap, RL, v2);
    if (rc) return rc;
    F->rank_ok = true;
    F->rank_v2 = v2;
    if (v2) {
        bool ident = RL.n_slots <= 16 && RL.n_slots == F->n_features;
        for (int j = 0; j < RL.n_slots && ident; ++j) ident = RL.slot_feat[j] == j && RL.slot_base[j] == 0;
        F->rank_identity = ident;
    }
    const int nfs = v2 ? 32 : 16;
    F->rank_offsets = RL.offsets;
    F->rank_nodes = (int64_t)RL.nodes.size();
    for (int f = 0; f < 32; ++f) {
        F->rthr_off[f] = f < nfs ? RL.thr_off[f] : 0;
        F->rthr_cnt[f] = f < nfs ? RL.thr_off[f + 1] - RL.thr_off[f] : 0;
    }
    F->rn_slots = RL.n_slots;
    for (int j = 0; j < 32; ++j) {
        F->rslot_feat[j] = RL.slot_feat[j];
        F->rslot_base[j] = RL.slot_base[j];
    }
    // two-level search tables (RankTab): smallest segment with <= kMaxRankSamples samples
    std::vector<float> useg, smp;
    std::vector<uint16_t> itab, rat;
    int seg = 16;
    for (;; seg *= 2) {
        int64_t m = 0;
        for (int f = 0; f < nfs; ++f) m += ceil_div(F->rthr_cnt[f], seg);
        if (m <= kMaxRankSamples) break;
    }
    F->rseg = seg;
    for (int f = 0; f < nfs; ++f) {
        const int32_t c = F->rthr_cnt[f], ns = (int32_t)ceil_div(c, seg);
        F->ruoff[f] = (int32_t)useg.size();
        F->rsoff[f] = (int32_t)smp.size();
        F->rscnt[f] = ns;
        for (int32_t j = 0; j < ns * seg; ++j) useg.push_back(j < c ? RL.thr[(size_t)(RL.thr_off[f] + j)] : INFINITY);
        for (int32_t j = 0; j < ns; ++j) smp.push_back(RL.thr[(size_t)(RL.thr_off[f] + j * seg)]);
    }
    F->rnsmp = (int32_t)smp.size();
    // Eytzinger tables of the searched features of k_zfill_grouped_w3 (15-feature forests with
    // 16-float segments): samples padded with +inf to 2^L - 1, laid out in BFS order
    std::vector<float> etab;
    F->rnetab = 0;
    if (F->n_features == 15 && seg == 16 && (!v2 || F->rank_identity)) {
        for (int s = 0; s < 4; ++s) {
            const int f = kW3Search[s];
            const int32_t ns = F->rscnt[f];
            int L = 0;
            while (((int64_t)1 << L) - 1 < ns) ++L;
            const int32_t m = (1 << L) - 1;
            F->reoff[s] = (int32_t)etab.size();
            F->relev[s] = L;
            std::vector<float> e((size_t)m + 1, INFINITY);  // e[0] unused
            int32_t i = 0;
            std::function<void(int32_t)> fill = [&](int32_t k) {  // in-order walk = sorted order
                if (k > m) return;
                fill(2 * k);
                e[(size_t)k] = i < ns ? smp[(size_t)(F->rsoff[f] + i)] : INFINITY;
                ++i;
                fill(2 * k + 1);
            };
            fill(1);
            etab.insert(etab.end(), e.begin(), e.end());
        }
        if (etab.size() > (size_t)kMaxRankSamples) etab.clear();  // over the LDS budget: generic kernel
        F->rnetab = (int32_t)etab.size();
    }
    // one whole +inf segment past the end: k_zfill_grouped_w3 reads a segment of every
    // searched feature unconditionally (a feature without thresholds points here)
    for (int j = 0; j < 16; ++j) useg.push_back(INFINITY);
    if (smp.empty()) smp.push_back(INFINITY);
    // integer / ratio rank tables of the scoring pipeline's prepares (the v1 row format: one
    // slot per feature): the same float64 scaling and float32 cast as zval(), then the
    // lower_bound the device search computes (bit-identical arithmetic on the host)
    itab.assign((size_t)16 * kIntTab, 0);
    rat.assign((size_t)16 * kRatN * kRatN, 0);
    for (int f = 0; f < 16 && f < F->n_features && (!v2 || F->rank_identity); ++f) {
        const float *u0 = RL.thr.data() + RL.thr_off[f], *u1 = RL.thr.data() + RL.thr_off[f + 1];
        const double *mean = F->h_mean.empty() ? nullptr : F->h_mean.data();
        const double *scale = F->h_scale.empty() ? nullptr : F->h_scale.data();
        for (int c = 0; c < kIntTab; ++c) {
            double x = (double)c;
            if (mean) x = x - mean[f];
            if (scale) x = x / scale[f];
            itab[(size_t)f * kIntTab + c] = (uint16_t)(std::lower_bound(u0, u1, (float)x) - u0);
        }
        for (int nb = 0; nb < kRatN; ++nb)  // term_risk(): nb > 0 ? fr / nb : 0.0
            for (int fr = 0; fr < kRatN; ++fr) {
                double x = nb > 0 ? (double)fr / (double)nb : 0.0;
                if (mean) x = x - mean[f];
                if (scale) x = x / scale[f];
                rat[((size_t)f * kRatN + nb) * kRatN + fr] = (uint16_t)(std::lower_bound(u0, u1, (float)x) - u0);
            }
    }
    const size_t rn = RL.nodes.size(), nt = (size_t)F->n_trees, nthr = std::max<size_t>(RL.thr.size(), 1);
    FDX_HIP(hipMalloc(&F->rnodes_d, 4 * rn));
    FDX_HIP(hipMalloc(&F->rorig_d, 4 * rn));
    FDX_HIP(hipMalloc(&F->rlval_d, 8 * rn));
    FDX_HIP(hipMalloc(&F->rml_d, rn));
    FDX_HIP(hipMalloc(&F->rroot_d, 4 * nt));
    FDX_HIP(hipMalloc(&F->rdepth_d, 4 * nt));
    FDX_HIP(hipMalloc(&F->rthr_d, 4 * nthr));
    FDX_HIP(hipMalloc(&F->rseg_d, 4 * useg.size()));
    FDX_HIP(hipMalloc(&F->rsmp_d, 4 * smp.size()));
    FDX_HIP(hipMalloc(&F->ritab_d, 2 * itab.size()));
    FDX_HIP(hipMalloc(&F->rrat_d, 2 * rat.size()));
    FDX_HIP(hipMemcpyAsync(F->rseg_d, useg.data(), 4 * useg.size(), hipMemcpyHostToDevice, st));
    FDX_HIP(hipMemcpyAsync(F->rsmp_d, smp.data(), 4 * smp.size(), hipMemcpyHostToDevice, st));
    FDX_HIP(hipMemcpyAsync(F->ritab_d, itab.data(), 2 * itab.size(), hipMemcpyHostToDevice, st));
    FDX_HIP(hipMemcpyAsync(F->rrat_d, rat.data(), 2 * rat.size(), hipMemcpyHostToDevice, st));
    if (!etab.empty()) {
        FDX_HIP(hipMalloc(&F->retab_d, 4 * etab.size()));
        FDX_HIP(hipMemcpyAsync(F->retab_d, etab.data(), 4 * etab.size(), hipMemcpyHostToDevice, st));
    }
    FDX_HIP(hipMemcpyAsync(F->rnodes_d, RL.nodes.data(), 4 * rn, hipMemcpyHostToDevice, st));
    FDX_HIP(hipMemcpyAsync(F->rorig_d, RL.orig.data(), 4 * rn, hipMemcpyHostToDevice, st));
    FDX_HIP(hipMemcpyAsync(F->rlval_d, RL.lval.data(), 8 * rn, hipMemcpyHostToDevice, st));
    FDX_HIP(hipMemcpyAsync(F->rml_d, RL.ml.data(), rn, hipMemcpyHostToDevice, st));
    FDX_HIP(hipMemcpyAsync(F->rroot_d, RL.root.data(), 4 * nt, hipMemcpyHostToDevice, st));
    FDX_HIP(hipMemcpyAsync(F->rdepth_d, RL.depth.data(), 4 * nt, hipMemcpyHostToDevice, st));
    if (!RL.thr.empty()) FDX_HIP(hipMemcpyAsync(F->rthr_d, RL.thr.data(), 4 * RL.thr.size(), hipMemcpyHostToDevice, st));
    FDX_HIP(hipStreamSynchronize(st));  // the host vectors die at return
    return FDX_OK;
}
}  // namespace
}  // namespace fdx

extern "C" int fdx_forest_create(const fdx_forest_desc *d, fdx_forest *out, void *stream) {
    FDX_REQUIRE(d && out, "null pointer");
    *out = nullptr;
    std::vector<uint64_t> packed;
    std::vector<int32_t> orig, root, depth;
    int rc = pack_forest(d, packed, orig, root, depth);
    if (rc) return rc;
    const int64_t total = (int64_t)packed.size();
    fdx_forest_s *F = new (std::nothrow) fdx_forest_s();
    FDX_REQUIRE(F, "out of host memory");
    F->n_trees = d->n_trees;
    F->n_features = d->n_features;
    F->zstride = d->n_features <= 16 ? 16 : 32;
    F->n_nodes = total;
    F->node_offsets.assign(d->node_offsets, d->node_offsets + d->n_trees + 1);
    F->h_packed = packed;
    F->h_orig = orig;
    F->h_depth = depth;
    if (d->scaler_mean) F->h_mean.assign(d->scaler_mean, d->scaler_mean + d->n_features);
    if (d->scaler_scale) F->h_scale.assign(d->scaler_scale, d->scaler_scale + d->n_features);
    hipStream_t st = as_stream(stream);
    auto fail = [&](hipError_t e, const char *what) {
        set_error("%s failed: %s", what, hipGetErrorString(e));
        fdx_forest_destroy(F);
        return FDX_E_HIP;
    };
    hipError_t e;
    {
        int dev = 0, ncu = 0;
        if ((e = hipGetDevice(&dev)) || (e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)))
            return fail(e, "hipDeviceGetAttribute");
        if (ncu > 0) F->n_cu = ncu;
    }
    // Rank layout choice: v1 when the forest fits it (measured fastest on MI355X for the bench
    // model: 8.06 vs 8.68 ms for the compact v2 planes, profiles/r02_v6_ab_*.json); else v2 (more
    // than 4,096 nodes under one threshold rank or ranks past 12 bits -- the deployed model);
    // else the wide 8-byte layout.  (fdx_forest_set_variant switches an existing forest to the
    // other rank format.)
    rc = install_rank_layout(F, false, st);
    if (rc == FDX_E_UNSUPPORTED) rc = install_rank_layout(F, true, st);
    if (rc == FDX_E_UNSUPPORTED) rc = FDX_OK;  // the wide layout serves it
    if (rc) {
        fdx_forest_destroy(F);
        return rc;
    }
    set_error("");
    // default kernel: the rank layout when the forest fits it, else the wide layout
    F->variant = !F->rank_ok ? 0
                             : (!F->rank_v2 ? kDefaultRankVariant
                                            : (F->rank_identity ? kDefaultRankCompactVariant : kDefaultRankV2Variant));
    build_chunks(F);
    if ((e = hipMalloc(&F->nodes_d, sizeof(uint64_t) * total)) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMalloc(&F->orig_d, sizeof(int32_t) * total)) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMalloc(&F->root_d, sizeof(int32_t) * d->n_trees)) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMalloc(&F->depth_d, sizeof(int32_t) * d->n_trees)) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMalloc(&F->chunk_t_d, sizeof(int32_t) * (d->n_trees + 1))) != hipSuccess) return fail(e, "hipMalloc");
    if ((e = hipMalloc(&F->chunk_base_d, sizeof(int64_t) * (d->n_trees + 1))) != hipSuccess)
        return fail(e, "hipMalloc");
    if ((e = hipMemcpyAsync(F->depth_d, depth.data(), sizeof(int32_t) * d->n_trees, hipMemcpyHostToDevice, st)))
        return fail(e, "hipMemcpyAsync");
    if ((e = hipMemcpyAsync(F->nodes_d, packed.data(), sizeof(uint64_t) * total, hipMemcpyHostToDevice, st)))
        return fail(e, "hipMemcpyAsync");
    if ((e = hipMemcpyAsync(F->orig_d, orig.data(), sizeof(int32_t) * total, hipMemcpyHostToDevice, st)))
        return fail(e, "hipMemcpyAsync");
    if ((e = hipMemcpyAsync(F->root_d, root.data(), sizeof(int32_t) * d->n_trees, hipMemcpyHostToDevice, st)))
        return fail(e, "hipMemcpyAsync");
    if (d->scaler_mean) {
        if ((e = hipMalloc(&F->mean_d, sizeof(double) * d->n_features))) return fail(e, "hipMalloc");
        if ((e = hipMemcpyAsync(F->mean_d, d->scaler_mean, sizeof(double) * d->n_features,
                                hipMemcpyHostToDevice, st)))
            return fail(e, "hipMemcpyAsync");
    }
    if (d->scaler_scale) {
        if ((e = hipMalloc(&F->scale_d, sizeof(double) * d->n_features))) return fail(e, "hipMalloc");
        if ((e = hipMemcpyAsync(F->scale_d, d->scaler_scale, sizeof(double) * d->n_features,
                                hipMemcpyHostToDevice, st)))
            return fail(e, "hipMemcpyAsync");
    }
    // host vectors die at return: make the uploads complete first
    if ((e = hipStreamSynchronize(st))) return fail(e, "hipStreamSynchronize");
    if (upload_chunks(F)) {
        fdx_forest_destroy(F);
        return FDX_E_HIP;
    }
    *out = F;
    return FDX_OK;
}

extern "C" int fdx_forest_destroy(fdx_forest F) {
    if (!F) return FDX_OK;
    (void)hipFree(F->nodes_d);
    (void)hipFree(F->orig_d);
    (void)hipFree(F->root_d);
    (void)hipFree(F->depth_d);
    (void)hipFree(F->chunk_t_d);
    (void)hipFree(F->chunk_base_d);
    free_rank_buffers(F);
    (void)hipFree(F->mean_d);
    (void)hipFree(F->scale_d);
    delete F;
    return FDX_OK;
}

extern "C" int fdx_forest_info(fdx_forest F, int32_t *n_trees, int32_t *n_features, int64_t *n_nodes,
                               int32_t *n_chunks) {
    FDX_REQUIRE(F, "null forest");
    if (n_trees) *n_trees = F->n_trees;
    if (n_features) *n_features = F->n_features;
    if (n_nodes) *n_nodes = F->n_nodes;
    if (n_chunks) *n_chunks = (int32_t)F->chunks.size();
    return FDX_OK;
}

// Batches of at most this many rows (a sequential chunk launch would leave CUs idle: one
// block per CU) run every LDS chunk at once and need per-tree values in the workspace.
static int64_t concurrent_rows(const fdx_forest_s *F) {
    if (!rank_mode(F)) return 0;
    const Variant v = kVariants[F->variant];
    return (int64_t)F->n_cu * v.block * v.rows / 2;
}

extern "C" size_t fdx_forest_workspace_size(fdx_forest F, int64_t n_rows);

// a workspace that serves every batch of up to n_rows rows at full speed
extern "C" size_t fdx_forest_workspace_size_max(fdx_forest F, int64_t n_rows) {
    if (!F || n_rows <= 0) return 256;
    const size_t a = fdx_forest_workspace_size(F, n_rows);
    const size_t b = fdx_forest_workspace_size(F, std::min<int64_t>(n_rows, concurrent_rows(F)));
    return a > b ? a : b;
}

// rows + running sums + NaN flag word: what every traversal needs
static size_t ws_base(const fdx_forest_s *F, int64_t n_rows) {
    return align_up(sizeof(float) * F->zstride * (size_t)n_rows) + align_up(sizeof(double) * (size_t)n_rows) + 256;
}

extern "C" size_t fdx_forest_workspace_size(fdx_forest F, int64_t n_rows) {
    if (!F || n_rows <= 0) return 256;
    size_t b = ws_base(F, n_rows);
    if (n_rows <= concurrent_rows(F) && F->chunks.size() > 1)
        b += align_up(sizeof(double) * (size_t)n_rows * F->n_trees);  // per-tree values
    return b;
}

static RankTab rank_tab(const fdx_forest_s *F) {
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

static int forest_ws(fdx_forest F, int64_t n, void *ws, size_t ws_bytes, float **z, double **acc,
                     int32_t **nan_flag = nullptr) {
    size_t need = ws_base(F, n);  // (a smaller batch's per-tree values are optional: see forest_traverse)
    if (!ws || ws_bytes < need) {
        set_error("forest workspace too small: %zu < %zu", ws_bytes, need);
        return FDX_E_WORKSPACE;
    }
    *z = reinterpret_cast<float *>(ws);
    *acc = reinterpret_cast<double *>(reinterpret_cast<char *>(ws) +
                                      align_up(sizeof(float) * F->zstride * (size_t)n));
    if (nan_flag)
        *nan_flag = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(*acc) + align_up(sizeof(double) * (size_t)n));
    return FDX_OK;
}

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
    if (rank_mode(F) && kVariants[F->variant].p16 == 2) {
        hipLaunchKernelGGL(k_prepare_v2, dim3(grid), dim3(256), 0, st, X_d, n, row_stride, col_stride, F->n_features,
                           F->mean_d, F->scale_d, reinterpret_cast<uint16_t *>(z), flag, rank_tab(F));
        FDX_LAUNCHED("k_prepare_v2");
        return FDX_OK;
    }
    FDX_PREP(k_prepare, dim3(grid), st, X_d, n, row_stride, col_stride, F->n_features, F->mean_d, F->scale_d,
             (void *)z, flag);
    FDX_LAUNCHED("k_prepare");
    return FDX_OK;
}

static int forest_traverse(fdx_forest F, int64_t n, double *proba_d, const int32_t *out_perm_d,
                           int32_t *leaf_d, void *ws, size_t ws_bytes, void *stream) {
    FDX_REQUIRE(F, "null forest");
    FDX_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(proba_d, "null pointer");
    float *z;
    double *acc;
    int32_t *flag;
    int rc = forest_ws(F, n, ws, ws_bytes, &z, &acc, &flag);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    if (rank_mode(F)) {
        const size_t nc = F->chunks.size();
        const uint16_t *zr = reinterpret_cast<const uint16_t *>(z);
        // small batch: all chunks in one launch (grid.y = chunk) + k_tree_sum
        double *tv = nullptr;
        if (nc > 1 && n <= concurrent_rows(F) && ws_bytes >= fdx_forest_workspace_size(F, n))
            tv = reinterpret_cast<double *>(reinterpret_cast<char *>(acc) + align_up(sizeof(double) * (size_t)n) + 256);
        for (size_t c = 0; c < (tv ? 1 : nc); ++c) {
            const auto &ch = F->chunks[c];
            const int first = c == 0, last = c + 1 == nc;
#define FDX_LAUNCH_RANK(B, R, G, P, PIPE)                                                                      \
    do {                                                                                                      \
        const int64_t tiles_ = ceil_div(n, (int64_t)(B) * (R));                                               \
        const dim3 grid(tv ? (unsigned)tiles_ : (unsigned)std::min<int64_t>(tiles_, F->n_cu), tv ? (unsigned)nc : 1u); \
        hipLaunchKernelGGL((k_forest_rank<B, R, G, P, PIPE>), grid, dim3(B), 0, st, F->rnodes_d, ch.node_base,    \
                           (int32_t)ch.nodes, F->rroot_d, F->rdepth_d, ch.t0, ch.t1, zr, flag, (int64_t)0, n,       \
                           F->rlval_d, F->rml_d, acc, proba_d, out_perm_d, leaf_d, F->rorig_d, F->n_trees, first,  \
                           last, F->chunk_t_d, F->chunk_base_d, tv, n);                                           \
    } while (0)
            switch (F->variant) {
                case 2: FDX_LAUNCH_RANK(1024, 1, 6, 2, 2); break;
                case 3: FDX_LAUNCH_RANK(1024, 1, 6, 3, 2); break;
                case 4: FDX_LAUNCH_RANK(1024, 1, 10, 2, 2); break;
                case 5: FDX_LAUNCH_RANK(1024, 1, 8, 3, 2); break;
                case 6: FDX_LAUNCH_RANK(1024, 1, 10, 3, 2); break;
                default: FDX_LAUNCH_RANK(1024, 1, 10, 0, 2); break;
            }
#undef FDX_LAUNCH_RANK
            FDX_LAUNCHED("k_forest_rank");
        }
        if (tv) {
            hipLaunchKernelGGL(k_tree_sum, dim3(stream_grid(n, 256, 4096)), dim3(256), 0, st, tv, n, F->n_trees,
                               out_perm_d, proba_d);
            FDX_LAUNCHED("k_tree_sum");
        }
        return FDX_OK;
    }
    // wide layout: k_forest_chunk, one launch per chunk (an oversized tree runs from global memory)
    const size_t nc = F->chunks.size();
    for (size_t c = 0; c < nc; ++c) {
        const auto &ch = F->chunks[c];
        const int first = c == 0, last = c + 1 == nc;
#define FDX_LAUNCH_CHUNK(FS, L)                                                                              \
    hipLaunchKernelGGL((k_forest_chunk<FS, L, 512, 1, 4>), dim3((unsigned)std::min<int64_t>(ceil_div(n, 512), 1024)), \
                       dim3(512), 0, st, F->nodes_d, ch.node_base, (int32_t)ch.nodes, F->root_d, F->depth_d, ch.t0,  \
                       ch.t1, z, flag, (int64_t)0, n, acc, proba_d, out_perm_d, leaf_d, F->orig_d, F->n_trees, first, \
                       last)
        if (F->zstride == 16) {
            if (ch.in_lds) FDX_LAUNCH_CHUNK(16, true); else FDX_LAUNCH_CHUNK(16, false);
        } else {
            if (ch.in_lds) FDX_LAUNCH_CHUNK(32, true); else FDX_LAUNCH_CHUNK(32, false);
        }
#undef FDX_LAUNCH_CHUNK
        FDX_LAUNCHED("k_forest_chunk");
    }
    return FDX_OK;
}

extern "C" int fdx_forest_traverse(fdx_forest F, int64_t n, double *proba_d, int32_t *leaf_d, void *ws,
                                   size_t ws_bytes, void *stream) {
    return forest_traverse(F, n, proba_d, nullptr, leaf_d, ws, ws_bytes, stream);
}

extern "C" int fdx_forest_traverse_perm(fdx_forest F, int64_t n, double *proba_d, const int32_t *out_perm_d,
                                        int32_t *leaf_d, void *ws, size_t ws_bytes, void *stream) {
    return forest_traverse(F, n, proba_d, out_perm_d, leaf_d, ws, ws_bytes, stream);
}

extern "C" int fdx_forest_predict(fdx_forest F, const double *X_d, int64_t n, int64_t row_stride,
                                  int64_t col_stride, double *proba_d, int32_t *leaf_d, void *ws,
                                  size_t ws_bytes, void *stream) {
    int rc = fdx_forest_prepare(F, X_d, n, row_stride, col_stride, ws, ws_bytes, stream);
    if (rc) return rc;
    return fdx_forest_traverse(F, n, proba_d, leaf_d, ws, ws_bytes, stream);
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
    FDX_REQUIRE(!(rank_mode(F) && kVariants[F->variant].p16 == 2),
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
    FDX_REQUIRE(!(rank_mode(F) && kVariants[F->variant].p16 == 2),
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
    FDX_REQUIRE(!(rank_mode(F) && kVariants[F->variant].p16 == 2),
                "the fused scoring rows need the v1 row format (one slot per feature)");
    FDX_REQUIRE(n >= 0 && n_windows >= 1 && n_windows <= FDX_MAX_WINDOWS, "bad argument");
    FDX_REQUIRE(flags_mode == FDX_FLAGS_NOTEBOOK || flags_mode == FDX_FLAGS_SPARK, "bad flags mode");
    FDX_REQUIRE(F->n_features == 3 + 4 * n_windows, "forest has %d features, expected %d", F->n_features,
                3 + 4 * n_windows);
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(cust_ts_d && cust_amount_d && cust_nb_d && cust_avg_d && term_rec_d, "null pointer");
    FDX_REQUIRE((cust_val_is_sum & ~5) == 0, "cust_val_is_sum: FDX_PREP_VAL_IS_SUM | FDX_PREP_TERM_COMPACT only");
    FDX_REQUIRE(!(cust_val_is_sum & 4) || (n_windows == 3 && ((uintptr_t)term_rec_d & 15) == 0),
                "compact terminal records: W = 3 and a 16-byte aligned record array");
    float *z;
    double *acc;
    int32_t *flag;
    int rc = forest_ws(F, n, ws, ws_bytes, &z, &acc, &flag);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    FDX_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), st));
    const unsigned grid = stream_grid(n, 256);
    const RankTab rt = rank_tab(F);
    if (rank_mode(F) && n_windows == 3 && F->rseg == 16 && rt.rat && rt.etab) {
#define FDX_ZFILL_W3(E)                                                                                          \
    hipLaunchKernelGGL(k_zfill_grouped_w3<E>, dim3(grid), dim3(256), 0, st, cust_ts_d, cust_amount_d, cust_nb_d,   \
                       cust_avg_d, cust_perm_d, term_inv_d, term_rec_d, n, flags_mode, cust_val_is_sum, F->mean_d, \
                       F->scale_d, (void *)z, flag, rt, reinterpret_cast<char *>(rows_out_d), out_cap)
        if (!rows_out_d)
            FDX_ZFILL_W3(0);
        else if (rows_order == FDX_ROWS_SLOT_ORDER)
            FDX_ZFILL_W3(FDX_ROWS_SLOT_ORDER);
        else
            FDX_ZFILL_W3(FDX_ROWS_INPUT_ORDER);
#undef FDX_ZFILL_W3
        FDX_LAUNCHED("k_zfill_grouped_w3");
        return FDX_OK;
    }
    FDX_REQUIRE(!rows_out_d, "feature rows: n_windows = 3, compact terminal records and the rank layout only");
    FDX_PREP(k_zfill_grouped, dim3(grid), st, cust_ts_d, cust_amount_d, cust_nb_d, cust_avg_d, cust_perm_d,
             term_inv_d, term_rec_d, n, n_windows, flags_mode, cust_val_is_sum, F->mean_d, F->scale_d, (void *)z, flag);
    FDX_LAUNCHED("k_zfill_grouped");
    return FDX_OK;
}
