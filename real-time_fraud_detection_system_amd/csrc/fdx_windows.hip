// fdx_windows.hip -- K1: time flags, customer spending windows, terminal delayed-risk
// windows on gfx950.  HBM-bound integer/FP64 scan work (no MFMA: nothing here is a
// contraction).
//
// Reference behaviour (see include/fdx.h for the per-entry citations):
//   flags     feature_transformation.ipynb:246-253, :294-301; fraud_detection.py:103-104
//   customer  feature_transformation.ipynb:601-628 (pandas rolling('{w}d').sum()/count())
//   terminal  feature_transformation.ipynb:1495-1522 (rolling(delay) vs rolling(delay+w))
#include <cstdlib>
#include <type_traits>

#include "fdx_internal.h"

namespace fdx {
namespace {

constexpr int64_t kNsPerDay = 86400LL * 1000000000LL;
constexpr int64_t kNsPerHour = 3600LL * 1000000000LL;

__device__ __forceinline__ int64_t floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

// ----------------------------------------------------------------------------- flags
// 8 rows per thread: 64 B of timestamps in, 8 B per flag array out (one u64 store each).
__global__ void __launch_bounds__(256) k_time_flags(const int64_t *__restrict__ ts, int64_t n,
                                                    int32_t mode, uint8_t *__restrict__ weekend,
                                                    uint8_t *__restrict__ night) {
    const int64_t n8 = n / 8;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n8; g += stride) {
        const int64_t *p = ts + g * 8;
        uint64_t we = 0, ni = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            int64_t t = p[k];
            int64_t day = floor_div(t, kNsPerDay);
            int64_t hour = (t - day * kNsPerDay) / kNsPerHour;
            int64_t wd = (day + 3) % 7;  // Monday=0 (1970-01-01 was a Thursday); day may be < 0
            if (wd < 0) wd += 7;
            bool w, nt;
            if (mode == FDX_FLAGS_NOTEBOOK) {
                w = wd >= 5;
                nt = hour <= 6;
            } else {
                int64_t dow = ((wd + 1) % 7) + 1;  // Spark dayofweek: Sunday=1 .. Saturday=7
                w = dow >= 5;
                nt = hour >= 20;
            }
            we |= (uint64_t)w << (8 * k);
            ni |= (uint64_t)nt << (8 * k);
        }
        reinterpret_cast<uint64_t *>(weekend)[g] = we;
        reinterpret_cast<uint64_t *>(night)[g] = ni;
    }
    // tail (< 8 rows) handled by block 0
    if (blockIdx.x == 0 && threadIdx.x < (unsigned)(n - n8 * 8)) {
        int64_t i = n8 * 8 + threadIdx.x;
        int64_t t = ts[i];
        int64_t day = floor_div(t, kNsPerDay);
        int64_t hour = (t - day * kNsPerDay) / kNsPerHour;
        int64_t wd = (day + 3) % 7;
        if (wd < 0) wd += 7;
        if (mode == FDX_FLAGS_NOTEBOOK) {
            weekend[i] = wd >= 5;
            night[i] = hour <= 6;
        } else {
            int64_t dow = ((wd + 1) % 7) + 1;
            weekend[i] = dow >= 5;
            night[i] = hour >= 20;
        }
    }
}

// ------------------------------------------------------------------ customer windows
struct WinArgs {
    int64_t w[FDX_MAX_WINDOWS];
};

// pandas roll_sum state (aggregations.pyx add_sum/remove_sum/calc_sum), emulated exactly.
struct RollSum {
    double sum, c_add, c_rem, prev;
    int32_t nobs, nsame;

    __device__ __forceinline__ void reset(double first) {
        sum = 0.0; c_add = 0.0; c_rem = 0.0; prev = first; nobs = 0; nsame = 0;
    }
    __device__ __forceinline__ void add(double v) {
        if (v == v) {
            nobs += 1;
            double y = v - c_add;
            double t = sum + y;
            c_add = (t - sum) - y;
            sum = t;
            nsame = (v == prev) ? nsame + 1 : 1;
            prev = v;
        }
    }
    __device__ __forceinline__ void remove(double v) {
        if (v == v) {
            nobs -= 1;
            double y = -v - c_rem;
            double t = sum + y;
            c_rem = (t - sum) - y;
            sum = t;
        }
    }
    // calc_sum with min_periods = 1 (offset windows)
    __device__ __forceinline__ double value() const {
        if (nobs >= 1) return (nsame >= nobs) ? prev * (double)nobs : sum;
        return __builtin_nan("");
    }
};

// One lane per (segment, window).  The lane walks its segment in time order with a tail
// pointer, reproducing pandas' variable-window bounds (closed='right': rows j <= i with
// t_j > t_i - w) and its add/remove/reset schedule, so the sums are bit-identical.
// Lanes k*W .. k*W+W-1 share segment k, so their row loads hit the same cache lines.
__global__ void __launch_bounds__(256) k_customer_exact(
    const int64_t *__restrict__ ts, const double *__restrict__ amount,
    const int64_t *__restrict__ seg_off, int64_t n_seg, int64_t n, WinArgs win, int32_t n_win,
    int32_t *__restrict__ nb_out, double *__restrict__ avg_out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t seg = gid / n_win;
    if (seg >= n_seg) return;
    const int wi = (int)(gid - seg * n_win);
    const int64_t W = win.w[wi];
    const int64_t b = seg_off[seg], e = seg_off[seg + 1];
    int32_t *nb = nb_out + (int64_t)wi * n;
    double *avg = avg_out + (int64_t)wi * n;

    RollSum s;
    int64_t tail = b;
    for (int64_t i = b; i < e; ++i) {
        const int64_t t = ts[i];
        const double v = amount[i];
        if (i == b) {
            s.reset(v);
            s.add(v);
        } else {
            const int64_t bound = t - W;
            int64_t nt = tail;
            while (nt < i && ts[nt] <= bound) ++nt;
            if (nt >= i) {  // start[i] >= end[i-1]: pandas re-initialises the window
                s.reset(v);
                s.add(v);
            } else {
                for (int64_t j = tail; j < nt; ++j) s.remove(amount[j]);
                s.add(v);
            }
            tail = nt;
        }
        const double sum = s.value();
        nb[i] = s.nobs;
        avg[i] = sum / (double)s.nobs;
    }
}

// ------------------------------------------------- customer windows, interleaved layout
// The scoring pipeline's customer layout ("lane-major"): segments are ordered by length
// (longest first) and cut into groups of S = 64 / W segments; group g owns S * L_g slots
// (L_g = its longest segment) starting at goff[g], and row t of the group's segment l sits
// in slot goff[g] + t*S + l.  One wave walks one group: lane k = (segment l = k / W,
// window w = k % W) runs the exact pandas recurrence of its segment while the W lanes of a
// segment share every head load, and every wave instruction touches S consecutive slots
// (coalesced) instead of 64 unrelated streams.  Outputs use the same slot index; slots
// past a segment's end are padding (row index -1).

// key = LMAX - min(len, LMAX): a stable sort by it orders segments by decreasing length
__global__ void k_seg_len_keys(const int64_t *__restrict__ seg_off, int64_t n_seg, int32_t lmax,
                               int32_t *__restrict__ key) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_seg;
         s += (int64_t)gridDim.x * blockDim.x) {
        const int64_t L = seg_off[s + 1] - seg_off[s];
        key[s] = lmax - (int32_t)(L < lmax ? L : lmax);
    }
}

// slots of group g = S * length of its first (longest) segment
__global__ void k_group_slots(const int64_t *__restrict__ seg_off, const int32_t *__restrict__ sorder,
                              int64_t n_seg, int32_t S, int64_t n_groups, uint32_t *__restrict__ gslots) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_groups;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = sorder[g * S];
        gslots[g] = (uint32_t)(S * (seg_off[s + 1] - seg_off[s]));
    }
}

// The layout plan in ONE launch for up to kPlanMaxSeg segments (the radix plan is ~17 small
// launches, each shorter than its launch: ~0.3 ms of a step went to the host launching them).
// One block of 16 waves; wave w owns the segments [w*per, (w+1)*per) in index order, 64 per
// chunk, at most kPlanChunks chunks, and keeps their bins in registers.  The order is exactly the
// radix plan's -- decreasing length (clamped at 65535), ties by index:
//   * segments of >= kPlanBins-1 rows ("long", rare): collected in LDS and ranked exactly;
//   * the others: counting sort on bin = kPlanBins-1-length -- wave-private LDS counters, a
//     bin-major / wave-minor prefix, then each wave places its chunks in order: the lanes of
//     one bin find each other by ballot multisplit over the 11 bin bits, read the bin's counter,
//     and the lowest of them advances it;
// then the group slot counts (S x the group's first = longest segment) and their exclusive scan
// into goff[0..n_groups].  *status = 1: more long segments than kPlanMaxLong (the host then
// plans with the radix path).
constexpr int kPlanWaves = 16, kPlanChunks = 64, kPlanBins = 2048, kPlanBinBits = 11, kPlanMaxLong = 512;
constexpr int64_t kPlanMaxSeg = (int64_t)kPlanWaves * kPlanChunks * kWave;  // 65,536
constexpr int64_t kPlanMaxGroups = 3200;                                       // (>= 65,536 / 21)
__global__ void __launch_bounds__(kPlanWaves * kWave) k_layout_plan_small(const int64_t *__restrict__ seg_off,
                                                                          int64_t n_seg, int32_t S, int64_t n_groups,
                                                                          int32_t *__restrict__ sorder,
                                                                          uint32_t *__restrict__ goff,
                                                                          int32_t *__restrict__ status,
                                                                          int32_t *plan_host = nullptr) {
    // plan_host (fdx_customer_layout_plan_async): the caller's pinned [slots, status] words, written
    // from here at system scope -- no copy after the kernel (its blit waited ~70 us behind the
    // terminal scatter's higher-priority blocks for a CU, r06au trace)
    auto to_host = [&](int i, int32_t v) {
        if (plan_host) __hip_atomic_store(plan_host + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    };
    __shared__ uint32_t s_h[kPlanWaves][kPlanBins];
    __shared__ int32_t s_long[kPlanMaxLong];
    __shared__ int32_t s_nlong;
    __shared__ uint32_t s_part[kPlanWaves * kWave];
    __shared__ uint32_t s_gs[kPlanMaxGroups];  // group slot counts
    constexpr int kT = kPlanWaves * kWave;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    for (int e = tid; e < kPlanWaves * kPlanBins; e += kT) (&s_h[0][0])[e] = 0;
    if (tid == 0) s_nlong = 0;
    __syncthreads();
    const int64_t per = (n_seg + kPlanWaves - 1) / kPlanWaves;
    const int64_t lo = wv * per, hi = imin64(n_seg, lo + per);
    // (lengths clamped at 0: out-of-range ids, rejected after the step, can leave the offsets
    // out of order -- never an out-of-bounds counter)
    auto len_of = [&](int64_t sg) -> int64_t { return imax64(seg_off[sg + 1] - seg_off[sg], 0); };
    // 1. bins of this wave's chunks (kept in registers, two u16 per VGPR: 0xFFFF = none, 0 =
    // long), wave-private counts
    uint32_t binp[kPlanChunks / 2] = {};
    auto bin_at = [&](int c) -> int32_t {
        const int32_t v = (int32_t)((binp[c >> 1] >> (16 * (c & 1))) & 0xFFFFu);
        return v == 0xFFFF ? -1 : v;
    };
    constexpr int kBatch = 8;  // chunks whose offsets are loaded together (one load per segment:
                                // the next offset comes from the next lane, lane 63 loads it)
    const int n_chunks = (int)((imax64(hi - lo, 0) + kWave - 1) / kWave);  // this wave's
#pragma unroll
    for (int c0 = 0; c0 < kPlanChunks; c0 += kBatch) {
        if (c0 >= n_chunks) continue;  // (uniform; phase 3 skips these chunks too)
        int64_t a[kBatch], e63[kBatch];
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
            const int64_t sg = imin64(lo + (int64_t)(c0 + j) * kWave + lane, n_seg);
            a[j] = seg_off[sg];
            e63[j] = lane == kWave - 1 ? seg_off[imin64(sg + 1, n_seg)] : 0;
        }
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
            const int64_t sg = lo + (int64_t)(c0 + j) * kWave + lane;
            const int64_t nx = __shfl_down(a[j], 1, kWave);
            const int64_t L = imax64((lane == kWave - 1 ? e63[j] : nx) - a[j], 0);
            const int32_t bn = sg >= hi ? 0xFFFF : (L >= kPlanBins - 1 ? 0 : (int32_t)(kPlanBins - 1 - L));
            binp[(c0 + j) >> 1] |= (uint32_t)bn << (16 * ((c0 + j) & 1));
            if (sg < hi) {
                if (bn == 0) {
                    const int at = atomicAdd(&s_nlong, 1);
                    if (at < kPlanMaxLong) s_long[at] = (int32_t)sg;
                } else {
                    atomicAdd(&s_h[wv][bn], 1u);
                }
            }
        }
    }
    __syncthreads();
    const int n_long = s_nlong;
    if (n_long > kPlanMaxLong) {  // uniform: the host falls back to the radix plan
        if (tid == 0) {
            *status = 1;
            to_host(0, 0);
            to_host(1, 1);
        }
        return;
    }
    // 2. exclusive prefix over (bin, wave) entries e = bin * 16 + wave, after the long segments
    constexpr int kE = kPlanWaves * kPlanBins, kPerT = kE / kT;
    uint32_t loc[kPerT], sum = 0;
#pragma unroll
    for (int j = 0; j < kPerT; ++j) {
        const int e = tid * kPerT + j;
        loc[j] = s_h[e % kPlanWaves][e / kPlanWaves];
        sum += loc[j];
    }
    s_part[tid] = sum;
    __syncthreads();
    for (int d = 1; d < kT; d <<= 1) {  // inclusive scan of the per-thread sums
        const uint32_t v = tid >= d ? s_part[tid - d] : 0u;
        __syncthreads();
        s_part[tid] += v;
        __syncthreads();
    }
    uint32_t run = s_part[tid] - sum + (uint32_t)n_long;
#pragma unroll
    for (int j = 0; j < kPerT; ++j) {
        const int e = tid * kPerT + j;
        s_h[e % kPlanWaves][e / kPlanWaves] = run;
        run += loc[j];
    }
    __syncthreads();
    // long segments: exact rank by (length desc, index asc), lengths clamped as the radix key
    for (int i = tid; i < n_long; i += kT) {
        const int32_t si = s_long[i];
        const int64_t li = imin64(len_of(si), 65535);
        int r = 0;
        for (int j = 0; j < n_long; ++j) {
            const int32_t sj = s_long[j];
            const int64_t lj = imin64(len_of(sj), 65535);
            r += (lj > li) || (lj == li && sj < si);
        }
        sorder[r] = si;
        if (r % S == 0) s_gs[r / S] = (uint32_t)(S * len_of(si));
    }
    // 3. each wave places its chunks in index order (chunks past the wave's range skipped:
    // uniform; the group index pos / S by a reciprocal multiply, exact for pos < 2^16)
    const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint32_t s_inv = (uint32_t)((0xFFFFFFFFull + (uint64_t)S) / (uint64_t)S);  // ceil(2^32 / S)
#pragma unroll
    for (int c = 0; c < kPlanChunks; ++c) {
        if (c >= n_chunks) continue;  // (not break: the loop stays unrolled, bin_at(c) static)
        const int32_t bn = bin_at(c);
        const bool valid = bn > 0;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < kPlanBinBits; ++bit) {
            const bool set = (bn >> bit) & 1;
            const uint64_t m = __ballot(set);
            peers &= set ? m : ~m;
        }
        // the counter's read (every lane of the bin) precedes the leader's update in the wave's
        // LDS instruction order, which the hardware keeps; no fence (a wavefront-scope fence
        // also waits for the global store below -- one HBM round trip per chunk)
        const uint32_t cnt = valid ? s_h[wv][bn] : 0u;
        if (valid) {
            const uint32_t below = (uint32_t)__popcll(peers & lt_mask);
            if (below == 0) s_h[wv][bn] = cnt + (uint32_t)__popcll(peers);
            const uint32_t pos = cnt + below;
            sorder[pos] = (int32_t)(lo + (int64_t)c * kWave + lane);
            const uint32_t grp = (uint32_t)(((uint64_t)pos * s_inv) >> 32);
            if (pos == grp * (uint32_t)S) s_gs[grp] = (uint32_t)(S * (kPlanBins - 1 - bn));  // a group's first
        }
    }
    __syncthreads();
    // 4. exclusive scan of the group slot counts (goff[n_groups] = total)
    const int64_t gper = (n_groups + kT - 1) / kT;
    const int64_t g0 = tid * gper, g1 = imin64(n_groups, g0 + gper);
    uint32_t gs = 0;
    for (int64_t g = g0; g < g1; ++g) gs += s_gs[g];
    // (a wave scan, then the 16 wave totals: 1 barrier instead of 20)
    uint32_t inc = gs;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t t = __shfl_up(inc, d, kWave);
        if (lane >= d) inc += t;
    }
    if (lane == kWave - 1) s_part[wv] = inc;
    __syncthreads();
    uint32_t wsum = 0;
    for (int w = 0; w < wv; ++w) wsum += s_part[w];
    uint32_t gr = wsum + inc - gs;
    for (int64_t g = g0; g < g1; ++g) {
        goff[g] = gr;
        gr += s_gs[g];
    }
    if (tid == kT - 1) {
        goff[n_groups] = wsum + inc;
        to_host(0, (int32_t)(wsum + inc));
    }
    if (tid == 0) {
        *status = 0;
        to_host(1, 0);
    }
}

// one block per group: slot (t, l) <- time-order row r = cperm[seg_off[s] + t]
// STARTS: the block then also computes every row's window starts (pandas' variable-window
// start, see k_customer_starts) -- one wave per segment, the segment's timestamps read back
// from the just-written slots (L2) into LDS, binary searches in LDS -- written
// segment-contiguous: starts[w * n_slots + goff[g] + l * Lg + t] (Lg = the group's longest
// segment), so both this writer and k_customer_walk's per-lane reads are contiguous.
// GROUPED: ts / amount are already in grouped order (fdx_rekey_payload carried them through
// the re-key): slot (t, l) reads ts[seg_off[s] + t] -- each segment a sequential stream --
// instead of ts[cperm[...]], a random HBM line per 8-byte element.
constexpr int kStartLds = 1024;  // segment rows staged per wave for the start searches
template <bool STARTS, bool GROUPED = false>
__global__ void __launch_bounds__(256) k_interleave(
    const int64_t *__restrict__ seg_off, const int32_t *__restrict__ sorder, const int32_t *__restrict__ cperm,
    const uint32_t *__restrict__ goff, int64_t n_seg, int32_t S, const int64_t *__restrict__ ts,
    const double *__restrict__ amount, int64_t *__restrict__ its, double *__restrict__ iamt,
    int32_t *__restrict__ irow, WinArgs win, int32_t n_win, int32_t *__restrict__ starts, int64_t n_slots) {
    __shared__ int64_t s_ts[STARTS ? 4 : 1][STARTS ? kStartLds : 1];
    const int64_t g = blockIdx.x;
    const int rows_per_iter = blockDim.x / S;
    const int l = threadIdx.x % S, tt = threadIdx.x / S;
    const int64_t s0 = sorder[g * S];
    const int64_t Lg = seg_off[s0 + 1] - seg_off[s0];
    const int64_t base = goff[g];
    if constexpr (STARTS && GROUPED) {
        // a tile = R rows of each of the group's S segments (R * S <= 1024 slots): loaded along
        // the segments (R consecutive rows each: whole lines, not the row-at-a-time form's 12
        // rows of 21 segments per wave load), transposed through LDS (the start phase's staging
        // arrays, free until then), written as R * S consecutive slots (0.371 -> 0.342 ms alone
        // at config 2, bit-equal, profiles/r04wxy_interleave_ab.txt)
        __shared__ int64_t s_sb[kWave];
        __shared__ int32_t s_sl[kWave];
        if ((int)threadIdx.x < S) {
            const int64_t si = g * S + threadIdx.x;
            const int64_t sx = si < n_seg ? sorder[si] : -1;
            s_sb[threadIdx.x] = sx >= 0 ? seg_off[sx] : 0;
            s_sl[threadIdx.x] = sx >= 0 ? (int32_t)(seg_off[sx + 1] - seg_off[sx]) : 0;
        }
        __syncthreads();
        int64_t *x_ts = s_ts[0];
        double *x_am = reinterpret_cast<double *>(s_ts[1]);
        int32_t *x_rw = reinterpret_cast<int32_t *>(s_ts[2]);
        const int R = kStartLds / S, TS = R * S;
        const uint32_t r_inv = ((1u << 20) + (uint32_t)R - 1) / (uint32_t)R;  // e / R = e * r_inv >> 20 (e * R < 2^20)
        constexpr int E = kStartLds / 256;
        for (int64_t t0 = 0; t0 < Lg; t0 += R) {
            int64_t vts[E];
            double vam[E];
            int32_t vr[E], xi[E];
            bool okv[E];
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const int e = j * 256 + (int)threadIdx.x;
                const bool valid = e < TS;
                const int ls = valid ? (int)(((uint32_t)e * r_inv) >> 20) : 0;
                const int r = e - ls * R;
                const int64_t t = t0 + r;
                const bool ok = valid && t < s_sl[ls];
                const int64_t k = ok ? s_sb[ls] + t : 0;  // row 0 stands in (n >= 1 here)
                vr[j] = cperm[k];
                vts[j] = ts[k];
                vam[j] = amount[k];
                okv[j] = ok;
                xi[j] = valid ? r * S + ls : e;  // (past TS: padding words, never read)
            }
#pragma unroll
            for (int j = 0; j < E; ++j) {
                x_ts[xi[j]] = okv[j] ? vts[j] : 0;
                x_am[xi[j]] = okv[j] ? vam[j] : 0.0;
                x_rw[xi[j]] = okv[j] ? vr[j] : -1;
            }
            __syncthreads();
            const int64_t lim = imin64(R, Lg - t0) * S;
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const int e = j * 256 + (int)threadIdx.x;
                if (e < lim) {
                    const int64_t slot = base + t0 * S + e;
                    its[slot] = x_ts[e];
                    iamt[slot] = x_am[e];
                    irow[slot] = x_rw[e];
                }
            }
            __syncthreads();
        }
    } else if (tt < rows_per_iter) {
        const int64_t si = g * S + l;
        const int64_t s = si < n_seg ? sorder[si] : -1;
        const int64_t b = s >= 0 ? seg_off[s] : 0;
        const int64_t L = s >= 0 ? seg_off[s + 1] - b : 0;
        // 4 rows per trip, every load issued before the first store (the loop is memory-latency
        // bound: one dependent load -> store round trip per row otherwise)
        constexpr int U = 4;
        for (int64_t t0 = tt; t0 < Lg; t0 += U * rows_per_iter) {
            int64_t vts[U];
            double vam[U];
            int32_t vr[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t t = t0 + (int64_t)u * rows_per_iter;
                vr[u] = t < L ? cperm[b + t] : -1;
                if (GROUPED) {
                    vts[u] = t < L ? ts[b + t] : 0;
                    vam[u] = t < L ? amount[b + t] : 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t t = t0 + (int64_t)u * rows_per_iter;
                if (!GROUPED) {
                    vts[u] = vr[u] >= 0 ? ts[vr[u]] : 0;
                    vam[u] = vr[u] >= 0 ? amount[vr[u]] : 0.0;
                }
                if (t < Lg) {
                    const int64_t slot = base + t * S + l;
                    its[slot] = vts[u];
                    iamt[slot] = vam[u];
                    irow[slot] = vr[u];
                }
            }
        }
    }
    if constexpr (STARTS) {
        if (!GROUPED) {  // the window starts read the timestamps back from the slots just written
            __threadfence_block();
            __syncthreads();
        }
        const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
        int64_t *lts = s_ts[wv];
        for (int ls = wv; ls < S; ls += (int)(blockDim.x / kWave)) {
            const int64_t si = g * S + ls;
            if (si >= n_seg) break;
            const int64_t sg = sorder[si];
            const int64_t L = seg_off[sg + 1] - seg_off[sg];
            // row t's ts: the grouped input (contiguous) or, gathering form, the slots just written
            const int64_t *gts = GROUPED ? ts + seg_off[sg] : its + base + ls;
            const int64_t gstride = GROUPED ? 1 : S;
            const bool in_lds = L <= kStartLds;
            if (in_lds && L > 0) {  // (an empty segment: nothing to stage or search)
                // the whole staged segment in one trip: every lane's 16 loads issued before its
                // first LDS store (a rolled loop waited on each load in turn: 0.41 -> 0.37 ms
                // alone at config 2, profiles/r04wxy_interleave_ab.txt); a row past the end
                // re-reads and re-stores the last row (the same value to the same word)
                constexpr int UF = kStartLds / kWave;
                int64_t v[UF];
#pragma unroll
                for (int j = 0; j < UF; ++j)
                    v[j] = __builtin_nontemporal_load(gts + (int64_t)min(lane + j * kWave, (int32_t)L - 1) * gstride);
#pragma unroll
                for (int j = 0; j < UF; ++j) lts[min(lane + j * kWave, (int32_t)L - 1)] = v[j];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // one loop per memory space (a load through `in_lds ? lds : global` compiles to a
            // flat load, which takes the vector-memory path even for LDS addresses), windows
            // unrolled (a runtime-indexed prev[] became a chain of v_cndmask per access)
            auto search = [&](auto T) {
                // (32-bit positions: a segment is < 2^31 rows; 64-bit index arithmetic doubled the
                // search's dependent instruction chain)
                int32_t prev[FDX_MAX_WINDOWS] = {};  // this lane's start of row t - 64: a lower bound (starts rise)
                for (int32_t t = lane; t < (int32_t)L; t += kWave) {
                    const int64_t tv = T(t);
#pragma unroll
                    for (int w = 0; w < FDX_MAX_WINDOWS; ++w) {
                        if (w < n_win) {
                            const int64_t bound = tv - win.w[w];
                            int32_t a = prev[w], e = t;  // first k in [prev, t] with ts_k > bound (k = t qualifies)
                            while (a < e) {
                                const int32_t m = (int32_t)((uint32_t)(a + e) >> 1);
                                if (T(m) > bound) e = m; else a = m + 1;
                            }
                            prev[w] = a;
                            starts[(int64_t)w * n_slots + base + (int64_t)ls * Lg + t] = a;
                        }
                    }
                }
            };
            if (in_lds)
                search([&](int64_t j) { return lts[j]; });
            else
                search([&](int64_t j) { return __builtin_nontemporal_load(gts + j * gstride); });
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
}

// One wave per group; the wave streams its group's rows through an LDS ring (coalesced
// chunk loads of C rows x S segments), so both the head row and the trailing rows that
// leave the window are read from LDS.  A trailing row older than the ring (window
// occupancy > kRing - kChunk rows) is copied from global memory instead (correct, slower).
constexpr int kChunk = 16;   // rows per cooperative load; divides every ring size below
// walk length classes: groups whose longest segment has >= kWalkSplitRows rows use the 256-row
// ring on the fork stream (fdx_customer_windows_walk)
// (r03 walk shapes: 3 waves per long group 0.94 ms, both classes split 1.08-1.11, one launch for
// every group 0.80, against 0.78 for this one: profiles/r03i_walk_shapes.jsonl, r03j_*)
constexpr int kWalkSplitRows = 480;
constexpr int kWalkLongWaves = 2;   // waves per group, long class (11 + 10 customers)
constexpr int kWalkShortWaves = 1;  // waves per group, short class
// rows per chunk of k_customer_walk: 8, not kChunk = 16 -- the per-chunk register arrays (outputs
// double-buffered over two chunks, window starts) take 116-124 VGPRs instead of 184-200, so a walk
// wave leaves room for other kernels' waves on its SIMD (the terminal re-key runs beside the walk):
// step minus forest 3.59-3.60 -> 3.56-3.57 ms on one box, the walk alone 0.72 -> 0.73 ms
// (profiles/r05aq_walk_chunk_ab.txt)
constexpr int kWalkChunk = 8;

// kRing rows per segment stay in LDS.  Launched once per ring size over length classes of
// groups (a block outside [lg_min, lg_max) exits at once): long segments belong to busy
// customers whose 30-day windows hold the most rows.
// The per-row work is straight-line: the tail loop removes rows as it advances (pandas
// first finds the new start, then removes rows [old start, new start) -- unless the
// window restarts, in which case the state is re-initialised; removing first and
// re-initialising afterwards leaves exactly the same state), and the re-initialisation is
// a predicated select, so a wave runs one instruction stream for its 1/7/30-day lanes.
// Memory schedule (the walk is a latency chain, so nothing in it may wait on HBM):
//  * the next chunk is loaded into registers while the current one is walked;
//  * a chunk's outputs are kept in registers and stored after its walk, alternating two
//    register sets, so no walk step overwrites a register an in-flight store still reads
//    (on gfx9 that forces a vmcnt wait);
//  * a ring miss copies the row into the lane's LDS miss slot, so the common path never
//    merges a pending global load into a VGPR.
template <int S_MAX, int kRing>
__global__ void __launch_bounds__(64) k_customer_ring(
    const int64_t *__restrict__ its, const double *__restrict__ iamt, const int64_t *__restrict__ seg_off,
    const int32_t *__restrict__ sorder, const uint32_t *__restrict__ goff, int64_t n_seg, int32_t S,
    int64_t n_slots, WinArgs win, int32_t n_win, int32_t *__restrict__ nb_out, double *__restrict__ sum_out,
    int32_t lg_min, int32_t lg_max) {
    static_assert(kRing % kChunk == 0, "ring holds whole chunks");
    constexpr int kPer = (kChunk * S_MAX + kWave - 1) / kWave;  // chunk elements per lane
    // ring rows [0, kRing) + one miss slot per lane
    constexpr int kRingEl = kRing * S_MAX + kWave;
    __shared__ int64_t r_ts[kRingEl];
    __shared__ double r_amt[kRingEl];
    const int lane = threadIdx.x;
    const int64_t g = blockIdx.x;
    const int64_t s0 = sorder[g * S];
    const int32_t Lg = (int32_t)(seg_off[s0 + 1] - seg_off[s0]);
    if (Lg < lg_min || Lg >= lg_max) return;  // another launch's length class
    const int l = lane / n_win, wi = lane - l * n_win;
    const int64_t si = g * S + l;
    const bool active = l < S && si < n_seg;
    const int64_t s = active ? sorder[si] : 0;
    const int32_t L = active ? (int32_t)(seg_off[s + 1] - seg_off[s]) : 0;
    int64_t W = win.w[0];  // select from the kernel arguments (no indexed load)
#pragma unroll
    for (int i = 1; i < FDX_MAX_WINDOWS; ++i) W = (active && wi == i) ? win.w[i] : W;
    const int64_t gbase = goff[g];
    const int64_t *g_ts = its + gbase + l;     // row t of this lane's segment: g_ts[t * S]
    const double *g_amt = iamt + gbase + l;
    int32_t *nb = nb_out + (int64_t)wi * n_slots + gbase + l;
    double *sm = sum_out + (int64_t)wi * n_slots + gbase + l;
    // chunk prefetch registers: element e = lane + j * 64 of a chunk is (row e / S, seg e % S)
    int64_t pts[kPer];
    double pam[kPer];
    auto fetch = [&](int32_t t0) {
        const int n_el = min(kChunk, Lg - t0) * S;
        const int64_t src0 = gbase + (int64_t)t0 * S;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int e = lane + j * kWave;
            if (e < n_el) {
                pts[j] = its[src0 + e];
                pam[j] = iamt[src0 + e];
            }
        }
    };
    auto commit = [&](int32_t t0) {
        const int n_el = min(kChunk, Lg - t0) * S;
        const int ring0 = t0 % kRing;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int e = lane + j * kWave;
            if (e < n_el) {
                const int tt = e / S, ll = e - tt * S;
                r_ts[(ring0 + tt) * S_MAX + ll] = pts[j];
                r_amt[(ring0 + tt) * S_MAX + ll] = pam[j];
            }
        }
    };
    // pandas roll_sum state (aggregations.pyx)
    double sum = 0.0, c_add = 0.0, c_rem = 0.0, prev = 0.0;
    int32_t nobs = 0, nsame = 0;
    int32_t tail = 0, tail_r = 0, head_r = 0;
    auto chunk = [&](int32_t t0, int32_t (&onb)[kChunk], double (&oval)[kChunk]) {
        commit(t0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (t0 + kChunk < Lg) fetch(t0 + kChunk);  // in flight while this chunk is walked
        const int32_t oldest = t0 + kChunk - kRing;  // first row still in the ring
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            const int32_t t = t0 + j;
            if (t < L) {
                const int64_t tv = r_ts[head_r * S_MAX + l];
                const double v = r_amt[head_r * S_MAX + l];
                const int64_t bound = tv - W;
                // advance the window start, removing each row that leaves (Kahan remove)
                while (tail < t) {
                    int e = tail_r * S_MAX + l;
                    if (tail < oldest) {  // older than the ring: via this lane's miss slot
                        e = kRing * S_MAX + lane;
                        r_ts[e] = g_ts[(int64_t)tail * S];
                        r_amt[e] = g_amt[(int64_t)tail * S];
                    }
                    const int64_t x = r_ts[e];
                    if (x > bound) break;
                    const double a = r_amt[e];
                    if (a == a) {
                        nobs -= 1;
                        const double y = -a - c_rem;
                        const double tt = sum + y;
                        c_rem = (tt - sum) - y;
                        sum = tt;
                    }
                    ++tail;
                    tail_r = tail_r + 1 == kRing ? 0 : tail_r + 1;
                }
                // start[i] >= end[i-1] (or i == 0): pandas re-initialises the window state
                if (tail >= t) {
                    sum = 0.0; c_add = 0.0; c_rem = 0.0; nobs = 0; nsame = 0; prev = v;
                }
                if (v == v) {  // Kahan add
                    nobs += 1;
                    const double y = v - c_add;
                    const double tt = sum + y;
                    c_add = (tt - sum) - y;
                    sum = tt;
                    nsame = (v == prev) ? nsame + 1 : 1;
                    prev = v;
                }
                onb[j] = nobs;
                oval[j] = nobs >= 1 ? ((nsame >= nobs) ? prev * (double)nobs : sum) : __builtin_nan("");
                head_r = head_r + 1 == kRing ? 0 : head_r + 1;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            if (t0 + j < L) {
                nb[(int64_t)(t0 + j) * S] = onb[j];
                sm[(int64_t)(t0 + j) * S] = oval[j];  // rolling SUM: the division by nb is the consumer's
            }
        }
    };
    int32_t nb_a[kChunk], nb_b[kChunk];
    double val_a[kChunk], val_b[kChunk];
    if (Lg > 0) fetch(0);
    for (int32_t t0 = 0; t0 < Lg; t0 += 2 * kChunk) {
        chunk(t0, nb_a, val_a);
        if (t0 + kChunk < Lg) chunk(t0 + kChunk, nb_b, val_b);
    }
}

// ---------------------------------------------------- customer windows, two-pass form
// Pass 1 (k_interleave<true, ...>, in the layout kernel): pandas' variable-window start of
//   every row, start_w(t) = first row j of the segment with ts_j > ts_t - W_w (closed='right').
// Pass 2 (k_customer_walk): the exact Kahan add/remove recurrence, one lane per (segment,
// window) -- the only sequential part -- free of timestamp compares: per row it removes
// rows [start(t-1), start(t)) (or re-initialises when start(t) == t) and adds row t.  Only
// the amounts ride in the LDS ring (8 B per row), so more waves fit per CU.
// starts: segment-contiguous (k_interleave<true>); nullptr = in nb_out, slot layout, overwritten
// by the counts.
// BUF: the per-row outputs stored by raw buffer stores, a lane past its segment's end given an
// out-of-range offset (the store is dropped) instead of a branch: behind a branch around stores,
// the next chunk's wait for its prefetched amounts had to assume the stores were skipped and
// waited for them too (vmcnt counts stores).  Needs the outputs within 2^31 bytes (the host picks).
typedef unsigned int fdx_u32x2 __attribute__((ext_vector_type(2)));
template <int S_MAX, int kRing, int P, bool BUF, int kChunk = fdx::kChunk>
__global__ void __launch_bounds__(64) k_customer_walk(
    const double *__restrict__ iamt, const int64_t *__restrict__ seg_off, const int32_t *__restrict__ sorder,
    const uint32_t *__restrict__ goff, int64_t n_seg, int32_t S, int64_t n_slots, int32_t n_win,
    int32_t *__restrict__ nb_out, double *__restrict__ sum_out, const int32_t *__restrict__ starts,
    int32_t lg_min = 0, int32_t lg_max = INT32_MAX) {
    static_assert((kRing & (kRing - 1)) == 0 && kRing % kChunk == 0, "power-of-two ring of whole chunks");
    constexpr int kPer = (kChunk * S_MAX + kWave - 1) / kWave;  // chunk elements per lane
    constexpr int kRingEl = kRing * S_MAX + kWave;             // + one miss slot per lane
    __shared__ double r_amt[kRingEl];
    const int lane = threadIdx.x;
    // P waves per group: wave h walks the group's segments [seg0, seg0 + Sw) (sorted by
    // decreasing length, so its first is its longest, Lw rows); the length class is the group's
    const int64_t g = blockIdx.x / P;
    const int h = (int)(blockIdx.x % P);
    const int Sh = (S + P - 1) / P, seg0 = h * Sh;
    const int64_t s0 = sorder[g * S];
    const int32_t Lg = (int32_t)(seg_off[s0 + 1] - seg_off[s0]);
    if (Lg < lg_min || Lg >= lg_max) return;  // another launch's length class
    if (seg0 >= S || g * S + seg0 >= n_seg) return;
    const int Sw = min(Sh, (int)imin64(S - seg0, n_seg - g * S - seg0));
    const int64_t sw0 = sorder[g * S + seg0];
    const int32_t Lw = (int32_t)(seg_off[sw0 + 1] - seg_off[sw0]);
    const int l = lane / n_win, wi = lane - l * n_win;
    const bool active = l < Sw;
    const int64_t s = active ? sorder[g * S + seg0 + l] : 0;
    const int32_t L = active ? (int32_t)(seg_off[s + 1] - seg_off[s]) : 0;
    const int64_t gbase = goff[g];
    const double *g_amt = iamt + gbase + seg0 + l;  // row t of this lane's segment: g_amt[t * S]
    int32_t *nb = nb_out + (int64_t)wi * n_slots + gbase + seg0 + l;
    double *sm = sum_out + (int64_t)wi * n_slots + gbase + seg0 + l;
    const int32_t n_out = (int32_t)imin64((int64_t)n_win * n_slots, INT32_MAX / 8);
    const __amdgpu_buffer_rsrc_t rnb = __builtin_amdgcn_make_buffer_rsrc(nb_out, (short)0, n_out * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsm = __builtin_amdgcn_make_buffer_rsrc(sum_out, (short)0, n_out * 8, 0x00020000);
    // chunk element e = lane + j * 64 of this wave's Sw segments: row e / Sw, segment e % Sw --
    // the same for every chunk, so its slot offset and ring position are computed once
    int32_t e_src[kPer], e_ring[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int e = lane + j * kWave;
        const int tt = e / Sw, ll = e - tt * Sw;
        e_src[j] = tt * S + ll;
        e_ring[j] = tt * S_MAX + ll;
    }
    double pam[kPer];
    int32_t pst[kChunk];
    auto fetch = [&](int32_t t0) {
        const int n_el = min(kChunk, Lw - t0) * Sw;
        const int64_t src0 = gbase + (int64_t)t0 * S + seg0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {  // (no branch: a conditional load's register merge waits for it)
            const int e = lane + j * kWave;
            pam[j] = iamt[src0 + (e < n_el ? e_src[j] : 0)];  // src0 is a slot of this wave's longest segment
        }
        if (starts) {
            const int32_t *sp = t0 < L ? starts + (int64_t)wi * n_slots + gbase + (int64_t)(seg0 + l) * Lg + t0 : starts;
#pragma unroll
            for (int j = 0; j < kChunk; ++j) pst[j] = sp[t0 + j < L ? j : 0];
        } else {
#pragma unroll
            for (int j = 0; j < kChunk; ++j)
                if (t0 + j < L) pst[j] = nb[(int64_t)(t0 + j) * S];
        }
    };
    // wave-uniform: has any amount this wave staged been NaN?  Every row a lane removes was staged
    // before (ring or not), so until then the removes need no NaN select (5 of the loop's 14 VALU)
    bool nan_seen = false;
    auto commit = [&](int32_t t0) {
        const int n_el = min(kChunk, Lw - t0) * Sw;
        const int ring0 = (t0 & (kRing - 1)) * S_MAX;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {  // elements past the chunk go to the lane's miss slot (scratch):
            const int e = lane + j * kWave;  // past the chunk, a ring row may still hold a live older row
            r_amt[e < n_el ? ring0 + e_ring[j] : kRing * S_MAX + lane] = pam[j];
        }
        bool nan_l = false;
#pragma unroll
        for (int j = 0; j < kPer; ++j) nan_l |= pam[j] != pam[j];
        nan_seen |= __builtin_amdgcn_ballot_w64(nan_l) != 0;
    };
    double sum = 0.0, c_add = 0.0, c_rem = 0.0, prev = 0.0;
    int32_t nobs = 0, nsame = 0, tail = 0;
    auto chunk = [&](int32_t t0, int32_t (&onb)[kChunk], double (&oval)[kChunk]) {
        int32_t cst[kChunk];
#pragma unroll
        for (int j = 0; j < kChunk; ++j) cst[j] = pst[j];
        commit(t0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int32_t oldest = t0 + kChunk - kRing;  // first row still in the ring
        // every row's amount and the first row it removes (its predecessor's start), read for the
        // whole chunk before the walk: the reads leave the add/remove chain, which otherwise waited
        // for an LDS round trip per row (the first removal from the miss slot stays in the loop)
        double pv[kChunk], pr[kChunk];
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            const int32_t r = j == 0 ? tail : cst[j - 1];
            pv[j] = r_amt[((t0 + j) & (kRing - 1)) * S_MAX + l];
            pr[j] = r_amt[r >= oldest ? (r & (kRing - 1)) * S_MAX + l : kRing * S_MAX + lane];
        }
        // (issued ahead of the next chunk's fetch: the branch around it keeps the compiler from
        // sinking row 0's reads into row 0's block, behind a full wait)
        if (t0 + kChunk < Lw) fetch(t0 + kChunk);  // in flight while this chunk is walked
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            const int32_t t = t0 + j;
            if (t < L) {
                const double v = pv[j];
                const int32_t st = cst[j];
                if (st >= t) {  // start[i] >= end[i-1] (or i == 0): pandas re-initialises
                    sum = 0.0; c_add = 0.0; c_rem = 0.0; nobs = 0; nsame = 0; prev = v;
                } else {
                    // rows [tail, st) leave the window (Kahan remove, in row order)
                    auto remove = [&](double a) {
                        if (a == a) {
                            nobs -= 1;
                            const double y = -a - c_rem;
                            const double tt = sum + y;
                            c_rem = (tt - sum) - y;
                            sum = tt;
                        }
                    };
                    int32_t k = tail;
                    for (; k < st && k < oldest; ++k) remove(g_amt[(int64_t)k * S]);  // older than the ring (rare)
                    if (k < st) {
                        // the ring rows, software-pipelined and branch-free: the next row's amount is
                        // read (in bounds whatever k) while this one is removed; the first was read
                        // with the chunk unless out-of-ring rows came before it
                        double a = k == tail ? pr[j] : r_amt[(k & (kRing - 1)) * S_MAX + l];
                        // settle it here: a read carried into the loop as pending makes the wait-count
                        // pass put lgkmcnt(0) -- the next read's too -- ahead of every trip's adds
                        __builtin_amdgcn_s_waitcnt(0xC07F);
                        if (!nan_seen) {
                            auto kahan = [&](double x) {
                                const double y = -x - c_rem;
                                const double tt = sum + y;
                                c_rem = (tt - sum) - y;
                                sum = tt;
                            };
                            nobs -= st - k;
                            // two rows a trip, the next two read ahead of the eight adds (rows past st
                            // are read in bounds and left unused)
                            double a1 = r_amt[((k + 1) & (kRing - 1)) * S_MAX + l];
                            for (; k + 1 < st; k += 2) {
                                const double n0 = r_amt[((k + 2) & (kRing - 1)) * S_MAX + l];
                                const double n1 = r_amt[((k + 3) & (kRing - 1)) * S_MAX + l];
                                __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the adds
                                kahan(a);
                                kahan(a1);
                                a = n0;
                                a1 = n1;
                            }
                            if (k < st) kahan(a);
                        } else {
                            for (; k < st; ++k) {
                                const double an = r_amt[((k + 1) & (kRing - 1)) * S_MAX + l];
                                __builtin_amdgcn_sched_barrier(0);
                                remove(a);
                                a = an;
                            }
                        }
                    }
                }
                tail = st;
                if (v == v) {  // Kahan add
                    nobs += 1;
                    const double y = v - c_add;
                    const double tt = sum + y;
                    c_add = (tt - sum) - y;
                    sum = tt;
                    nsame = (v == prev) ? nsame + 1 : 1;
                    prev = v;
                }
                onb[j] = nobs;
                oval[j] = nobs >= 1 ? ((nsame >= nobs) ? prev * (double)nobs : sum) : __builtin_nan("");
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if constexpr (BUF) {
            const uint32_t o0 = (uint32_t)((int64_t)wi * n_slots + gbase + seg0 + l);  // element index of row 0
#pragma unroll
            for (int j = 0; j < kChunk; ++j) {
                const bool ok = t0 + j < L;
                const uint32_t el = o0 + (uint32_t)(t0 + j) * (uint32_t)S;
                __builtin_amdgcn_raw_buffer_store_b32(onb[j], rnb, ok ? (int)(el * 4u) : (int)0x80000000, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(fdx_u32x2, oval[j]), rsm,
                                                      ok ? (int)(el * 8u) : (int)0x80000000, 0, 0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < kChunk; ++j) {
                if (t0 + j < L) {
                    nb[(int64_t)(t0 + j) * S] = onb[j];
                    sm[(int64_t)(t0 + j) * S] = oval[j];
                }
            }
        }
    };
    int32_t nb_a[kChunk], nb_b[kChunk];
    double val_a[kChunk], val_b[kChunk];
    if (Lw > 0) fetch(0);
    for (int32_t t0 = 0; t0 < Lw; t0 += 2 * kChunk) {
        chunk(t0, nb_a, val_a);
        if (t0 + kChunk < Lw) chunk(t0 + kChunk, nb_b, val_b);
    }
}

// ------------------------------------------------ customer windows, scan mode
// The averages from float64 prefix sums instead of pandas' sequential Kahan add/remove
// recurrence: fully parallel, one wave per segment.  Counts are exact; sums agree with pandas
// to ~1e-13 relative (the prefix magnitude over the window sum times 2^-52; tests use rtol
// 1e-10); pandas' "n equal values -> prev * n" rule is not applied.  Per segment (grouped,
// time-sorted rows): E[j] = sum of the non-NaN amounts of rows [0, j), C[j] = their count
// (wave scans of 64 rows + carry; LDS for segments <= kScanLds rows, else the segment's
// range of the global scratch), ts staged in LDS alike.  Row t, window w:
//   start = first j in [0, t] with ts_j > ts_t - W_w   (pandas closed='right')
//   NB = C[t+1] - C[start],  SUM = E[t+1] - E[start]   (NaN when NB == 0)
// Output position: slot goff[si / S] + t*S + si % S of the interleaved layout (sorder given,
// segment s = sorder[si]) -- val = SUM, the walk's outputs -- or grouped position
// seg_off[s] + t -- val = SUM / NB (val_is_sum = 0) or SUM.
constexpr int kScanLds = 1024;
__global__ void __launch_bounds__(64) k_customer_scan(
    const int64_t *__restrict__ gts, const double *__restrict__ gamt, const int64_t *__restrict__ seg_off,
    int64_t n_seg, const int32_t *__restrict__ sorder, const uint32_t *__restrict__ goff, int32_t S, int64_t n_out,
    WinArgs win, int32_t n_win, int32_t *__restrict__ nb_out, double *__restrict__ val_out, int val_is_sum,
    double *__restrict__ ge, int32_t *__restrict__ gc) {
    __shared__ int64_t s_ts[kScanLds];
    __shared__ double s_e[kScanLds + 1];
    __shared__ int32_t s_c[kScanLds + 1];
    const int lane = threadIdx.x;
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    for (int64_t si = blockIdx.x; si < n_seg; si += gridDim.x) {
        const int64_t s = sorder ? sorder[si] : si;
        const int64_t b = seg_off[s], L = seg_off[s + 1] - b;
        if (L <= 0) continue;
        const bool in_lds = L <= kScanLds;
        const int64_t *T = gts + b;
        const int64_t obase = sorder ? (int64_t)goff[si / S] + si % S : b;
        const int64_t ostride = sorder ? S : 1;
        // E / C: L + 1 entries in LDS or in the segment's scratch range; the body is expanded once
        // per memory space (through a runtime-selected pointer every access is a flat one)
        auto body = [&](double *E, int32_t *C, auto ts_at) {
            if (lane == 0) {
                E[0] = 0.0;
                C[0] = 0;
            }
            double carry = 0.0;
            int32_t ccarry = 0;
            for (int64_t t0 = 0; t0 < L; t0 += kWave) {
                const int64_t t = t0 + lane;
                double v = 0.0;
                int32_t c = 0;
                if (t < L) {
                    const double a = gamt[b + t];
                    if (in_lds) s_ts[t] = T[t];
                    if (a == a) {
                        v = a;
                        c = 1;
                    }
                }
#pragma unroll
                for (int d = 1; d < kWave; d <<= 1) {
                    const double u = __shfl_up(v, d, kWave);
                    const int32_t uc = __shfl_up(c, d, kWave);
                    if (lane >= d) {
                        v += u;
                        c += uc;
                    }
                }
                const double e = carry + v;
                const int32_t cc = ccarry + c;
                if (t < L) {
                    E[t + 1] = e;
                    C[t + 1] = cc;
                }
                carry = __shfl(e, kWave - 1, kWave);
                ccarry = __shfl(cc, kWave - 1, kWave);
            }
            if (!in_lds) __threadfence();  // this wave's scratch writes before its reads below
            wave_sync();
            int64_t prev[FDX_MAX_WINDOWS] = {};  // this lane's start of row t - 64: a lower bound
            for (int64_t t = lane; t < L; t += kWave) {
                const int64_t tv = ts_at(t);
                const double et = E[t + 1];
                const int32_t ct = C[t + 1];
#pragma unroll
                for (int w = 0; w < FDX_MAX_WINDOWS; ++w) {
                    if (w < n_win) {
                        const int64_t bound = tv - win.w[w];
                        int64_t a = prev[w], e = t;  // first j in [prev, t] with ts_j > bound (j = t qualifies)
                        while (a < e) {
                            const int64_t m = (a + e) >> 1;
                            if (ts_at(m) > bound) e = m; else a = m + 1;
                        }
                        prev[w] = a;
                        const int32_t nb = ct - C[a];
                        const double sum = nb > 0 ? et - E[a] : __builtin_nan("");
                        const int64_t o = (int64_t)w * n_out + obase + t * ostride;
                        nb_out[o] = nb;
                        val_out[o] = val_is_sum ? sum : sum / (double)nb;
                    }
                }
            }
        };
        if (in_lds)
            body(s_e, s_c, [&](int64_t j) { return s_ts[j]; });
        else
            body(ge + b + s, gc + b + s, [&](int64_t j) { return T[j]; });
        wave_sync();
    }
}

// Slot form of the scan mode, in two coalesced passes around the layout's window starts
// (k_interleave<true, true>, segment-contiguous): k_seg_prefix writes every segment's E / C
// (grouped order, E[seg_off[s] + s + j], one wave per segment), then k_scan_slots -- one
// block per group of S segments, threads over slots (t, l) as k_interleave's copy -- reads
// the starts and four prefix entries per window and writes NB / SUM by slot, coalesced.
__global__ void __launch_bounds__(256) k_seg_prefix(const double *__restrict__ gamt, const int64_t *__restrict__ seg_off,
                                                    int64_t n_seg, double *__restrict__ ge, int32_t *__restrict__ gc) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
    const int64_t nw = (int64_t)gridDim.x * blockDim.x / kWave;
    for (int64_t s = w0; s < n_seg; s += nw) {
        const int64_t b = seg_off[s], L = seg_off[s + 1] - b;
        double *E = ge + b + s;
        int32_t *C = gc + b + s;
        if (lane == 0) {
            E[0] = 0.0;
            C[0] = 0;
        }
        double carry = 0.0;
        int32_t ccarry = 0;
        for (int64_t t0 = 0; t0 < L; t0 += kWave) {
            const int64_t t = t0 + lane;
            double v = 0.0;
            int32_t c = 0;
            if (t < L) {
                const double a = gamt[b + t];
                if (a == a) {
                    v = a;
                    c = 1;
                }
            }
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const double u = __shfl_up(v, d, kWave);
                const int32_t uc = __shfl_up(c, d, kWave);
                if (lane >= d) {
                    v += u;
                    c += uc;
                }
            }
            const double e = carry + v;
            const int32_t cc = ccarry + c;
            if (t < L) {
                E[t + 1] = e;
                C[t + 1] = cc;
            }
            carry = __shfl(e, kWave - 1, kWave);
            ccarry = __shfl(cc, kWave - 1, kWave);
        }
    }
}

__global__ void __launch_bounds__(256) k_scan_slots(
    const int64_t *__restrict__ seg_off, const int32_t *__restrict__ sorder, const uint32_t *__restrict__ goff,
    int64_t n_seg, int32_t S, int64_t n_slots, int32_t n_win, const int32_t *__restrict__ starts,
    const double *__restrict__ ge, const int32_t *__restrict__ gc, int32_t *__restrict__ nb_out,
    double *__restrict__ sum_out) {
    const int64_t g = blockIdx.x;
    const int rows_per_iter = blockDim.x / S;
    const int l = threadIdx.x % S, tt = threadIdx.x / S;
    if (tt >= rows_per_iter) return;
    const int64_t s0 = sorder[g * S];
    const int64_t Lg = seg_off[s0 + 1] - seg_off[s0];
    const int64_t base = goff[g];
    const int64_t si = g * S + l;
    if (si >= n_seg) return;
    const int64_t s = sorder[si];
    const int64_t b = seg_off[s], L = seg_off[s + 1] - b;
    const double *E = ge + b + s;
    const int32_t *C = gc + b + s;
    for (int64_t t = tt; t < L; t += rows_per_iter) {
        const double et = E[t + 1];
        const int32_t ct = C[t + 1];
        for (int w = 0; w < n_win; ++w) {
            const int32_t st = starts[(int64_t)w * n_slots + base + (int64_t)l * Lg + t];
            const int32_t nb = ct - C[st];
            const int64_t o = (int64_t)w * n_slots + base + t * S + l;
            nb_out[o] = nb;
            sum_out[o] = nb > 0 ? et - E[st] : __builtin_nan("");
        }
    }
}

// ------------------------------------------------------------------ terminal windows
constexpr int kTermBlock = 256;
constexpr int kTermWaves = kTermBlock / kWave;
constexpr int kTermLdsRows = 1024;  // rows of one segment staged per wave (12 KB)
// The short-segment pass: segments of <= kTermShortRows rows run in a kernel with a 256-row
// stage (3 KB per wave instead of 12: about twice the resident waves for this latency-bound
// kernel), the longer ones in a second launch with the full stage (see terminal_launch).
constexpr int kTermShortRows = 256;


__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        int u = __shfl_up(v, d, kWave);
        if (lane >= d) v += u;
    }
    return v;
}

// Output either column-major (nb_out/risk_out [W][n], grouped order) or, when rec_out !=
// nullptr, one count record per row (W words NB | FRAUD << 32, see fdx.h) at rec_out[row].
__device__ __forceinline__ void term_store(int32_t *nb_out, double *risk_out, int64_t *rec_out, int64_t n,
                                           int32_t n_win, int64_t q, int64_t row, int w, int32_t cnt,
                                           int32_t fr) {
    if (rec_out) {
        rec_out[row * n_win + w] = term_word(cnt, fr);
    } else {
        nb_out[(int64_t)w * n + q] = cnt;
        risk_out[(int64_t)w * n + q] = cnt > 0 ? (double)fr / (double)cnt : 0.0;
    }
}

// Run starts (RUNS: wherever ts descends) kept per wave: kMaxRuns in s_runs for segments
// staged in LDS; a long segment does not use the LDS stage, so its run list takes the stage's
// timestamp words instead (kMaxRunsLong entries).
constexpr int kMaxRuns = 64;

// One row's window counts out: the compact W = 3 record (+ the full record in the overflow
// area), the 24-byte record as two stores (8 + 16 or 16 + 8 bytes by its 16-byte alignment:
// fewer random write transactions than three), or the general forms of term_store.
__device__ __forceinline__ void term_emit(int32_t *nb_out, double *risk_out, int64_t *rec_out, int64_t n,
                                          int32_t n_win, int64_t compact_n, int64_t q, int64_t row,
                                          const int32_t (&cn)[FDX_MAX_WINDOWS], const int32_t (&cf)[FDX_MAX_WINDOWS]) {
    if (compact_n > 0) {
        const bool fits = cn[0] <= kCompactMax && cn[1] <= kCompactMax && cn[2] <= kCompactMax;
        int64_t lo, hi;
        if (fits) {
            lo = (int64_t)cn[0] | ((int64_t)cn[1] << kCompactBits) | ((int64_t)cn[2] << (2 * kCompactBits));
            hi = (int64_t)cf[0] | ((int64_t)cf[1] << kCompactBits) | ((int64_t)cf[2] << (2 * kCompactBits));
        } else {
            const int64_t off = 2 * compact_n + 3 * row;
#pragma unroll
            for (int w = 0; w < 3; ++w) rec_out[off + w] = term_word(cn[w], cf[w]);
            lo = off | INT64_MIN;
            hi = 0;
        }
        *reinterpret_cast<longlong2 *>(rec_out + 2 * row) = make_longlong2(lo, hi);
    } else if (rec_out && n_win == 3 && ((uintptr_t)rec_out & 15) == 0) {
        int64_t *dst = rec_out + row * 3;
        const int64_t w0 = term_word(cn[0], cf[0]), w1 = term_word(cn[1], cf[1]), w2 = term_word(cn[2], cf[2]);
        if ((row & 1) == 0) {
            *reinterpret_cast<longlong2 *>(dst) = make_longlong2(w0, w1);
            dst[2] = w2;
        } else {
            dst[0] = w0;
            *reinterpret_cast<longlong2 *>(dst + 1) = make_longlong2(w1, w2);
        }
    } else {
        for (int w = 0; w < n_win; ++w) term_store(nb_out, risk_out, rec_out, n, n_win, q, row, w, cn[w], cf[w]);
    }
}

// Terminal windows over GROUPED inputs (fdx_rekey_payload carried ts -- and the fraud bit in
// bit 31 of the perm -- through the re-key): every read is sequential within a segment.
//   gts[q]    ts of grouped position q; segments time-sorted, or (RUNS) concatenations of
//             time-sorted runs (the multi-GPU owner side: one run per source rank)
//   fraud(q)  gfraud ? gfraud[q] : rows[q] >> 31
//   rows[q]   destination row of q's record (bits 30..0; NULL: q itself)
// Output: count records rec_out[row] (W words NB | FRAUD << 32), or nb_out/risk_out[w*n + q].
// One wave per segment (grid-stride over segments).  Closed form of the reference's
// rolling(delay+w) - rolling(delay) (bitwise-identical, tie-order independent because every
// counted row is strictly older than the current one):
//   hi   = #rows with t <= t_i - delay,  lo_w = #rows with t <= t_i - delay - w
//   NB_w = hi - lo_w,  FRAUD_w = F[hi] - F[lo_w]  (F = prefix count of fraud rows)
//   RISK_w = NB_w > 0 ? FRAUD_w / NB_w : 0   (fillna(0) of 0/0)
// RUNS: every count is summed over the segment's time-sorted runs, each searched separately.
// Segments of <= LR rows are staged in LDS.  Longer ones -- a hot terminal, or one
// terminal's rows from every rank on its owner -- use global memory: the segment's wave
// first writes the inclusive prefix fraud count of every position to scratch[q], then each
// row binary-searches its window bounds in gts (per run) and reads two prefix counts:
// O(L log L) per segment.  Only a segment of more unsorted runs than its run list holds
// (> 64 in LDS, > 2 LR - 1 long -- never the owner side, which has one run per source rank)
// is counted directly, O(L) per row.  Only segments with len_lo < L <= len_hi are processed
// (the short / long passes of terminal_launch).
template <bool RUNS, int LR = kTermLdsRows>
__global__ void __launch_bounds__(kTermBlock) k_terminal_g(
    const int64_t *__restrict__ gts, const uint8_t *__restrict__ gfraud, const int32_t *__restrict__ rows,
    const int64_t *__restrict__ seg_off, int64_t n_seg, int64_t n, int64_t delay, WinArgs win, int32_t n_win,
    int32_t *__restrict__ nb_out, double *__restrict__ risk_out, int64_t *__restrict__ rec_out,
    int32_t *__restrict__ scratch, int64_t len_lo, int64_t len_hi, int64_t compact_n) {
    static_assert(LR % kWave == 0 && LR <= 32768, "the merge packs a staging index in 15 bits");
    constexpr int kMaxRunsLong = 2 * LR - 1;  // a long segment's run list in the stage's ts words
    __shared__ int64_t s_ts[kTermWaves][LR];
    __shared__ int32_t s_f[kTermWaves][LR + 1];
    __shared__ int32_t s_runs[RUNS ? kTermWaves : 1][kMaxRuns + 1];
    // RUNS, LDS-staged segments: the merged order's staging index | fraud << 15
    __shared__ uint16_t s_q[RUNS ? kTermWaves : 1][RUNS ? LR : 1];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int64_t gwave = (int64_t)blockIdx.x * kTermWaves + wv;
    const int64_t nwaves = (int64_t)gridDim.x * kTermWaves;
    int64_t *lts = s_ts[wv];
    int32_t *lf = s_f[wv];
    auto fraud_of = [&](int64_t q) -> int { return gfraud ? (gfraud[q] != 0) : (int)((uint32_t)rows[q] >> 31); };
    auto dest_of = [&](int64_t q) -> int64_t { return rows ? (int64_t)(rows[q] & 0x7FFFFFFF) : q; };
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    for (int64_t seg = gwave; seg < n_seg; seg += nwaves) {
        const int64_t b = seg_off[seg], e = seg_off[seg + 1];
        const int64_t L = e - b;
        if (L <= len_lo || L > len_hi) continue;
        const bool in_lds = L <= LR;
        // stage ts (LDS) and the inclusive prefix fraud counts (LDS: lf[j + 1]; global: scratch[b + j])
        int carry = 0;
        if (in_lds && lane == 0) lf[0] = 0;
        for (int64_t c = 0; c < L; c += kWave) {
            const int64_t j = c + lane;
            int f = 0;
            if (j < L) {
                f = fraud_of(b + j);
                if (in_lds) lts[j] = gts[b + j];
            }
            const int inc = wave_incl_scan(f, lane) + carry;
            if (j < L) {
                if (in_lds) lf[j + 1] = inc;
                else scratch[b + j] = inc;
            }
            carry = __shfl(inc, kWave - 1, kWave);
        }
        // this wave's scratch writes before its reads below; an agent-scope fence also drops
        // L1 lines another wave of this CU may hold for a neighbouring segment's scratch
        if (!in_lds) __threadfence();
        wave_sync();
        // timestamps and prefix counts F(j) = # fraud rows in [0, j) of the segment, one accessor
        // pair per memory space: every loop below is instantiated for each (a load through
        // `in_lds ? lds : global` compiles to a flat load, which takes the vector-memory path and
        // its latency even for LDS addresses -- the binary searches are chains of such loads)
        auto T_lds = [&](int64_t j) -> int64_t { return lts[j]; };
        auto F_lds = [&](int64_t j) -> int32_t { return lf[j]; };
        auto T_glb = [&](int64_t j) -> int64_t { return __builtin_nontemporal_load(gts + b + j); };
        auto F_glb = [&](int64_t j) -> int32_t { return j == 0 ? 0 : __builtin_nontemporal_load(scratch + b + j - 1); };
        int nruns = 1;
        int32_t *lr = in_lds ? s_runs[RUNS ? wv : 0] : reinterpret_cast<int32_t *>(lts);
        const int max_runs = in_lds ? kMaxRuns : kMaxRunsLong;
        if (RUNS) {  // run starts: wherever ts descends
            if (lane == 0) lr[0] = 0;
            auto find_runs = [&](auto T) {
                int nr = 1;
                for (int64_t c = 0; c < L; c += kWave) {
                    const int64_t j = c + lane;
                    const bool dsc = j > 0 && j < L && T(j) < T(j - 1);
                    const uint64_t m = __ballot(dsc);
                    const int at = nr + __popcll(m & ((1ull << lane) - 1ull));
                    if (dsc && at < max_runs) lr[at] = (int32_t)j;
                    nr += __popcll(m);
                }
                return nr;
            };
            const int nr = in_lds ? find_runs(T_lds) : find_runs(T_glb);
            if (lane == 0 && nr <= max_runs) lr[nr] = (int32_t)L;
            nruns = nr;
            wave_sync();
        }
        // LDS-staged segment of several runs: merge the runs in LDS (each element's merged
        // position = its index in its run + the elements of the other runs before it, by
        // binary search; ties: lower run first), then the single-run closed form -- (runs - 1)
        // searches per element once, instead of runs x 4 searches per element
        bool merged = false;
        if constexpr (RUNS) {
            if (in_lds && nruns > 1 && nruns <= max_runs) {
                uint16_t *lq = s_q[wv];
                constexpr int kCh = LR / kWave;
                int32_t mpos[kCh];
                int64_t mts[kCh];
#pragma unroll
                for (int k = 0; k < kCh; ++k) {
                    const int64_t j = (int64_t)k * kWave + lane;
                    mpos[k] = -1;
                    if (j < L) {
                        const int64_t tj = lts[j];
                        int r = 0;
                        while (r + 1 < nruns && lr[r + 1] <= j) ++r;
                        int64_t m = j - lr[r];
                        for (int r2 = 0; r2 < nruns; ++r2) {
                            if (r2 == r) continue;
                            int64_t lo = lr[r2], hi = lr[r2 + 1];
                            while (lo < hi) {  // r2 < r: count ts <= tj; r2 > r: count ts < tj
                                const int64_t mid = (lo + hi) >> 1;
                                const int64_t x = lts[mid];
                                if (r2 < r ? x <= tj : x < tj) lo = mid + 1; else hi = mid;
                            }
                            m += lo - lr[r2];
                        }
                        mpos[k] = (int32_t)m;
                        mts[k] = tj;
                    }
                }
                wave_sync();  // every read of the staging order's timestamps done
#pragma unroll
                for (int k = 0; k < kCh; ++k)
                    if (mpos[k] >= 0) {
                        const int64_t j = (int64_t)k * kWave + lane;
                        lts[mpos[k]] = mts[k];
                        lq[mpos[k]] = (uint16_t)(j | ((lf[j + 1] - lf[j]) << 15));  // lf: still staging order
                    }
                wave_sync();
                int c2 = 0;  // prefix fraud counts in the merged order
                for (int64_t c = 0; c < L; c += kWave) {
                    const int64_t j = c + lane;
                    const int f = j < L ? (int)(lq[j] >> 15) : 0;
                    const int inc = wave_incl_scan(f, lane) + c2;
                    if (j < L) lf[j + 1] = inc;
                    c2 = __shfl(inc, kWave - 1, kWave);
                }
                wave_sync();
                merged = true;
            }
        }
        auto rows_loop = [&](auto T, auto F) {
            auto ub = [&](int64_t lo, int64_t hi, int64_t x) -> int64_t {  // first j in [lo, hi) with T(j) > x
                while (lo < hi) {
                    const int64_t mid = (lo + hi) >> 1;
                    if (T(mid) <= x) lo = mid + 1; else hi = mid;
                }
                return lo;
            };
            for (int64_t i = lane; i < L; i += kWave) {
                const int64_t t = T(i);
                // merged: i is a position in the merged order; its record belongs to staging index qi
                const int64_t qi = merged ? (int64_t)(s_q[RUNS ? wv : 0][i] & 0x7FFF) : i;
                const int64_t row = dest_of(b + qi);
                int32_t nbh = 0, frh = 0;
                int32_t cn[FDX_MAX_WINDOWS], cf[FDX_MAX_WINDOWS];
                if (!RUNS || nruns == 1 || merged) {
                    const int64_t hi = ub(0, i, t - delay);  // rows strictly older than t - delay < t
                    nbh = (int32_t)hi;
                    frh = F(hi);
    #pragma unroll
                    for (int w = 0; w < FDX_MAX_WINDOWS; ++w) {
                        if (w < n_win) {
                            const int64_t lo = ub(0, hi, t - delay - win.w[w]);
                            cn[w] = (int32_t)(hi - lo);
                            cf[w] = frh - F(lo);
                        }
                    }
                } else if (nruns <= max_runs) {
                    for (int r = 0; r < nruns; ++r) {
                        const int64_t h = ub(lr[r], lr[r + 1], t - delay);
                        nbh += (int32_t)(h - lr[r]);
                        frh += F(h) - F(lr[r]);
                    }
    #pragma unroll
                    for (int w = 0; w < FDX_MAX_WINDOWS; ++w) {
                        if (w < n_win) {
                            int32_t nbl = 0, frl = 0;
                            for (int r = 0; r < nruns; ++r) {
                                const int64_t lo = ub(lr[r], lr[r + 1], t - delay - win.w[w]);
                                nbl += (int32_t)(lo - lr[r]);
                                frl += F(lo) - F(lr[r]);
                            }
                            cn[w] = nbh - nbl;
                            cf[w] = frh - frl;
                        }
                    }
                } else {  // more unsorted runs than the run list holds: count directly (any order)
                    int32_t nbl[FDX_MAX_WINDOWS] = {}, frl[FDX_MAX_WINDOWS] = {};
                    for (int64_t j = 0; j < L; ++j) {
                        const int64_t tj = T(j);
                        if (tj > t - delay) continue;
                        const int fj = F(j + 1) - F(j);
                        ++nbh;
                        frh += fj;
                        for (int w = 0; w < n_win; ++w)
                            if (tj <= t - delay - win.w[w]) {
                                ++nbl[w];
                                frl[w] += fj;
                            }
                    }
    #pragma unroll
                    for (int w = 0; w < FDX_MAX_WINDOWS; ++w) {
                        cn[w] = nbh - nbl[w];
                        cf[w] = frh - frl[w];
                    }
                }
                term_emit(nb_out, risk_out, rec_out, n, n_win, compact_n, b + qi, row, cn, cf);
            }
        };
        if (in_lds)
            rows_loop(T_lds, F_lds);
        else
            rows_loop(T_glb, F_glb);
        wave_sync();
    }
}

// The short-segment pass of the single-run case (segments of 1..kTermShortRows rows, 99.95 % of
// the rows at config 2), software-pipelined across a wave's segments: the next segment's
// timestamps and rows words are loaded into registers while the current one is searched, and
// the rows words (destination row | fraud << 31) are staged in LDS beside the timestamps, so
// neither the staging nor the record stores wait on a global load (the one-segment-at-a-time
// form spent 73 % of its wave time in s_waitcnt on HBM round trips, r03r PMC).  Same closed
// form, same outputs as k_terminal_g.
// NW > 0 (compile-time window count; the launch uses 3 for W = 3): every search of the segment
// runs at once -- a branchless fixed-depth binary search over [0, i) per (row chunk, bound), all
// (chunks x (NW + 1)) chains interleaved, so that a segment costs one search's LDS latency
// (8 dependent reads) rather than chunks x (hi search, then the window searches inside [0, hi)).
// Bounds over [0, i) equal those over [0, hi): ts is sorted and every ts in [hi, i) exceeds
// t - delay >= each window's bound.  NW = 0: the runtime window count, one row at a time.
template <int NW>
__global__ void __launch_bounds__(kTermBlock) k_terminal_short(
    const int64_t *__restrict__ gts, const uint8_t *__restrict__ gfraud, const int32_t *__restrict__ rows,
    const int64_t *__restrict__ seg_off, int64_t n_seg, int64_t n, int64_t delay, WinArgs win, int32_t n_win,
    int32_t *__restrict__ nb_out, double *__restrict__ risk_out, int64_t *__restrict__ rec_out, int64_t compact_n) {
    constexpr int LR = kTermShortRows, CH = LR / kWave;
    __shared__ int64_t s_ts[kTermWaves][LR];
    __shared__ int32_t s_f[kTermWaves][LR + 1];
    __shared__ int32_t s_r[kTermWaves][LR];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const int64_t nwaves = (int64_t)gridDim.x * kTermWaves;
    int64_t *lts = s_ts[wv];
    int32_t *lf = s_f[wv], *lr = s_r[wv];
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // the wave's next segment of this pass at or after s (wave-uniform scalar loads)
    auto next_seg = [&](int64_t s, int64_t &b, int64_t &L) -> int64_t {
        for (; s < n_seg; s += nwaves) {
            b = seg_off[s];
            L = seg_off[s + 1] - b;
            if (L > 0 && L <= LR) return s;
        }
        return n_seg;
    };
    int64_t pts[CH];
    int32_t prw[CH];
    uint32_t pfr[CH];
    auto load = [&](int64_t b, int64_t L) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int64_t j = imin64(c * kWave + lane, L - 1);  // clamped: no branch
            pts[c] = gts[b + j];
            prw[c] = rows ? rows[b + j] : (int32_t)(b + j);
            pfr[c] = gfraud ? gfraud[b + j] : 0u;
        }
    };
    int64_t cb = 0, cl = 0;
    int64_t cur = next_seg((int64_t)blockIdx.x * kTermWaves + wv, cb, cl);
    if (cur < n_seg) load(cb, cl);
    while (cur < n_seg) {
        // stage the current segment from registers: ts, rows words, prefix fraud counts
        if (lane == 0) lf[0] = 0;
        int carry = 0;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int64_t j = c * kWave + lane;
            const bool in = j < cl;
            const int f = in ? (gfraud ? (pfr[c] != 0) : (int)((uint32_t)prw[c] >> 31)) : 0;
            if (in) {
                lts[j] = pts[c];
                lr[j] = prw[c] & 0x7FFFFFFF;
            }
            const int inc = wave_incl_scan(f, lane) + carry;
            if (in) lf[j + 1] = inc;
            carry = __shfl(inc, kWave - 1, kWave);
        }
        wave_sync();
        // the next segment's loads, in flight during this one's searches
        int64_t nb = 0, nl = 0;
        const int64_t nxt = next_seg(cur + nwaves, nb, nl);
        if (nxt < n_seg) load(nb, nl);
        if constexpr (NW > 0) {
            const int32_t L32 = (int32_t)cl;
            auto chunks = [&](auto nc) {
                constexpr int NC = decltype(nc)::value;
                int32_t pos[NC][NW + 1];
                int64_t x[NC][NW + 1];
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    const int64_t t = lts[c * kWave + lane];  // past the segment: stale, never emitted
                    x[c][0] = t - delay;
#pragma unroll
                    for (int w = 0; w < NW; ++w) x[c][w + 1] = t - delay - win.w[w];
#pragma unroll
                    for (int k = 0; k <= NW; ++k) pos[c][k] = 0;
                }
                // pos = #j < i with ts_j <= x (ts sorted): steps LR/2 .. 1 reach any i < LR
#pragma unroll
                for (int step = LR / 2; step >= 1; step >>= 1) {
#pragma unroll
                    for (int c = 0; c < NC; ++c) {
                        const int32_t i = c * kWave + lane;
#pragma unroll
                        for (int k = 0; k <= NW; ++k) {
                            const int32_t q = pos[c][k] + step;
                            const bool take = (q <= i) & (lts[q - 1] <= x[c][k]);  // q - 1 < LR
                            pos[c][k] = take ? q : pos[c][k];
                        }
                    }
                }
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    const int32_t i = c * kWave + lane;
                    if (i < L32) {
                        int32_t cn[FDX_MAX_WINDOWS], cf[FDX_MAX_WINDOWS];
                        const int32_t hi = pos[c][0], frh = lf[hi];
#pragma unroll
                        for (int w = 0; w < NW; ++w) {
                            cn[w] = hi - pos[c][w + 1];
                            cf[w] = frh - lf[pos[c][w + 1]];
                        }
                        term_emit(nb_out, risk_out, rec_out, n, NW, compact_n, cb + i, lr[i], cn, cf);
                    }
                }
            };
            static_assert(CH == 4, "the chunk switch below covers 1..4 chunks of 64 rows");
            switch ((L32 + kWave - 1) / kWave) {
                case 1: chunks(std::integral_constant<int, 1>{}); break;
                case 2: chunks(std::integral_constant<int, 2>{}); break;
                case 3: chunks(std::integral_constant<int, 3>{}); break;
                default: chunks(std::integral_constant<int, 4>{}); break;
            }
            wave_sync();
            cur = nxt;
            cb = nb;
            cl = nl;
            continue;
        }
        auto ub = [&](int32_t lo, int32_t hi, int64_t x) -> int32_t {  // first j in [lo, hi) with ts_j > x
            while (lo < hi) {
                const int32_t mid = (int32_t)((uint32_t)(lo + hi) >> 1);
                if (lts[mid] <= x) lo = mid + 1; else hi = mid;
            }
            return lo;
        };
        for (int32_t i = lane; i < (int32_t)cl; i += kWave) {
            const int64_t t = lts[i];
            const int64_t row = lr[i];
            int32_t cn[FDX_MAX_WINDOWS], cf[FDX_MAX_WINDOWS];
            const int32_t hi = ub(0, i, t - delay);  // rows strictly older than t - delay < t
            const int32_t frh = lf[hi];
#pragma unroll
            for (int w = 0; w < FDX_MAX_WINDOWS; ++w) {
                if (w < n_win) {
                    const int32_t lo = ub(0, hi, t - delay - win.w[w]);
                    cn[w] = (int32_t)(hi - lo);
                    cf[w] = frh - lf[lo];
                }
            }
            term_emit(nb_out, risk_out, rec_out, n, n_win, compact_n, cb + i, row, cn, cf);
        }
        wave_sync();
        cur = nxt;
        cb = nb;
        cl = nl;
    }
}

// X[r][0..2] = amount, weekend, night (rows already in output order)
__global__ void __launch_bounds__(256) k_assemble_time(const double *__restrict__ amount,
                                                       const uint8_t *__restrict__ weekend,
                                                       const uint8_t *__restrict__ night, int64_t n,
                                                       double *__restrict__ X, int64_t ld) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        double *x = X + r * ld;
        x[0] = amount[r];
        x[1] = (double)weekend[r];
        x[2] = (double)night[r];
    }
}

// X[perm[i]][col0 + 2w] = nb[w][i], X[perm[i]][col0 + 2w + 1] = val[w][i]
__global__ void __launch_bounds__(256) k_assemble_group(const int32_t *__restrict__ perm,
                                                        const int32_t *__restrict__ nb,
                                                        const double *__restrict__ val, int64_t n,
                                                        int32_t n_win, double *__restrict__ X, int64_t ld,
                                                        int32_t col0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double *x = X + (int64_t)perm[i] * ld + col0;
        for (int w = 0; w < n_win; ++w) {
            x[2 * w] = (double)nb[(int64_t)w * n + i];
            x[2 * w + 1] = val[(int64_t)w * n + i];
        }
    }
}

int check_windows(const int64_t *window_ns, int32_t n_windows, WinArgs *wa) {
    FDX_REQUIRE(window_ns != nullptr, "window_ns is NULL");
    FDX_REQUIRE(n_windows >= 1 && n_windows <= FDX_MAX_WINDOWS, "n_windows must be in [1, %d]",
                FDX_MAX_WINDOWS);
    for (int i = 0; i < FDX_MAX_WINDOWS; ++i) wa->w[i] = 0;
    for (int i = 0; i < n_windows; ++i) {
        FDX_REQUIRE(window_ns[i] > 0, "window %d must be > 0 ns", i);
        wa->w[i] = window_ns[i];
    }
    return FDX_OK;
}

}  // namespace
}  // namespace fdx

using namespace fdx;

extern "C" int fdx_time_flags(const int64_t *ts_ns_d, int64_t n, int32_t mode, uint8_t *weekend_d,
                              uint8_t *night_d, void *stream) {
    FDX_REQUIRE(n >= 0, "n < 0");
    FDX_REQUIRE(mode == FDX_FLAGS_NOTEBOOK || mode == FDX_FLAGS_SPARK, "bad flags mode %d", mode);
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(ts_ns_d && weekend_d && night_d, "null pointer");
    FDX_REQUIRE(((uintptr_t)weekend_d % 8) == 0 && ((uintptr_t)night_d % 8) == 0,
                "flag outputs must be 8-byte aligned");
    const int block = 256;
    unsigned grid = stream_grid(ceil_div(n, 8), block);
    hipLaunchKernelGGL(k_time_flags, dim3(grid), dim3(block), 0, as_stream(stream), ts_ns_d, n, mode,
                       weekend_d, night_d);
    FDX_LAUNCHED("k_time_flags");
    return FDX_OK;
}

extern "C" int fdx_customer_windows(const int64_t *ts_ns_d, const double *amount_d,
                                    const int64_t *seg_off_d, int64_t n_seg, int64_t n,
                                    const int64_t *window_ns, int32_t n_windows, int32_t *nb_d,
                                    double *avg_d, void *stream) {
    WinArgs wa;
    int rc = check_windows(window_ns, n_windows, &wa);
    if (rc) return rc;
    FDX_REQUIRE(n_seg >= 0 && n >= 0, "negative size");
    if (n_seg == 0 || n == 0) return FDX_OK;
    FDX_REQUIRE(ts_ns_d && amount_d && seg_off_d && nb_d && avg_d, "null pointer");
    const int block = 256;
    const int64_t lanes = n_seg * n_windows;
    hipLaunchKernelGGL(k_customer_exact, dim3((unsigned)ceil_div(lanes, block)), dim3(block), 0,
                       as_stream(stream), ts_ns_d, amount_d, seg_off_d, n_seg, n, wa, n_windows,
                       nb_d, avg_d);
    FDX_LAUNCHED("k_customer_exact");
    return FDX_OK;
}

// Every terminal-window launch: the short-segment pass (<= kTermShortRows rows, small LDS
// stage, more resident waves) then the long pass (the 1,024-row stage, global memory beyond);
// each skips the other's segments.
static void terminal_launch(bool runs, const int64_t *gts, const uint8_t *gfr, const int32_t *rows,
                            const int64_t *seg_off, int64_t n_seg, int64_t n, int64_t delay_ns, const WinArgs &wa,
                            int32_t n_windows, int32_t *nb_d, double *risk_d, int64_t *rec_d, int32_t *scratch,
                            hipStream_t st, int64_t compact_n = 0) {
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n_seg, kTermWaves), 256 * 16);
    const int64_t lo = kTermShortRows, inf = INT64_MAX;
#define FDX_TERM_LAUNCH(R, LRV, A, B)                                                                           \
    hipLaunchKernelGGL((k_terminal_g<R, LRV>), dim3(grid), dim3(kTermBlock), 0, st, gts, gfr, rows, seg_off, n_seg, \
                       n, delay_ns, wa, n_windows, nb_d, risk_d, rec_d, scratch, (int64_t)(A), (int64_t)(B), \
                       compact_n)
    if (runs) {
        FDX_TERM_LAUNCH(true, kTermShortRows, 0, kTermShortRows);
        FDX_TERM_LAUNCH(true, kTermLdsRows, lo, inf);
    } else {
        if (n_windows == 3)  // every search of a segment interleaved
            hipLaunchKernelGGL(k_terminal_short<3>, dim3(grid), dim3(kTermBlock), 0, st, gts, gfr, rows, seg_off,
                               n_seg, n, delay_ns, wa, n_windows, nb_d, risk_d, rec_d, compact_n);
        else
            hipLaunchKernelGGL(k_terminal_short<0>, dim3(grid), dim3(kTermBlock), 0, st, gts, gfr, rows, seg_off,
                               n_seg, n, delay_ns, wa, n_windows, nb_d, risk_d, rec_d, compact_n);
        FDX_TERM_LAUNCH(false, kTermLdsRows, lo, inf);
    }
#undef FDX_TERM_LAUNCH
}

extern "C" size_t fdx_terminal_windows_workspace_size(int64_t n) {
    return round_up((size_t)(n > 0 ? n : 0) * 4, 256) + 256;
}

// Grouped rows (time order inside each segment): the grouped kernel, its long-segment prefix
// counts in the caller's workspace.
extern "C" int fdx_terminal_windows(const int64_t *ts_ns_d, const uint8_t *fraud_d,
                                    const int64_t *seg_off_d, int64_t n_seg, int64_t n,
                                    int64_t delay_ns, const int64_t *window_ns, int32_t n_windows,
                                    int32_t *nb_d, double *risk_d, void *workspace_d, size_t workspace_bytes,
                                    void *stream) {
    WinArgs wa;
    int rc = check_windows(window_ns, n_windows, &wa);
    if (rc) return rc;
    FDX_REQUIRE(delay_ns > 0, "delay must be > 0 ns");
    FDX_REQUIRE(n_seg >= 0 && n >= 0, "negative size");
    if (n_seg == 0 || n == 0) return FDX_OK;
    FDX_REQUIRE(ts_ns_d && fraud_d && seg_off_d && nb_d && risk_d, "null pointer");
    const size_t need = fdx_terminal_windows_workspace_size(n);
    if (!workspace_d || workspace_bytes < need) {
        set_error("terminal windows workspace too small: %zu < %zu", workspace_bytes, need);
        return FDX_E_WORKSPACE;
    }
    terminal_launch(false, ts_ns_d, fraud_d, nullptr, seg_off_d, n_seg, n, delay_ns, wa, n_windows, nb_d, risk_d,
                    nullptr, reinterpret_cast<int32_t *>(workspace_d), as_stream(stream));
    FDX_LAUNCHED("k_terminal_g");
    return FDX_OK;
}

static int terminal_grouped(const int64_t *gts_d, const uint8_t *gfraud_d, const int32_t *rows_d,
                            const int64_t *seg_off_d, int64_t n_seg, int64_t n, int64_t delay_ns,
                            const int64_t *window_ns, int32_t n_windows, int32_t runs, int32_t *nb_d, double *risk_d,
                            int64_t *rec_d, int32_t *scratch_d, void *stream, bool compact = false) {
    WinArgs wa;
    int rc = check_windows(window_ns, n_windows, &wa);
    if (rc) return rc;
    FDX_REQUIRE(delay_ns > 0, "delay must be > 0 ns");
    FDX_REQUIRE(n_seg >= 0 && n >= 0, "negative size");
    if (n_seg == 0 || n == 0) return FDX_OK;
    FDX_REQUIRE(gts_d && seg_off_d && scratch_d, "null pointer");
    FDX_REQUIRE(gfraud_d || rows_d, "fraud comes from gfraud_d or bit 31 of rows_d");
    FDX_REQUIRE(rec_d || (nb_d && risk_d), "no output");
    FDX_REQUIRE(!compact || (rec_d && n_windows == 3 && ((uintptr_t)rec_d & 15) == 0),
                "compact records: W = 3, a 16-byte aligned record array");
    terminal_launch(runs != 0, gts_d, gfraud_d, rows_d, seg_off_d, n_seg, n, delay_ns, wa, n_windows, nb_d, risk_d,
                    rec_d, scratch_d, as_stream(stream), compact ? n : 0);
    FDX_LAUNCHED("k_terminal_g");
    return FDX_OK;
}

extern "C" int fdx_terminal_windows_grouped(const int64_t *gts_d, const uint8_t *gfraud_d, const int32_t *rows_d,
                                            const int64_t *seg_off_d, int64_t n_seg, int64_t n, int64_t delay_ns,
                                            const int64_t *window_ns, int32_t n_windows, int32_t runs, int32_t *nb_d,
                                            double *risk_d, int64_t *rec_d, int32_t *scratch_d, void *stream) {
    return terminal_grouped(gts_d, gfraud_d, rows_d, seg_off_d, n_seg, n, delay_ns, window_ns, n_windows, runs, nb_d,
                            risk_d, rec_d, scratch_d, stream);
}

extern "C" int fdx_terminal_windows_grouped_compact(const int64_t *gts_d, const uint8_t *gfraud_d,
                                                    const int32_t *rows_d, const int64_t *seg_off_d, int64_t n_seg,
                                                    int64_t n, int64_t delay_ns, const int64_t *window_ns,
                                                    int32_t n_windows, int32_t runs, int64_t *rec_d,
                                                    int32_t *scratch_d, void *stream) {
    return terminal_grouped(gts_d, gfraud_d, rows_d, seg_off_d, n_seg, n, delay_ns, window_ns, n_windows, runs,
                            nullptr, nullptr, rec_d, scratch_d, stream, true);
}

extern "C" int fdx_assemble_features(int64_t n, int32_t n_windows, const double *amount_d,
                                     const uint8_t *weekend_d, const uint8_t *night_d,
                                     const int32_t *cust_perm_d, const int32_t *cust_nb_d,
                                     const double *cust_avg_d, const int32_t *term_perm_d,
                                     const int32_t *term_nb_d, const double *term_risk_d, double *X_d,
                                     int64_t ld, void *stream) {
    FDX_REQUIRE(n >= 0, "n < 0");
    FDX_REQUIRE(n_windows >= 1 && n_windows <= FDX_MAX_WINDOWS, "bad n_windows");
    FDX_REQUIRE(ld >= 3 + 4 * n_windows, "ld too small");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(amount_d && weekend_d && night_d && cust_perm_d && cust_nb_d && cust_avg_d && X_d,
                "null pointer");
    hipStream_t st = as_stream(stream);
    const unsigned grid = stream_grid(n, 256);
    hipLaunchKernelGGL(k_assemble_time, dim3(grid), dim3(256), 0, st, amount_d, weekend_d, night_d, n, X_d, ld);
    FDX_LAUNCHED("k_assemble_time");
    hipLaunchKernelGGL(k_assemble_group, dim3(grid), dim3(256), 0, st, cust_perm_d, cust_nb_d, cust_avg_d, n,
                       n_windows, X_d, ld, 3);
    FDX_LAUNCHED("k_assemble_group");
    if (term_perm_d && term_nb_d && term_risk_d) {  // NULL: filled later (multi-GPU reply path)
        hipLaunchKernelGGL(k_assemble_group, dim3(grid), dim3(256), 0, st, term_perm_d, term_nb_d, term_risk_d,
                           n, n_windows, X_d, ld, 3 + 2 * n_windows);
        FDX_LAUNCHED("k_assemble_group");
    }
    return FDX_OK;
}

static size_t al256(size_t x) { return (x + 255) / 256 * 256; }

extern "C" size_t fdx_customer_layout_workspace_size(int64_t n_seg) {
    if (n_seg < 0) n_seg = 0;
    return al256((size_t)n_seg * 4) + al256((size_t)(65535 + 2) * 8) + fdx_rekey_workspace_size(n_seg, 16) +
           fdx_exclusive_scan_u32_workspace_size(n_seg + 1) + 256;
}

// The layout in two halves.  Plan (segment lengths only, so it can run while the rows are
// still being re-keyed): segments sorted by decreasing length, the slot offset of every group
// and the slot count (read back: the one host synchronisation of the layout).  Fill: the slots
// (and the window starts) from the grouped rows.
extern "C" int fdx_customer_layout_plan(const int64_t *seg_off_d, int64_t n_seg, int32_t n_windows, int32_t *sorder_d,
                                        uint32_t *goff_d, int64_t *n_slots_h, void *ws, size_t ws_bytes,
                                        void *stream) {
    FDX_REQUIRE(n_seg >= 1 && n_windows >= 1 && n_windows <= 64, "bad argument");
    FDX_REQUIRE(seg_off_d && sorder_d && goff_d && n_slots_h && ws, "null pointer");
    FDX_REQUIRE(ws_bytes >= fdx_customer_layout_workspace_size(n_seg), "workspace too small");
    hipStream_t st = as_stream(stream);
    const int32_t S = kWave / n_windows;
    const int64_t n_groups = ceil_div(n_seg, S);
    const int32_t lmax = 65535;
    char *w = reinterpret_cast<char *>(ws);
    int32_t *keys = reinterpret_cast<int32_t *>(w);
    w += al256((size_t)n_seg * 4);
    int32_t *status = reinterpret_cast<int32_t *>(w);  // (in the reserved range)
    w += al256((size_t)(lmax + 2) * 8);
    if (n_seg <= kPlanMaxSeg && n_groups <= kPlanMaxGroups) {  // one launch; the radix plan below if it
                                                               // reports too many long segments
        struct {
            uint32_t total;
            int32_t status;
        } h{};
        hipLaunchKernelGGL(k_layout_plan_small, dim3(1), dim3(kPlanWaves * kWave), 0, st, seg_off_d, n_seg, S, n_groups,
                           sorder_d, goff_d, status);
        FDX_LAUNCHED("k_layout_plan_small");
        FDX_HIP(hipMemcpyAsync(&h.status, status, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        FDX_HIP(hipMemcpyAsync(&h.total, goff_d + n_groups, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        FDX_HIP(hipStreamSynchronize(st));
        if (h.status == 0) {
            *n_slots_h = h.total;
            return FDX_OK;
        }
    }
    hipLaunchKernelGGL(k_seg_len_keys, dim3(stream_grid(n_seg, 256)), dim3(256), 0, st, seg_off_d, n_seg, lmax, keys);
    FDX_LAUNCHED("k_seg_len_keys");
    const size_t rws = fdx_rekey_workspace_size(n_seg, 16);
    int rc = fdx_rekey(keys, n_seg, 16, lmax + 1, sorder_d, nullptr, nullptr, w, rws, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_group_slots, dim3(stream_grid(n_groups, 256)), dim3(256), 0, st, seg_off_d, sorder_d,
                       n_seg, S, n_groups, goff_d);
    FDX_LAUNCHED("k_group_slots");
    // goff[0..n_groups] = exclusive scan of the slot counts (total in goff[n_groups])
    FDX_HIP(hipMemsetAsync(goff_d + n_groups, 0, sizeof(uint32_t), st));
    rc = fdx_exclusive_scan_u32(goff_d, n_groups + 1, w + rws, stream);
    if (rc) return rc;
    uint32_t total = 0;
    FDX_HIP(hipMemcpyAsync(&total, goff_d + n_groups, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    FDX_HIP(hipStreamSynchronize(st));
    *n_slots_h = total;
    return FDX_OK;
}

// The one-launch plan without the host synchronisation: the slot count and the plan's status go
// to caller-owned pinned host memory (plan_h[0] = slots, plan_h[1] = status: 0 = done, 1 = too
// many long segments -- plan again with fdx_customer_layout_plan), read once the stream is past
// this call.  FDX_E_UNSUPPORTED for more than 65,536 segments.
extern "C" int fdx_customer_layout_plan_async(const int64_t *seg_off_d, int64_t n_seg, int32_t n_windows,
                                              int32_t *sorder_d, uint32_t *goff_d, int32_t *plan_h, void *ws,
                                              size_t ws_bytes, void *stream) {
    FDX_REQUIRE(n_seg >= 1 && n_windows >= 1 && n_windows <= 64, "bad argument");
    FDX_REQUIRE(seg_off_d && sorder_d && goff_d && plan_h && ws, "null pointer");
    FDX_REQUIRE(ws_bytes >= fdx_customer_layout_workspace_size(n_seg), "workspace too small");
    hipStream_t st = as_stream(stream);
    const int32_t S = kWave / n_windows;
    const int64_t n_groups = ceil_div(n_seg, S);
    if (n_seg > kPlanMaxSeg || n_groups > kPlanMaxGroups) {
        set_error("the one-launch plan takes <= %lld segments and <= %lld groups", (long long)kPlanMaxSeg,
                  (long long)kPlanMaxGroups);
        return FDX_E_UNSUPPORTED;
    }
    int32_t *status = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(ws) + al256((size_t)n_seg * 4));
    // pinned memory of the HIP allocator (torch's pin_memory included) maps into the device's
    // address space: the kernel writes the two words itself; other host memory gets the copies
    void *plan_dev = nullptr;
    if (hipHostGetDevicePointer(&plan_dev, plan_h, 0) != hipSuccess) {
        (void)hipGetLastError();  // (not an error of this call: the copy path follows)
        plan_dev = nullptr;
    }
    hipLaunchKernelGGL(k_layout_plan_small, dim3(1), dim3(kPlanWaves * kWave), 0, st, seg_off_d, n_seg, S, n_groups,
                       sorder_d, goff_d, status, reinterpret_cast<int32_t *>(plan_dev));
    FDX_LAUNCHED("k_layout_plan_small");
    if (!plan_dev) {
        FDX_HIP(hipMemcpyAsync(plan_h, goff_d + n_groups, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        FDX_HIP(hipMemcpyAsync(plan_h + 1, status, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    }
    return FDX_OK;
}

static int customer_layout_fill(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d, const int64_t *ts_d,
                                const double *amount_d, int32_t n_windows, const int32_t *sorder_d,
                                const uint32_t *goff_d, int64_t n_slots, int64_t *its_d, double *iamt_d,
                                int32_t *irow_d, hipStream_t st, const WinArgs *wa, int32_t *starts_d, bool grouped) {
    FDX_REQUIRE(n_seg >= 1 && n_windows >= 1 && n_windows <= 64 && n_slots >= 0, "bad argument");
    FDX_REQUIRE(seg_off_d && cperm_d && ts_d && amount_d && sorder_d && goff_d && its_d && iamt_d && irow_d,
                "null pointer");
    const int32_t S = kWave / n_windows;
    const int64_t n_groups = ceil_div(n_seg, S);
    if (!starts_d && grouped)
        hipLaunchKernelGGL((k_interleave<false, true>), dim3((unsigned)n_groups), dim3(256), 0, st, seg_off_d,
                           sorder_d, cperm_d, goff_d, n_seg, S, ts_d, amount_d, its_d, iamt_d, irow_d, WinArgs{},
                           n_windows, (int32_t *)nullptr, n_slots);
    else if (starts_d && grouped)
        hipLaunchKernelGGL((k_interleave<true, true>), dim3((unsigned)n_groups), dim3(256), 0, st, seg_off_d, sorder_d,
                           cperm_d, goff_d, n_seg, S, ts_d, amount_d, its_d, iamt_d, irow_d, *wa, n_windows, starts_d,
                           n_slots);
    else if (starts_d)
        hipLaunchKernelGGL(k_interleave<true>, dim3((unsigned)n_groups), dim3(256), 0, st, seg_off_d, sorder_d,
                           cperm_d, goff_d, n_seg, S, ts_d, amount_d, its_d, iamt_d, irow_d, *wa, n_windows, starts_d,
                           n_slots);
    else
        hipLaunchKernelGGL(k_interleave<false>, dim3((unsigned)n_groups), dim3(256), 0, st, seg_off_d, sorder_d,
                           cperm_d, goff_d, n_seg, S, ts_d, amount_d, its_d, iamt_d, irow_d, WinArgs{}, n_windows,
                           (int32_t *)nullptr, n_slots);
    FDX_LAUNCHED("k_interleave");
    return FDX_OK;
}

extern "C" int fdx_customer_layout_fill_starts_grouped(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                                                       const int64_t *gts_d, const double *gamount_d,
                                                       const int64_t *window_ns, int32_t n_windows,
                                                       const int32_t *sorder_d, const uint32_t *goff_d,
                                                       int64_t n_slots, int64_t *its_d, double *iamt_d,
                                                       int32_t *irow_d, int32_t *starts_d, void *stream) {
    WinArgs wa;
    int rc = check_windows(window_ns, n_windows, &wa);
    if (rc) return rc;
    FDX_REQUIRE(starts_d, "null pointer");
    return customer_layout_fill(seg_off_d, n_seg, cperm_d, gts_d, gamount_d, n_windows, sorder_d, goff_d, n_slots,
                                its_d, iamt_d, irow_d, as_stream(stream), &wa, starts_d, true);
}

// plan + fill in one call (the slot count must fit max_slots: FDX_E_WORKSPACE with *n_slots_h
// set otherwise)
static int customer_layout(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                           const int64_t *ts_d, const double *amount_d, int32_t n_windows,
                           int32_t *sorder_d, uint32_t *goff_d, int64_t *its_d, double *iamt_d,
                           int32_t *irow_d, int64_t max_slots, int64_t *n_slots_h, void *ws,
                           size_t ws_bytes, void *stream, const WinArgs *wa, int32_t *starts_d, bool grouped = false) {
    FDX_REQUIRE(cperm_d && ts_d && amount_d && its_d && iamt_d && irow_d, "null pointer");
    int rc = fdx_customer_layout_plan(seg_off_d, n_seg, n_windows, sorder_d, goff_d, n_slots_h, ws, ws_bytes, stream);
    if (rc) return rc;
    if (*n_slots_h > max_slots) {
        set_error("interleaved layout needs %lld slots > max_slots %lld", (long long)*n_slots_h, (long long)max_slots);
        return FDX_E_WORKSPACE;
    }
    return customer_layout_fill(seg_off_d, n_seg, cperm_d, ts_d, amount_d, n_windows, sorder_d, goff_d, *n_slots_h,
                                its_d, iamt_d, irow_d, as_stream(stream), wa, starts_d, grouped);
}

extern "C" int fdx_customer_layout(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                                   const int64_t *ts_d, const double *amount_d, int32_t n_windows,
                                   int32_t *sorder_d, uint32_t *goff_d, int64_t *its_d, double *iamt_d,
                                   int32_t *irow_d, int64_t max_slots, int64_t *n_slots_h, void *ws,
                                   size_t ws_bytes, void *stream) {
    return customer_layout(seg_off_d, n_seg, cperm_d, ts_d, amount_d, n_windows, sorder_d, goff_d, its_d, iamt_d,
                           irow_d, max_slots, n_slots_h, ws, ws_bytes, stream, nullptr, nullptr);
}

extern "C" int fdx_customer_layout_starts(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                                          const int64_t *ts_d, const double *amount_d, const int64_t *window_ns,
                                          int32_t n_windows, int32_t *sorder_d, uint32_t *goff_d, int64_t *its_d,
                                          double *iamt_d, int32_t *irow_d, int32_t *starts_d, int64_t max_slots,
                                          int64_t *n_slots_h, void *ws, size_t ws_bytes, void *stream) {
    WinArgs wa;
    int rc = check_windows(window_ns, n_windows, &wa);
    if (rc) return rc;
    FDX_REQUIRE(starts_d, "null pointer");
    return customer_layout(seg_off_d, n_seg, cperm_d, ts_d, amount_d, n_windows, sorder_d, goff_d, its_d, iamt_d,
                           irow_d, max_slots, n_slots_h, ws, ws_bytes, stream, &wa, starts_d);
}

extern "C" int fdx_customer_layout_starts_grouped(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                                                  const int64_t *gts_d, const double *gamount_d,
                                                  const int64_t *window_ns, int32_t n_windows, int32_t *sorder_d,
                                                  uint32_t *goff_d, int64_t *its_d, double *iamt_d, int32_t *irow_d,
                                                  int32_t *starts_d, int64_t max_slots, int64_t *n_slots_h, void *ws,
                                                  size_t ws_bytes, void *stream) {
    WinArgs wa;
    int rc = check_windows(window_ns, n_windows, &wa);
    if (rc) return rc;
    FDX_REQUIRE(starts_d, "null pointer");
    return customer_layout(seg_off_d, n_seg, cperm_d, gts_d, gamount_d, n_windows, sorder_d, goff_d, its_d, iamt_d,
                           irow_d, max_slots, n_slots_h, ws, ws_bytes, stream, &wa, starts_d, true);
}

extern "C" int fdx_customer_layout_grouped(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                                           const int64_t *gts_d, const double *gamount_d, int32_t n_windows,
                                           int32_t *sorder_d, uint32_t *goff_d, int64_t *its_d, double *iamt_d,
                                           int32_t *irow_d, int64_t max_slots, int64_t *n_slots_h, void *ws,
                                           size_t ws_bytes, void *stream) {
    return customer_layout(seg_off_d, n_seg, cperm_d, gts_d, gamount_d, n_windows, sorder_d, goff_d, its_d, iamt_d,
                           irow_d, max_slots, n_slots_h, ws, ws_bytes, stream, nullptr, nullptr, true);
}

/* slot form of the scan mode over a layout built WITH window starts (fdx.h) */
extern "C" int fdx_customer_windows_scan_slots(const double *gamount_d, const int64_t *seg_off_d, int64_t n_seg,
                                               int64_t n, const int32_t *sorder_d, const uint32_t *goff_d,
                                               int64_t n_slots, int32_t n_windows, const int32_t *starts_d,
                                               int32_t *nb_d, double *sum_d, void *ws, size_t ws_bytes,
                                               void *stream);

extern "C" size_t fdx_customer_windows_scan_workspace_size(int64_t n, int64_t n_seg) {
    if (n < 0 || n_seg < 0) return 0;
    return al256((size_t)(n + n_seg + 1) * 8) + al256((size_t)(n + n_seg + 1) * 4);
}

extern "C" int fdx_customer_windows_scan(const int64_t *gts_d, const double *gamount_d, const int64_t *seg_off_d,
                                         int64_t n_seg, int64_t n, const int64_t *window_ns, int32_t n_windows,
                                         const int32_t *sorder_d, const uint32_t *goff_d, int64_t n_out,
                                         int32_t *nb_d, double *val_d, int32_t val_is_sum, void *ws, size_t ws_bytes,
                                         void *stream) {
    WinArgs wa;
    int rc = check_windows(window_ns, n_windows, &wa);
    if (rc) return rc;
    FDX_REQUIRE(n_seg >= 0 && n >= 0 && n_out >= 0, "negative size");
    if (n_seg == 0 || n == 0) return FDX_OK;
    FDX_REQUIRE(gts_d && gamount_d && seg_off_d && nb_d && val_d && ws, "null pointer");
    FDX_REQUIRE(!sorder_d || goff_d, "sorder_d needs goff_d");
    FDX_REQUIRE(ws_bytes >= fdx_customer_windows_scan_workspace_size(n, n_seg), "workspace too small");
    const int32_t S = kWave / n_windows;
    FDX_REQUIRE(sorder_d || n_out >= n, "n_out < n");
    double *ge = reinterpret_cast<double *>(ws);
    int32_t *gc = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(ws) + al256((size_t)(n + n_seg + 1) * 8));
    const unsigned grid = (unsigned)std::min<int64_t>(n_seg, 256 * 64);
    hipLaunchKernelGGL(k_customer_scan, dim3(grid), dim3(kWave), 0, as_stream(stream), gts_d, gamount_d, seg_off_d,
                       n_seg, sorder_d, goff_d, S, n_out, wa, n_windows, nb_d, val_d, val_is_sum, ge, gc);
    FDX_LAUNCHED("k_customer_scan");
    return FDX_OK;
}

// A side stream (per device, created once) for launches that fork from the caller's stream
// and join back before the call returns: the caller still sees one stream-ordered call.
// Created at the HIGH priority level: HIP gives each priority level its own pool of
// GPU_MAX_HW_QUEUES hardware queues, and a normal-priority stream created after torch's and
// RCCL's was measured on the caller's own hardware queue (rocprofv3 Queue_Id) -- the two
// walks then ran back to back.
struct ForkStream {
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};
static int fork_stream(ForkStream **out) {
    static ForkStream per_dev[64];
    int dev = 0;
    FDX_HIP(hipGetDevice(&dev));
    FDX_REQUIRE(dev >= 0 && dev < 64, "device id out of range");
    ForkStream &f = per_dev[dev];
    if (!f.side) {
        int least = 0, greatest = 0;
        FDX_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        (void)least;
        FDX_HIP(hipStreamCreateWithPriority(&f.side, hipStreamNonBlocking, greatest));
        FDX_HIP(hipEventCreateWithFlags(&f.fork, hipEventDisableTiming));
        FDX_HIP(hipEventCreateWithFlags(&f.join, hipEventDisableTiming));
    }
    *out = &f;
    return FDX_OK;
}

extern "C" int fdx_customer_windows_walk(const double *iamt_d, const int64_t *seg_off_d, const int32_t *sorder_d,
                                         const uint32_t *goff_d, int64_t n_seg, int64_t n_slots, int32_t n_windows,
                                         const int32_t *starts_d, int32_t *nb_d, double *sum_d, void *stream) {
    FDX_REQUIRE(n_seg >= 0 && n_slots >= 0, "negative size");
    FDX_REQUIRE(n_windows >= 1 && n_windows <= FDX_MAX_WINDOWS, "bad n_windows");
    if (n_seg == 0) return FDX_OK;
    FDX_REQUIRE(iamt_d && seg_off_d && sorder_d && goff_d && starts_d && nb_d && sum_d, "null pointer");
    const int32_t S = kWave / n_windows;
    FDX_REQUIRE(S <= 21, "the walk kernel is built for <= 21 segments per wave (>= 3 windows)");
    const int64_t n_groups = ceil_div(n_seg, S);
    hipStream_t st = as_stream(stream);
    // Length classes: the groups of the longest segments (the busiest customers, whose
    // longest window holds more rows than the 128-row ring minus a chunk, so nearly every
    // removal would miss the ring and wait on a dependent global load) walk with a 256-row
    // ring on a forked stream, concurrently with the rest on the 128-row ring (twice the
    // blocks per CU); the class boundary is kWalkSplitRows.
    constexpr int split = kWalkSplitRows;
    // buffer stores while the outputs fit 2^31 bytes (raw buffer offsets are 32-bit)
    const bool buf = (int64_t)n_windows * n_slots * 8 < (int64_t)INT32_MAX / 8 * 8;
#define FDX_WALK(SM, RING, P, STREAM, LO, HI)                                                                 \
    if (buf)                                                                                                  \
        hipLaunchKernelGGL((k_customer_walk<SM, RING, P, true, kWalkChunk>), dim3((unsigned)(n_groups * (P))), dim3(64), 0, \
                           STREAM, iamt_d, seg_off_d, sorder_d, goff_d, n_seg, S, n_slots, n_windows, nb_d, sum_d, \
                           starts_d, LO, HI);                                                                  \
    else                                                                                                      \
        hipLaunchKernelGGL((k_customer_walk<SM, RING, P, false, kWalkChunk>), dim3((unsigned)(n_groups * (P))), dim3(64), 0, \
                           STREAM, iamt_d, seg_off_d, sorder_d, goff_d, n_seg, S, n_slots, n_windows, nb_d, sum_d, \
                           starts_d, LO, HI);                                                                  \
    FDX_LAUNCHED("k_customer_walk")
    ForkStream *f;
    int rc = fork_stream(&f);
    if (rc) return rc;
    FDX_HIP(hipEventRecord(f->fork, st));
    FDX_HIP(hipStreamWaitEvent(f->side, f->fork, 0));
    FDX_WALK((21 + kWalkLongWaves - 1) / kWalkLongWaves, 256, kWalkLongWaves, f->side, split, INT32_MAX);
    FDX_WALK((21 + kWalkShortWaves - 1) / kWalkShortWaves, 128, kWalkShortWaves, st, 0, split);
    FDX_HIP(hipEventRecord(f->join, f->side));
    FDX_HIP(hipStreamWaitEvent(st, f->join, 0));
    return FDX_OK;
#undef FDX_WALK
}

extern "C" int fdx_customer_windows_interleaved(const int64_t *its_d, const double *iamt_d,
                                                const int64_t *seg_off_d, const int32_t *sorder_d,
                                                const uint32_t *goff_d, int64_t n_seg, int64_t n_slots,
                                                const int64_t *window_ns, int32_t n_windows, int32_t *nb_d,
                                                double *avg_d, void *stream) {
    WinArgs wa;
    int rc = check_windows(window_ns, n_windows, &wa);
    if (rc) return rc;
    FDX_REQUIRE(n_seg >= 0 && n_slots >= 0, "negative size");
    if (n_seg == 0) return FDX_OK;
    FDX_REQUIRE(its_d && iamt_d && seg_off_d && sorder_d && goff_d && nb_d && avg_d, "null pointer");
    const int32_t S = kWave / n_windows;
    const int64_t n_groups = ceil_div(n_seg, S);
    // One pass per group (the ring kernel: window starts found in the walk itself) -- the form
    // for any window count; the scoring pipeline's 3-window layouts use the two-kernel
    // layout-starts + fdx_customer_windows_walk instead.  Ring rows: measured (r01, config 2)
    // 96 rows for every group 1.74 ms (occupancy wins), a 192-row ring for the longest groups
    // 2.33-2.48 ms.
    hipStream_t st = as_stream(stream);
#define FDX_RING(SM, RG)                                                                                   \
    hipLaunchKernelGGL((k_customer_ring<SM, RG>), dim3((unsigned)n_groups), dim3(64), 0, st, its_d, iamt_d, seg_off_d, \
                       sorder_d, goff_d, n_seg, S, n_slots, wa, n_windows, nb_d, avg_d, 0, INT32_MAX)
    if (S <= 21)
        FDX_RING(21, 96);
    else if (S <= 32)
        FDX_RING(32, 192);
    else
        FDX_RING(64, 96);
#undef FDX_RING
    FDX_LAUNCHED("k_customer_ring");
    return FDX_OK;
}

extern "C" int fdx_customer_windows_scan_slots(const double *gamount_d, const int64_t *seg_off_d, int64_t n_seg,
                                               int64_t n, const int32_t *sorder_d, const uint32_t *goff_d,
                                               int64_t n_slots, int32_t n_windows, const int32_t *starts_d,
                                               int32_t *nb_d, double *sum_d, void *ws, size_t ws_bytes,
                                               void *stream) {
    FDX_REQUIRE(n_seg >= 0 && n >= 0 && n_slots >= 0, "negative size");
    FDX_REQUIRE(n_windows >= 1 && n_windows <= FDX_MAX_WINDOWS, "bad n_windows");
    if (n_seg == 0 || n == 0) return FDX_OK;
    FDX_REQUIRE(gamount_d && seg_off_d && sorder_d && goff_d && starts_d && nb_d && sum_d && ws, "null pointer");
    FDX_REQUIRE(ws_bytes >= fdx_customer_windows_scan_workspace_size(n, n_seg), "workspace too small");
    hipStream_t st = as_stream(stream);
    const int32_t S = kWave / n_windows;
    const int64_t n_groups = ceil_div(n_seg, S);
    double *ge = reinterpret_cast<double *>(ws);
    int32_t *gc = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(ws) + al256((size_t)(n + n_seg + 1) * 8));
    hipLaunchKernelGGL(k_seg_prefix, dim3(stream_grid(n_seg * kWave, 256, 256 * 32)), dim3(256), 0, st, gamount_d,
                       seg_off_d, n_seg, ge, gc);
    FDX_LAUNCHED("k_seg_prefix");
    hipLaunchKernelGGL(k_scan_slots, dim3((unsigned)n_groups), dim3(256), 0, st, seg_off_d, sorder_d, goff_d, n_seg,
                       S, n_slots, n_windows, starts_d, ge, gc, nb_d, sum_d);
    FDX_LAUNCHED("k_scan_slots");
    return FDX_OK;
}
