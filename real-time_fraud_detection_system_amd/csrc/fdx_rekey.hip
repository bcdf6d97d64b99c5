// fdx_rekey.hip -- K2: stable LSD radix key-sort + segment compaction (re-keying
// CUSTOMER_ID -> TERMINAL_ID), plus permutation gather/scatter.
//
// Replaces the regrouping implied by pandas groupby('CUSTOMER_ID') -> sort_values
// ('TX_DATETIME') -> groupby('TERMINAL_ID') (feature_transformation.ipynb:1092-1093,
// :2435-2436).  Because the input table is already in time order, a STABLE sort on the key
// alone yields per-key time order, which is what the window kernels need.
//
// Per pass (8- or 9-bit digit): hist (per-tile digit counts, wave-private counters fed by a
// ballot multisplit) -> device-wide exclusive scan over the digit-major [bins][tiles] table ->
// scatter (the same multisplit gives the stable in-tile rank; the tile is re-ordered in LDS
// so that the global writes are runs of consecutive addresses).  All traffic is HBM-streaming.
#include <algorithm>
#include <type_traits>

#include "fdx_internal.h"

namespace fdx {
namespace {

constexpr int kRadixBits = 8;   // default digit; 9-bit digits when they save a pass (17-18-bit keys)
constexpr int kMaxBins = 512;
constexpr int kBlock = 256;
constexpr int kItems = 16;
constexpr int kTile = kBlock * kItems;  // 4096 keys per tile
constexpr int kWavesPerBlock = kBlock / kWave;

// ---------------------------------------------------------------- device-wide scan
constexpr int kScanBlock = 256;
constexpr int kScanItems = 16;
constexpr int kScanChunk = kScanBlock * kScanItems;

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint32_t u = __shfl_up(v, d, kWave);
        if (lane >= d) v += u;
    }
    return v;
}

// exclusive block scan of one value per thread; returns the block total via *total
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *total) {
    __shared__ uint32_t s_w[kScanBlock / kWave];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    uint32_t inc = wave_incl_scan_u32(v, lane);
    if (lane == kWave - 1) s_w[wv] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kScanBlock / kWave; ++w) {
        uint32_t x = s_w[w];
        if (w < wv) base += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

__global__ void __launch_bounds__(kScanBlock) k_scan_partials(const uint32_t *__restrict__ in,
                                                              int64_t m, uint32_t *__restrict__ part) {
    const int64_t base = (int64_t)blockIdx.x * kScanChunk;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        int64_t i = base + (int64_t)k * kScanBlock + threadIdx.x;
        if (i < m) s += in[i];
    }
    uint32_t tot;
    block_excl_scan(s, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// single block: exclusive scan of part[0..P) in place
__global__ void __launch_bounds__(kScanBlock) k_scan_single(uint32_t *__restrict__ part, int64_t P) {
    uint32_t carry = 0;
    for (int64_t c = 0; c < P; c += kScanBlock) {
        int64_t i = c + threadIdx.x;
        uint32_t v = i < P ? part[i] : 0u;
        uint32_t tot;
        uint32_t ex = block_excl_scan(v, &tot);
        if (i < P) part[i] = ex + carry;
        carry += tot;
    }
}

// out = exclusive_scan(in) using the per-chunk bases in part (may alias in == out)
__global__ void __launch_bounds__(kScanBlock) k_scan_apply(const uint32_t *in, int64_t m,
                                                           const uint32_t *__restrict__ part,
                                                           uint32_t *out) {
    const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        int64_t i = base + k;
        v[k] = i < m ? in[i] : 0u;
        s += v[k];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan(s, &tot) + part[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        int64_t i = base + k;
        if (i < m) out[i] = ex;
        ex += v[k];
    }
}

int64_t scan_partials_count(int64_t m) { return ceil_div(m, kScanChunk); }

// scratch words of exclusive_scan (uint32): the partials.  (Round 4 measured a single-launch
// decoupled look-back scan in their place: bit-identical and no faster in the re-keys -- 0.591 /
// 0.513 vs 0.555 / 0.504 ms alone, profiles/r04h_bench*.json -- and removed it.)
int64_t scan_scratch_words(int64_t m) { return scan_partials_count(m) + 1; }

int exclusive_scan(uint32_t *data, int64_t m, uint32_t *part, hipStream_t st) {
    if (m == 0) return FDX_OK;
    const int64_t P = scan_partials_count(m);
    hipLaunchKernelGGL(k_scan_partials, dim3((unsigned)P), dim3(kScanBlock), 0, st, data, m, part);
    FDX_LAUNCHED("k_scan_partials");
    hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(kScanBlock), 0, st, part, P);
    FDX_LAUNCHED("k_scan_single");
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)P), dim3(kScanBlock), 0, st, data, m, part, data);
    FDX_LAUNCHED("k_scan_apply");
    return FDX_OK;
}

// ------------------------------------------------------------------- radix passes
template <typename K, int BITS>
__device__ __forceinline__ uint32_t digit_of(K k, int shift, K flip) {
    return (uint32_t)(((k ^ flip) >> shift) & (K)((1 << BITS) - 1));
}

// Per-tile digit counts, in the scatter's blocked order (wave w counts the 1,024 consecutive
// keys [w * 1024, (w + 1) * 1024) of the tile).  Each wave keeps its own LDS counters (one
// block-shared atomicAdd per key spent ~70 % of its LDS cycles on same-address conflicts, r02
// PMC); each key is one LDS atomic add on them (the ballot multisplit -- only the lowest lane
// of each group of equal digits adds the group's size -- took BITS ballots per key, which the
// counts alone do not need: re-keys 0.585 / 0.553 -> 0.553 / 0.534 ms, r03am_radix_hist_ab.txt).
// bad != nullptr (first pass of fdx_rekey_payload_checked): also count the keys >= key_limit
// (as unsigned: negative int32 ids count too) -- the id range check rides on this pass's reads.
template <typename K, int BITS>
__global__ void __launch_bounds__(kBlock) k_radix_hist(const K *__restrict__ keys, int64_t n, int shift,
                                                       K flip, int64_t n_tiles,
                                                       uint32_t *__restrict__ hist, uint64_t key_limit = 0,
                                                       int32_t *__restrict__ bad = nullptr) {
    constexpr int kBins = 1 << BITS;
    constexpr int kWaveSpan = kTile / kWavesPerBlock;
    __shared__ uint32_t s_h[kWavesPerBlock][kBins];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    for (int d = tid; d < kWavesPerBlock * kBins; d += kBlock) (&s_h[0][0])[d] = 0;
    __syncthreads();
    const int64_t wbase = (int64_t)blockIdx.x * kTile + (int64_t)wv * kWaveSpan + lane;
    uint32_t *h = s_h[wv];
    K key[kItems];
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const int64_t i = wbase + (int64_t)r * kWave;
        key[r] = i < n ? keys[i] : (K)0;
    }
    // counts only (no ranks): one LDS atomic add per key on the wave's own counters -- lanes of
    // one digit in one instruction serialise on their address
#pragma unroll
    for (int r = 0; r < kItems; ++r)
        if (wbase + (int64_t)r * kWave < n) atomicAdd(&h[digit_of<K, BITS>(key[r], shift, flip)], 1u);
    if (bad) {
        int nb = 0;
#pragma unroll
        for (int r = 0; r < kItems; ++r)
            nb += __popcll(__ballot(wbase + (int64_t)r * kWave < n && (uint64_t)key[r] >= key_limit));
        if (lane == 0 && nb) atomicAdd(bad, nb);
    }
    __syncthreads();
    for (int d = tid; d < kBins; d += kBlock) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; ++w) c += s_h[w][d];
        hist[(int64_t)d * n_tiles + blockIdx.x] = c;
    }
}

// Tile of this scatter block, XCD-aware: workgroups go to the 8 XCDs round robin, so block b
// takes tile (b % 8) * ceil(n_tiles / 8) + b / 8 -- each XCD scatters a contiguous range of
// tiles, and the digit runs that neighbouring tiles write side by side meet in that XCD's L2
// instead of leaving as partial lines from two L2s (config 2: customer re-key 0.78 -> 0.66 ms,
// terminal 0.70 -> 0.61 ms, 64-bit argsort 1.60 -> 1.48 ms; bit-identical, profiles/r03q*).
__device__ __forceinline__ int64_t scatter_tile(int64_t n_tiles) {
    const int64_t per = (n_tiles + 7) / 8;
    return (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
}
inline unsigned scatter_grid(int64_t n_tiles) { return (unsigned)((n_tiles + 7) / 8 * 8); }

// Stable scatter of one tile (BLOCKED: wave w owns the 1,024 consecutive input positions
// [w * 1024, (w + 1) * 1024) of the tile, item r of lane l at w * 1024 + r * 64 + l -- still
// coalesced loads).  vals_in == nullptr means "the value is the row index" (with bit 31 =
// flag_in[row] != 0 when flag_in is given: fdx_rekey_payload's packed flag).  PW > 0: PW
// 8-byte payload streams ride along: after the keys are out, each stream is loaded coalesced
// in input order, re-ordered through LDS (reusing the key/value buffers as 4,096 8-byte slots)
// with the same tile permutation, and written to the destinations the key pass computed --
// the same coalesced runs as the keys, so the grouped payload reads sequentially downstream
// (gathering it through the permutation took a random HBM line per 8-byte element: round-1
// PMC 3-6x the algorithmic bytes).  Input order inside the tile is then (wave, item, lane), so each
// wave ranks its 16 items against wave-private digit counters (ballot multisplit; the leader
// lane of each digit group bumps the counter) with no block barrier, and one barrier later the
// per-digit scan over the four waves' counts gives each wave its offset: 3 barriers per tile
// instead of 3 per item (measured on MI355X at config 2: terminal re-key 0.686 -> 0.611 ms,
// 64-bit argsort 2.43 -> 1.59 ms, customer re-key unchanged; bit-identical,
// tools/radix_ab.py).  The tile's global digit offsets are staged in LDS once.
template <typename K, int BITS, int PW>
__global__ void __launch_bounds__(kBlock) k_radix_scatter(
    const K *__restrict__ keys_in, const uint32_t *__restrict__ vals_in, int64_t n, int shift, K flip,
    int64_t n_tiles, const uint32_t *__restrict__ offsets, K *__restrict__ keys_out,
    uint32_t *__restrict__ vals_out, const uint8_t *__restrict__ flag_in, const uint64_t *__restrict__ p0_in,
    const uint64_t *__restrict__ p1_in, uint64_t *__restrict__ p0_out, uint64_t *__restrict__ p1_out) {
    constexpr int kBins = 1 << BITS, kPer = kBins / kBlock;
    static_assert(kBins % kBlock == 0, "digit bins must be a multiple of the block");
    constexpr int kWaveSpan = kTile / kWavesPerBlock;  // 1,024 input positions per wave
    __shared__ uint32_t s_cnt[kWavesPerBlock][kBins];  // wave-private counts, then wave offsets
    __shared__ int32_t s_goff[kBins];                  // global destination of tile position 0 per digit
    constexpr int kKeyWords = (int)(sizeof(K) / 4);
    __shared__ __align__(16) uint32_t s_kv[(kKeyWords + 1) * kTile];
    K *s_key = reinterpret_cast<K *>(s_kv);
    uint32_t *s_val = s_kv + kKeyWords * kTile;

    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
    const int64_t tile = scatter_tile(n_tiles);
    if (tile >= n_tiles) return;
    const int64_t base = tile * kTile;
    const int64_t wbase = base + (int64_t)wv * kWaveSpan + lane;  // + r * 64: item r of this lane
    for (int d = tid; d < kBins; d += kBlock)
#pragma unroll
        for (int w = 0; w < kWavesPerBlock; ++w) s_cnt[w][d] = 0;
    __syncthreads();

    K key[kItems];
    uint32_t val[kItems], rank[kItems], dig[kItems];
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t *cnt = s_cnt[wv];
    // every load of the tile issued before the first use: one straight-line copy per uniform
    // case and for full tiles (all but the last) no per-item bound test -- with the case and the
    // bound tested per item, the flag byte's use right after its load made the compiler wait
    // for each item in turn (16 dependent HBM round trips per tile)
    const bool full = base + kTile <= n;  // uniform
    if (vals_in) {
        if (full) {
#pragma unroll
            for (int r = 0; r < kItems; ++r) {
                const int64_t i = wbase + (int64_t)r * kWave;
                key[r] = keys_in[i];
                val[r] = vals_in[i];
            }
        } else {
#pragma unroll
            for (int r = 0; r < kItems; ++r) {
                const int64_t i = wbase + (int64_t)r * kWave, j = min(i, n - 1);
                key[r] = i < n ? keys_in[j] : (K)0;
                val[r] = i < n ? vals_in[j] : 0u;
            }
        }
    } else if (flag_in) {
        uint32_t fl[kItems];
#pragma unroll
        for (int r = 0; r < kItems; ++r) {
            const int64_t i = min(wbase + (int64_t)r * kWave, n - 1);  // (full tiles: never clamped)
            key[r] = keys_in[i];
            fl[r] = flag_in[i];
        }
#pragma unroll
        for (int r = 0; r < kItems; ++r) {
            const int64_t i = wbase + (int64_t)r * kWave;
            val[r] = (uint32_t)i | (fl[r] ? 0x80000000u : 0u);
            if (i >= n) key[r] = (K)0;
        }
    } else {
#pragma unroll
        for (int r = 0; r < kItems; ++r) {
            const int64_t i = wbase + (int64_t)r * kWave;
            key[r] = i < n ? keys_in[min(i, n - 1)] : (K)0;
            val[r] = (uint32_t)i;
        }
    }
    // payload registers: stream q's 16 values of this lane, coalesced in input order (clamped:
    // no branch); the loads of stream 0 go out behind the key re-order and those of stream q + 1
    // while stream q is re-ordered (r03: each after the previous phase's stores, or stream 0 with
    // the keys -- 170 VGPRs -- measured slower)
    uint64_t pv[PW > 0 ? kItems : 1];
    auto load_pay = [&](const uint64_t *pin) {
#pragma unroll
        for (int r = 0; r < kItems; ++r) pv[r] = pin[min(wbase + (int64_t)r * kWave, n - 1)];
    };
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const int64_t i = wbase + (int64_t)r * kWave;
        const bool valid = i < n;
        const uint32_t d = digit_of<K, BITS>(key[r], shift, flip);
        dig[r] = d;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < BITS; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t in_wave = (uint32_t)__popcll(peers & lt_mask);
        const uint32_t old = valid ? cnt[d] : 0u;
        // every lane's read of the counter before the leader's update (LDS ops of a wave
        // execute in order; the fences keep the compiler from moving them)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (valid && in_wave == 0) cnt[d] = old + (uint32_t)__popcll(peers);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        rank[r] = old + in_wave;
    }
    __syncthreads();
    // per digit: tile start (exclusive scan over digits of the tile totals), each wave's offset
    // (tile start + the counts of the earlier waves) and the global destination of position 0
    {
        uint32_t c[kPer][kWavesPerBlock], tot_d[kPer], sum = 0;
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            tot_d[q] = 0;
#pragma unroll
            for (int w = 0; w < kWavesPerBlock; ++w) {
                c[q][w] = s_cnt[w][tid * kPer + q];
                tot_d[q] += c[q][w];
            }
            sum += tot_d[q];
        }
        uint32_t tot;
        uint32_t ex = block_excl_scan(sum, &tot);  // (its own barriers: every s_cnt read above is done)
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int d = tid * kPer + q;
            uint32_t o = ex;
#pragma unroll
            for (int w = 0; w < kWavesPerBlock; ++w) {
                s_cnt[w][d] = o;
                o += c[q][w];
            }
            s_goff[d] = (int32_t)offsets[(int64_t)d * n_tiles + tile] - (int32_t)ex;
            ex += tot_d[q];
        }
    }
    __syncthreads();
    uint32_t pos[kItems];
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        if (wbase + (int64_t)r * kWave < n) {
            const uint32_t p = cnt[dig[r]] + rank[r];
            pos[r] = p;
            s_key[p] = key[r];
            s_val[p] = val[r];
        }
    }
    if constexpr (PW > 0) load_pay(p0_in);
    __syncthreads();
    const int64_t tcnt = std::min<int64_t>(kTile, n - base);
    int32_t dsts[kItems];  // destination of tile position tid + j * kBlock
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const int p = tid + j * kBlock;
        if (p < tcnt) {
            const K k = s_key[p];
            const int32_t dst = s_goff[digit_of<K, BITS>(k, shift, flip)] + p;
            dsts[j] = dst;
            keys_out[dst] = k;
            vals_out[dst] = s_val[p];
        }
    }
    if constexpr (PW > 0) {
        uint64_t *s_pay = reinterpret_cast<uint64_t *>(s_kv);
#pragma unroll
        for (int q = 0; q < PW; ++q) {
            uint64_t *pout = q == 0 ? p0_out : p1_out;
            __syncthreads();  // the previous contents of the LDS slots are consumed
#pragma unroll
            for (int r = 0; r < kItems; ++r)
                if (wbase + (int64_t)r * kWave < n) s_pay[pos[r]] = pv[r];
            if (q + 1 < PW) load_pay(p1_in);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kItems; ++j) {
                const int p = tid + j * kBlock;
                if (p < tcnt) pout[dsts[j]] = s_pay[p];
            }
        }
    }
}

__global__ void k_iota(uint32_t *__restrict__ out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)i;
}

__global__ void k_copy_u32(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

// seg_off[q] = first sorted position whose key >= q, for q in [0, n_keys], in ONE pass over the
// sorted keys: every boundary i (key sk[i-1] < sk[i], or i = 0) writes seg_off[q] = i for the keys
// q in (sk[i-1], sk[i]] -- absent keys included, so no search -- and the last row writes n for
// (sk[n-1], n_keys].  Each q is written once when the keys are sorted and in range.  (Three
// launches before -- fill -1, mark the present keys, binary-search the absent ones.)  The buffer
// is zeroed first, so that out-of-range ids -- which sort out of key order and are rejected
// after the step (fdx_rekey_payload_checked) -- can never leave an offset outside [0, n].
__device__ __forceinline__ void seg_bound(int64_t i, int64_t prev, int64_t cur, int64_t n_keys,
                                          int64_t *__restrict__ seg_off) {
    const int64_t q1 = min(cur, n_keys);
    for (int64_t q = prev + 1; q <= q1; ++q) seg_off[q] = i;
}

__global__ void k_seg_bounds(const uint32_t *__restrict__ sk, int64_t n, int64_t n_keys,
                             int64_t *__restrict__ seg_off) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t cur = sk[i];
        seg_bound(i, i > 0 ? (int64_t)sk[i - 1] : -1, cur, n_keys, seg_off);
        if (i == n - 1) seg_bound(n, cur, n_keys, n_keys, seg_off);
    }
}

// k_seg_bounds over 16-byte aligned keys, 4 per thread and trip (one 16-byte load; the previous
// key an L1 / L2 hit, the neighbouring thread's line)
__global__ void k_seg_bounds4(const uint32_t *__restrict__ sk, int64_t n, int64_t n_keys,
                              int64_t *__restrict__ seg_off) {
    const int64_t n4 = n / 4;
    const uint4 *sk4 = reinterpret_cast<const uint4 *>(sk);
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
        const uint4 v = sk4[q];
        const int64_t i = 4 * q;
        seg_bound(i, q > 0 ? (int64_t)sk[i - 1] : -1, v.x, n_keys, seg_off);
        seg_bound(i + 1, v.x, v.y, n_keys, seg_off);
        seg_bound(i + 2, v.y, v.z, n_keys, seg_off);
        seg_bound(i + 3, v.z, v.w, n_keys, seg_off);
        if (i + 3 == n - 1) seg_bound(n, v.w, n_keys, n_keys, seg_off);
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {  // the last n % 4 keys
        const int64_t cur = sk[i];
        seg_bound(i, i > 0 ? (int64_t)sk[i - 1] : -1, cur, n_keys, seg_off);
        if (i == n - 1) seg_bound(n, cur, n_keys, n_keys, seg_off);
    }
}

__global__ void k_zero_i64(int64_t *__restrict__ p, int64_t m) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = 0;
}

int seg_offsets(const uint32_t *sk, int64_t n, int64_t n_keys, int64_t *seg_off, hipStream_t st) {
    // (one launch: hipMemsetAsync of the (n_keys + 1) x 8 bytes took two fill kernels, ~12 us on
    // the terminal half's chain between its last scatter and its windows, r06ax trace)
    hipLaunchKernelGGL(k_zero_i64, dim3(stream_grid(n_keys + 1, 256)), dim3(256), 0, st, seg_off, n_keys + 1);
    FDX_LAUNCHED("k_zero_i64");
    if (((uintptr_t)sk & 15) == 0) {  // (the radix buffers; a caller's sorted_keys_d may not be)
        hipLaunchKernelGGL(k_seg_bounds4, dim3(stream_grid(ceil_div(n, 4), 256)), dim3(256), 0, st, sk, n, n_keys,
                           seg_off);
        FDX_LAUNCHED("k_seg_bounds4");
    } else {
        hipLaunchKernelGGL(k_seg_bounds, dim3(stream_grid(n, 256)), dim3(256), 0, st, sk, n, n_keys, seg_off);
        FDX_LAUNCHED("k_seg_bounds");
    }
    return FDX_OK;
}

// Key histogram -> the segment offsets of the stable grouping by key (= fdx_rekey's seg_off for
// keys in [0, n_keys)), without sorting: what the customer layout's plan needs, so that it can
// run while the rows are being re-keyed.  Keys outside the range are counted in *bad.
__global__ void k_key_hist(const int32_t *__restrict__ keys, int64_t n, int64_t n_keys, uint32_t *__restrict__ cnt,
                           int32_t *__restrict__ bad) {
    int nbad = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t k = keys[i];
        if (k >= 0 && (int64_t)k < n_keys) atomicAdd(&cnt[k], 1u);
        else ++nbad;
    }
    if (bad) {
        for (int d = kWave / 2; d > 0; d >>= 1) nbad += __shfl_down(nbad, d, kWave);
        if ((threadIdx.x & (kWave - 1)) == 0 && nbad) atomicAdd(bad, nbad);
    }
}

__global__ void k_widen_u32(const uint32_t *__restrict__ in, int64_t m, int64_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

template <typename T>
__global__ void k_gather(const T *__restrict__ src, const int32_t *__restrict__ perm, int64_t n,
                         T *__restrict__ dst) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[perm[i]];
}

template <typename T>
__global__ void k_scatter(const T *__restrict__ src, const int32_t *__restrict__ perm, int64_t n,
                          T *__restrict__ dst) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        dst[perm[i]] = src[i];
}

__global__ void k_check_sorted_i64(const int64_t *__restrict__ k, int64_t n, int32_t *__restrict__ flag) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        if (k[i] < k[i - 1]) *flag = 0;
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace of one radix sort of n keys of type K: two ping-pong key/value buffers, the
// digit histogram table and the scan partials.
template <typename K>
struct SortWs {
    K *k0, *k1;
    uint32_t *v0, *v1, *hist, *part;
    uint64_t *q[2][2];  // payload ping-pong buffers [stream][parity] (PW streams)
};

template <typename K>
size_t sort_ws(int64_t n, SortWs<K> *w, char *base, int pw = 0) {
    const int64_t tiles = std::max<int64_t>(1, ceil_div(n, kTile));
    const int64_t hm = tiles * kMaxBins;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char *p = base ? base + off : nullptr;
        off += align_up(bytes);
        return p;
    };
    SortWs<K> t;
    t.k0 = reinterpret_cast<K *>(take(sizeof(K) * n));
    t.k1 = reinterpret_cast<K *>(take(sizeof(K) * n));
    t.v0 = reinterpret_cast<uint32_t *>(take(sizeof(uint32_t) * n));
    t.v1 = reinterpret_cast<uint32_t *>(take(sizeof(uint32_t) * n));
    t.hist = reinterpret_cast<uint32_t *>(take(sizeof(uint32_t) * hm));
    t.part = reinterpret_cast<uint32_t *>(take(sizeof(uint32_t) * (scan_scratch_words(hm) + 2)));
    for (int q = 0; q < 2; ++q)
        for (int par = 0; par < 2; ++par)
            t.q[q][par] = q < pw ? reinterpret_cast<uint64_t *>(take(sizeof(uint64_t) * n)) : nullptr;
    if (w) *w = t;
    return off;
}

// Stable LSD radix sort of (key, row index) pairs over the low `bits` bits of (key ^ flip).
// vals_out receives the input row index of each sorted position (| flag << 31 with flag_in);
// keys_out (optional) the sorted keys; pay_out[q] (PW streams) the payload in sorted order.
// Returns the buffer that holds the sorted keys.
template <typename K, int BITS, int PW>
void launch_scatter(const K *kin, const uint32_t *vin, int64_t n, int shift, K flip, int64_t tiles,
                    const uint32_t *hist, K *kout, uint32_t *vout, const uint8_t *flag_in, const uint64_t *const (&pin)[2],
                    uint64_t *const (&pout)[2], hipStream_t st) {
    hipLaunchKernelGGL((k_radix_scatter<K, BITS, PW>), dim3(scatter_grid(tiles)), dim3(kBlock), 0, st, kin, vin, n, shift,
                       flip, tiles, hist, kout, vout, flag_in, pin[0], pin[1], pout[0], pout[1]);
}

// The digit schedule of a `bits`-bit key: passes, and how many leading passes take 9 bits.
// 9-bit digits only where they save a pass (17- and 18-bit keys: 2 passes, not 3), and then
// only as many as the key needs: 17 bits = 9 + 8 -- an 8-bit pass writes runs of ~16 keys
// per digit and 4,096-key tile (a 9-bit pass ~8: twice the partial lines)
void digit_plan(int bits, int *passes_out, int *n9_out) {
    const int p8 = (bits + kRadixBits - 1) / kRadixBits, p9 = (bits + 8) / 9;
    const int passes = std::min(p8, p9);
    *passes_out = passes;
    *n9_out = p9 < p8 ? std::max(0, bits - kRadixBits * passes) : 0;
}

// The first pass's per-tile digit table, scanned (what its scatter reads), into hist / part.
template <typename K>
int pass0_table(const K *keys, int64_t n, int bits, K flip, uint32_t *hist, uint32_t *part, uint64_t key_limit,
                int32_t *bad, hipStream_t st) {
    int passes, n9;
    digit_plan(bits, &passes, &n9);
    const int64_t tiles = ceil_div(n, kTile);
    const int dbits = n9 > 0 ? 9 : kRadixBits;
    if (dbits == 9)
        hipLaunchKernelGGL((k_radix_hist<K, 9>), dim3((unsigned)tiles), dim3(kBlock), 0, st, keys, n, 0, flip, tiles,
                           hist, key_limit, bad);
    else
        hipLaunchKernelGGL((k_radix_hist<K, kRadixBits>), dim3((unsigned)tiles), dim3(kBlock), 0, st, keys, n, 0, flip,
                           tiles, hist, key_limit, bad);
    FDX_LAUNCHED("k_radix_hist");
    return exclusive_scan(hist, tiles * ((int64_t)1 << dbits), part, st);
}

// hist0 != nullptr: the first pass's scanned table, computed beforehand by pass0_table (e.g. on
// another stream, while something else runs) -- the pass goes straight to its scatter.
template <typename K>
int radix_sort(const K *keys, int64_t n, int bits, K flip, K *keys_out, uint32_t *vals_out,
               const SortWs<K> &w, hipStream_t st, const K **sorted, int pw = 0, const uint8_t *flag_in = nullptr,
               const uint64_t *const *pay_in = nullptr, uint64_t *const *pay_out = nullptr, uint64_t key_limit = 0,
               int32_t *bad = nullptr, const uint32_t *hist0 = nullptr) {
    const int64_t tiles = ceil_div(n, kTile);
    int passes, n9;
    digit_plan(bits, &passes, &n9);
    const K *kin = keys;
    const uint32_t *vin = nullptr;  // identity on the first pass
    const uint64_t *pin[2] = {pw > 0 ? pay_in[0] : nullptr, pw > 1 ? pay_in[1] : nullptr};
    if (passes == 0) {
        if (flag_in) {
            set_error("a packed flag needs at least one radix pass");
            return FDX_E_INVALID;
        }
        hipLaunchKernelGGL(k_iota, dim3(stream_grid(n, 256)), dim3(256), 0, st, vals_out, n);
        FDX_LAUNCHED("k_iota");
        for (int q = 0; q < pw; ++q)
            FDX_HIP(hipMemcpyAsync(pay_out[q], pay_in[q], sizeof(uint64_t) * n, hipMemcpyDeviceToDevice, st));
        *sorted = keys;
        return FDX_OK;
    }
    for (int p = 0; p < passes; ++p) {
        const int dbits = p < n9 ? 9 : kRadixBits;
        const int shift = p < n9 ? 9 * p : 9 * n9 + kRadixBits * (p - n9);
        const bool last = p == passes - 1;
        K *kout = (p & 1) ? w.k1 : w.k0;
        if (last && keys_out) kout = keys_out;
        uint32_t *vout = last ? vals_out : ((p & 1) ? w.v1 : w.v0);
        uint64_t *pout[2] = {nullptr, nullptr};
        for (int q = 0; q < pw; ++q) pout[q] = last ? pay_out[q] : w.q[q][p & 1];
        int32_t *bad_p = p == 0 ? bad : nullptr;
        const uint32_t *htab = p == 0 && hist0 ? hist0 : w.hist;
        if (htab == w.hist) {
            if (dbits == 9)
                hipLaunchKernelGGL((k_radix_hist<K, 9>), dim3((unsigned)tiles), dim3(kBlock), 0, st, kin, n, shift,
                                   flip, tiles, w.hist, key_limit, bad_p);
            else
                hipLaunchKernelGGL((k_radix_hist<K, kRadixBits>), dim3((unsigned)tiles), dim3(kBlock), 0, st, kin, n,
                                   shift, flip, tiles, w.hist, key_limit, bad_p);
            FDX_LAUNCHED("k_radix_hist");
            int rc = exclusive_scan(w.hist, tiles * ((int64_t)1 << dbits), w.part, st);
            if (rc) return rc;
        }
        const uint8_t *fl = p == 0 ? flag_in : nullptr;
#define FDX_SCATTER(B, PWV) \
    launch_scatter<K, B, PWV>(kin, vin, n, shift, flip, tiles, htab, kout, vout, fl, pin, pout, st)
        if (dbits == 9) {
            if (pw == 2) FDX_SCATTER(9, 2); else if (pw == 1) FDX_SCATTER(9, 1); else FDX_SCATTER(9, 0);
        } else {
            if (pw == 2) FDX_SCATTER(kRadixBits, 2); else if (pw == 1) FDX_SCATTER(kRadixBits, 1); else FDX_SCATTER(kRadixBits, 0);
        }
#undef FDX_SCATTER
        FDX_LAUNCHED("k_radix_scatter");
        kin = kout;
        vin = vout;
        for (int q = 0; q < pw; ++q) pin[q] = pout[q];
    }
    *sorted = kin;
    return FDX_OK;
}

}  // namespace
}  // namespace fdx

using namespace fdx;

extern "C" size_t fdx_rekey_workspace_size(int64_t n, int32_t key_bits) {
    (void)key_bits;
    if (n < 0) n = 0;
    return sort_ws<uint32_t>(n, nullptr, nullptr);
}

extern "C" int fdx_rekey(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys,
                         int32_t *perm_d, int32_t *sorted_keys_d, int64_t *seg_off_d,
                         void *workspace_d, size_t workspace_bytes, void *stream) {
    FDX_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "n out of range");
    FDX_REQUIRE(key_bits >= 0 && key_bits <= 31, "key_bits must be in [0, 31]");
    FDX_REQUIRE(n_keys >= 1 && n_keys <= (int64_t(1) << key_bits), "n_keys must be in [1, 2^key_bits]");
    hipStream_t st = as_stream(stream);
    if (n == 0) {
        if (seg_off_d) FDX_HIP(hipMemsetAsync(seg_off_d, 0, sizeof(int64_t) * (n_keys + 1), st));
        return FDX_OK;
    }
    FDX_REQUIRE(keys_d && perm_d, "null keys/perm");
    SortWs<uint32_t> w;
    size_t need = sort_ws<uint32_t>(n, &w, reinterpret_cast<char *>(workspace_d));
    if (!workspace_d || workspace_bytes < need) {
        set_error("rekey workspace too small: %zu < %zu", workspace_bytes, need);
        return FDX_E_WORKSPACE;
    }
    const uint32_t *sorted = nullptr;
    int rc = radix_sort<uint32_t>(reinterpret_cast<const uint32_t *>(keys_d), n, key_bits, 0u,
                                  reinterpret_cast<uint32_t *>(sorted_keys_d),
                                  reinterpret_cast<uint32_t *>(perm_d), w, st, &sorted);
    if (rc) return rc;
    if (sorted_keys_d && sorted != reinterpret_cast<const uint32_t *>(sorted_keys_d)) {
        hipLaunchKernelGGL(k_copy_u32, dim3(stream_grid(n, 256)), dim3(256), 0, st, sorted,
                           reinterpret_cast<uint32_t *>(sorted_keys_d), n);
        FDX_LAUNCHED("k_copy_u32");
    }
    if (seg_off_d) return seg_offsets(sorted, n, n_keys, seg_off_d, st);
    return FDX_OK;
}

extern "C" size_t fdx_rekey_payload_workspace_size(int64_t n, int32_t key_bits, int32_t n_payload) {
    (void)key_bits;
    if (n < 0) n = 0;
    return sort_ws<uint32_t>(n, nullptr, nullptr, n_payload < 0 ? 0 : (n_payload > 2 ? 2 : n_payload));
}

static int rekey_payload(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys, const uint8_t *flag_d,
                         const uint64_t *pay0_d, const uint64_t *pay1_d, int32_t *perm_d, int64_t *seg_off_d,
                         uint64_t *pay0_out_d, uint64_t *pay1_out_d, int32_t *bad_d, void *workspace_d,
                         size_t workspace_bytes, void *stream, int32_t *sorted_keys_d = nullptr,
                         const uint32_t *hist0_d = nullptr);

extern "C" int fdx_rekey_payload(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys,
                                 const uint8_t *flag_d, const uint64_t *pay0_d, const uint64_t *pay1_d, int32_t *perm_d,
                                 int64_t *seg_off_d, uint64_t *pay0_out_d, uint64_t *pay1_out_d, void *workspace_d,
                                 size_t workspace_bytes, void *stream) {
    return rekey_payload(keys_d, n, key_bits, n_keys, flag_d, pay0_d, pay1_d, perm_d, seg_off_d, pay0_out_d,
                         pay1_out_d, nullptr, workspace_d, workspace_bytes, stream);
}

extern "C" int fdx_rekey_payload_checked(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys,
                                         const uint8_t *flag_d, const uint64_t *pay0_d, const uint64_t *pay1_d,
                                         int32_t *perm_d, int64_t *seg_off_d, uint64_t *pay0_out_d,
                                         uint64_t *pay1_out_d, int32_t *bad_d, void *workspace_d,
                                         size_t workspace_bytes, void *stream) {
    FDX_REQUIRE(bad_d, "null bad_d");
    return rekey_payload(keys_d, n, key_bits, n_keys, flag_d, pay0_d, pay1_d, perm_d, seg_off_d, pay0_out_d,
                         pay1_out_d, bad_d, workspace_d, workspace_bytes, stream);
}

extern "C" int fdx_rekey_payload_keys(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys,
                                      const uint8_t *flag_d, const uint64_t *pay0_d, const uint64_t *pay1_d,
                                      int32_t *perm_d, int32_t *sorted_keys_d, uint64_t *pay0_out_d,
                                      uint64_t *pay1_out_d, int32_t *bad_d, void *workspace_d, size_t workspace_bytes,
                                      void *stream) {
    FDX_REQUIRE(n == 0 || sorted_keys_d, "null sorted_keys_d");
    FDX_REQUIRE(((uintptr_t)sorted_keys_d & 15) == 0, "sorted_keys_d must be 16-byte aligned");
    return rekey_payload(keys_d, n, key_bits, n_keys, flag_d, pay0_d, pay1_d, perm_d, nullptr, pay0_out_d,
                         pay1_out_d, bad_d, workspace_d, workspace_bytes, stream, sorted_keys_d);
}

extern "C" size_t fdx_rekey_hist0_size(int64_t n, int32_t key_bits) {
    if (n < 0) n = 0;
    int passes, n9;
    digit_plan(key_bits, &passes, &n9);
    const int64_t hm = std::max<int64_t>(1, ceil_div(n, kTile)) * ((int64_t)1 << (n9 > 0 ? 9 : kRadixBits));
    return align_up(sizeof(uint32_t) * (size_t)hm) + sizeof(uint32_t) * (size_t)(scan_scratch_words(hm) + 2);
}

extern "C" int fdx_rekey_hist0(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys, void *hist0_d,
                               size_t hist0_bytes, int32_t *bad_d, void *stream) {
    FDX_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "n out of range");
    FDX_REQUIRE(key_bits >= 1 && key_bits <= 31, "key_bits must be in [1, 31]");
    FDX_REQUIRE(n_keys >= 1 && n_keys <= (int64_t(1) << key_bits), "n_keys must be in [1, 2^key_bits]");
    FDX_REQUIRE(hist0_d && (n == 0 || keys_d), "null pointer");
    FDX_REQUIRE(hist0_bytes >= fdx_rekey_hist0_size(n, key_bits), "hist0 buffer too small");
    hipStream_t st = as_stream(stream);
    if (bad_d) FDX_HIP(hipMemsetAsync(bad_d, 0, sizeof(int32_t), st));
    if (n == 0) return FDX_OK;
    int passes, n9;
    digit_plan(key_bits, &passes, &n9);
    const int64_t hm = ceil_div(n, kTile) * ((int64_t)1 << (n9 > 0 ? 9 : kRadixBits));
    uint32_t *hist = reinterpret_cast<uint32_t *>(hist0_d);
    uint32_t *part = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(hist0_d) +
                                                  align_up(sizeof(uint32_t) * (size_t)hm));
    return pass0_table<uint32_t>(reinterpret_cast<const uint32_t *>(keys_d), n, key_bits, 0u, hist, part,
                                 (uint64_t)n_keys, bad_d, st);
}

extern "C" int fdx_rekey_payload_hist0(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys,
                                       const uint8_t *flag_d, const uint64_t *pay0_d, const uint64_t *pay1_d,
                                       int32_t *perm_d, int64_t *seg_off_d, uint64_t *pay0_out_d, uint64_t *pay1_out_d,
                                       const void *hist0_d, void *workspace_d, size_t workspace_bytes, void *stream) {
    FDX_REQUIRE(n == 0 || hist0_d, "null hist0_d");
    return rekey_payload(keys_d, n, key_bits, n_keys, flag_d, pay0_d, pay1_d, perm_d, seg_off_d, pay0_out_d,
                         pay1_out_d, nullptr, workspace_d, workspace_bytes, stream, nullptr,
                         reinterpret_cast<const uint32_t *>(hist0_d));
}

extern "C" int fdx_segment_offsets_sorted(const int32_t *sorted_keys_d, int64_t n, int64_t n_keys, int64_t *seg_off_d,
                                          void *stream) {
    FDX_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "n out of range");
    FDX_REQUIRE(n_keys >= 1 && n_keys < (int64_t)INT32_MAX, "n_keys out of range");
    FDX_REQUIRE(seg_off_d && (n == 0 || sorted_keys_d), "null pointer");
    hipStream_t st = as_stream(stream);
    if (n == 0) {
        FDX_HIP(hipMemsetAsync(seg_off_d, 0, sizeof(int64_t) * (n_keys + 1), st));
        return FDX_OK;
    }
    return seg_offsets(reinterpret_cast<const uint32_t *>(sorted_keys_d), n, n_keys, seg_off_d, st);
}

static int rekey_payload(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys, const uint8_t *flag_d,
                         const uint64_t *pay0_d, const uint64_t *pay1_d, int32_t *perm_d, int64_t *seg_off_d,
                         uint64_t *pay0_out_d, uint64_t *pay1_out_d, int32_t *bad_d, void *workspace_d,
                         size_t workspace_bytes, void *stream, int32_t *sorted_keys_d,
                         const uint32_t *hist0_d) {
    FDX_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "n out of range");
    FDX_REQUIRE(key_bits >= 1 && key_bits <= 31, "key_bits must be in [1, 31]");
    FDX_REQUIRE(n_keys >= 1 && n_keys <= (int64_t(1) << key_bits), "n_keys must be in [1, 2^key_bits]");
    FDX_REQUIRE((pay0_d == nullptr) == (pay0_out_d == nullptr) && (pay1_d == nullptr) == (pay1_out_d == nullptr) &&
                    (pay1_d == nullptr || pay0_d != nullptr),
                "payload inputs and outputs go together (stream 1 needs stream 0)");
    hipStream_t st = as_stream(stream);
    if (bad_d && !hist0_d) FDX_HIP(hipMemsetAsync(bad_d, 0, sizeof(int32_t), st));  // (hist0: counted there)
    if (n == 0) {
        if (seg_off_d) FDX_HIP(hipMemsetAsync(seg_off_d, 0, sizeof(int64_t) * (n_keys + 1), st));
        return FDX_OK;
    }
    FDX_REQUIRE(keys_d && perm_d, "null keys/perm");
    const int pw = pay1_d ? 2 : (pay0_d ? 1 : 0);
    SortWs<uint32_t> w;
    size_t need = sort_ws<uint32_t>(n, &w, reinterpret_cast<char *>(workspace_d), pw);
    if (!workspace_d || workspace_bytes < need) {
        set_error("rekey workspace too small: %zu < %zu", workspace_bytes, need);
        return FDX_E_WORKSPACE;
    }
    const uint64_t *pin[2] = {pay0_d, pay1_d};
    uint64_t *pout[2] = {pay0_out_d, pay1_out_d};
    const uint32_t *sorted = nullptr;
    uint32_t *kout = reinterpret_cast<uint32_t *>(sorted_keys_d);
    int rc = radix_sort<uint32_t>(reinterpret_cast<const uint32_t *>(keys_d), n, key_bits, 0u, kout,
                                  reinterpret_cast<uint32_t *>(perm_d), w, st, &sorted, pw, flag_d, pin, pout,
                                  (uint64_t)n_keys, hist0_d ? nullptr : bad_d, hist0_d);
    if (rc) return rc;
    if (kout && sorted != kout) {  // (no radix pass: the input order is the sorted one)
        hipLaunchKernelGGL(k_copy_u32, dim3(stream_grid(n, 256)), dim3(256), 0, st, sorted, kout, n);
        FDX_LAUNCHED("k_copy_u32");
    }
    if (seg_off_d) return seg_offsets(sorted, n, n_keys, seg_off_d, st);
    return FDX_OK;
}

extern "C" size_t fdx_argsort_i64_workspace_size(int64_t n) {
    if (n < 0) n = 0;
    return sort_ws<uint64_t>(n, nullptr, nullptr);
}

extern "C" int fdx_argsort_i64(const int64_t *keys_d, int64_t n, int32_t *perm_d, void *workspace_d,
                               size_t workspace_bytes, void *stream) {
    FDX_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "n out of range");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(keys_d && perm_d, "null pointer");
    SortWs<uint64_t> w;
    size_t need = sort_ws<uint64_t>(n, &w, reinterpret_cast<char *>(workspace_d));
    if (!workspace_d || workspace_bytes < need) {
        set_error("argsort workspace too small: %zu < %zu", workspace_bytes, need);
        return FDX_E_WORKSPACE;
    }
    const uint64_t *sorted = nullptr;
    // signed order: flip the sign bit so that negative keys sort first
    return radix_sort<uint64_t>(reinterpret_cast<const uint64_t *>(keys_d), n, 64, 1ull << 63, nullptr,
                                reinterpret_cast<uint32_t *>(perm_d), w, as_stream(stream), &sorted);
}

// ---- dense ids of arbitrary int64 keys (the drop-ins' groupby on ids that are not dense) ----
// flags[i] = 1 where the sorted key differs from its predecessor (sorted = sign-flipped u64)
__global__ void k_new_key_flags(const uint64_t *__restrict__ sorted, int64_t n, uint32_t *__restrict__ flags) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        flags[i] = i > 0 && sorted[i] != sorted[i - 1];
}
// ids[perm[i]] = #distinct keys among sorted[0..i] - 1 (= exclusive count + own flag)
__global__ void k_dense_scatter(const uint64_t *__restrict__ sorted, const uint32_t *__restrict__ excl,
                                const int32_t *__restrict__ perm, int64_t n, int32_t *__restrict__ ids,
                                int64_t *__restrict__ n_unique) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = (int32_t)(excl[i] + (i > 0 && sorted[i] != sorted[i - 1] ? 1u : 0u));
        ids[perm[i]] = r;
        if (i == n - 1) *n_unique = (int64_t)r + 1;
    }
}

static size_t dense_ids_parts(int64_t n, size_t *off_perm, size_t *off_flags, size_t *off_scan) {
    const size_t a = align_up(sort_ws<uint64_t>(n, nullptr, nullptr));
    const size_t b = align_up(sizeof(int32_t) * (size_t)n);
    const size_t c = align_up(sizeof(uint32_t) * (size_t)n);
    if (off_perm) *off_perm = a;
    if (off_flags) *off_flags = a + b;
    if (off_scan) *off_scan = a + b + c;
    return a + b + c + fdx_exclusive_scan_u32_workspace_size(n);
}

extern "C" size_t fdx_dense_ids_i64_workspace_size(int64_t n) {
    return dense_ids_parts(n < 0 ? 0 : n, nullptr, nullptr, nullptr);
}

extern "C" int fdx_dense_ids_i64(const int64_t *keys_d, int64_t n, int32_t *ids_d, int64_t *n_unique_d,
                                 void *workspace_d, size_t workspace_bytes, void *stream) {
    FDX_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "n out of range");
    FDX_REQUIRE(n_unique_d, "null n_unique");
    hipStream_t st = as_stream(stream);
    if (n == 0) {
        FDX_HIP(hipMemsetAsync(n_unique_d, 0, sizeof(int64_t), st));
        return FDX_OK;
    }
    FDX_REQUIRE(keys_d && ids_d && workspace_d, "null pointer");
    size_t o_perm, o_flags, o_scan;
    const size_t need = dense_ids_parts(n, &o_perm, &o_flags, &o_scan);
    if (workspace_bytes < need) {
        set_error("dense ids workspace too small: %zu < %zu", workspace_bytes, need);
        return FDX_E_WORKSPACE;
    }
    char *ws = reinterpret_cast<char *>(workspace_d);
    int32_t *perm = reinterpret_cast<int32_t *>(ws + o_perm);
    uint32_t *flags = reinterpret_cast<uint32_t *>(ws + o_flags);
    SortWs<uint64_t> w;
    sort_ws<uint64_t>(n, &w, ws);
    const uint64_t *sorted = nullptr;
    int rc = radix_sort<uint64_t>(reinterpret_cast<const uint64_t *>(keys_d), n, 64, 1ull << 63, nullptr,
                                  reinterpret_cast<uint32_t *>(perm), w, st, &sorted);
    if (rc) return rc;
    hipLaunchKernelGGL(k_new_key_flags, dim3(stream_grid(n, 256)), dim3(256), 0, st, sorted, n, flags);
    FDX_LAUNCHED("k_new_key_flags");
    rc = exclusive_scan(flags, n, reinterpret_cast<uint32_t *>(ws + o_scan), st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_dense_scatter, dim3(stream_grid(n, 256)), dim3(256), 0, st, sorted, flags, perm, n, ids_d,
                       n_unique_d);
    FDX_LAUNCHED("k_dense_scatter");
    return FDX_OK;
}

extern "C" int fdx_is_sorted_i64(const int64_t *keys_d, int64_t n, int32_t *flag_d, void *stream) {
    FDX_REQUIRE(n >= 0 && flag_d, "bad argument");
    hipStream_t st = as_stream(stream);
    FDX_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(flag_d), 1, 1, st));
    if (n < 2) return FDX_OK;
    FDX_REQUIRE(keys_d, "null keys");
    hipLaunchKernelGGL(k_check_sorted_i64, dim3(stream_grid(n, 256)), dim3(256), 0, st, keys_d, n, flag_d);
    FDX_LAUNCHED("k_check_sorted_i64");
    return FDX_OK;
}

// ---- multi-GPU terminal exchange (fdx.distributed) ----------------------------------
__global__ void k_key_map(const int32_t *__restrict__ in, int64_t n, int32_t op, int32_t param,
                          int32_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t k = in[i];
        out[i] = op == FDX_KEY_MOD ? k % param : (op == FDX_KEY_DIV ? k / param : k - param);
    }
}

// count of keys outside [lo, hi): per-wave ballot count, one atomic per wave
__global__ void __launch_bounds__(256) k_count_out_of_range(const int32_t *__restrict__ keys, int64_t n, int32_t lo,
                                                            int32_t hi, int32_t *__restrict__ count) {
    int32_t bad = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t k = keys[i];
        bad += (k < lo || k >= hi) ? 1 : 0;
    }
    const uint64_t any = __ballot(bad != 0);
    if (any == 0) return;
#pragma unroll
    for (int d = kWave / 2; d >= 1; d >>= 1) bad += __shfl_xor(bad, d, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) atomicAdd(count, bad);
}

// rec[j] = {ts[r], term[r] << 32 | fraud[r] << 31 | r}, r = perm[j] (destination-grouped)
__global__ void k_exchange_pack(const int64_t *__restrict__ ts, const int32_t *__restrict__ term,
                                const uint8_t *__restrict__ fraud, const int32_t *__restrict__ perm,
                                int64_t n, int64_t *__restrict__ rec) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = perm[j];
        rec[2 * j] = ts[r];
        rec[2 * j + 1] = ((int64_t)term[r] << 32) | ((int64_t)(fraud[r] != 0) << 31) | (int64_t)r;
    }
}

__global__ void k_exchange_unpack(const int64_t *__restrict__ rec, int64_t m, int32_t world,
                                  int64_t *__restrict__ ts, int32_t *__restrict__ term_local,
                                  uint8_t *__restrict__ fraud) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m;
         j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t w = rec[2 * j + 1];
        ts[j] = rec[2 * j];
        term_local[j] = (int32_t)(w >> 32) / world;
        fraud[j] = (uint8_t)((w >> 31) & 1);
    }
}

// X[perm[j]][col0 + 2w] = nb_w, X[perm[j]][col0 + 2w + 1] = risk_w from count records
__global__ void k_reply_assemble(const int64_t *__restrict__ reply, const int32_t *__restrict__ perm,
                                 int64_t n, int32_t W, double *__restrict__ X, int64_t ld, int32_t col0) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t *r = reply + j * W;
        double *x = X + (int64_t)perm[j] * ld + col0;
        for (int w = 0; w < W; ++w) {
            x[2 * w] = (double)term_nb(r[w]);
            x[2 * w + 1] = term_risk(r[w]);
        }
    }
}

__global__ void k_invert_perm(const int32_t *__restrict__ perm, int64_t n, int32_t *__restrict__ inv) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        inv[perm[i]] = (int32_t)i;
}

template <typename T>
static int launch_perm(bool gather, const void *src, const int32_t *perm, int64_t n, void *dst,
                       hipStream_t st) {
    unsigned grid = stream_grid(n, 256);
    if (gather)
        hipLaunchKernelGGL(k_gather<T>, dim3(grid), dim3(256), 0, st, (const T *)src, perm, n, (T *)dst);
    else
        hipLaunchKernelGGL(k_scatter<T>, dim3(grid), dim3(256), 0, st, (const T *)src, perm, n, (T *)dst);
    FDX_LAUNCHED(gather ? "k_gather" : "k_scatter");
    return FDX_OK;
}

static int perm_op(bool gather, const void *src_d, int32_t elem_bytes, const int32_t *perm_d, int64_t n,
                   void *dst_d, void *stream) {
    FDX_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(src_d && perm_d && dst_d, "null pointer");
    hipStream_t st = as_stream(stream);
    switch (elem_bytes) {
        case 1: return launch_perm<uint8_t>(gather, src_d, perm_d, n, dst_d, st);
        case 2: return launch_perm<uint16_t>(gather, src_d, perm_d, n, dst_d, st);
        case 4: return launch_perm<uint32_t>(gather, src_d, perm_d, n, dst_d, st);
        case 8: return launch_perm<uint64_t>(gather, src_d, perm_d, n, dst_d, st);
        default: set_error("elem_bytes must be 1, 2, 4 or 8"); return FDX_E_INVALID;
    }
}

extern "C" int fdx_gather(const void *src_d, int32_t elem_bytes, const int32_t *perm_d, int64_t n,
                          void *dst_d, void *stream) {
    return perm_op(true, src_d, elem_bytes, perm_d, n, dst_d, stream);
}

extern "C" int fdx_scatter(const void *src_d, int32_t elem_bytes, const int32_t *perm_d, int64_t n,
                           void *dst_d, void *stream) {
    return perm_op(false, src_d, elem_bytes, perm_d, n, dst_d, stream);
}

extern "C" int fdx_key_map(const int32_t *keys_d, int64_t n, int32_t op, int32_t param, int32_t *out_d,
                           void *stream) {
    FDX_REQUIRE(n >= 0, "n < 0");
    FDX_REQUIRE(op == FDX_KEY_MOD || op == FDX_KEY_DIV || op == FDX_KEY_SUB, "bad op %d", op);
    FDX_REQUIRE(op == FDX_KEY_SUB || param >= 1, "param must be >= 1");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(keys_d && out_d, "null pointer");
    hipLaunchKernelGGL(k_key_map, dim3(stream_grid(n, 256)), dim3(256), 0, as_stream(stream), keys_d, n, op,
                       param, out_d);
    FDX_LAUNCHED("k_key_map");
    return FDX_OK;
}

extern "C" int fdx_count_out_of_range(const int32_t *keys_d, int64_t n, int32_t lo, int32_t hi, int32_t *count_d,
                                      void *stream) {
    FDX_REQUIRE(n >= 0 && count_d, "bad argument");
    hipStream_t st = as_stream(stream);
    FDX_HIP(hipMemsetAsync(count_d, 0, 4, st));
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(keys_d, "null keys");
    hipLaunchKernelGGL(k_count_out_of_range, dim3(stream_grid(n, 256)), dim3(256), 0, st, keys_d, n, lo, hi, count_d);
    FDX_LAUNCHED("k_count_out_of_range");
    return FDX_OK;
}

extern "C" int fdx_exchange_pack(const int64_t *ts_d, const int32_t *term_d, const uint8_t *fraud_d,
                                 const int32_t *perm_d, int64_t n, int64_t *rec_d, void *stream) {
    FDX_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(ts_d && term_d && fraud_d && perm_d && rec_d, "null pointer");
    hipLaunchKernelGGL(k_exchange_pack, dim3(stream_grid(n, 256)), dim3(256), 0, as_stream(stream), ts_d,
                       term_d, fraud_d, perm_d, n, rec_d);
    FDX_LAUNCHED("k_exchange_pack");
    return FDX_OK;
}

extern "C" int fdx_exchange_unpack(const int64_t *rec_d, int64_t m, int32_t world, int64_t *ts_d,
                                   int32_t *term_local_d, uint8_t *fraud_d, void *stream) {
    FDX_REQUIRE(m >= 0 && world >= 1, "bad argument");
    if (m == 0) return FDX_OK;
    FDX_REQUIRE(rec_d && ts_d && term_local_d && fraud_d, "null pointer");
    hipLaunchKernelGGL(k_exchange_unpack, dim3(stream_grid(m, 256)), dim3(256), 0, as_stream(stream), rec_d,
                       m, world, ts_d, term_local_d, fraud_d);
    FDX_LAUNCHED("k_exchange_unpack");
    return FDX_OK;
}

extern "C" int fdx_reply_assemble(const int64_t *reply_d, const int32_t *perm_d, int64_t n, int32_t n_windows,
                                  double *X_d, int64_t ld, int32_t col0, void *stream) {
    FDX_REQUIRE(n >= 0 && n_windows >= 1 && n_windows <= FDX_MAX_WINDOWS, "bad argument");
    FDX_REQUIRE(col0 >= 0 && col0 + 2 * n_windows <= ld, "columns out of range");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(reply_d && perm_d && X_d, "null pointer");
    hipLaunchKernelGGL(k_reply_assemble, dim3(stream_grid(n, 256)), dim3(256), 0, as_stream(stream), reply_d,
                       perm_d, n, n_windows, X_d, ld, col0);
    FDX_LAUNCHED("k_reply_assemble");
    return FDX_OK;
}

extern "C" int fdx_invert_perm(const int32_t *perm_d, int64_t n, int32_t *inv_d, void *stream) {
    FDX_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(perm_d && inv_d, "null pointer");
    hipLaunchKernelGGL(k_invert_perm, dim3(stream_grid(n, 256)), dim3(256), 0, as_stream(stream), perm_d, n, inv_d);
    FDX_LAUNCHED("k_invert_perm");
    return FDX_OK;
}

extern "C" size_t fdx_exclusive_scan_u32_workspace_size(int64_t m) {
    return sizeof(uint32_t) * (size_t)(scan_scratch_words(m) + 2) + 256;
}

extern "C" int fdx_exclusive_scan_u32(uint32_t *data_d, int64_t m, void *workspace_d, void *stream) {
    FDX_REQUIRE(m >= 0, "m < 0");
    if (m == 0) return FDX_OK;
    FDX_REQUIRE(data_d && workspace_d, "null pointer");
    return exclusive_scan(data_d, m, reinterpret_cast<uint32_t *>(workspace_d), as_stream(stream));
}

extern "C" size_t fdx_key_segments_workspace_size(int64_t n_keys) {
    if (n_keys < 0) n_keys = 0;
    return align_up(sizeof(uint32_t) * (size_t)(n_keys + 1)) + fdx_exclusive_scan_u32_workspace_size(n_keys + 1);
}

extern "C" int fdx_key_segments(const int32_t *keys_d, int64_t n, int64_t n_keys, int64_t *seg_off_d, int32_t *bad_d,
                                void *workspace_d, size_t workspace_bytes, void *stream) {
    FDX_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "n out of range");
    FDX_REQUIRE(n_keys >= 1 && n_keys < (int64_t)INT32_MAX, "n_keys out of range");
    FDX_REQUIRE(seg_off_d && workspace_d && (n == 0 || keys_d), "null pointer");
    FDX_REQUIRE(workspace_bytes >= fdx_key_segments_workspace_size(n_keys), "workspace too small");
    hipStream_t st = as_stream(stream);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(workspace_d);
    void *sws = reinterpret_cast<char *>(workspace_d) + align_up(sizeof(uint32_t) * (size_t)(n_keys + 1));
    FDX_HIP(hipMemsetAsync(cnt, 0, sizeof(uint32_t) * (size_t)(n_keys + 1), st));
    if (bad_d) FDX_HIP(hipMemsetAsync(bad_d, 0, sizeof(int32_t), st));
    if (n > 0) {
        hipLaunchKernelGGL(k_key_hist, dim3(stream_grid(n, 256)), dim3(256), 0, st, keys_d, n, n_keys, cnt, bad_d);
        FDX_LAUNCHED("k_key_hist");
    }
    int rc = fdx_exclusive_scan_u32(cnt, n_keys + 1, sws, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_widen_u32, dim3(stream_grid(n_keys + 1, 256)), dim3(256), 0, st, cnt, n_keys + 1, seg_off_d);
    FDX_LAUNCHED("k_widen_u32");
    return FDX_OK;
}
