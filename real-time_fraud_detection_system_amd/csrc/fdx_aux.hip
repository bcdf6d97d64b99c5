// fdx_aux.hip -- SURVEY.md §8(f): the callers and data formats either side of the hot path.
//
//   f-1 feature-snapshot export (the serving tables the streaming job LEFT JOINs):
//       latest row per terminal   feature_transformation.ipynb:2914-2918
//           df.loc[df.groupby('TERMINAL_ID').TX_DATETIME.idxmax()]
//       customer row of a date    :3606-3635, :4182
//           df[df.tx_datetime.dt.date == d].drop_duplicates(subset=['customer_id'])  (keep='first')
//   f-2 Debezium CDC decode + dedup of a micro-batch
//       pyspark/scripts/kafka_s3_sink_transactions.py:64-71  tx_amount: big-endian two's-
//           complement unscaled integer, scale 2 (Decimal(unscaled) / 10**2)
//       :167  to_timestamp(from_unixtime(tx_datetime / 1000000))  (microseconds -> whole seconds)
//       :180  ROW_NUMBER() OVER (PARTITION BY tx_id ORDER BY timestamp DESC) = 1
//   f-4 delay-aware train/test split and Card-Precision@k (model-quality parity on GPU outputs)
//       shared_functions.py:133-188  get_train_test_set
//       shared_functions.py:352-411  card_precision_top_k_day / card_precision_top_k
//
// All HBM-bound byte/integer work: one wave per segment (reductions) or one lane per record.
#include "fdx_internal.h"

namespace fdx {
namespace {

// (ts, pos) lexicographic "better" for idxmax: larger ts, then earlier position
__device__ __forceinline__ bool better_latest(int64_t ta, int64_t pa, int64_t tb, int64_t pb) {
    return ta > tb || (ta == tb && pa < pb);
}

// One wave per segment: the first position (segment order = frame order, stable grouping)
// holding the segment's maximum timestamp -> out_row[k] = perm[pos] (-1: empty segment).
__global__ void __launch_bounds__(256) k_segment_latest(const int64_t *__restrict__ ts,
                                                        const int32_t *__restrict__ perm,
                                                        const int64_t *__restrict__ seg_off, int64_t n_seg,
                                                        int32_t *__restrict__ out_row) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / kWave);
    for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave; k < n_seg; k += nw) {
        const int64_t b = seg_off[k], e = seg_off[k + 1];
        int64_t bt = INT64_MIN, bp = INT64_MAX;
        for (int64_t p = b + lane; p < e; p += kWave) {
            const int64_t t = ts[perm ? perm[p] : p];
            if (better_latest(t, p, bt, bp)) {
                bt = t;
                bp = p;
            }
        }
#pragma unroll
        for (int d = kWave / 2; d > 0; d >>= 1) {
            const int64_t ot = __shfl_xor(bt, d, kWave), op = __shfl_xor(bp, d, kWave);
            if (better_latest(ot, op, bt, bp)) {
                bt = ot;
                bp = op;
            }
        }
        if (lane == 0) out_row[k] = e > b ? (perm ? perm[bp] : (int32_t)bp) : -1;
    }
}

// One wave per segment: the first position with t_lo <= ts < t_hi (-1: none).
__global__ void __launch_bounds__(256) k_segment_first_in_range(const int64_t *__restrict__ ts,
                                                                const int32_t *__restrict__ perm,
                                                                const int64_t *__restrict__ seg_off, int64_t n_seg,
                                                                int64_t t_lo, int64_t t_hi,
                                                                int32_t *__restrict__ out_row) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / kWave);
    for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave; k < n_seg; k += nw) {
        const int64_t b = seg_off[k], e = seg_off[k + 1];
        int64_t first = INT64_MAX;
        for (int64_t c = b; c < e && first == INT64_MAX; c += kWave) {  // chunks in order: stop at a hit
            const int64_t p = c + lane;
            bool hit = false;
            if (p < e) {
                const int64_t t = ts[perm ? perm[p] : p];
                hit = t >= t_lo && t < t_hi;
            }
            const uint64_t m = __ballot(hit);
            if (m) first = c + __ffsll((long long)m) - 1;
        }
        if (lane == 0) out_row[k] = first == INT64_MAX ? -1 : (perm ? perm[first] : (int32_t)first);
    }
}

// Debezium DECIMAL(10,2) bytes -> unscaled int64 (big-endian two's complement, 1..8 bytes),
// amount = unscaled / 100.0 (the IEEE-correctly-rounded double of Decimal(unscaled) / 100,
// as float(Decimal) gives); microseconds -> whole seconds as Spark's
// from_unixtime(us / 1000000) (double division, truncation) -> ns.
__global__ void __launch_bounds__(256) k_cdc_decode(const uint8_t *__restrict__ bytes,
                                                    const int64_t *__restrict__ offsets, const int64_t *__restrict__ us,
                                                    int64_t n, int64_t *__restrict__ unscaled,
                                                    double *__restrict__ amount, int64_t *__restrict__ ts_ns,
                                                    int32_t *__restrict__ bad) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (bytes && offsets) {
            const int64_t b = offsets[i], e = offsets[i + 1];
            const int64_t len = e - b;
            int64_t v = 0;
            if (len >= 1 && len <= 8) {
                uint64_t u = 0;
                for (int64_t j = b; j < e; ++j) u = (u << 8) | bytes[j];
                const int sh = 64 - 8 * (int)len;  // sign-extend from the top byte
                v = (int64_t)(u << sh) >> sh;
            } else {
                *bad = 1;
            }
            if (unscaled) unscaled[i] = v;
            if (amount) amount[i] = (double)v / 100.0;
        }
        if (us && ts_ns) {
            const double q = (double)us[i] / 1000000.0;
            ts_ns[i] = (int64_t)q * 1000000000LL;
        }
    }
}

// Latest record per key (ROW_NUMBER() OVER (PARTITION BY tx_id ORDER BY timestamp DESC) = 1)
// with an open-addressing hash table in the caller's workspace -- O(n), four short launches,
// no sort (a micro-batch's dedup was a full 64-bit radix argsort: 8 passes).  Slot h holds
// the key (EMPTY until claimed), the largest Kafka timestamp seen (order-preserving unsigned
// encoding) and the largest batch position holding that timestamp (ties: the last record in
// batch order, the documented choice where Spark's tie order is arbitrary).
constexpr unsigned long long kDedupEmpty = 0xFFFFFFFFFFFFFFFFull;  // reserved: key INT64_MAX ^ sign... see below
__device__ __forceinline__ unsigned long long dedup_ukey(int64_t k) { return (unsigned long long)k; }
__device__ __forceinline__ unsigned long long dedup_uts(int64_t t) {  // signed -> order-preserving unsigned
    return (unsigned long long)t ^ 0x8000000000000000ull;
}
__device__ __forceinline__ uint32_t dedup_hash(unsigned long long k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return (uint32_t)k;
}
__global__ void __launch_bounds__(256) k_dedup_init(unsigned long long *__restrict__ tkey,
                                                    unsigned long long *__restrict__ tts, int32_t *__restrict__ tpos,
                                                    int64_t cap) {
    for (int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; h < cap; h += (int64_t)gridDim.x * blockDim.x) {
        tkey[h] = kDedupEmpty;
        tts[h] = 0ull;
        tpos[h] = -1;
    }
}
// claim (or find) the key's slot, raise its timestamp; slot_of[i] = the slot.  A key equal
// to the EMPTY pattern (-1 as int64 tx_id) would alias empty slots: flagged as bad.
__global__ void __launch_bounds__(256) k_dedup_insert(const int64_t *__restrict__ key, const int64_t *__restrict__ kts,
                                                      int64_t n, unsigned long long *__restrict__ tkey,
                                                      unsigned long long *__restrict__ tts, int64_t cap,
                                                      int32_t *__restrict__ slot_of, int32_t *__restrict__ bad) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long k = dedup_ukey(key[i]);
        if (k == kDedupEmpty) {
            *bad = 1;
            slot_of[i] = -1;
            continue;
        }
        uint32_t h = dedup_hash(k) & (uint32_t)(cap - 1);
        for (;;) {  // cap >= 2 n: a free slot always exists, the probe ends
            const unsigned long long prev = atomicCAS(tkey + h, kDedupEmpty, k);
            if (prev == kDedupEmpty || prev == k) break;
            h = (h + 1) & (uint32_t)(cap - 1);
        }
        atomicMax(tts + h, dedup_uts(kts[i]));
        slot_of[i] = (int32_t)h;
    }
}
__global__ void __launch_bounds__(256) k_dedup_pos(const int64_t *__restrict__ kts, int64_t n,
                                                   const unsigned long long *__restrict__ tts,
                                                   const int32_t *__restrict__ slot_of, int32_t *__restrict__ tpos) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t h = slot_of[i];
        if (h >= 0 && dedup_uts(kts[i]) == tts[h]) atomicMax(tpos + h, (int32_t)i);
    }
}
__global__ void __launch_bounds__(256) k_dedup_keep(int64_t n, const int32_t *__restrict__ slot_of,
                                                    const int32_t *__restrict__ tpos, uint8_t *__restrict__ keep) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t h = slot_of[i];
        keep[i] = (h >= 0 && tpos[h] == (int32_t)i) ? 1 : 0;
    }
}

// The kept records of a micro-batch, compacted in batch order into the stream state's input
// columns: pos = exclusive scan of keep; ids narrowed to int32 (an id outside int32 becomes
// -1, which fdx_stream_update reports as a key out of range instead of wrapping into range).
__global__ void __launch_bounds__(256) k_cdc_compact(const uint8_t *__restrict__ keep, const uint32_t *__restrict__ pos,
                                                     int64_t n, const int64_t *__restrict__ cust,
                                                     const int64_t *__restrict__ term, const int64_t *__restrict__ ts,
                                                     const double *__restrict__ amt, const uint8_t *__restrict__ fraud,
                                                     int32_t *__restrict__ cust_out, int32_t *__restrict__ term_out,
                                                     int64_t *__restrict__ ts_out, double *__restrict__ amt_out,
                                                     uint8_t *__restrict__ fraud_out, int32_t *__restrict__ row_out,
                                                     int64_t *__restrict__ count) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i == n - 1) *count = (int64_t)pos[i] + (keep[i] ? 1 : 0);
        if (!keep[i]) continue;
        const int64_t j = pos[i];
        const int64_t c = cust[i], t = term[i];
        cust_out[j] = (c >= 0 && c <= INT32_MAX) ? (int32_t)c : -1;
        term_out[j] = (t >= 0 && t <= INT32_MAX) ? (int32_t)t : -1;
        ts_out[j] = ts[i];
        amt_out[j] = amt[i];
        fraud_out[j] = fraud ? (uint8_t)(fraud[i] != 0) : 0;
        if (row_out) row_out[j] = (int32_t)i;
    }
}

// ---------------------------------------------------------------- f-4: split, CP@k
// get_train_test_set: train rows t_lo <= ts < t_hi; per customer: a fraud among the train
// rows (train_fraud) and the first delay-period day index d' (TX_TIME_DAYS == day_base - 1
// + d', 0 <= d' < delta_test) with a fraud (delay_first); test day d keeps a row of day
// day_base + delta_delay + d iff its customer is known neither from training nor by day d.
__global__ void __launch_bounds__(256) k_split_pass1(const int64_t *__restrict__ ts, const int32_t *__restrict__ day,
                                                     const int32_t *__restrict__ cust, const uint8_t *__restrict__ fraud,
                                                     int64_t n, int64_t t_lo, int64_t t_hi, int32_t *__restrict__ day_min,
                                                     uint8_t *__restrict__ train) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const bool tr = ts[i] >= t_lo && ts[i] < t_hi;
        train[i] = tr;
        if (tr) atomicMin(day_min, day[i]);
    }
}
__global__ void __launch_bounds__(256) k_split_pass2(const int32_t *__restrict__ day, const int32_t *__restrict__ cust,
                                                     const uint8_t *__restrict__ fraud, const uint8_t *__restrict__ train,
                                                     int64_t n, int32_t day_base, int32_t delta_test,
                                                     uint8_t *__restrict__ train_fraud, int32_t *__restrict__ delay_first) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!fraud[i]) continue;
        const int32_t c = cust[i];
        if (train[i]) train_fraud[c] = 1;
        const int32_t dp = day[i] - (day_base - 1);
        if (dp >= 0 && dp < delta_test) atomicMin(&delay_first[c], dp);
    }
}
__global__ void __launch_bounds__(256) k_split_pass3(const int32_t *__restrict__ day, const int32_t *__restrict__ cust,
                                                     int64_t n, int32_t test_day0, int32_t delta_test,
                                                     const uint8_t *__restrict__ train_fraud,
                                                     const int32_t *__restrict__ delay_first, uint8_t *__restrict__ test) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t d = day[i] - test_day0;
        const int32_t c = cust[i];
        test[i] = d >= 0 && d < delta_test && !train_fraud[c] && delay_first[c] > d;
    }
}

// card_precision_top_k_day over the rows of one day, customers not yet detected:
// per customer max(prediction) (order-preserving u64 keys; predictions are >= 0) and max(label)
__global__ void __launch_bounds__(256) k_cpk_day_max(const int32_t *__restrict__ day, const int32_t *__restrict__ cust,
                                                     const double *__restrict__ pred, const uint8_t *__restrict__ fraud,
                                                     int64_t n, int32_t d, const uint8_t *__restrict__ detected,
                                                     unsigned long long *__restrict__ cmax, uint8_t *__restrict__ cfraud,
                                                     uint8_t *__restrict__ present) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (day[i] != d) continue;
        const int32_t c = cust[i];
        if (detected[c]) continue;
        present[c] = 1;
        atomicMax(&cmax[c], (unsigned long long)__double_as_longlong(pred[i]));
        if (fraud[i]) cfraud[c] = 1;
    }
}
// rank of every present customer in (prediction desc, customer asc) order; the top k are
// "detected" when compromised.  out[0] += compromised customers of the day, out[1] += top-k hits.
__global__ void __launch_bounds__(256) k_cpk_day_topk(const unsigned long long *__restrict__ cmax,
                                                      const uint8_t *__restrict__ cfraud,
                                                      const uint8_t *__restrict__ present, int32_t n_cust,
                                                      int32_t top_k, uint8_t *__restrict__ detected,
                                                      int32_t *__restrict__ out) {
    for (int32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n_cust; c += gridDim.x * blockDim.x) {
        if (!present[c]) continue;
        if (cfraud[c]) atomicAdd(&out[0], 1);
        const unsigned long long v = cmax[c];
        int32_t rank = 0;
        for (int32_t o = 0; o < n_cust && rank < top_k; ++o)
            if (present[o] && (cmax[o] > v || (cmax[o] == v && o < c))) ++rank;
        if (rank < top_k && cfraud[c]) {
            atomicAdd(&out[1], 1);
            detected[c] = 1;
        }
    }
}

// f-1 from the featurized table itself (FeatureTable, slot order: slot s holds input row row[s],
// -1 for padding), without a grouping of the input: per key, atomics over the slots.
//   LATEST: the max ts of the key (pass 1), then the smallest input row holding it (pass 2) --
//           input rows are in time order (frame order), so this is groupby(key).idxmax()
//   FIRST_IN_RANGE: the smallest input row with t_lo <= ts < t_hi (drop_duplicates keep='first')
// best[k] = (row << 32) | slot, so the minimum carries the chosen row's slot.
__global__ void __launch_bounds__(256) k_tsel_init(int64_t *__restrict__ best_ts, uint64_t *__restrict__ best,
                                                   int64_t n_keys) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_keys; k += (int64_t)gridDim.x * blockDim.x) {
        best_ts[k] = INT64_MIN;
        best[k] = UINT64_MAX;
    }
}

__global__ void __launch_bounds__(256) k_tsel_max(const int32_t *__restrict__ row, int64_t n_slots,
                                                  const int64_t *__restrict__ ts, const int32_t *__restrict__ key,
                                                  int64_t n_keys, int64_t *__restrict__ best_ts) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_slots; s += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = row[s];
        if (r < 0) continue;
        const int32_t k = key[r];
        if ((uint32_t)k < (uint64_t)n_keys) atomicMax(reinterpret_cast<long long *>(best_ts + k), (long long)ts[r]);
    }
}

template <bool LATEST>
__global__ void __launch_bounds__(256) k_tsel_min(const int32_t *__restrict__ row, int64_t n_slots,
                                                  const int64_t *__restrict__ ts, const int32_t *__restrict__ key,
                                                  int64_t n_keys, int64_t t_lo, int64_t t_hi,
                                                  const int64_t *__restrict__ best_ts, uint64_t *__restrict__ best) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_slots; s += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = row[s];
        if (r < 0) continue;
        const int32_t k = key[r];
        if ((uint32_t)k >= (uint64_t)n_keys) continue;
        const int64_t t = ts[r];
        if (LATEST ? t == best_ts[k] : (t >= t_lo && t < t_hi))
            atomicMin(reinterpret_cast<unsigned long long *>(best + k),
                      (unsigned long long)(((uint64_t)(uint32_t)r << 32) | (uint64_t)(uint32_t)s));
    }
}

__global__ void __launch_bounds__(256) k_tsel_out(const uint64_t *__restrict__ best, int64_t n_keys,
                                                  int32_t *__restrict__ out_slot) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_keys; k += (int64_t)gridDim.x * blockDim.x)
        out_slot[k] = best[k] == UINT64_MAX ? -1 : (int32_t)(uint32_t)(best[k] & 0xFFFFFFFFu);
}

}  // namespace
}  // namespace fdx

using namespace fdx;

extern "C" int fdx_train_test_split(const int64_t *ts_d, const int32_t *day_d, const int32_t *cust_d,
                                    const uint8_t *fraud_d, int64_t n, int32_t n_cust, int64_t t_lo, int64_t t_hi,
                                    int32_t delta_train, int32_t delta_delay, int32_t delta_test, uint8_t *train_d,
                                    uint8_t *test_d, void *workspace_d, size_t workspace_bytes, int32_t *day_min_h,
                                    void *stream) {
    FDX_REQUIRE(n >= 0 && n_cust >= 0 && delta_test >= 0, "bad argument");
    FDX_REQUIRE(workspace_bytes >= (size_t)n_cust * 5 + 64, "workspace too small");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(ts_d && day_d && cust_d && fraud_d && train_d && test_d && workspace_d && day_min_h, "null pointer");
    hipStream_t st = as_stream(stream);
    char *w = reinterpret_cast<char *>(workspace_d);
    int32_t *day_min = reinterpret_cast<int32_t *>(w);
    int32_t *delay_first = reinterpret_cast<int32_t *>(w + 64);
    uint8_t *train_fraud = reinterpret_cast<uint8_t *>(w + 64 + (size_t)n_cust * 4);
    const int32_t big = INT32_MAX;
    FDX_HIP(hipMemcpyAsync(day_min, &big, 4, hipMemcpyHostToDevice, st));
    FDX_HIP(hipMemsetAsync(delay_first, 0x7F, (size_t)n_cust * 4, st));  // 0x7F7F7F7F: "never"
    FDX_HIP(hipMemsetAsync(train_fraud, 0, (size_t)n_cust, st));
    const unsigned grid = stream_grid(n, 256);
    hipLaunchKernelGGL(k_split_pass1, dim3(grid), dim3(256), 0, st, ts_d, day_d, cust_d, fraud_d, n, t_lo, t_hi,
                       day_min, train_d);
    FDX_LAUNCHED("k_split_pass1");
    FDX_HIP(hipMemcpyAsync(day_min_h, day_min, 4, hipMemcpyDeviceToHost, st));
    FDX_HIP(hipStreamSynchronize(st));
    if (*day_min_h == INT32_MAX) {  // empty training set: no test days either
        FDX_HIP(hipMemsetAsync(test_d, 0, (size_t)n, st));
        return FDX_OK;
    }
    const int32_t day_base = *day_min_h + delta_train;
    hipLaunchKernelGGL(k_split_pass2, dim3(grid), dim3(256), 0, st, day_d, cust_d, fraud_d, train_d, n, day_base,
                       delta_test, train_fraud, delay_first);
    FDX_LAUNCHED("k_split_pass2");
    hipLaunchKernelGGL(k_split_pass3, dim3(grid), dim3(256), 0, st, day_d, cust_d, n, day_base + delta_delay,
                       delta_test, train_fraud, delay_first, test_d);
    FDX_LAUNCHED("k_split_pass3");
    return FDX_OK;
}

extern "C" size_t fdx_card_precision_workspace_size(int32_t n_cust) {
    return (size_t)(n_cust < 0 ? 0 : n_cust) * 12 + 256;
}

extern "C" int fdx_card_precision_top_k(const int32_t *day_d, const int32_t *cust_d, const double *pred_d,
                                        const uint8_t *fraud_d, int64_t n, int32_t n_cust, const int32_t *days_h,
                                        int32_t n_days, int32_t top_k, int32_t remove_detected,
                                        int32_t *nb_compromised_h, double *cp_h, void *workspace_d,
                                        size_t workspace_bytes, void *stream) {
    FDX_REQUIRE(n >= 0 && n_cust >= 0 && n_days >= 0 && top_k >= 1, "bad argument");
    FDX_REQUIRE(workspace_bytes >= fdx_card_precision_workspace_size(n_cust), "workspace too small");
    if (n_days == 0) return FDX_OK;
    FDX_REQUIRE(day_d && cust_d && pred_d && fraud_d && days_h && nb_compromised_h && cp_h && workspace_d,
                "null pointer");
    hipStream_t st = as_stream(stream);
    char *w = reinterpret_cast<char *>(workspace_d);
    int32_t *out = reinterpret_cast<int32_t *>(w);
    unsigned long long *cmax = reinterpret_cast<unsigned long long *>(w + 256);
    uint8_t *detected = reinterpret_cast<uint8_t *>(w + 256 + (size_t)n_cust * 8);
    uint8_t *cfraud = detected + n_cust;
    uint8_t *present = cfraud + n_cust;
    uint8_t *scratch = present + n_cust;  // the day's detections when they are not carried over
    FDX_HIP(hipMemsetAsync(detected, 0, (size_t)n_cust, st));
    const unsigned grid = stream_grid(n, 256);
    const unsigned cgrid = stream_grid(n_cust, 256);
    for (int32_t k = 0; k < n_days; ++k) {
        FDX_HIP(hipMemsetAsync(out, 0, 8, st));
        FDX_HIP(hipMemsetAsync(cmax, 0, (size_t)n_cust * 8, st));
        FDX_HIP(hipMemsetAsync(cfraud, 0, (size_t)n_cust * 2, st));  // cfraud + present
        hipLaunchKernelGGL(k_cpk_day_max, dim3(grid), dim3(256), 0, st, day_d, cust_d, pred_d, fraud_d, n, days_h[k],
                           detected, cmax, cfraud, present);
        FDX_LAUNCHED("k_cpk_day_max");
        hipLaunchKernelGGL(k_cpk_day_topk, dim3(cgrid), dim3(256), 0, st, cmax, cfraud, present, n_cust, top_k,
                           remove_detected ? detected : scratch, out);
        FDX_LAUNCHED("k_cpk_day_topk");
        int32_t o[2];
        FDX_HIP(hipMemcpyAsync(o, out, 8, hipMemcpyDeviceToHost, st));
        FDX_HIP(hipStreamSynchronize(st));
        nb_compromised_h[k] = o[0];
        cp_h[k] = (double)o[1] / (double)top_k;
    }
    return FDX_OK;
}

extern "C" int fdx_segment_latest(const int64_t *ts_d, const int32_t *perm_d, const int64_t *seg_off_d, int64_t n_seg,
                                  int32_t *out_row_d, void *stream) {
    FDX_REQUIRE(n_seg >= 0, "negative size");
    if (n_seg == 0) return FDX_OK;
    FDX_REQUIRE(ts_d && seg_off_d && out_row_d, "null pointer");
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n_seg * kWave, 256), 256 * 16);
    hipLaunchKernelGGL(k_segment_latest, dim3(grid), dim3(256), 0, as_stream(stream), ts_d, perm_d, seg_off_d, n_seg,
                       out_row_d);
    FDX_LAUNCHED("k_segment_latest");
    return FDX_OK;
}

extern "C" int fdx_segment_first_in_range(const int64_t *ts_d, const int32_t *perm_d, const int64_t *seg_off_d,
                                          int64_t n_seg, int64_t t_lo, int64_t t_hi, int32_t *out_row_d,
                                          void *stream) {
    FDX_REQUIRE(n_seg >= 0, "negative size");
    if (n_seg == 0) return FDX_OK;
    FDX_REQUIRE(ts_d && seg_off_d && out_row_d, "null pointer");
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n_seg * kWave, 256), 256 * 16);
    hipLaunchKernelGGL(k_segment_first_in_range, dim3(grid), dim3(256), 0, as_stream(stream), ts_d, perm_d, seg_off_d,
                       n_seg, t_lo, t_hi, out_row_d);
    FDX_LAUNCHED("k_segment_first_in_range");
    return FDX_OK;
}

extern "C" int fdx_cdc_decode(const uint8_t *bytes_d, const int64_t *offsets_d, const int64_t *us_d, int64_t n,
                              int64_t *unscaled_d, double *amount_d, int64_t *ts_ns_d, int32_t *bad_d, void *stream) {
    FDX_REQUIRE(n >= 0, "negative size");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(bad_d, "null pointer");
    FDX_REQUIRE((bytes_d != nullptr) == (offsets_d != nullptr), "bytes and offsets go together");
    hipLaunchKernelGGL(k_cdc_decode, dim3(stream_grid(n, 256)), dim3(256), 0, as_stream(stream), bytes_d, offsets_d,
                       us_d, n, unscaled_d, amount_d, ts_ns_d, bad_d);
    FDX_LAUNCHED("k_cdc_decode");
    return FDX_OK;
}

static int64_t dedup_cap(int64_t n) {
    int64_t cap = 2;
    while (cap < 2 * n) cap <<= 1;
    return cap;
}

extern "C" size_t fdx_dedup_latest_workspace_size(int64_t n) {
    if (n < 0) n = 0;
    const int64_t cap = dedup_cap(n);
    return round_up((size_t)cap * 8, 256) * 2 + round_up((size_t)cap * 4, 256) + round_up((size_t)n * 4, 256) + 256;
}

extern "C" int fdx_dedup_latest(const int64_t *key_d, const int64_t *kafka_ts_d, int64_t n, uint8_t *keep_d,
                                int32_t *bad_d, void *workspace_d, size_t workspace_bytes, void *stream) {
    // hash slots are stored as int32 (negative = no slot) and the table holds up to 2n+ slots:
    // n <= 2^30 keeps every slot index below 2^31
    FDX_REQUIRE(n >= 0 && n <= (int64_t(1) << 30), "n out of range (dedup batches hold at most 2^30 records)");
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(key_d && kafka_ts_d && keep_d && bad_d, "null pointer");
    const size_t need = fdx_dedup_latest_workspace_size(n);
    if (!workspace_d || workspace_bytes < need) {
        set_error("dedup workspace too small: %zu < %zu", workspace_bytes, need);
        return FDX_E_WORKSPACE;
    }
    const int64_t cap = dedup_cap(n);
    char *w = reinterpret_cast<char *>(workspace_d);
    auto *tkey = reinterpret_cast<unsigned long long *>(w);
    auto *tts = reinterpret_cast<unsigned long long *>(w + round_up((size_t)cap * 8, 256));
    auto *tpos = reinterpret_cast<int32_t *>(w + 2 * round_up((size_t)cap * 8, 256));
    auto *slot = reinterpret_cast<int32_t *>(w + 2 * round_up((size_t)cap * 8, 256) + round_up((size_t)cap * 4, 256));
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_dedup_init, dim3(stream_grid(cap, 256)), dim3(256), 0, st, tkey, tts, tpos, cap);
    FDX_LAUNCHED("k_dedup_init");
    hipLaunchKernelGGL(k_dedup_insert, dim3(stream_grid(n, 256)), dim3(256), 0, st, key_d, kafka_ts_d, n, tkey, tts,
                       cap, slot, bad_d);
    FDX_LAUNCHED("k_dedup_insert");
    hipLaunchKernelGGL(k_dedup_pos, dim3(stream_grid(n, 256)), dim3(256), 0, st, kafka_ts_d, n, tts, slot, tpos);
    FDX_LAUNCHED("k_dedup_pos");
    hipLaunchKernelGGL(k_dedup_keep, dim3(stream_grid(n, 256)), dim3(256), 0, st, n, slot, tpos, keep_d);
    FDX_LAUNCHED("k_dedup_keep");
    return FDX_OK;
}

extern "C" size_t fdx_cdc_compact_workspace_size(int64_t n) {
    if (n < 0) n = 0;
    return round_up((size_t)n * 4, 256) + fdx_exclusive_scan_u32_workspace_size(n) + 256;
}

__global__ void k_u8_to_u32(const uint8_t *__restrict__ in, int64_t n, uint32_t *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[i] ? 1u : 0u;
}

extern "C" int fdx_cdc_compact(const uint8_t *keep_d, int64_t n, const int64_t *customer_d, const int64_t *terminal_d,
                               const int64_t *ts_ns_d, const double *amount_d, const uint8_t *fraud_d,
                               int32_t *customer_out_d, int32_t *terminal_out_d, int64_t *ts_out_d,
                               double *amount_out_d, uint8_t *fraud_out_d, int32_t *row_out_d, int64_t *count_d,
                               void *workspace_d, size_t workspace_bytes, void *stream) {
    FDX_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "n out of range");
    FDX_REQUIRE(count_d, "null count");
    hipStream_t st = as_stream(stream);
    if (n == 0) {
        FDX_HIP(hipMemsetAsync(count_d, 0, sizeof(int64_t), st));
        return FDX_OK;
    }
    FDX_REQUIRE(keep_d && customer_d && terminal_d && ts_ns_d && amount_d && customer_out_d && terminal_out_d &&
                    ts_out_d && amount_out_d && fraud_out_d,
                "null pointer");
    const size_t need = fdx_cdc_compact_workspace_size(n);
    if (!workspace_d || workspace_bytes < need) {
        set_error("cdc compact workspace too small: %zu < %zu", workspace_bytes, need);
        return FDX_E_WORKSPACE;
    }
    auto *pos = reinterpret_cast<uint32_t *>(workspace_d);
    void *scan_ws = reinterpret_cast<char *>(workspace_d) + round_up((size_t)n * 4, 256);
    hipLaunchKernelGGL(k_u8_to_u32, dim3(stream_grid(n, 256)), dim3(256), 0, st, keep_d, n, pos);
    FDX_LAUNCHED("k_u8_to_u32");
    int rc = fdx_exclusive_scan_u32(pos, n, scan_ws, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_cdc_compact, dim3(stream_grid(n, 256)), dim3(256), 0, st, keep_d, pos, n, customer_d,
                       terminal_d, ts_ns_d, amount_d, fraud_d, customer_out_d, terminal_out_d, ts_out_d, amount_out_d,
                       fraud_out_d, row_out_d, count_d);
    FDX_LAUNCHED("k_cdc_compact");
    return FDX_OK;
}

extern "C" size_t fdx_table_select_workspace_size(int64_t n_keys) {
    return (size_t)(n_keys > 0 ? n_keys : 0) * 16 + 256;
}

extern "C" int fdx_table_select(const int32_t *row_d, int64_t n_slots, const int64_t *ts_d, const int32_t *key_d,
                                int64_t n_keys, int32_t mode, int64_t t_lo, int64_t t_hi, int32_t *out_slot_d,
                                void *ws, size_t ws_bytes, void *stream) {
    FDX_REQUIRE(n_slots >= 0 && n_keys >= 0 && n_keys <= INT32_MAX, "bad size");
    FDX_REQUIRE(mode == FDX_SELECT_LATEST || mode == FDX_SELECT_FIRST_IN_RANGE, "mode must be FDX_SELECT_*");
    if (n_keys == 0) return FDX_OK;
    FDX_REQUIRE(out_slot_d && (n_slots == 0 || (row_d && ts_d && key_d)), "null pointer");
    FDX_REQUIRE(n_slots <= INT32_MAX, "more than 2^31 slots");
    if (!ws || ws_bytes < fdx_table_select_workspace_size(n_keys)) {
        set_error("table select workspace too small: %zu < %zu", ws_bytes, fdx_table_select_workspace_size(n_keys));
        return FDX_E_WORKSPACE;
    }
    int64_t *best_ts = reinterpret_cast<int64_t *>(ws);
    uint64_t *best = reinterpret_cast<uint64_t *>(best_ts + n_keys);
    hipStream_t st = as_stream(stream);
    const unsigned gk = stream_grid(n_keys, 256), gs = stream_grid(std::max<int64_t>(n_slots, 1), 256);
    hipLaunchKernelGGL(k_tsel_init, dim3(gk), dim3(256), 0, st, best_ts, best, n_keys);
    FDX_LAUNCHED("k_tsel_init");
    if (n_slots > 0) {
        if (mode == FDX_SELECT_LATEST) {
            hipLaunchKernelGGL(k_tsel_max, dim3(gs), dim3(256), 0, st, row_d, n_slots, ts_d, key_d, n_keys, best_ts);
            FDX_LAUNCHED("k_tsel_max");
            hipLaunchKernelGGL(k_tsel_min<true>, dim3(gs), dim3(256), 0, st, row_d, n_slots, ts_d, key_d, n_keys, t_lo,
                               t_hi, best_ts, best);
        } else {
            hipLaunchKernelGGL(k_tsel_min<false>, dim3(gs), dim3(256), 0, st, row_d, n_slots, ts_d, key_d, n_keys, t_lo,
                               t_hi, best_ts, best);
        }
        FDX_LAUNCHED("k_tsel_min");
    }
    hipLaunchKernelGGL(k_tsel_out, dim3(gk), dim3(256), 0, st, best, n_keys, out_slot_d);
    FDX_LAUNCHED("k_tsel_out");
    return FDX_OK;
}
