/*
 * fdx.h -- C ABI of the MI355X-native fraud-feature + scoring engine (libfdx.so).
 *
 * The reference (sauravtanwar786/Real-time_fraud_detection_system) has no FFI layer: its
 * hot path is a set of Python functions called per group by pandas and a Spark pandas
 * UDF.  Each entry point below replaces the arithmetic behind one of those calls for a
 * WHOLE table (one call per table / Arrow batch, not per group); the Python drop-in
 * (real-time_fraud_detection_system_amd/fdx) keeps the reference's names, signatures and
 * DataFrame column contract on top of it.  See INTEGRATION.md for the bindings.
 *
 * Conventions
 *   - Every pointer argument named *_d is DEVICE memory owned by the caller (e.g. a torch
 *     tensor's data_ptr()); the library never frees caller memory and never allocates in
 *     a compute call (scratch comes from a caller-passed workspace, see *_workspace_size).
 *   - Host arrays (window lengths, tree descriptions) are read during the call only.
 *   - `stream` is a hipStream_t (NULL = legacy default stream).  Every compute call is
 *     stream-ordered and asynchronous; calls on different streams are independent.
 *   - Return value: FDX_OK (0) or a negative FDX_E_* code; fdx_last_error() returns a
 *     thread-local message for the last failing call on this thread.
 *   - Timestamps are int64 nanoseconds since the Unix epoch (pandas datetime64[ns]).
 *   - Grouped inputs: rows of key k occupy [seg_off_d[k], seg_off_d[k+1]) and are in
 *     time order inside the segment (fdx_rekey produces exactly this layout).
 */
#ifndef FDX_H_
#define FDX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FDX_ABI_VERSION 2

#define FDX_OK 0
#define FDX_E_INVALID (-1)     /* bad argument (null pointer, size, unsupported shape) */
#define FDX_E_HIP (-2)         /* a HIP runtime call failed */
#define FDX_E_UNSUPPORTED (-3) /* input the engine does not implement (e.g. regressor forest) */
#define FDX_E_WORKSPACE (-4)   /* workspace smaller than *_workspace_size() */

#define FDX_MAX_WINDOWS 8
#define FDX_MAX_FEATURES 32

/* flag semantics: notebook (feature_transformation.ipynb:246-253, :294-301) or the Spark
 * SQL of the streaming job (pyspark/scripts/fraud_detection.py:103-104). */
#define FDX_FLAGS_NOTEBOOK 0 /* weekend = weekday()>=5 (Sat,Sun); night = hour<=6       */
#define FDX_FLAGS_SPARK 1    /* weekend = dayofweek>=5 (Thu,Fri,Sat); night = hour>=20 (UTC) */

const char *fdx_last_error(void);
int fdx_abi_version(void);

/* ---- a-1 / a-6: TX_DURING_WEEKEND, TX_DURING_NIGHT ------------------------------------
 * Replaces `transactions_df.TX_DATETIME.apply(is_weekend|is_night)`
 * (fraud_detection_model/feature_transformation.ipynb:278, :319) and the Spark SQL
 * `if(dayofweek(tx_datetime) >= 5,1,0)`, `if(hour(tx_datetime) >= 20,1,0)`
 * (pyspark/scripts/fraud_detection.py:103-104).  Outputs are 0/1 bytes, length n. */
int fdx_time_flags(const int64_t *ts_ns_d, int64_t n, int32_t mode, uint8_t *weekend_d,
                   uint8_t *night_d, void *stream);

/* ---- a-2: customer spending-behaviour windows -----------------------------------------
 * Replaces get_customer_spending_behaviour_features(customer_transactions,
 * windows_size_in_days) (feature_transformation.ipynb:601-628) applied through
 * `groupby('CUSTOMER_ID').apply(...)` (:1092), for all segments at once.
 *   nb_d[w*n + i]  = rolling('{w}d').count()  (int32; the reference stores it as float64)
 *   avg_d[w*n + i] = rolling('{w}d').sum() / count, bit-identical to pandas' Kahan
 *                    add/remove roll_sum (exact emulation).
 * window_ns: host array of n_windows window lengths in ns.  n = seg_off_d[n_seg]. */
int fdx_customer_windows(const int64_t *ts_ns_d, const double *amount_d, const int64_t *seg_off_d,
                         int64_t n_seg, int64_t n, const int64_t *window_ns, int32_t n_windows,
                         int32_t *nb_d, double *avg_d, void *stream);

/* Scoring-pipeline layout of the customer windows (coalesced form of the same arithmetic):
 * segments ordered by decreasing length (sorder_d [n_seg]) and cut into groups of
 * S = 64 / n_windows; group g owns slots [goff_d[g], goff_d[g+1]) and row t of its l-th
 * segment is slot goff_d[g] + t*S + l.  fdx_customer_layout fills its_d / iamt_d (ts and
 * amount per slot) and irow_d (time-order row of each slot, -1 = padding) from the
 * time-ordered ts/amount through cperm_d (fdx_rekey output), writes the slot count to
 * *n_slots_h (host; this call synchronises the stream once) and fails with
 * FDX_E_WORKSPACE if it exceeds max_slots (it is at most n + (S-1)*max segment length).
 * goff_d needs n_groups+1 = ceil(n_seg/S)+1 entries. */
size_t fdx_customer_layout_workspace_size(int64_t n_seg);
int fdx_customer_layout(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                        const int64_t *ts_d, const double *amount_d, int32_t n_windows,
                        int32_t *sorder_d, uint32_t *goff_d, int64_t *its_d, double *iamt_d,
                        int32_t *irow_d, int64_t max_slots, int64_t *n_slots_h, void *workspace_d,
                        size_t workspace_bytes, void *stream);
/* fdx_customer_layout that also writes every row's window starts (pandas' variable-window
 * start: the first row j of the segment with ts_j > ts_t - window_ns[w], closed='right'),
 * computed in the same kernel from the freshly gathered timestamps, segment-contiguous:
 * row t of segment l of group g at starts_d[w * n_slots + goff_d[g] + l * Lg + t] (Lg = the
 * group's longest segment; starts_d: room for n_windows * max_slots int32).  Follow with
 * fdx_customer_windows_walk. */
int fdx_customer_layout_starts(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                               const int64_t *ts_d, const double *amount_d, const int64_t *window_ns,
                               int32_t n_windows, int32_t *sorder_d, uint32_t *goff_d, int64_t *its_d,
                               double *iamt_d, int32_t *irow_d, int32_t *starts_d, int64_t max_slots,
                               int64_t *n_slots_h, void *workspace_d, size_t workspace_bytes, void *stream);
/* The layout in two halves, for callers that overlap them with the re-key:
 * plan -- from the segment offsets alone: sorder_d, goff_d and *n_slots_h (synchronises the
 * stream: the slot count is read back); fill -- fdx_customer_layout_starts_grouped's slots and
 * window starts for that plan (its_d / iamt_d / irow_d of n_slots entries, starts_d of
 * n_windows * n_slots).  fdx_customer_layout* = plan + fill. */
int fdx_customer_layout_plan(const int64_t *seg_off_d, int64_t n_seg, int32_t n_windows, int32_t *sorder_d,
                             uint32_t *goff_d, int64_t *n_slots_h, void *workspace_d, size_t workspace_bytes,
                             void *stream);
/* fdx_customer_layout_plan without the host synchronisation, for <= 65,536 segments (else
 * FDX_E_UNSUPPORTED): plan_h (caller-owned pinned host int32[2]) receives [slot count, status]
 * once the stream reaches them; status 1 = plan again with fdx_customer_layout_plan.  Pinned
 * memory HIP maps into the device (hipHostMalloc, torch's pin_memory) is written by the plan
 * kernel itself at system scope; other host memory gets two copies after it. */
int fdx_customer_layout_plan_async(const int64_t *seg_off_d, int64_t n_seg, int32_t n_windows, int32_t *sorder_d,
                                   uint32_t *goff_d, int32_t *plan_h, void *workspace_d, size_t workspace_bytes,
                                   void *stream);
int fdx_customer_layout_fill_starts_grouped(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                                            const int64_t *gts_d, const double *gamount_d, const int64_t *window_ns,
                                            int32_t n_windows, const int32_t *sorder_d, const uint32_t *goff_d,
                                            int64_t n_slots, int64_t *its_d, double *iamt_d, int32_t *irow_d,
                                            int32_t *starts_d, void *stream);

/* fdx_customer_layout_starts over GROUPED ts / amount (fdx_rekey_payload outputs: row j of
 * the grouping is gts_d[j], gamount_d[j]) -- the layout then reads every segment as a
 * sequential stream instead of gathering through cperm_d (which still gives irow_d). */
int fdx_customer_layout_starts_grouped(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                                       const int64_t *gts_d, const double *gamount_d, const int64_t *window_ns,
                                       int32_t n_windows, int32_t *sorder_d, uint32_t *goff_d, int64_t *its_d,
                                       double *iamt_d, int32_t *irow_d, int32_t *starts_d, int64_t max_slots,
                                       int64_t *n_slots_h, void *workspace_d, size_t workspace_bytes, void *stream);
/* fdx_customer_layout over GROUPED ts / amount without the window starts (the scan mode's
 * layout: fdx_customer_windows_scan computes the windows itself). */
int fdx_customer_layout_grouped(const int64_t *seg_off_d, int64_t n_seg, const int32_t *cperm_d,
                                const int64_t *gts_d, const double *gamount_d, int32_t n_windows,
                                int32_t *sorder_d, uint32_t *goff_d, int64_t *its_d, double *iamt_d,
                                int32_t *irow_d, int64_t max_slots, int64_t *n_slots_h, void *workspace_d,
                                size_t workspace_bytes, void *stream);
/* Customer windows, SCAN mode (SURVEY.md §7 step 4 / §8(b) "exact|scan" mode flag;
 * replaces the same feature_transformation.ipynb:1092-1093 call as fdx_customer_windows):
 * the rolling sums from float64 prefix sums over each segment instead of pandas' sequential
 * Kahan add/remove recurrence -- fully parallel (one wave per segment).  NB is exact; the
 * SUM agrees with pandas to ~1e-13 relative, ~1e-13 absolute for a window whose amounts
 * sum to 0 (NOT bit-exact; pandas' "n equal values -> prev * n" rule is not applied); SUM
 * is NaN when NB == 0.  Inputs are grouped
 * (fdx_rekey_payload outputs: segment s = rows [seg_off_d[s], seg_off_d[s+1]), time-sorted).
 * Output: with sorder_d / goff_d (an interleaved layout of the same segments, n_out =
 * n_slots): nb_d / val_d [W][n_out] by slot, exactly the shape of fdx_customer_windows_walk;
 * else by grouped position (n_out >= n).  val = SUM when val_is_sum, else SUM / NB (the
 * average, IEEE division).  Workspace: fdx_customer_windows_scan_workspace_size(n, n_seg)
 * bytes (segments longer than 1,024 rows keep their prefix sums there). */
size_t fdx_customer_windows_scan_workspace_size(int64_t n, int64_t n_seg);
int fdx_customer_windows_scan(const int64_t *gts_d, const double *gamount_d, const int64_t *seg_off_d,
                              int64_t n_seg, int64_t n, const int64_t *window_ns, int32_t n_windows,
                              const int32_t *sorder_d, const uint32_t *goff_d, int64_t n_out, int32_t *nb_d,
                              double *val_d, int32_t val_is_sum, void *workspace_d, size_t workspace_bytes,
                              void *stream);
/* The slot form of the scan mode over a layout built WITH window starts
 * (fdx_customer_layout_starts_grouped): the window starts come from the layout, so the scan
 * is two coalesced passes -- per-segment prefix sums (grouped order), then NB / SUM by slot.
 * Same outputs and precision as fdx_customer_windows_scan(sorder_d, goff_d, ...); gamount_d
 * grouped; workspace fdx_customer_windows_scan_workspace_size(n, n_seg). */
int fdx_customer_windows_scan_slots(const double *gamount_d, const int64_t *seg_off_d, int64_t n_seg, int64_t n,
                                    const int32_t *sorder_d, const uint32_t *goff_d, int64_t n_slots,
                                    int32_t n_windows, const int32_t *starts_d, int32_t *nb_d, double *sum_d,
                                    void *workspace_d, size_t workspace_bytes, void *stream);
/* The sequential half of fdx_customer_windows_interleaved over the starts of
 * fdx_customer_layout_starts: nb_d / sum_d as there ([W][n_slots] by slot; n_windows >= 3,
 * i.e. <= 21 segments per wave). */
int fdx_customer_windows_walk(const double *iamt_d, const int64_t *seg_off_d, const int32_t *sorder_d,
                              const uint32_t *goff_d, int64_t n_seg, int64_t n_slots, int32_t n_windows,
                              const int32_t *starts_d, int32_t *nb_d, double *sum_d, void *stream);
/* fdx_customer_windows over that layout: nb_d / sum_d are [W][n_slots] indexed by slot, with
 * sum_d the rolling SUM (pandas roll_sum, bit-exact); the average is sum / nb (IEEE float64
 * division, done by the consumer -- fdx_forest_prepare_grouped with cust_val_is_sum = 1 --
 * so that the division is off the sequential recurrence's critical path). */
int fdx_customer_windows_interleaved(const int64_t *its_d, const double *iamt_d,
                                     const int64_t *seg_off_d, const int32_t *sorder_d,
                                     const uint32_t *goff_d, int64_t n_seg, int64_t n_slots,
                                     const int64_t *window_ns, int32_t n_windows, int32_t *nb_d,
                                     double *sum_d, void *stream);

/* ---- a-3: terminal delayed-risk windows -----------------------------------------------
 * Replaces get_count_risk_rolling_window(terminal_transactions, delay_period,
 * windows_size_in_days, feature) (feature_transformation.ipynb:1495-1522) applied through
 * `groupby('TERMINAL_ID').apply(...)` (:2435), for all segments at once.
 *   nb_d[w*n+i]   = #rows of the segment with t in (t_i - delay - w, t_i - delay]
 *   risk_d[w*n+i] = (#fraud rows in that window) / nb, or 0.0 when nb == 0 (fillna(0))
 * fraud_d: 0/1 bytes.  Rows grouped by segment (seg_off_d), time order inside each segment
 * (fdx_rekey of a time-ordered table; fdx_argsort_i64 first otherwise).  workspace_d: caller
 * device memory of at least fdx_terminal_windows_workspace_size(n) bytes (the prefix fraud
 * counts of segments longer than the kernel's 1,024-row LDS stage); the call allocates nothing. */
size_t fdx_terminal_windows_workspace_size(int64_t n);
int fdx_terminal_windows(const int64_t *ts_ns_d, const uint8_t *fraud_d, const int64_t *seg_off_d,
                         int64_t n_seg, int64_t n, int64_t delay_ns, const int64_t *window_ns,
                         int32_t n_windows, int32_t *nb_d, double *risk_d, void *workspace_d,
                         size_t workspace_bytes, void *stream);

/* Assemble the 15-feature scoring matrix in the column order of `input_features`
 * (model_training.ipynb:457-463 = pyspark/scripts/fraud_detection.py:126-132):
 * X_d row r (leading dimension ld >= 3 + 4*n_windows, float64):
 *   [TX_AMOUNT, TX_DURING_WEEKEND, TX_DURING_NIGHT,
 *    CUSTOMER_ID_NB_TX_w, CUSTOMER_ID_AVG_AMOUNT_w (w = each window),
 *    TERMINAL_ID_NB_TX_w, TERMINAL_ID_RISK_w (w = each window)]
 * amount/weekend/night are in output row order; the grouped outputs of
 * fdx_customer_windows / fdx_terminal_windows are scattered back through their perms.
 * The three term_* pointers may all be NULL (the multi-GPU path fills those columns with
 * fdx_reply_assemble after the return exchange). */
int fdx_assemble_features(int64_t n, int32_t n_windows, const double *amount_d,
                          const uint8_t *weekend_d, const uint8_t *night_d, const int32_t *cust_perm_d,
                          const int32_t *cust_nb_d, const double *cust_avg_d, const int32_t *term_perm_d,
                          const int32_t *term_nb_d, const double *term_risk_d, double *X_d, int64_t ld,
                          void *stream);

/* The terminal windows over GROUPED inputs (the scoring pipeline's form): gts_d[q] = ts of
 * grouped position q (fdx_rekey_payload output); fraud of q = gfraud_d[q], or bit 31 of
 * rows_d[q] when gfraud_d is NULL (fdx_rekey_payload's packed flag); rows_d[q] & 0x7FFFFFFF =
 * the row whose record is written (NULL: q).  Output: COUNT RECORDS rec_d[row][n_windows] --
 * word w = NB_w | FRAUD_w << 32 (both uint32; RISK_w = NB_w > 0 ? (double)FRAUD_w / NB_w : 0,
 * the IEEE division fdx_terminal_windows does; the consumers fdx_forest_prepare_grouped,
 * fdx_forest_prepare_reply and fdx_reply_assemble divide) -- or, when rec_d is NULL,
 * nb_d / risk_d [w*n + q].  runs != 0:
 * segments are concatenations of time-sorted runs (multi-GPU owner side).  scratch_d: int32[n]
 * (prefix fraud counts of segments longer than the kernel's LDS stage, 1,024 rows; such
 * segments cost O(L log L)). */
int fdx_terminal_windows_grouped(const int64_t *gts_d, const uint8_t *gfraud_d, const int32_t *rows_d,
                                 const int64_t *seg_off_d, int64_t n_seg, int64_t n, int64_t delay_ns,
                                 const int64_t *window_ns, int32_t n_windows, int32_t runs, int32_t *nb_d,
                                 double *risk_d, int64_t *rec_d, int32_t *scratch_d, void *stream);
/* fdx_terminal_windows_grouped (count records by row) in the COMPACT format, n_windows = 3:
 * rec_d is int64[5 n], 16-byte aligned.  Words [2 r, 2 r + 2) hold row r's record as
 * lo = NB_0 | NB_1 << 21 | NB_2 << 42, hi = FRAUD_0 | FRAUD_1 << 21 | FRAUD_2 << 42 -- one
 * aligned 16-byte store (and load, FDX_PREP_TERM_COMPACT) per row instead of a 24-byte record
 * across two.  A row with a window count above 2^21 - 1 instead gets lo = (1 << 63) | o,
 * hi = 0, with its full 3-word record (NB | FRAUD << 32 per window) at rec_d[o], o = 2 n + 3 r
 * (the overflow area [2 n, 5 n), written only for such rows).  Exact for any counts. */
int fdx_terminal_windows_grouped_compact(const int64_t *gts_d, const uint8_t *gfraud_d, const int32_t *rows_d,
                                         const int64_t *seg_off_d, int64_t n_seg, int64_t n, int64_t delay_ns,
                                         const int64_t *window_ns, int32_t n_windows, int32_t runs, int64_t *rec_d,
                                         int32_t *scratch_d, void *stream);

/* ---- a-4: re-key (stable radix sort by key + segment offsets) -------------------------
 * Replaces the regrouping done by pandas groupby('CUSTOMER_ID') / sort_values /
 * groupby('TERMINAL_ID') (feature_transformation.ipynb:1092-1093, :2435-2436).
 * keys_d[i] in [0, n_keys); key_bits = bits needed for n_keys-1 (<= 31).
 * Outputs: perm_d[j] = input row placed at grouped position j (stable: equal keys keep
 * input order), sorted_keys_d (optional, may be NULL), seg_off_d[0..n_keys] (CSR by key
 * value; empty keys get empty segments; may be NULL when only the order is needed). */
size_t fdx_rekey_workspace_size(int64_t n, int32_t key_bits);
int fdx_rekey(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys, int32_t *perm_d,
              int32_t *sorted_keys_d, int64_t *seg_off_d, void *workspace_d, size_t workspace_bytes,
              void *stream);

/* fdx_rekey that also carries up to two 8-byte payload streams through the radix passes
 * (pay0_d / pay1_d in input row order -> pay0_out_d / pay1_out_d in grouped order), so that the
 * window kernels read the grouped table sequentially.  flag_d (optional, uint8 per row):
 * perm_d[j] = row | (flag_d[row] != 0) << 31 (e.g. TX_FRAUD packed beside the row index).
 * Workspace: fdx_rekey_payload_workspace_size(n, key_bits, number of payload streams). */
size_t fdx_rekey_payload_workspace_size(int64_t n, int32_t key_bits, int32_t n_payload);
int fdx_rekey_payload(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys, const uint8_t *flag_d,
                      const uint64_t *pay0_d, const uint64_t *pay1_d, int32_t *perm_d, int64_t *seg_off_d,
                      uint64_t *pay0_out_d, uint64_t *pay1_out_d, void *workspace_d, size_t workspace_bytes,
                      void *stream);
/* fdx_rekey_payload that also counts the keys outside [0, n_keys) into *bad_d (device int32,
 * zeroed by the call, written on `stream`) inside the first radix pass's histogram -- the id
 * range check of the reference's groupby without a kernel of its own.  Out-of-range keys never
 * make the call write out of bounds; the caller raises when *bad_d != 0 (the grouping would be
 * wrong), as fdx/ops.py:KeyRangeCheck does. */
int fdx_rekey_payload_checked(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys,
                              const uint8_t *flag_d, const uint64_t *pay0_d, const uint64_t *pay1_d, int32_t *perm_d,
                              int64_t *seg_off_d, uint64_t *pay0_out_d, uint64_t *pay1_out_d, int32_t *bad_d,
                              void *workspace_d, size_t workspace_bytes, void *stream);
/* fdx_rekey_payload_checked (bad_d optional here) with the sorted keys written to the caller's
 * sorted_keys_d (int32 [n], 16-byte aligned) instead of the segment offsets: the workspace is
 * free again when the call's last pass ends, so a second re-key sharing it can start before
 * the offsets are derived (fdx_segment_offsets_sorted, from sorted_keys_d, on any stream
 * ordered after this call). */
int fdx_rekey_payload_keys(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys, const uint8_t *flag_d,
                           const uint64_t *pay0_d, const uint64_t *pay1_d, int32_t *perm_d, int32_t *sorted_keys_d,
                           uint64_t *pay0_out_d, uint64_t *pay1_out_d, int32_t *bad_d, void *workspace_d,
                           size_t workspace_bytes, void *stream);
/* The first radix pass's scanned digit table of a payload re-key, computed ahead of it (on
 * another stream, e.g. while a re-key that shares the workspace still runs): hist0_d
 * (fdx_rekey_hist0_size bytes, the caller's, not the workspace) also receives the id-range count
 * into bad_d (optional, zeroed by the call) -- the check fdx_rekey_payload_checked does in that
 * pass.  fdx_rekey_payload_hist0 is fdx_rekey_payload whose first pass goes straight to its
 * scatter with that table; keys_d must be unchanged in between. */
size_t fdx_rekey_hist0_size(int64_t n, int32_t key_bits);
int fdx_rekey_hist0(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys, void *hist0_d,
                    size_t hist0_bytes, int32_t *bad_d, void *stream);
int fdx_rekey_payload_hist0(const int32_t *keys_d, int64_t n, int32_t key_bits, int64_t n_keys, const uint8_t *flag_d,
                            const uint64_t *pay0_d, const uint64_t *pay1_d, int32_t *perm_d, int64_t *seg_off_d,
                            uint64_t *pay0_out_d, uint64_t *pay1_out_d, const void *hist0_d, void *workspace_d,
                            size_t workspace_bytes, void *stream);
/* seg_off_d[0..n_keys] from keys sorted ascending (fdx_rekey's seg_off: rows of key k at
 * [seg_off_d[k], seg_off_d[k+1])), one pass over the keys; keys outside [0, n_keys) never put an
 * offset outside [0, n]. */
int fdx_segment_offsets_sorted(const int32_t *sorted_keys_d, int64_t n, int64_t n_keys, int64_t *seg_off_d,
                               void *stream);

/* Stable argsort of int64 keys (e.g. TX_DATETIME ns): perm_d[j] = input row at sorted
 * position j, ties keep input order.  Used when a caller's frame is not in time order
 * (the reference sorts every group with sort_values('TX_DATETIME'),
 * feature_transformation.ipynb:604, :1497). */
size_t fdx_argsort_i64_workspace_size(int64_t n);
int fdx_argsort_i64(const int64_t *keys_d, int64_t n, int32_t *perm_d, void *workspace_d,
                    size_t workspace_bytes, void *stream);
/* Dense ids of arbitrary int64 keys, order-preserving: ids_d[i] = the rank of keys_d[i] among
 * the distinct keys (0-based), *n_unique_d (device int64) = the number of distinct keys --
 * what pandas' groupby does with ids that are not dense in [0, n) (the drop-in's sparse-id
 * path; feature_transformation.ipynb:1092, :2435).  Sort-based (fdx_argsort_i64), no host sync. */
size_t fdx_dense_ids_i64_workspace_size(int64_t n);
int fdx_dense_ids_i64(const int64_t *keys_d, int64_t n, int32_t *ids_d, int64_t *n_unique_d, void *workspace_d,
                      size_t workspace_bytes, void *stream);
/* *flag_d = 1 if keys_d is non-decreasing, else 0 (stream-ordered). */
int fdx_is_sorted_i64(const int64_t *keys_d, int64_t n, int32_t *flag_d, void *stream);

/* Device-wide exclusive prefix sum of m uint32 values, in place. */
/* seg_off_d[0..n_keys] of the stable grouping by key -- equal to fdx_rekey's seg_off when every
 * key lies in [0, n_keys) -- from a key histogram, without sorting (the group sizes of
 * groupby('CUSTOMER_ID'), feature_transformation.ipynb:1092; the customer layout's plan needs
 * only these, so it can run while the rows are being re-keyed).  bad_d (optional, int32):
 * the number of keys outside [0, n_keys). */
size_t fdx_key_segments_workspace_size(int64_t n_keys);
int fdx_key_segments(const int32_t *keys_d, int64_t n, int64_t n_keys, int64_t *seg_off_d, int32_t *bad_d,
                     void *workspace_d, size_t workspace_bytes, void *stream);

size_t fdx_exclusive_scan_u32_workspace_size(int64_t m);
int fdx_exclusive_scan_u32(uint32_t *data_d, int64_t m, void *workspace_d, void *stream);

/* inv_d[perm_d[i]] = i */
int fdx_invert_perm(const int32_t *perm_d, int64_t n, int32_t *inv_d, void *stream);

/* dst[j] = src[perm[j]] for 1-, 2-, 4- or 8-byte elements (elem_bytes). */
int fdx_gather(const void *src_d, int32_t elem_bytes, const int32_t *perm_d, int64_t n, void *dst_d,
               void *stream);
/* dst[perm[j]] = src[j]  (inverse of fdx_gather). */
int fdx_scatter(const void *src_d, int32_t elem_bytes, const int32_t *perm_d, int64_t n, void *dst_d,
                void *stream);

/* ---- multi-GPU re-key exchange ------------------------------------
 * Rows are sharded by customer; the terminal windows need every row of a terminal on its
 * owner rank, owner(t) = t % world.  Per step: fdx_key_map(MOD) -> fdx_rekey(owner) ->
 * fdx_exchange_pack -> RCCL all-to-all (16 B/row) -> fdx_exchange_unpack (local terminal
 * id = t / world) -> fdx_rekey_payload (ts payload, fraud flag) -> fdx_terminal_windows_grouped
 * with runs = 1 (a segment = one time-sorted run per source rank; count records indexed by
 * receive position) -> RCCL all-to-all back -> fdx_forest_prepare_grouped / fdx_reply_assemble.
 * Record layouts: exchange rec[j] = {ts, term<<32 | fraud<<31 | source row}; reply rows
 * are count records (n_windows words, fdx_terminal_windows_grouped). */
#define FDX_KEY_MOD 0 /* out = key % param  (owner rank of a terminal)          */
#define FDX_KEY_DIV 1 /* out = key / param  (owner-local terminal id)           */
#define FDX_KEY_SUB 2 /* out = key - param  (shard-local customer id)           */
int fdx_key_map(const int32_t *keys_d, int64_t n, int32_t op, int32_t param, int32_t *out_d,
                void *stream);
/* *count_d = #{i : keys_d[i] < lo or keys_d[i] >= hi} (stream-ordered; count_d is zeroed by
 * the call).  fdx_rekey requires keys in [0, n_keys): a shard's customer ids outside its
 * range would be mis-grouped, so the callers check with this before trusting the segments. */
int fdx_count_out_of_range(const int32_t *keys_d, int64_t n, int32_t lo, int32_t hi, int32_t *count_d,
                           void *stream);
int fdx_exchange_pack(const int64_t *ts_d, const int32_t *term_d, const uint8_t *fraud_d,
                      const int32_t *perm_d, int64_t n, int64_t *rec_d, void *stream);
int fdx_exchange_unpack(const int64_t *rec_d, int64_t m, int32_t world, int64_t *ts_d,
                        int32_t *term_local_d, uint8_t *fraud_d, void *stream);
int fdx_reply_assemble(const int64_t *reply_d, const int32_t *perm_d, int64_t n, int32_t n_windows,
                       double *X_d, int64_t ld, int32_t col0, void *stream);

/* ---- a-5 + a-7/a-8: StandardScaler + tree-ensemble predict_proba ----------------------
 * Replaces `loaded_scaler.transform(features)` + `model.predict_proba(scaled)[:, 1]`
 * (pyspark/scripts/fraud_detection.py:190-193) and the predict_proba inside
 * fit_model_and_get_predictions (shared_functions.py:304-333 /
 * model_training.ipynb:491-520) for sklearn DecisionTreeClassifier /
 * RandomForestClassifier with 2 classes and one output.
 *
 * The forest is described with sklearn's own per-tree arrays concatenated over trees:
 * tree t owns nodes [node_offsets[t], node_offsets[t+1]); child indices are tree-local
 * (-1 = leaf), value1[i] = tree_.value[i, 0, 1] (class-1 fraction).  Scaler arrays are
 * optional (NULL = no scaling). */
/* StandardScaler.transform alone (shared_functions.py:114-120 scaleData):
 * out[r,f] = (X[r,f] - mean[f]) / scale[f] in float64; mean_d/scale_d are device arrays
 * (either may be NULL = skip that step).  Element (r, f) of X is X_d[r*row_stride +
 * f*col_stride]; of out, out_d[r*out_row_stride + f*out_col_stride]. */
int fdx_standard_scale(const double *X_d, int64_t n, int32_t n_features, int64_t row_stride,
                       int64_t col_stride, const double *mean_d, const double *scale_d, double *out_d,
                       int64_t out_row_stride, int64_t out_col_stride, void *stream);

typedef struct fdx_forest_s *fdx_forest;

typedef struct {
    int32_t n_trees;
    int32_t n_features;
    const int64_t *node_offsets;   /* [n_trees+1] */
    const int64_t *children_left;  /* [total nodes] */
    const int64_t *children_right; /* [total nodes] */
    const int64_t *feature;        /* [total nodes] */
    const double *threshold;       /* [total nodes] */
    const uint8_t *missing_go_to_left; /* [total nodes] (NULL = all 0) */
    const double *value1;          /* [total nodes] */
    const double *scaler_mean;     /* [n_features] or NULL */
    const double *scaler_scale;    /* [n_features] or NULL */
} fdx_forest_desc;

int fdx_forest_create(const fdx_forest_desc *desc, fdx_forest *out, void *stream);
/* Host-only: validate + pack the forest exactly as fdx_forest_create does (no GPU needed).
 * nodes_out [total nodes] packed 8-byte nodes, orig_out [total] sklearn node id of each
 * packed node, root_out [n_trees] packed position of each root. */
int fdx_forest_pack(const fdx_forest_desc *desc, uint64_t *nodes_out, int32_t *orig_out,
                    int32_t *root_out);
/* Host-only: the RANK layout fdx_forest_create builds when the forest fits it (<= 15
 * features, <= 32767 distinct float32 thresholds per feature, every tree within the LDS
 * node budget; else FDX_E_UNSUPPORTED and the wide 8-byte layout is used).  Per feature f,
 * U_f = thr_out[thr_off_out[f] .. thr_off_out[f+1]) are the sorted distinct thresholds
 * (float32 rounded toward -inf); a row value x becomes r = #{u in U_f : u < x}.
 * nodes_out (4 B): [30:16] threshold rank k, [15:12] feature (15 = leaf / jump),
 * [11:0] right-child offset (left child = next node; go left iff r <= k); a leaf is
 * 0x7FFFF000, a jump node 0x0000F000 | d forwards to the node d further.  orig_out = sklearn
 * node id per node (-1 for jumps), leaf_value_out = value1 of leaves, missing_left_out =
 * missing_go_to_left, root_out/depth_out per tree (depth = max steps incl. jumps),
 * thr_off_out [17].  Sizes from fdx_forest_rank_layout_size. */
int fdx_forest_rank_layout_size(const fdx_forest_desc *desc, int64_t *n_nodes, int32_t *n_thresholds);
int fdx_forest_pack_rank(const fdx_forest_desc *desc, uint32_t *nodes_out, int32_t *orig_out,
                         double *leaf_value_out, uint8_t *missing_left_out, int32_t *root_out,
                         int32_t *depth_out, float *thr_out, int32_t *thr_off_out);
/* Rank layout v2 (forests whose features have more than 32,767 distinct thresholds -- e.g. the
 * reference's deployed RandomForestClassifier(random_state=0), model_training.ipynb:2212): 32
 * u16 threshold-rank SLOTS, feature f spanning ceil(|U_f| / 32767) consecutive slots; slot s
 * holds min(max(r_f - slot_base[s], 0), 32767).  Node (4 B): [30:16] k' | [15:11] slot |
 * [10:0] right offset; leaf 0x7FFF0000; jump 0xFFFF0000 | offset.  version = 1 or 2 (1 = the
 * fdx_forest_pack_rank layout; thr_off_out then has 17 meaningful entries of 33, slot tables 0).
 * fdx_forest_create picks v1 when the forest fits it, else v2 when <= 16 features need <= 32
 * slots, else the wide 8-byte layout.  v2 forests score through fdx_forest_predict /
 * prepare + traverse (the fused scoring-pipeline prepares need v1). */
int fdx_forest_rank_layout_size2(const fdx_forest_desc *desc, int32_t version, int64_t *n_nodes,
                                 int32_t *n_thresholds, int32_t *n_slots);
int fdx_forest_pack_rank2(const fdx_forest_desc *desc, int32_t version, uint32_t *nodes_out, int32_t *orig_out,
                          double *leaf_value_out, uint8_t *missing_left_out, int32_t *root_out, int32_t *depth_out,
                          float *thr_out, int32_t *thr_off_out /* [33] */, int32_t *slot_feat_out /* [32] */,
                          int32_t *slot_base_out /* [32] */);
/* Host form of the fused row assembly's search tables (tests; fdx_forest_prepare_grouped*):
 * for a 15-feature forest, every 4th v1-layout threshold of features 0, 4, 6, 8 (amount and the
 * three customer averages) as a complete 9-ary tree of 8-key nodes, keys in in-order (= sorted)
 * order, +inf padded.  Feature s's node k (children 9k+1..9k+9) is trees_out[8*(eoff_out[s]+k)
 * ...+7]; elev_out[s] levels.  A descent that goes to child c = #keys < v at every level
 * counts the samples < v in base 9.  trees_out may be NULL (sizes only); *n_floats = 0 when
 * the trees exceed the kernel's LDS budget (the generic prepare kernel is used then). */
int fdx_forest_search_trees(const fdx_forest_desc *desc, float *trees_out, int64_t cap, int64_t *n_floats,
                            int32_t *eoff_out /* [4] */, int32_t *elev_out /* [4] */);
/* *layout = 0 (wide 8-byte nodes), 1 (rank v1, the default when the forest fits it), 2 (rank
 * v2) or 3 (rank v2 with one slot per feature: v1 row format, compact 32 KiB row planes);
 * *n_slots = rank slots.  fdx_forest_set_variant rebuilds the rank layout in the other node
 * format when the requested variant needs it. */
int fdx_forest_layout(fdx_forest forest, int32_t *layout, int32_t *n_slots);
int fdx_forest_destroy(fdx_forest forest);
int fdx_forest_info(fdx_forest forest, int32_t *n_trees, int32_t *n_features, int64_t *n_nodes,
                    int32_t *n_chunks);
/* Workspace for a traversal of n_rows rows.  Small batches (that cannot fill the CUs with
 * one LDS chunk at a time) also get room for per-tree values, so that every chunk runs in
 * one launch; a workspace without that room still works (chunk-sequential launches).
 * fdx_forest_workspace_size_max: one workspace for every batch size up to n_rows. */
size_t fdx_forest_workspace_size(fdx_forest forest, int64_t n_rows);
size_t fdx_forest_workspace_size_max(fdx_forest forest, int64_t n_rows);
/* X element (r, f) is X_d[r*row_stride + f*col_stride] (float64, raw unscaled features;
 * NaN allowed = missing).  proba_d[r] = predict_proba(X)[r, 1]; leaf_d (optional) is
 * [n][n_trees] int32 sklearn node ids (tree_.apply). */
int fdx_forest_predict(fdx_forest forest, const double *X_d, int64_t n, int64_t row_stride,
                       int64_t col_stride, double *proba_d, int32_t *leaf_d, void *workspace_d,
                       size_t workspace_bytes, void *stream);

/* The two halves of fdx_forest_predict, for callers that time or overlap them:
 * prepare = scale + float32 cast (+ threshold ranks) into the workspace; traverse = the tree
 * walk over the LDS-sized chunks of trees (one launch for all of them when each chunk is one walk
 * group, see fdx_forest_traverse_launches) reading that workspace. */
int fdx_forest_prepare(fdx_forest forest, const double *X_d, int64_t n, int64_t row_stride,
                       int64_t col_stride, void *workspace_d, size_t workspace_bytes, void *stream);
int fdx_forest_traverse(fdx_forest forest, int64_t n, double *proba_d, int32_t *leaf_d,
                        void *workspace_d, size_t workspace_bytes, void *stream);
/* *launches = the tree-walk kernel launches fdx_forest_traverse makes for n rows (with a full
 * fdx_forest_workspace_size workspace): 1 when every LDS chunk is one walk group and no leaf ids
 * are asked for (one launch walks the chunks in turn), or for small batches (all chunks at
 * once); else one per chunk (n_chunks of fdx_forest_info). */
int fdx_forest_traverse_launches(fdx_forest forest, int64_t n, int32_t with_leaves, int32_t *launches);
/* Traversal kernel shape (one default per layout):
 *   0 = wide layout (8-byte nodes, float32 rows; any forest, the only one for > 15 features),
 *   1 = rank layout v1, 1,024 threads x 10 trees per lane (the default when the forest fits v1),
 *   2 = rank layout v2, 32 threshold slots (the default for forests v1 cannot hold),
 *   3 = v2 nodes over 16 compact u16 planes (every feature in one slot),
 *   4 = rank layout v2 with 10 trees per lane,
 *   5 = rank layout v2 over paired planes: two rows per lane, only the forest's threshold slots
 *       staged (the v2 default when every tree fits the node budget left beside them: the
 *       reference's deployed RF(100, unlimited depth), 22 slots).
 * Variants > 0 need <= 15 features (the rank rows' 16th slot is the v1 sentinel) and the
 * rank layout (FDX_E_UNSUPPORTED otherwise; a
 * refused call leaves the forest's node format, variant and chunks as they were).
 * Re-cuts the LDS chunks; results are identical for every variant.  The row format of a
 * prepared workspace depends on the layout: prepare again after switching layouts. */
int fdx_forest_set_variant(fdx_forest forest, int32_t variant);
int fdx_forest_get_variant(fdx_forest forest, int32_t *variant);
/* Rows per traversal range (rounded down to a multiple of 1,024; 0 = the default, as many as
 * the walk's 32-bit offsets allow): every chunk walks one range before the next range starts. */
int fdx_forest_set_range_rows(fdx_forest forest, int64_t rows);

/* Fused assemble + scale for the scoring pipeline: writes the forest's float32 feature
 * rows in the workspace straight from the window kernels' grouped outputs (same columns
 * and arithmetic as fdx_assemble_features followed by fdx_forest_prepare), so
 * fdx_forest_traverse can follow.  term_* may be NULL (filled by fdx_forest_prepare_reply
 * in the multi-GPU path, col0 = 3 + 2*n_windows). */
int fdx_forest_prepare_features(fdx_forest forest, int64_t n, int32_t n_windows,
                                const double *amount_d, const uint8_t *weekend_d,
                                const uint8_t *night_d, const int32_t *cust_perm_d,
                                const int32_t *cust_nb_d, const double *cust_avg_d,
                                const int32_t *term_perm_d, const int32_t *term_nb_d,
                                const double *term_risk_d, void *workspace_d,
                                size_t workspace_bytes, void *stream);
int fdx_forest_prepare_reply(fdx_forest forest, const int64_t *reply_d, const int32_t *perm_d,
                             int64_t n, int32_t n_windows, int32_t col0, void *workspace_d,
                             size_t workspace_bytes, void *stream);

/* The scoring rows in CUSTOMER-grouped order, each written whole (coalesced): row i is
 * transaction r = cust_perm[i]; cust_ts/cust_amount/cust_nb/cust_avg are the customer-grouped
 * copies and outputs (flags are derived from cust_ts with flags_mode), the terminal half
 * is the count record term_rec[term_inv[r]] (term_inv may be NULL = identity: the
 * fdx_terminal_windows_grouped output with rows_d = the terminal perm is already in row
 * order; the multi-GPU reply records need term_inv = inverse of the send perm).  Follow
 * with fdx_forest_traverse_perm(out_perm = cust_perm)
 * so that proba lands in row order.  The same call serves the interleaved customer layout
 * (cust_* = slot arrays, cust_perm = irow): slots with cust_perm < 0 are padding (zero
 * row, never written back).  cust_val_is_sum: FDX_PREP_* option bits (1 = cust_avg_d
 * holds rolling sums and the average is computed here as sum / nb; 4 = compact terminal
 * records). */
#define FDX_PREP_VAL_IS_SUM 1   /* cust_avg_d holds rolling sums: average = sum / nb here      */
#define FDX_PREP_TERM_COMPACT 4 /* term_rec_d holds COMPACT records (fdx_terminal_windows_
                                   grouped_compact; n_windows = 3, 16-byte aligned)          */
#define FDX_PREP_FLAG_CLEARED 8 /* the workspace's NaN flag was cleared by fdx_forest_clear_flag
                                   (earlier, e.g. on another stream): no clearing memset here   */
/* Clears the NaN flag of a forest workspace sized for n rows (a 4-byte memset on `stream`): with
 * FDX_PREP_FLAG_CLEARED, the prepare call that follows skips its own clearing -- the scoring step
 * enqueues this off its critical path (fdx.pipeline). */
int fdx_forest_clear_flag(fdx_forest forest, int64_t n, void *workspace_d, size_t workspace_bytes, void *stream);
int fdx_forest_prepare_grouped(fdx_forest forest, int64_t n, int32_t n_windows, int32_t flags_mode,
                               int32_t cust_val_is_sum, const int64_t *cust_ts_d, const double *cust_amount_d,
                               const int32_t *cust_nb_d, const double *cust_avg_d,
                               const int32_t *cust_perm_d, const int32_t *term_inv_d,
                               const int64_t *term_rec_d, void *workspace_d, size_t workspace_bytes,
                               void *stream);
/* The featurized table the reference writes (feature_transformation.ipynb:2890-2905; columns
 * added at :613-622 and :1509-1520): one 80-byte record per transaction in the compact form of
 * SURVEY §8(d) -- window counts as int32 (pandas holds the same integers as float64),
 * averages / risks float64 bit-equal to the reference's, the two flags as bytes -- plus the
 * transaction's input row.  Windows in windows_days order (1, 7, 30 for the reference). */
typedef struct fdx_feature_row {
    int32_t cust_nb[3];     /* CUSTOMER_ID_NB_TX_{w}DAY_WINDOW          */
    int32_t term_nb[3];     /* TERMINAL_ID_NB_TX_{w}DAY_WINDOW          */
    double cust_avg[3];     /* CUSTOMER_ID_AVG_AMOUNT_{w}DAY_WINDOW     */
    double term_risk[3];    /* TERMINAL_ID_RISK_{w}DAY_WINDOW           */
    uint8_t weekend, night; /* TX_DURING_WEEKEND, TX_DURING_NIGHT       */
    uint8_t pad[2];
    int32_t row;            /* input row of the transaction (-1: a padding slot's record) */
} fdx_feature_row;
/* rows_order of fdx_forest_prepare_grouped_rows */
#define FDX_ROWS_INPUT_ORDER 1 /* out_d = fdx_feature_row records, out_d[r] = input row r (time order,
                                  as the reference's table after its sort_values('TX_DATETIME')):
                                  one random 80-byte write per row (rows >= out_cap: not written) */
#define FDX_ROWS_SLOT_ORDER 2  /* out_d = the same fields as COLUMNS, by scoring slot i < n (padding
                                  slots: row -1, zero features), each column written coalesced:
                                  FDX_FEATURE_COL(c, cap) bytes into out_d, cap = rows per column */
/* Column c of the slot-order table (a buffer of FDX_FEATURE_TABLE_BYTES(cap) bytes, cap >= n,
 * cap % 64 == 0): 0-2 cust_nb[w] int32, 3-5 term_nb[w] int32, 6-8 cust_avg[w] float64,
 * 9-11 term_risk[w] float64, 12 row int32, 13 flags uint8[2] per slot (weekend, night). */
#define FDX_FEATURE_COL(c, cap)                                                                  \
    ((c) < 6 ? (int64_t)(c) * 4 * (cap) : (c) < 12 ? (int64_t)24 * (cap) + ((c) - 6) * (int64_t)8 * (cap) \
                                       : (c) == 12 ? (int64_t)72 * (cap) : (int64_t)76 * (cap))
#define FDX_FEATURE_TABLE_BYTES(cap) ((int64_t)78 * (cap))
/* fdx_forest_prepare_grouped that also writes the featurized table, in rows_order, with the
 * same values the scoring row is built from (n_windows = 3 and the rank layout; other shapes:
 * FDX_E_UNSUPPORTED).  out_d NULL = fdx_forest_prepare_grouped; out_cap = records (input order)
 * or rows per column (slot order) the buffer holds. */
int fdx_forest_prepare_grouped_rows(fdx_forest forest, int64_t n, int32_t n_windows, int32_t flags_mode,
                                    int32_t cust_val_is_sum, const int64_t *cust_ts_d,
                                    const double *cust_amount_d, const int32_t *cust_nb_d,
                                    const double *cust_avg_d, const int32_t *cust_perm_d,
                                    const int32_t *term_inv_d, const int64_t *term_rec_d, void *out_d,
                                    int64_t out_cap, int32_t rows_order, void *workspace_d, size_t workspace_bytes,
                                    void *stream);
/* fdx_forest_traverse writing proba_d[out_perm_d[row]] (and leaf rows likewise). */
int fdx_forest_traverse_perm(fdx_forest forest, int64_t n, double *proba_d, const int32_t *out_perm_d,
                             int32_t *leaf_d, void *workspace_d, size_t workspace_bytes, void *stream);

/* ---- §8(f): callers and data formats either side of the path (csrc/fdx_aux.hip) ----------
 * f-1 feature snapshots for the serving tables (feature_transformation.ipynb:2914-2918,
 * :3606-3635, :4182).  Over a STABLE grouping (perm_d = fdx_rekey perm, seg_off_d) of the
 * frame's rows -- i.e. frame order inside each segment; perm_d NULL = rows already grouped:
 *   fdx_segment_latest:         out_row_d[k] = the first row of segment k holding its maximum
 *                               ts (pandas groupby(key).TX_DATETIME.idxmax()), -1 if empty;
 *   fdx_segment_first_in_range: out_row_d[k] = the first row of segment k with
 *                               t_lo <= ts < t_hi (date filter + drop_duplicates keep='first'),
 *                               -1 if none. */
int fdx_segment_latest(const int64_t *ts_d, const int32_t *perm_d, const int64_t *seg_off_d, int64_t n_seg,
                       int32_t *out_row_d, void *stream);
int fdx_segment_first_in_range(const int64_t *ts_d, const int32_t *perm_d, const int64_t *seg_off_d,
                               int64_t n_seg, int64_t t_lo, int64_t t_hi, int32_t *out_row_d, void *stream);
/* The same two snapshots straight from the featurized table the scoring path writes
 * (fdx_forest_prepare_grouped_rows, FDX_ROWS_SLOT_ORDER: row_d = its FDX_FEATURE_COL(12) column,
 * slot -> input row, -1 = padding), input rows in time order; ts_d / key_d by input row:
 *   FDX_SELECT_LATEST:         out_slot_d[k] = the slot of the first input row holding key k's
 *                              maximum ts (groupby(key).TX_DATETIME.idxmax(), :2914-2918)
 *   FDX_SELECT_FIRST_IN_RANGE: out_slot_d[k] = the slot of key k's first input row with
 *                              t_lo <= ts < t_hi (:3606-3635)
 * -1 for a key without such a row; the feature columns of the chosen rows are read at those
 * slots.  Workspace: fdx_table_select_workspace_size(n_keys). */
#define FDX_SELECT_LATEST 0
#define FDX_SELECT_FIRST_IN_RANGE 1
size_t fdx_table_select_workspace_size(int64_t n_keys);
int fdx_table_select(const int32_t *row_d, int64_t n_slots, const int64_t *ts_d, const int32_t *key_d,
                     int64_t n_keys, int32_t mode, int64_t t_lo, int64_t t_hi, int32_t *out_slot_d, void *workspace_d,
                     size_t workspace_bytes, void *stream);
/* f-2 Debezium CDC records of a micro-batch (pyspark/scripts/kafka_s3_sink_transactions.py):
 *   fdx_cdc_decode: tx_amount bytes (record i = bytes_d[offsets_d[i] .. offsets_d[i+1]),
 *     big-endian two's complement, 1..8 bytes; :64-71) -> unscaled_d (int64 cents) and
 *     amount_d (= unscaled / 100.0, the double of Decimal(unscaled) / 10**2); tx_datetime
 *     microseconds us_d -> ts_ns_d = whole seconds as from_unixtime(us / 1000000) (:167),
 *     in ns.  Any output may be NULL; *bad_d = 1 if a record has 0 or > 8 bytes.
 *   fdx_dedup_latest: ROW_NUMBER() OVER (PARTITION BY tx_id ORDER BY timestamp DESC) = 1
 *     (:180): keep_d[i] = 1 for the record with the largest Kafka timestamp of each key (ties:
 *     the last in batch order), 0 otherwise.  O(n): an open-addressing hash table in the
 *     workspace (fdx_dedup_latest_workspace_size), no sort.  *bad_d = 1 if a key is -1 (the
 *     table's empty pattern; bad_d is not cleared by the call).
 *   fdx_cdc_compact: the kept records (keep_d) of a decoded micro-batch, in batch order, as the
 *     stream state's input columns -- customer / terminal ids narrowed to int32 (an id outside
 *     int32 becomes -1: fdx_stream_update then reports it out of range), ts (ns), amount,
 *     fraud (fraud_d may be NULL: zeros; the CDC topic carries no label), row_out_d (optional)
 *     = the batch position of each kept record; *count_d = the number kept (device int64).
 *     The chain decode -> dedup -> compact -> fdx_stream_update -> forest stays on the device
 *     (one host read: count_d, to size the update). */
int fdx_cdc_decode(const uint8_t *bytes_d, const int64_t *offsets_d, const int64_t *us_d, int64_t n,
                   int64_t *unscaled_d, double *amount_d, int64_t *ts_ns_d, int32_t *bad_d, void *stream);
size_t fdx_dedup_latest_workspace_size(int64_t n);
int fdx_dedup_latest(const int64_t *key_d, const int64_t *kafka_ts_d, int64_t n, uint8_t *keep_d, int32_t *bad_d,
                     void *workspace_d, size_t workspace_bytes, void *stream);
size_t fdx_cdc_compact_workspace_size(int64_t n);
int fdx_cdc_compact(const uint8_t *keep_d, int64_t n, const int64_t *customer_d, const int64_t *terminal_d,
                    const int64_t *ts_ns_d, const double *amount_d, const uint8_t *fraud_d, int32_t *customer_out_d,
                    int32_t *terminal_out_d, int64_t *ts_out_d, double *amount_out_d, uint8_t *fraud_out_d,
                    int32_t *row_out_d, int64_t *count_d, void *workspace_d, size_t workspace_bytes, void *stream);
/* ---- config 5: streaming micro-batches with incremental window state ------------------
 * BASELINE.json config 5 ("micro-batches of 64k CDC transactions: incremental window-state
 * update + scoring").  The reference's streaming job (pyspark/scripts/fraud_detection.py:
 * 88-201) joins each micro-batch against snapshot tables; this engine instead keeps, per
 * customer and per terminal, the state the batch recurrences of fdx_customer_windows /
 * fdx_terminal_windows hold at a key's last row, so that feeding a history batch by batch
 * yields the same features, bit for bit, as one fdx_customer_windows / fdx_terminal_windows
 * call over the whole history (rows of one key in (ts, batch row) order).
 * fdx_stream_create allocates the state (customer_ring / terminal_ring rows of recent history
 * per key, powers of two: a key's rows of the longest window, resp. of delay + the longest
 * window, must fit, else fdx_stream_status reports a ring overflow).  window_ns: n_windows
 * customer windows = terminal windows (ns); delay_ns: the terminal label delay.
 * fdx_stream_update(rows ts/cust/amount/term/fraud, n <= max_batch): customer ids in
 *   [0, n_customers), terminal ids in [0, n_terminals); a key's rows must not go back in time
 *   across batches.  cust_d == NULL skips the customer half, term_d == NULL the terminal half.
 *   Writes X_d row r (leading dimension ld): [amount, weekend, night, (NB_w, AVG_w) x W] from
 *   the customer half and (NB_w, RISK_w) x W at column term_col0 (-1 = 3 + 2W) from the
 *   terminal half -- or, when term_rec_d != NULL, the terminal half as count records
 *   term_rec_d[r][W] (NB | FRAUD << 32, as fdx_terminal_windows_grouped) for the multi-GPU
 *   return exchange.  When cust_nb_d / cust_sum_d are given, the customer half goes there
 *   instead ([W][n] planes: NB int32 and the rolling SUM, bit-exact pandas roll_sum), and X_d
 *   may be NULL: the scoring layout of fdx_forest_prepare_grouped (cust_val_is_sum = 1,
 *   cust_perm_d = NULL, term_inv_d = NULL, cust_ts_d / cust_amount_d = the batch's ts / amount).
 *   Asynchronous; errors inside the kernels are collected as bits:
 * fdx_stream_status: synchronises, returns and clears them (1 customer ring overflow, 2
 *   terminal ring overflow, 4 key out of range, 8 rows out of time order). */
typedef struct fdx_stream_s *fdx_stream;
int fdx_stream_create(int64_t n_customers, int64_t n_terminals, int32_t customer_ring, int32_t terminal_ring,
                      int32_t n_windows, const int64_t *window_ns, int64_t delay_ns, int32_t flags_mode,
                      int64_t max_batch, fdx_stream *out, void *stream);
int fdx_stream_reset(fdx_stream s, void *stream);
int fdx_stream_memory(fdx_stream s, size_t *bytes);
int fdx_stream_update(fdx_stream s, const int64_t *ts_d, const int32_t *cust_d, const double *amount_d,
                      const int32_t *term_d, const uint8_t *fraud_d, int64_t n, double *X_d, int64_t ld,
                      int32_t term_col0, int32_t *cust_nb_d, double *cust_sum_d, int64_t *term_rec_d,
                      void *stream);
int fdx_stream_status(fdx_stream s, int32_t *flags_h, void *stream);
/* Non-blocking form: enqueues the copy of the status bits to flags_pinned_h (pinned host
 * memory, valid once the stream reaches this point); does not clear them. */
int fdx_stream_status_async(fdx_stream s, int32_t *flags_pinned_h, void *stream);
int fdx_stream_destroy(fdx_stream s);

/* f-4 delay-aware split and Card-Precision@k (shared_functions.py:133-188, :352-411).
 * fdx_train_test_split: train_d[i] = t_lo <= ts_d[i] < t_hi; test_d[i] = the row is on test
 *   day d = day_d[i] - (min train day + delta_train + delta_delay), 0 <= d < delta_test, and
 *   its customer (dense id < n_cust) has no fraud among the train rows nor on the days
 *   min train day + delta_train - 1 + [0, d] (the reference's growing known-defrauded set).
 *   workspace: n_cust * 5 + 64 bytes; *day_min_h = the min train day (host; one sync).
 * fdx_card_precision_top_k: for each day days_h[k] (ascending), customers max(prediction),
 *   max(TX_FRAUD) over the day's rows of customers not yet detected; the top_k customers by
 *   (prediction desc, customer asc) that are compromised are detected (carried over when
 *   remove_detected); nb_compromised_h[k] = compromised customers of the day, cp_h[k] =
 *   detected / top_k.  Predictions must be >= 0.  The reference sorts with pandas' default
 *   (unstable) quicksort: equal predictions straddling the k-th place may order differently.
 *   workspace: fdx_card_precision_workspace_size(n_cust); one host sync per day. */
int fdx_train_test_split(const int64_t *ts_d, const int32_t *day_d, const int32_t *cust_d, const uint8_t *fraud_d,
                         int64_t n, int32_t n_cust, int64_t t_lo, int64_t t_hi, int32_t delta_train,
                         int32_t delta_delay, int32_t delta_test, uint8_t *train_d, uint8_t *test_d,
                         void *workspace_d, size_t workspace_bytes, int32_t *day_min_h, void *stream);
size_t fdx_card_precision_workspace_size(int32_t n_cust);
int fdx_card_precision_top_k(const int32_t *day_d, const int32_t *cust_d, const double *pred_d,
                             const uint8_t *fraud_d, int64_t n, int32_t n_cust, const int32_t *days_h,
                             int32_t n_days, int32_t top_k, int32_t remove_detected, int32_t *nb_compromised_h,
                             double *cp_h, void *workspace_d, size_t workspace_bytes, void *stream);

/* f-3 synthetic transactions with the handbook generator's distributions, on the GPU
 * (fraud_detection_model/data_generator.ipynb :113-140 customers, :285-303 terminals, :420-437
 * terminals within radius, :786-834 daily Poisson transactions, :1339-1371 time sort, :1732-1782
 * add_frauds).  Profiles, the terminal sampler's band-sorted arrays and the compromised lists
 * come from the host (fdx.synth.generate_device); every random draw is Philox4x32-10 keyed by
 * `seed` with counter (customer + customer_offset, day, slot, purpose) -- the distributions of
 * the reference, not its Python RNG stream.  The descriptor describes customers
 * [customer_offset, customer_offset + n_customers) of a population (profile arrays indexed by
 * the local id): with the population's profiles and compromised lists, a range generates
 * exactly the population's rows of those customers, in the same order.  Two phases:
 * fdx_synth_plan (one host sync) returns the row count n_tx; fdx_synth_fill writes the
 * time-ordered rows (ts ns, customer + customer_offset, terminal, amount, fraud; scenario_d /
 * day_d optional).  comp_term_d: n_comp_term (terminal id, first day) int32 pairs sorted by
 * terminal (compromised for 28 days); comp_cust_d: (LOCAL customer id, first day) pairs sorted
 * by customer (14 days, 1/3 of the rows x5). */
typedef struct {
    int64_t n_customers, n_terminals;
    int32_t n_days;
    double radius;
    uint64_t seed;
    const double *cx_d, *cy_d, *mean_amount_d, *mean_nb_d; /* [n_customers] */
    const double *tx_sorted_d, *ty_sorted_d;               /* [n_terminals], sorted by (band of r, x) */
    const int32_t *t_order_d;                              /* sorted position -> terminal id */
    const int32_t *range_lo_d, *range_hi_d;                /* [n_customers][3] runs of the 3 bands */
    const int32_t *comp_term_d;
    int32_t n_comp_term;
    const int32_t *comp_cust_d;
    int32_t n_comp_cust;
    int64_t start_ns;
    int32_t customer_offset;
} fdx_synth_desc;
size_t fdx_synth_workspace_size(const fdx_synth_desc *desc, int64_t n_tx);
int fdx_synth_plan(const fdx_synth_desc *desc, void *workspace_d, size_t workspace_bytes, int64_t *n_tx_h,
                   void *stream);
int fdx_synth_fill(const fdx_synth_desc *desc, int64_t n_tx, void *workspace_d, size_t workspace_bytes, int64_t *ts_d,
                   int32_t *customer_d, int32_t *terminal_d, double *amount_d, uint8_t *fraud_d, uint8_t *scenario_d,
                   int32_t *day_d, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* FDX_H_ */
