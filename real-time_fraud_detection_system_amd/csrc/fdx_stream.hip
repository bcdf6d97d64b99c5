// fdx_stream.hip -- config 5 (BASELINE.json): streaming micro-batches of CDC transactions with
// INCREMENTAL window state, so that a batch costs O(batch) instead of a re-scan of history.
//
// The state carried between batches is exactly what the batch kernels' recurrences hold at
// the last row of a key, so a stream of batches gives bit-identical features to one batch
// call over the concatenated history (tests/test_gpu_stream.py):
//   customer (feature_transformation.ipynb:601-628): per window the pandas roll_sum state
//     (sum, Kahan add/remove compensations, nobs, n-same run, prev -- aggregations.pyx
//     add_sum/remove_sum/calc_sum, see RollSum in fdx_windows.hip) and the window's tail
//     (pandas' variable-window start), plus a ring of the customer's recent (ts, amount) rows
//     from which the tails remove;
//   terminal (:1495-1522): per window boundary (delay, delay + w) the count of the terminal's
//     rows with ts <= t - boundary and their fraud count, plus a ring of recent (ts, fraud).
//
// HBM layout (one record per key, 8-byte words, so a key's state is 2-3 cache lines):
//   customer record  [n, last_ts, (tail, sum, c_add, c_rem, prev, nobs | nsame << 32) x W]
//   customer ring    C entries of {ts, amount} per customer (C a power of two)
//   terminal record  [n, last_ts, (p_k, F_k) x (W + 1)]     k = 0: delay, k = w+1: delay + w
//   terminal ring    T entries of (ts << 1 | fraud) per terminal
// Row r of a key's history sits in ring slot r & (C-1); a ring slot is overwritten only once
// every window has passed the row in it (else status bit 1/2: ring too small).
//
// One update = two launches over the batch:
//   k_stream_link    per row: push the row on its customer's and terminal's chain (one
//                    atomic exchange each on a head array), write amount + flags;
//   k_stream_process per row: the thread whose row ended up at the head of a chain owns the
//                    key: it walks the chain in (ts, row) order, advances the key's state
//                    row by row, writes that row's features, stores the state back and clears
//                    the head.  Rows of one key in one batch are few (64k rows over 1M
//                    customers: mostly one), so the chain selection (quadratic in the rows of
//                    one key in one batch) is short; big bootstrap batches pay it per key.
// Latency-bound (a handful of dependent HBM reads per key), no MFMA, no LDS.
#include <climits>

#include "fdx_internal.h"

namespace fdx {
namespace {

constexpr int kMaxW = FDX_MAX_WINDOWS;
constexpr int64_t kNsPerDay = 86400LL * 1000000000LL;
constexpr int64_t kNsPerHour = 3600LL * 1000000000LL;

enum : int32_t {
    kStCustRing = 1,    // a customer ring slot still inside a window was overwritten
    kStTermRing = 2,    // same for a terminal ring
    kStKey = 4,         // customer / terminal id outside [0, capacity)
    kStOrder = 8,       // a key's rows went back in time across batches
};

struct StreamWin {
    int64_t win[kMaxW];         // customer windows (ns)
    int64_t tb[kMaxW + 1];      // terminal boundaries: delay, delay + win[w] (ns)
};

struct alignas(16) CEnt {
    int64_t ts;
    double amt;
};

// pandas roll_sum (aggregations.pyx add_sum / remove_sum / calc_sum), same as fdx_windows.hip
struct Roll {
    double sum, c_add, c_rem, prev;
    int32_t nobs, nsame;
    __device__ __forceinline__ void reset(double first) {
        sum = 0.0; c_add = 0.0; c_rem = 0.0; prev = first; nobs = 0; nsame = 0;
    }
    __device__ __forceinline__ void add(double v) {
        if (v == v) {
            nobs += 1;
            double y = v - c_add, t = sum + y;
            c_add = (t - sum) - y;
            sum = t;
            nsame = (v == prev) ? nsame + 1 : 1;
            prev = v;
        }
    }
    __device__ __forceinline__ void remove(double v) {
        if (v == v) {
            nobs -= 1;
            double y = -v - c_rem, t = sum + y;
            c_rem = (t - sum) - y;
            sum = t;
        }
    }
    __device__ __forceinline__ double value() const {
        if (nobs >= 1) return (nsame >= nobs) ? prev * (double)nobs : sum;
        return __builtin_nan("");
    }
};

__device__ __forceinline__ void time_flags(int64_t t, int32_t mode, double &we, double &ni) {
    int64_t day = t / kNsPerDay;
    if (t % kNsPerDay != 0 && t < 0) --day;
    const int64_t hour = (t - day * kNsPerDay) / kNsPerHour;
    int64_t wd = (day + 3) % 7;  // Monday = 0 (1970-01-01 was a Thursday)
    if (wd < 0) wd += 7;
    if (mode == FDX_FLAGS_NOTEBOOK) {
        we = wd >= 5; ni = hour <= 6;
    } else {
        const int64_t dow = ((wd + 1) % 7) + 1;  // Spark dayofweek: Sunday = 1 .. Saturday = 7
        we = dow >= 5; ni = hour >= 20;
    }
}

__global__ void __launch_bounds__(256) k_stream_link(
    const int64_t *__restrict__ ts, const int32_t *__restrict__ cust, const double *__restrict__ amount,
    const int32_t *__restrict__ term, int64_t n, int64_t n_cust, int64_t n_term, int32_t *__restrict__ chead,
    int32_t *__restrict__ cnext, int32_t *__restrict__ thead, int32_t *__restrict__ tnext, int32_t mode,
    double *__restrict__ X, int64_t ld, int32_t *__restrict__ status) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (cust) {
            const int32_t c = cust[i];
            if (c < 0 || c >= n_cust) {
                atomicOr(status, kStKey);
            } else {
                cnext[i] = atomicExch(&chead[c], (int32_t)i);
            }
            if (X) {
                double we, ni;
                time_flags(ts[i], mode, we, ni);
                double *x = X + i * ld;
                x[0] = amount[i]; x[1] = we; x[2] = ni;
            }
        }
        if (term) {
            const int32_t t = term[i];
            if (t < 0 || t >= n_term) {
                atomicOr(status, kStKey);
            } else {
                tnext[i] = atomicExch(&thead[t], (int32_t)i);
            }
        }
    }
}

// Visit the rows of the chain at `head` in (ts, row) order.
template <class F>
__device__ __forceinline__ void chain_in_order(int32_t head, const int32_t *__restrict__ next,
                                               const int64_t *__restrict__ ts, F &&visit) {
    int cnt = 0;
    int64_t bt = INT64_MAX;
    int32_t br = INT32_MAX;
    for (int32_t j = head; j >= 0; j = next[j]) {
        ++cnt;
        const int64_t t = ts[j];
        if (t < bt || (t == bt && j < br)) { bt = t; br = j; }
    }
    visit(br, bt);
    for (int k = 1; k < cnt; ++k) {
        int64_t nt = INT64_MAX;
        int32_t nr = INT32_MAX;
        for (int32_t j = head; j >= 0; j = next[j]) {
            const int64_t t = ts[j];
            const bool after = t > bt || (t == bt && j > br);
            const bool before = t < nt || (t == nt && j < nr);
            if (after && before) { nt = t; nr = j; }
        }
        bt = nt; br = nr;
        visit(br, bt);
    }
}

template <int W>
__device__ void customer_key(int32_t c, int32_t head, const int32_t *__restrict__ cnext,
                             const int64_t *__restrict__ ts, const double *__restrict__ amount,
                             const StreamWin &sw, int64_t *__restrict__ cstate, CEnt *__restrict__ cring,
                             int32_t C, double *__restrict__ X, int64_t ld, int32_t *__restrict__ cnb_out,
                             double *__restrict__ csum_out, int64_t n_rows, int32_t *__restrict__ status) {
    int64_t *rec = cstate + (int64_t)c * (2 + 6 * W);
    CEnt *ring = cring + (int64_t)c * C;
    const int64_t mask = C - 1;
    int64_t n = rec[0], last = rec[1];
    int64_t tail[W];
    Roll s[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const int64_t *r = rec + 2 + 6 * w;
        tail[w] = r[0];
        s[w].sum = __longlong_as_double(r[1]);
        s[w].c_add = __longlong_as_double(r[2]);
        s[w].c_rem = __longlong_as_double(r[3]);
        s[w].prev = __longlong_as_double(r[4]);
        s[w].nobs = (int32_t)(uint32_t)((uint64_t)r[5] & 0xFFFFFFFFu);
        s[w].nsame = (int32_t)(uint32_t)((uint64_t)r[5] >> 32);
    }
    int32_t bad = 0;
    chain_in_order(head, cnext, ts, [&](int32_t row, int64_t t) {
        const double v = amount[row];
        if (n > 0 && t < last) bad |= kStOrder;
        // the first ring entry each window's tail looks at, loaded together
        CEnt e[W];
#pragma unroll
        for (int w = 0; w < W; ++w) e[w] = tail[w] < n ? ring[tail[w] & mask] : CEnt{INT64_MAX, 0.0};
        int64_t tmin = n;
        double *x = cnb_out ? nullptr : X + (int64_t)row * ld + 3;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int64_t bound = t - sw.win[w];
            int64_t nt = tail[w];
            // pandas removes rows start[i-1] .. start[i]-1 (Kahan, c_rem) then adds row i;
            // when the window restarts (start[i] >= end[i-1]) it re-initialises instead, which
            // discards whatever the removals did -- so removing while advancing is exact.
            while (e[w].ts <= bound) {
                s[w].remove(e[w].amt);
                ++nt;
                e[w] = nt < n ? ring[nt & mask] : CEnt{INT64_MAX, 0.0};
            }
            if (nt >= n) s[w].reset(v);
            s[w].add(v);
            tail[w] = nt;
            tmin = nt < tmin ? nt : tmin;
            if (cnb_out) {  // scoring planes: NB and the rolling SUM (the consumer divides)
                cnb_out[(int64_t)w * n_rows + row] = s[w].nobs;
                csum_out[(int64_t)w * n_rows + row] = s[w].value();
            } else {
                x[2 * w] = (double)s[w].nobs;
                x[2 * w + 1] = s[w].value() / (double)s[w].nobs;
            }
        }
        if (n >= C && n - C >= tmin) bad |= kStCustRing;
        ring[n & mask] = CEnt{t, v};
        ++n;
        last = t;
    });
    rec[0] = n;
    rec[1] = last;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        int64_t *r = rec + 2 + 6 * w;
        r[0] = tail[w];
        r[1] = __double_as_longlong(s[w].sum);
        r[2] = __double_as_longlong(s[w].c_add);
        r[3] = __double_as_longlong(s[w].c_rem);
        r[4] = __double_as_longlong(s[w].prev);
        r[5] = (int64_t)(((uint64_t)(uint32_t)s[w].nsame << 32) | (uint32_t)s[w].nobs);
    }
    if (bad) atomicOr(status, bad);
}

template <int W>
__device__ void terminal_key(int32_t tk, int32_t head, const int32_t *__restrict__ tnext,
                             const int64_t *__restrict__ ts, const uint8_t *__restrict__ fraud,
                             const StreamWin &sw, int64_t *__restrict__ tstate, int64_t *__restrict__ tring,
                             int32_t T, double *__restrict__ X, int64_t ld, int32_t tcol0, int64_t *__restrict__ rec_out,
                             int32_t *__restrict__ status) {
    constexpr int K = W + 1;
    int64_t *rec = tstate + (int64_t)tk * (2 + 2 * K);
    int64_t *ring = tring + (int64_t)tk * T;
    const int64_t mask = T - 1;
    int64_t n = rec[0], last = rec[1];
    int64_t p[K], F[K];
#pragma unroll
    for (int k = 0; k < K; ++k) { p[k] = rec[2 + 2 * k]; F[k] = rec[3 + 2 * k]; }
    int32_t bad = 0;
    chain_in_order(head, tnext, ts, [&](int32_t row, int64_t t) {
        if (n > 0 && t < last) bad |= kStOrder;
        int64_t e[K];
#pragma unroll
        for (int k = 0; k < K; ++k) e[k] = p[k] < n ? ring[p[k] & mask] : INT64_MAX;
        int64_t pmin = n;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t bound = t - sw.tb[k];
            while ((e[k] >> 1) <= bound) {   // rows with ts <= t - boundary
                F[k] += e[k] & 1;
                ++p[k];
                e[k] = p[k] < n ? ring[p[k] & mask] : INT64_MAX;
            }
            pmin = p[k] < pmin ? p[k] : pmin;
        }
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int32_t nb = (int32_t)(p[0] - p[w + 1]), fr = (int32_t)(F[0] - F[w + 1]);
            if (rec_out) {
                rec_out[(int64_t)row * W + w] = term_word(nb, fr);
            } else {
                double *x = X + (int64_t)row * ld + tcol0 + 2 * w;
                x[0] = (double)nb;
                x[1] = nb > 0 ? (double)fr / (double)nb : 0.0;  // fillna(0) of 0/0
            }
        }
        if (n >= T && n - T >= pmin) bad |= kStTermRing;
        ring[n & mask] = (int64_t)(((uint64_t)t << 1) | (fraud[row] ? 1u : 0u));
        ++n;
        last = t;
    });
    rec[0] = n;
    rec[1] = last;
#pragma unroll
    for (int k = 0; k < K; ++k) { rec[2 + 2 * k] = p[k]; rec[3 + 2 * k] = F[k]; }
    if (bad) atomicOr(status, bad);
}

template <int W>
__global__ void __launch_bounds__(256) k_stream_process(
    const int64_t *__restrict__ ts, const int32_t *__restrict__ cust, const double *__restrict__ amount,
    const int32_t *__restrict__ term, const uint8_t *__restrict__ fraud, int64_t n, int64_t n_cust, int64_t n_term,
    StreamWin sw, int32_t *__restrict__ chead, const int32_t *__restrict__ cnext, int32_t *__restrict__ thead,
    const int32_t *__restrict__ tnext, int64_t *__restrict__ cstate, CEnt *__restrict__ cring, int32_t C,
    int64_t *__restrict__ tstate, int64_t *__restrict__ tring, int32_t T, double *__restrict__ X, int64_t ld,
    int32_t tcol0, int32_t *__restrict__ cnb_out, double *__restrict__ csum_out, int64_t *__restrict__ rec_out,
    int32_t *__restrict__ status) {
    // grid.y = 2 when both halves run: the customer and terminal keys of a row are walked by
    // different threads, so their dependent-load chains overlap instead of adding up
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool do_c = cust && (gridDim.y == 1 || blockIdx.y == 0);
    const bool do_t = term && (gridDim.y == 1 || blockIdx.y == 1);
    if (do_c) {
        const int32_t c = cust[i];
        if (c >= 0 && c < n_cust && chead[c] == (int32_t)i) {
            customer_key<W>(c, (int32_t)i, cnext, ts, amount, sw, cstate, cring, C, X, ld, cnb_out, csum_out, n,
                            status);
            chead[c] = -1;
        }
    }
    if (do_t) {
        const int32_t t = term[i];
        if (t >= 0 && t < n_term && thead[t] == (int32_t)i) {
            terminal_key<W>(t, (int32_t)i, tnext, ts, fraud, sw, tstate, tring, T, X, ld, tcol0, rec_out, status);
            thead[t] = -1;
        }
    }
}

bool pow2(int64_t x) { return x > 0 && (x & (x - 1)) == 0; }

}  // namespace
}  // namespace fdx

using namespace fdx;

struct fdx_stream_s {
    int64_t n_cust = 0, n_term = 0, max_batch = 0;
    int32_t C = 0, T = 0, W = 0, mode = 0;
    StreamWin sw{};
    CEnt *cring_d = nullptr;
    int64_t *cstate_d = nullptr, *tring_d = nullptr, *tstate_d = nullptr;
    int32_t *chead_d = nullptr, *thead_d = nullptr, *cnext_d = nullptr, *tnext_d = nullptr, *status_d = nullptr;
    size_t bytes = 0;
};

namespace {
size_t cust_rec_bytes(int W) { return (size_t)(2 + 6 * W) * 8; }
size_t term_rec_bytes(int W) { return (size_t)(2 + 2 * (W + 1)) * 8; }
}  // namespace

extern "C" int fdx_stream_destroy(fdx_stream s) {
    if (!s) return FDX_OK;
    (void)hipFree(s->cring_d);
    (void)hipFree(s->cstate_d);
    (void)hipFree(s->tring_d);
    (void)hipFree(s->tstate_d);
    (void)hipFree(s->chead_d);
    (void)hipFree(s->thead_d);
    (void)hipFree(s->cnext_d);
    (void)hipFree(s->tnext_d);
    (void)hipFree(s->status_d);
    delete s;
    return FDX_OK;
}

extern "C" int fdx_stream_reset(fdx_stream s, void *stream) {
    FDX_REQUIRE(s, "null stream state");
    hipStream_t st = as_stream(stream);
    if (s->n_cust) {
        FDX_HIP(hipMemsetAsync(s->cstate_d, 0, (size_t)s->n_cust * cust_rec_bytes(s->W), st));
        FDX_HIP(hipMemsetAsync(s->chead_d, 0xFF, (size_t)s->n_cust * 4, st));
    }
    if (s->n_term) {
        FDX_HIP(hipMemsetAsync(s->tstate_d, 0, (size_t)s->n_term * term_rec_bytes(s->W), st));
        FDX_HIP(hipMemsetAsync(s->thead_d, 0xFF, (size_t)s->n_term * 4, st));
    }
    FDX_HIP(hipMemsetAsync(s->status_d, 0, 4, st));
    return FDX_OK;
}

extern "C" int fdx_stream_create(int64_t n_customers, int64_t n_terminals, int32_t customer_ring,
                                 int32_t terminal_ring, int32_t n_windows, const int64_t *window_ns,
                                 int64_t delay_ns, int32_t flags_mode, int64_t max_batch, fdx_stream *out,
                                 void *stream) {
    FDX_REQUIRE(out, "null pointer");
    *out = nullptr;
    FDX_REQUIRE(n_customers >= 0 && n_customers <= INT32_MAX && n_terminals >= 0 && n_terminals <= INT32_MAX,
                "key capacity out of range");
    FDX_REQUIRE(n_windows >= 1 && n_windows <= kMaxW && window_ns, "n_windows must be in [1, %d]", kMaxW);
    FDX_REQUIRE(!n_customers || pow2(customer_ring), "customer_ring must be a power of two");
    FDX_REQUIRE(!n_terminals || pow2(terminal_ring), "terminal_ring must be a power of two");
    FDX_REQUIRE(max_batch >= 1 && max_batch <= INT32_MAX, "max_batch out of range");
    FDX_REQUIRE(delay_ns >= 0, "negative delay");
    FDX_REQUIRE(flags_mode == FDX_FLAGS_NOTEBOOK || flags_mode == FDX_FLAGS_SPARK, "bad flags mode");
    fdx_stream s = new fdx_stream_s;
    s->n_cust = n_customers; s->n_term = n_terminals; s->max_batch = max_batch;
    s->C = n_customers ? customer_ring : 0; s->T = n_terminals ? terminal_ring : 0;
    s->W = n_windows; s->mode = flags_mode;
    s->sw.tb[0] = delay_ns;
    for (int w = 0; w < n_windows; ++w) {
        if (window_ns[w] <= 0) {
            delete s;
            FDX_REQUIRE(false, "window lengths must be positive");
        }
        s->sw.win[w] = window_ns[w];
        s->sw.tb[w + 1] = delay_ns + window_ns[w];
    }
    auto alloc = [&](void **p, size_t b) -> hipError_t {
        s->bytes += b;
        return b ? hipMalloc(p, b) : hipSuccess;
    };
    hipError_t e = hipSuccess;
    const size_t nc = (size_t)n_customers, nt = (size_t)n_terminals;
    if ((e = alloc((void **)&s->cring_d, nc * s->C * sizeof(CEnt))) ||
        (e = alloc((void **)&s->cstate_d, nc * cust_rec_bytes(n_windows))) ||
        (e = alloc((void **)&s->chead_d, nc * 4)) ||
        (e = alloc((void **)&s->tring_d, nt * s->T * 8)) ||
        (e = alloc((void **)&s->tstate_d, nt * term_rec_bytes(n_windows))) ||
        (e = alloc((void **)&s->thead_d, nt * 4)) ||
        (e = alloc((void **)&s->cnext_d, (size_t)max_batch * 4)) ||
        (e = alloc((void **)&s->tnext_d, (size_t)max_batch * 4)) || (e = alloc((void **)&s->status_d, 4))) {
        set_error("hipMalloc of the stream state (%zu bytes so far) failed: %s", s->bytes, hipGetErrorString(e));
        fdx_stream_destroy(s);
        return FDX_E_HIP;
    }
    const int rc = fdx_stream_reset(s, stream);
    if (rc) {
        fdx_stream_destroy(s);
        return rc;
    }
    *out = s;
    return FDX_OK;
}

extern "C" int fdx_stream_memory(fdx_stream s, size_t *bytes) {
    FDX_REQUIRE(s && bytes, "null pointer");
    *bytes = s->bytes;
    return FDX_OK;
}

#define FDX_STREAM_PROCESS(WW)                                                                                   \
    case WW:                                                                                                     \
        hipLaunchKernelGGL(k_stream_process<WW>, grid, dim3(256), 0, st, ts_d, cust_d, amount_d, term_d,         \
                           fraud_d, n, s->n_cust, s->n_term, s->sw, s->chead_d, s->cnext_d, s->thead_d,          \
                           s->tnext_d, s->cstate_d, s->cring_d, s->C, s->tstate_d, s->tring_d, s->T, X_d, ld,     \
                           tcol, cust_nb_d, cust_sum_d, term_rec_d, s->status_d);                                \
        break;

extern "C" int fdx_stream_update(fdx_stream s, const int64_t *ts_d, const int32_t *cust_d, const double *amount_d,
                                 const int32_t *term_d, const uint8_t *fraud_d, int64_t n, double *X_d, int64_t ld,
                                 int32_t term_col0, int32_t *cust_nb_d, double *cust_sum_d, int64_t *term_rec_d,
                                 void *stream) {
    FDX_REQUIRE(s, "null stream state");
    FDX_REQUIRE(n >= 0 && n <= s->max_batch, "batch of %lld rows exceeds max_batch %lld", (long long)n,
                (long long)s->max_batch);
    if (n == 0) return FDX_OK;
    FDX_REQUIRE(ts_d, "null ts");
    FDX_REQUIRE(!cust_d || (amount_d && s->n_cust), "customer half needs amounts and customer state");
    FDX_REQUIRE(!term_d || (fraud_d && s->n_term), "terminal half needs fraud labels and terminal state");
    const int W = s->W;
    const int32_t tcol = term_col0 < 0 ? 3 + 2 * W : term_col0;
    FDX_REQUIRE(!cust_nb_d == !cust_sum_d, "cust_nb_d and cust_sum_d go together");
    FDX_REQUIRE(!cust_d || cust_nb_d || (X_d && ld >= 3 + 2 * W), "X needs ld >= 3 + 2 * n_windows");
    FDX_REQUIRE(!X_d || ld >= 3, "X needs ld >= 3");
    FDX_REQUIRE(!term_d || term_rec_d || (X_d && ld >= tcol + 2 * W), "terminal columns do not fit ld");
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_stream_link, dim3(stream_grid(n, 256)), dim3(256), 0, st, ts_d, cust_d, amount_d, term_d, n,
                       s->n_cust, s->n_term, s->chead_d, s->cnext_d, s->thead_d, s->tnext_d, s->mode, X_d, ld,
                       s->status_d);
    FDX_LAUNCHED("k_stream_link");
    const dim3 grid((unsigned)ceil_div(n, 256), cust_d && term_d ? 2u : 1u);
    switch (W) {
        FDX_STREAM_PROCESS(1)
        FDX_STREAM_PROCESS(2)
        FDX_STREAM_PROCESS(3)
        FDX_STREAM_PROCESS(4)
        FDX_STREAM_PROCESS(5)
        FDX_STREAM_PROCESS(6)
        FDX_STREAM_PROCESS(7)
        FDX_STREAM_PROCESS(8)
    }
    FDX_LAUNCHED("k_stream_process");
    return FDX_OK;
}

extern "C" int fdx_stream_status(fdx_stream s, int32_t *flags_h, void *stream) {
    FDX_REQUIRE(s && flags_h, "null pointer");
    hipStream_t st = as_stream(stream);
    FDX_HIP(hipMemcpyAsync(flags_h, s->status_d, 4, hipMemcpyDeviceToHost, st));
    FDX_HIP(hipStreamSynchronize(st));
    if (*flags_h) FDX_HIP(hipMemsetAsync(s->status_d, 0, 4, st));
    return FDX_OK;
}

extern "C" int fdx_stream_status_async(fdx_stream s, int32_t *flags_pinned_h, void *stream) {
    FDX_REQUIRE(s && flags_pinned_h, "null pointer");
    FDX_HIP(hipMemcpyAsync(flags_pinned_h, s->status_d, 4, hipMemcpyDeviceToHost, as_stream(stream)));
    return FDX_OK;
}

