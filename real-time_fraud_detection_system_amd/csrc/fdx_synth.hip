// fdx_synth.hip -- §8(f) row 3: synthetic transactions with the distributions of the
// reference's handbook generator, generated on the GPU (bench / large-config input).
//
// Reference (fraud_detection_model/data_generator.ipynb): customers on a 100x100 grid with
// mean_amount ~ U(5,100), std = mean/2, mean_nb_tx_per_day ~ U(0,4) (:113-140); terminals
// ~ U(0,100)^2 (:285-303); a customer's terminals are those at distance < r (:420-437);
// per customer and day nb_tx ~ Poisson(mean_nb), each tx at int(N(43200, 20000)) seconds,
// kept when 0 < t < 86400, amount N(mean, std) (a negative draw redrawn U(0, 2 mean)),
// rounded to cents, terminal uniform among the customer's (:786-834); global time sort
// (:1339-1371); add_frauds (:1732-1782): scenario 1 amount > 220, scenario 2 two terminals
// compromised per day for 28 days, scenario 3 three customers per day for 14 days with a
// third of their transactions x5 and fraudulent.
//
// Same distributions, not the reference's RNG stream (pure Python, ~100 s per 1.75M rows):
// every draw comes from Philox4x32-10 keyed by the seed with counter (GLOBAL customer id =
// local id + customer_offset, day, transaction slot, purpose), so the counting pass and the
// filling pass see the same draws, the output does not depend on the launch shape, and a
// rank generating customers [offset, offset + n) of a population gets exactly the rows the
// whole population's generation holds for them, in the same order (the multi-GPU bench's
// union is the same data at every N).  Parity of the statistics with the
// reference generator at config 1: tests/test_gpu_synth.py vs tests/golden/config1_stats.json.
#include <algorithm>
#include <cmath>

#include "fdx_internal.h"

namespace fdx {
namespace {

// ------------------------------------------------------------------------ Philox4x32-10
struct U4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// uniform double in (0, 1] from 53 random bits (never 0: safe for log)
__device__ __forceinline__ double unit(uint32_t a, uint32_t b) {
    const uint64_t m = ((uint64_t)a << 21) ^ (uint64_t)(b >> 11);
    return ((double)(m & ((1ull << 53) - 1)) + 1.0) * (1.0 / 9007199254740992.0);
}

struct Rng {
    uint32_t k0, k1;
    __device__ __forceinline__ U4 at(uint32_t c, uint32_t d, uint32_t slot, uint32_t purpose) const {
        return philox(U4{c, d, slot, purpose}, k0, k1);
    }
};

// standard normal (Box-Muller, cosine branch) from one Philox block
__device__ __forceinline__ double normal01(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const double u0 = unit(a, b), u1 = unit(c, d);
    return sqrt(-2.0 * log(u0)) * cos(6.283185307179586 * u1);
}

// Poisson(lambda) by inversion (lambda <= 4 here; capped at 64 for safety)
__device__ __forceinline__ int poisson(double lam, double u) {
    double p = exp(-lam), F = p;
    int k = 0;
    while (u > F && k < 64) {
        ++k;
        p *= lam / (double)k;
        F += p;
    }
    return k;
}

constexpr uint32_t kPurposeCount = 0, kPurposeTx = 1, kPurposeNeg = 2, kPurposeAmt = 3, kPurposeTerm = 8,
                   kPurposeFraud = 1 << 16;

// the time of slot k of (c, d): int(N(43200, 20000)) (Python int() truncates toward zero)
__device__ __forceinline__ int32_t tx_time(const Rng &g, uint32_t c, uint32_t d, uint32_t k) {
    const U4 r = g.at(c, d, k + 1, kPurposeTx);
    return (int32_t)(43200.0 + 20000.0 * normal01(r.x, r.y, r.z, r.w));
}

__device__ __forceinline__ int day_count(const Rng &g, uint32_t c, uint32_t d, double lam) {
    const U4 r = g.at(c, d, 0, kPurposeCount);
    return poisson(lam, unit(r.x, r.y));
}

__device__ __forceinline__ bool in_disk(double x, double y, double px, double py, double rad) {
    const double dx = x - px, dy = y - py;
    return sqrt(dx * dx + dy * dy) < rad;  // get_list_terminals_within_radius: dist < r
}

__global__ void __launch_bounds__(256) k_synth_has_terminal(fdx_synth_desc s, uint8_t *__restrict__ has) {
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < s.n_customers;
         c += (int64_t)gridDim.x * blockDim.x) {
        const double px = s.cx_d[c], py = s.cy_d[c];
        bool found = false;
        for (int b = 0; b < 3 && !found; ++b)
            for (int32_t i = s.range_lo_d[3 * c + b]; i < s.range_hi_d[3 * c + b]; ++i)
                if (in_disk(s.tx_sorted_d[i], s.ty_sorted_d[i], px, py, s.radius)) {
                    found = true;
                    break;
                }
        has[c] = found;
    }
}

// kept[c * D + d] = transactions of customer c on day d that survive the time filter
__global__ void __launch_bounds__(256) k_synth_count(fdx_synth_desc s, const uint8_t *__restrict__ has,
                                                     uint32_t *__restrict__ kept) {
    const Rng g{(uint32_t)s.seed, (uint32_t)(s.seed >> 32)};
    const int64_t total = s.n_customers * (int64_t)s.n_days;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t c = (uint32_t)(i / s.n_days), d = (uint32_t)(i - (int64_t)c * s.n_days);
        const uint32_t cg = c + (uint32_t)s.customer_offset;  // the draws' counter: the global id
        uint32_t k_kept = 0;
        if (has[c]) {
            const int n = day_count(g, cg, d, s.mean_nb_d[c]);
            for (int k = 0; k < n; ++k) {
                const int32_t t = tx_time(g, cg, d, (uint32_t)k);
                k_kept += (t > 0 && t < 86400) ? 1u : 0u;
            }
        }
        kept[i] = k_kept;
    }
}

// first index of pairs[2*j] (sorted by key) >= key
__device__ __forceinline__ int32_t pair_lower(const int32_t *pairs, int32_t n, int32_t key) {
    int32_t lo = 0, hi = n;
    while (lo < hi) {
        const int32_t m = (lo + hi) >> 1;
        if (pairs[2 * m] < key) lo = m + 1; else hi = m;
    }
    return lo;
}

__global__ void __launch_bounds__(256) k_synth_fill(fdx_synth_desc s, const uint8_t *__restrict__ has,
                                                    const uint32_t *__restrict__ offsets, uint32_t *__restrict__ secs,
                                                    int32_t *__restrict__ cust, int32_t *__restrict__ term,
                                                    double *__restrict__ amount, uint8_t *__restrict__ scen) {
    const Rng g{(uint32_t)s.seed, (uint32_t)(s.seed >> 32)};
    const int64_t total = s.n_customers * (int64_t)s.n_days;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t c = (uint32_t)(i / s.n_days), d = (uint32_t)(i - (int64_t)c * s.n_days);
        if (!has[c]) continue;
        const uint32_t cg = c + (uint32_t)s.customer_offset;  // the draws' counter: the global id
        const double mean = s.mean_amount_d[c], px = s.cx_d[c], py = s.cy_d[c];
        const int n = day_count(g, cg, d, s.mean_nb_d[c]);
        int64_t o = offsets[i];
        for (int k = 0; k < n; ++k) {
            const int32_t t = tx_time(g, cg, d, (uint32_t)k);
            if (!(t > 0 && t < 86400)) continue;
            // amount: N(mean, mean / 2); negative -> U(0, 2 mean); np.round(a, 2) = rint(a * 100) / 100
            const U4 r2 = g.at(cg, d, (uint32_t)k + 1, kPurposeAmt);
            double a = mean + 0.5 * mean * normal01(r2.x, r2.y, r2.z, r2.w);
            if (a < 0.0) {
                const U4 rn = g.at(cg, d, (uint32_t)k + 1, kPurposeNeg);
                a = unit(rn.x, rn.y) * (mean * 2.0);
            }
            a = rint(a * 100.0) / 100.0;
            // terminal: uniform over the three band runs, rejected outside the disk
            int32_t sel = -1;
            const int32_t *lo = s.range_lo_d + 3 * (int64_t)c, *hi = s.range_hi_d + 3 * (int64_t)c;
            const int64_t s0 = hi[0] - lo[0], s1 = s0 + (hi[1] - lo[1]), s2 = s1 + (hi[2] - lo[2]);
            for (uint32_t att = 0; att < 64 && sel < 0; ++att) {
                const U4 rt = g.at(cg, d, (uint32_t)k + 1, kPurposeTerm + att);
                const int64_t u = (int64_t)(unit(rt.x, rt.y) * (double)s2);  // in [0, s2] (unit may be 1)
                const int64_t uu = u >= s2 ? s2 - 1 : u;
                const int b = uu >= s0 ? (uu >= s1 ? 2 : 1) : 0;
                const int64_t cand = lo[b] + (uu - (b == 0 ? 0 : (b == 1 ? s0 : s1)));
                if (in_disk(s.tx_sorted_d[cand], s.ty_sorted_d[cand], px, py, s.radius)) sel = (int32_t)cand;
            }
            if (sel < 0) {  // exact fallback: the j-th in-disk terminal of the runs
                int64_t m = 0;
                for (int b = 0; b < 3; ++b)
                    for (int32_t j = lo[b]; j < hi[b]; ++j) m += in_disk(s.tx_sorted_d[j], s.ty_sorted_d[j], px, py, s.radius);
                const U4 rt = g.at(cg, d, (uint32_t)k + 1, kPurposeTerm + 64);
                int64_t want = (int64_t)(unit(rt.x, rt.y) * (double)m);
                if (want >= m) want = m - 1;
                for (int b = 0; b < 3 && sel < 0; ++b)
                    for (int32_t j = lo[b]; j < hi[b]; ++j)
                        if (in_disk(s.tx_sorted_d[j], s.ty_sorted_d[j], px, py, s.radius) && want-- == 0) {
                            sel = j;
                            break;
                        }
            }
            const int32_t tid = s.t_order_d[sel];
            // add_frauds: scenario 1 on the drawn amount, then 2 (terminal), then 3 (customer)
            uint8_t sc = a > 220.0 ? 1 : 0;
            for (int32_t j = pair_lower(s.comp_term_d, s.n_comp_term, tid); j < s.n_comp_term && s.comp_term_d[2 * j] == tid;
                 ++j) {
                const int32_t d0 = s.comp_term_d[2 * j + 1];
                if ((int32_t)d >= d0 && (int32_t)d < d0 + 28) sc = 2;
            }
            for (int32_t j = pair_lower(s.comp_cust_d, s.n_comp_cust, (int32_t)c); j < s.n_comp_cust &&
                                                                                  s.comp_cust_d[2 * j] == (int32_t)c;
                 ++j) {
                const int32_t d0 = s.comp_cust_d[2 * j + 1];
                if ((int32_t)d >= d0 && (int32_t)d < d0 + 14) {
                    const U4 rf = g.at(cg, d, (uint32_t)k + 1, kPurposeFraud + (uint32_t)d0);
                    if (unit(rf.x, rf.y) <= 1.0 / 3.0) {
                        a = a * 5.0;
                        sc = 3;
                    }
                }
            }
            secs[o] = (uint32_t)(d * 86400u + (uint32_t)t);
            cust[o] = (int32_t)c;
            term[o] = tid;
            amount[o] = a;
            scen[o] = sc;
            ++o;
        }
    }
}

// time order: out[j] = in[perm[j]], ts = start + secs * 1e9 ns, customer id + offset
__global__ void __launch_bounds__(256) k_synth_emit(const int32_t *__restrict__ perm, int64_t n,
                                                    const uint32_t *__restrict__ secs, const int32_t *__restrict__ cust,
                                                    const int32_t *__restrict__ term, const double *__restrict__ amount,
                                                    const uint8_t *__restrict__ scen, int64_t start_ns, int32_t cust_offset,
                                                    int64_t *__restrict__ ts_o, int32_t *__restrict__ cust_o,
                                                    int32_t *__restrict__ term_o, double *__restrict__ amount_o,
                                                    uint8_t *__restrict__ fraud_o, uint8_t *__restrict__ scen_o,
                                                    int32_t *__restrict__ day_o) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = perm[j];
        const uint32_t sc = secs[r];
        ts_o[j] = start_ns + (int64_t)sc * 1000000000LL;
        cust_o[j] = cust[r] + cust_offset;
        term_o[j] = term[r];
        amount_o[j] = amount[r];
        fraud_o[j] = scen[r] != 0;
        if (scen_o) scen_o[j] = scen[r];
        if (day_o) day_o[j] = (int32_t)(sc / 86400u);
    }
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

int check_desc(const fdx_synth_desc *s) {
    FDX_REQUIRE(s, "null descriptor");
    FDX_REQUIRE(s->n_customers >= 1 && s->n_customers < (int64_t(1) << 31) && s->n_terminals >= 1 &&
                    s->n_terminals < (int64_t(1) << 31) && s->n_days >= 1 && s->n_days <= 24000,
                "bad sizes");
    FDX_REQUIRE(s->cx_d && s->cy_d && s->mean_amount_d && s->mean_nb_d && s->tx_sorted_d && s->ty_sorted_d &&
                    s->t_order_d && s->range_lo_d && s->range_hi_d,
                "null profile array");
    FDX_REQUIRE((s->n_comp_term == 0 || s->comp_term_d) && (s->n_comp_cust == 0 || s->comp_cust_d),
                "null compromised list");
    FDX_REQUIRE(s->radius > 0, "radius must be > 0");
    return FDX_OK;
}

}  // namespace
}  // namespace fdx

using namespace fdx;

extern "C" size_t fdx_synth_workspace_size(const fdx_synth_desc *s, int64_t n_tx) {
    if (!s || n_tx < 0) return 0;
    const int64_t cd = s->n_customers * (int64_t)s->n_days;
    const int key_bits = (int)(64 - __builtin_clzll((unsigned long long)std::max<int64_t>(s->n_days * 86400LL - 1, 1)));
    return al256((size_t)cd * 4 + 4) + al256((size_t)s->n_customers) + al256(fdx_exclusive_scan_u32_workspace_size(cd + 1)) +
           al256((size_t)n_tx * 4) * 4 + al256((size_t)n_tx * 8) + al256((size_t)n_tx) +
           al256(fdx_rekey_workspace_size(n_tx, key_bits)) + 256;
}

// layout of the workspace: offsets [cd+1] u32 | has [n_c] u8 | scan scratch | secs | cust | term |
// perm | amount | scen | rekey scratch
struct SynthWs {
    uint32_t *off;
    uint8_t *has;
    void *scan;
    uint32_t *secs;
    int32_t *cust, *term, *perm;
    double *amount;
    uint8_t *scen;
    void *rk;
    size_t rk_bytes;
};

static SynthWs synth_ws(const fdx_synth_desc *s, int64_t n_tx, void *ws) {
    const int64_t cd = s->n_customers * (int64_t)s->n_days;
    char *p = reinterpret_cast<char *>(ws);
    SynthWs w;
    w.off = reinterpret_cast<uint32_t *>(p); p += al256((size_t)cd * 4 + 4);
    w.has = reinterpret_cast<uint8_t *>(p); p += al256((size_t)s->n_customers);
    w.scan = p; p += al256(fdx_exclusive_scan_u32_workspace_size(cd + 1));
    w.secs = reinterpret_cast<uint32_t *>(p); p += al256((size_t)n_tx * 4);
    w.cust = reinterpret_cast<int32_t *>(p); p += al256((size_t)n_tx * 4);
    w.term = reinterpret_cast<int32_t *>(p); p += al256((size_t)n_tx * 4);
    w.perm = reinterpret_cast<int32_t *>(p); p += al256((size_t)n_tx * 4);
    w.amount = reinterpret_cast<double *>(p); p += al256((size_t)n_tx * 8);
    w.scen = reinterpret_cast<uint8_t *>(p); p += al256((size_t)n_tx);
    w.rk = p;
    const int key_bits = (int)(64 - __builtin_clzll((unsigned long long)std::max<int64_t>(s->n_days * 86400LL - 1, 1)));
    w.rk_bytes = fdx_rekey_workspace_size(n_tx, key_bits);
    return w;
}

extern "C" int fdx_synth_plan(const fdx_synth_desc *s, void *workspace_d, size_t workspace_bytes, int64_t *n_tx_h,
                              void *stream) {
    int rc = check_desc(s);
    if (rc) return rc;
    FDX_REQUIRE(workspace_d && n_tx_h, "null pointer");
    FDX_REQUIRE(workspace_bytes >= fdx_synth_workspace_size(s, 0), "workspace too small");
    hipStream_t st = as_stream(stream);
    SynthWs w = synth_ws(s, 0, workspace_d);
    const int64_t cd = s->n_customers * (int64_t)s->n_days;
    hipLaunchKernelGGL(k_synth_has_terminal, dim3(stream_grid(s->n_customers, 256)), dim3(256), 0, st, *s, w.has);
    FDX_LAUNCHED("k_synth_has_terminal");
    hipLaunchKernelGGL(k_synth_count, dim3(stream_grid(cd, 256, 256 * 32)), dim3(256), 0, st, *s, w.has, w.off);
    FDX_LAUNCHED("k_synth_count");
    FDX_HIP(hipMemsetAsync(w.off + cd, 0, 4, st));
    rc = fdx_exclusive_scan_u32(w.off, cd + 1, w.scan, stream);
    if (rc) return rc;
    uint32_t total = 0;
    FDX_HIP(hipMemcpyAsync(&total, w.off + cd, 4, hipMemcpyDeviceToHost, st));
    FDX_HIP(hipStreamSynchronize(st));
    *n_tx_h = total;
    return FDX_OK;
}

extern "C" int fdx_synth_fill(const fdx_synth_desc *s, int64_t n_tx, void *workspace_d, size_t workspace_bytes,
                              int64_t *ts_d, int32_t *customer_d, int32_t *terminal_d, double *amount_d,
                              uint8_t *fraud_d, uint8_t *scenario_d, int32_t *day_d, void *stream) {
    int rc = check_desc(s);
    if (rc) return rc;
    FDX_REQUIRE(n_tx >= 0 && n_tx < (int64_t)INT32_MAX, "n_tx out of range");
    FDX_REQUIRE(workspace_d && workspace_bytes >= fdx_synth_workspace_size(s, n_tx), "workspace too small");
    if (n_tx == 0) return FDX_OK;
    FDX_REQUIRE(ts_d && customer_d && terminal_d && amount_d && fraud_d, "null output");
    hipStream_t st = as_stream(stream);
    // the plan's offsets / has live at the front of the same workspace layout
    SynthWs w = synth_ws(s, n_tx, workspace_d);
    const int64_t cd = s->n_customers * (int64_t)s->n_days;
    hipLaunchKernelGGL(k_synth_fill, dim3(stream_grid(cd, 256, 256 * 32)), dim3(256), 0, st, *s, w.has, w.off, w.secs,
                       w.cust, w.term, w.amount, w.scen);
    FDX_LAUNCHED("k_synth_fill");
    const int key_bits = (int)(64 - __builtin_clzll((unsigned long long)std::max<int64_t>(s->n_days * 86400LL - 1, 1)));
    rc = fdx_rekey(reinterpret_cast<const int32_t *>(w.secs), n_tx, key_bits, (int64_t)s->n_days * 86400, w.perm,
                   nullptr, nullptr, w.rk, w.rk_bytes, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_synth_emit, dim3(stream_grid(n_tx, 256)), dim3(256), 0, st, w.perm, n_tx, w.secs, w.cust,
                       w.term, w.amount, w.scen, s->start_ns, s->customer_offset, ts_d, customer_d, terminal_d,
                       amount_d, fraud_d, scenario_d, day_d);
    FDX_LAUNCHED("k_synth_emit");
    return FDX_OK;
}
