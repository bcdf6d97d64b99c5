// fdx_forest.hip -- K3: tree-ensemble predict_proba on gfx950 (the walk; the scoring rows are
// built by fdx_assemble.hip, the node layouts by fdx_forest_layout.cpp).
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
#include "fdx_forest_internal.h"

namespace fdx {
namespace {

__device__ __forceinline__ double leaf_value(uint64_t nd) { return __longlong_as_double((long long)nd); }

template <bool LDS>
__device__ __forceinline__ uint64_t node_at(const uint64_t *s_nodes, const char *gbase, uint32_t byte_off) {
    if (LDS) return *reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(s_nodes) + byte_off);
    return *reinterpret_cast<const uint64_t *>(gbase + byte_off);
}


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
constexpr int kExitEvery = 4;
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
constexpr uint32_t kSlotMask = P16 >= 2 ? 0xF800u : 0xF000u;
template <int P16>
constexpr uint32_t kOffMask = P16 >= 2 ? 0x7FFu : 0xFFFu;
// 3 = the v2 node format over 16 u16 planes of 1,024 rows (32 KiB): forests whose every feature
// fits one slot (slot = feature, the v1 row format); the node region starts at 32 KiB, so a
// chunk holds a third more nodes than with 64 KiB of planes (fewer chunk launches per batch)
// 4 = the v2 node format, TWO rows per lane (2,048 rows per 1,024-lane block): plane s holds one
// dword per lane -- its first row's u16 rank in the low half, its second row's in the high half --
// and only the forest's n_slots planes are staged, at the TOP of the LDS (byte pb = kLdsTotal -
// 4,096 n_slots); the nodes start at byte 0.  A rank address is 2 (node & 0xF800) + pb + 4 lane
// (+ 2 for the second row): one VALU more than the OR form, and lanes read 64 different banks
// whatever slots they test.  The deployed model (22 slots, trees up to 16.9k nodes) walks one
// tree per chunk: with one row per lane that is ONE dependency chain per lane (latency-bound,
// r06d PMC: 67 % of wave time in s_waitcnt); two rows double the chains in flight per CU.
template <int P16>
constexpr uint32_t kNodeB = P16 == 3 ? 32768u : (P16 == 4 ? 0u : kRankNodeB);
template <int P16>
__device__ __forceinline__ uint32_t plane_addr(uint32_t nd, uint32_t lane_base) {
    if constexpr (P16 == 4) {
        // 2 VALU (the compiler's own form was shift, and, add: 3 -- r06ag ISA)
        uint32_t t, a;
        asm("v_and_b32 %0, 0xf800, %2\n\tv_lshl_add_u32 %1, %0, 1, %3" : "=&v"(t), "=v"(a) : "v"(nd), "v"(lane_base));
        return a;
    } else
        return (nd & kSlotMask<P16>) | lane_base;
}

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
        x[k] = rank_x<P16>(lds, plane_addr<P16>(nd[k], lane_base[k]));
        if (P16 == 3) x[k] = (x[k] >> (16u - sh)) & 0xFFFFu;  // this lane's half
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint32_t st;
        if (NAN_AWARE && x[k] == (P16 ? 0xFFFFu : 0xFFFF0000u)) {  // (u32 planes: stage_planes_u32)
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
// PIPE = 102 (chains in interleaved pairs; u32 planes, the default variant):
// the group's VALU of a phase issued round-robin over its chains (sub, sub, and, and, med3,
// med3, ...), so that no instruction waits on the one issued right before it, then the group's
// reads; one asm block per group and phase.
// The step of two chains (u32 planes): d = x - nd, st = med3(d, 1, nd & 0xFFF), pa += 4 st.
__device__ __forceinline__ void il_node2(uint32_t &p0, uint32_t &p1, uint32_t x0, uint32_t x1, uint32_t n0, uint32_t n1) {
    uint32_t d0, d1, o0, o1;
    asm("v_sub_u32 %[d0], %[x0], %[n0]\n\tv_sub_u32 %[d1], %[x1], %[n1]\n\t"
        "v_and_b32 %[o0], 0xfff, %[n0]\n\tv_and_b32 %[o1], 0xfff, %[n1]\n\t"
        "v_med3_i32 %[d0], %[d0], 1, %[o0]\n\tv_med3_i32 %[d1], %[d1], 1, %[o1]\n\t"
        "v_lshl_add_u32 %[p0], %[d0], 2, %[p0]\n\tv_lshl_add_u32 %[p1], %[d1], 2, %[p1]"
        : [p0] "+v"(p0), [p1] "+v"(p1), [d0] "=&v"(d0), [d1] "=&v"(d1), [o0] "=&v"(o0), [o1] "=&v"(o1)
        : [x0] "v"(x0), [x1] "v"(x1), [n0] "v"(n0), [n1] "v"(n1));
}
__device__ __forceinline__ void il_node1(uint32_t &p0, uint32_t x0, uint32_t n0) {
    uint32_t d0, o0;
    asm("v_sub_u32 %[d0], %[x0], %[n0]\n\tv_and_b32 %[o0], 0xfff, %[n0]\n\t"
        "v_med3_i32 %[d0], %[d0], 1, %[o0]\n\tv_lshl_add_u32 %[p0], %[d0], 2, %[p0]"
        : [p0] "+v"(p0), [d0] "=&v"(d0), [o0] "=&v"(o0) : [x0] "v"(x0), [n0] "v"(n0));
}

template <int P16, int K, int PW>
__device__ __forceinline__ int rank_walk_pipe(const char *lds, const uint32_t (&lane_base)[K], uint32_t (&pa)[K],
                                              uint32_t (&nd)[K], int depth, int pre = 0) {
    auto fetch_x = [&](int k) -> uint32_t { return rank_x<P16>(lds, plane_addr<P16>(nd[k], lane_base[k])); };
    const uint32_t sh = plane_shift<P16>();
    uint32_t x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = fetch_x(k);
    auto step = [&]() {
        if constexpr (PW >= 100) {
            static_assert(PW == 102 && P16 == 0, "interleaved pairs: u32 planes");
#pragma unroll
            for (int g = 0; g < K; g += 2) {
                if (g + 1 < K) {
                    il_node2(pa[g], pa[g + 1], x[g], x[g + 1], nd[g], nd[g + 1]);
                    nd[g + 1] = lds32(lds, pa[g + 1]);
                    nd[g] = lds32(lds, pa[g]);
                } else {
                    il_node1(pa[g], x[g], nd[g]);
                    nd[g] = lds32(lds, pa[g]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int g = 0; g < K; g += 2) {
                const uint32_t a0 = (nd[g] & kSlotMask<P16>) | lane_base[g];
                const uint32_t a1 = g + 1 < K ? (nd[g + 1] & kSlotMask<P16>) | lane_base[g + 1] : 0u;
                x[g] = rank_x<P16>(lds, a0);
                if (g + 1 < K) x[g + 1] = rank_x<P16>(lds, a1);
                __builtin_amdgcn_sched_barrier(0);
            }
            return;
        }
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
    // The walk's last possible step (d = depth - 1) moves every chain to its leaf and reads
    // nothing: the node and rank reads a step issues serve the NEXT step, and after the last one
    // only the leaf ADDRESS is used (leaf values / ids are indexed by it).  The bench rows walk
    // ~19.8 of 20 steps per tree, so this drops 2 of ~40 LDS reads per tree.
    auto last_step = [&]() {
        if constexpr (PW >= 100) {
#pragma unroll
            for (int g = 0; g < K; g += 2) {
                if (g + 1 < K)
                    il_node2(pa[g], pa[g + 1], x[g], x[g + 1], nd[g], nd[g + 1]);
                else
                    il_node1(pa[g], x[g], nd[g]);
            }
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int32_t d = P16 ? (int32_t)((x[k] << (P16 == 3 ? sh : 16u)) + nd[k]) : (int32_t)(x[k] - nd[k]);
                uint32_t st, pn;
                asm("v_med3_i32 %1, %2, 1, %3\n\tv_lshl_add_u32 %0, %1, 2, %4"
                    : "=v"(pn), "=&v"(st) : "v"(d), "v"(nd[k] & kOffMask<P16>), "v"(pa[k]));
                pa[k] = pn;
            }
        }
    };
    int d = 0;
    // whole unrolled intervals; the exit test only past the first `pre` steps (pre <= depth -
    // kExitEvery: never the last step).  One loop, not a test-free loop and a testing one: two
    // loops over the same step got different registers, and the copies between them cost ~30
    // v_mov per tile.
    for (; d + kExitEvery < depth; d += kExitEvery) {
#pragma unroll
        for (int e = 0; e < kExitEvery; ++e) step();
        if (d + kExitEvery > pre) {  // (uniform)
            uint32_t moving = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) moving |= nd[k] & kOffMask<P16>;
            if (!__any(moving != 0)) return d + kExitEvery;
        }
    }
    if (d < depth) {  // 1 .. kExitEvery steps left, the last without reads
        if (d + kExitEvery == depth) {
#pragma unroll
            for (int e = 0; e < kExitEvery - 1; ++e) step();
        } else {
            for (; d < depth - 1; ++d) step();
        }
        last_step();
    }
    return depth;
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
    if constexpr (PIPE == 102) {
        // the first step from the launch-uniform root words (SGPRs): d = x - root,
        // med3(d, 1, root & 0xFFF) with the offset masked on the scalar unit, pa = root address +
        // 4 step -- 3 VALU and no copy of the roots into VGPRs (4 VALU + 2 v_mov per chain)
        if (dmax <= 0) return 0;
        uint32_t x[K];
#pragma unroll
        for (int g = 0; g < GG; ++g)
#pragma unroll
            for (int r = 0; r < R; ++r) x[r * GG + g] = lds32(lds, (rn[g] & 0xF000u) | lane_base[r * GG + g]);
#pragma unroll
        for (int g = 0; g < GG; ++g) {
            const uint32_t off = __builtin_amdgcn_readfirstlane(rn[g] & 0xFFFu);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int k = r * GG + g;
                uint32_t dd, st;
                asm("v_sub_u32 %[d], %[x], %[n]\n\t"
                    "v_med3_i32 %[s], %[d], 1, %[o]\n\t"
                    "v_lshl_add_u32 %[p], %[s], 2, %[b]"
                    : [p] "=v"(pa[k]), [d] "=&v"(dd), [s] "=&v"(st)
                    : [x] "v"(x[k]), [n] "s"(rn[g]), [o] "s"(off), [b] "s"(rp[g]));
            }
        }
        if (dmax == 1) return 1;  // (the walk's last step reads nothing)
#pragma unroll
        for (int k = 0; k < K; ++k) nd[k] = lds32(lds, pa[k]);
        return 1 + rank_walk_pipe<P16, K, PIPE>(lds, lane_base, pa, nd, dmax - 1, pre - 1);
    } else {
        return rank_walk_pipe<P16, K, PIPE>(lds, lane_base, pa, nd, dmax, pre);
    }
}

template <int K>
__device__ __forceinline__ void rank_leaf_values(const uint32_t (&pa)[K], int64_t node_base,
                                                 const double *__restrict__ lval, double (&v)[K],
                                                 uint32_t nodeb = kRankNodeB) {
    // lval[node_base + (pa - nodeb) / 4] as a uniform 64-bit base + a 32-bit byte offset 2 * pa:
    // one VALU per load (global_load saddr + voffset) instead of a 64-bit address per lane
    const char *base = reinterpret_cast<const char *>(lval + node_base) - (size_t)(nodeb >> 2) * sizeof(double);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = *reinterpret_cast<const double *>(base + (uint32_t)(pa[k] << 1));
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
// The loads go out kTreeSumBatch at a time before their additions (the rolled loop had one or
// two in flight per lane: 27 us for a 64k-row stream batch of 100 trees, r06e trace).
constexpr int kTreeSumBatch = 25;
__global__ void __launch_bounds__(256) k_tree_sum(const double *__restrict__ tv, int64_t n, int32_t n_trees,
                                                  const int32_t *__restrict__ out_perm, double *__restrict__ proba) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        double a = 0.0;
        int t = 0;
        for (; t + kTreeSumBatch <= n_trees; t += kTreeSumBatch) {
            double v[kTreeSumBatch];
#pragma unroll
            for (int j = 0; j < kTreeSumBatch; ++j) v[j] = tv[(int64_t)(t + j) * n + r];
#pragma unroll
            for (int j = 0; j < kTreeSumBatch; ++j) a += v[j];  // tree order
        }
        for (; t < n_trees; ++t) a += tv[(int64_t)t * n + r];
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
// persist > 0 (every chunk one walk group): ONE launch walks chunks 0 .. persist-1 in turn, each
// block refilling its LDS nodes between chunks; the running sum crosses chunks through acc,
// written and read back by the same lane (a block owns the same tiles in every chunk).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
// The 15 u32 plane words of row slot r * BLOCK + tid (rank << 16, NaN 0xFFFF0000).  With
// ds_write_addtid_b32 (address = M0 + offset + 4 * lane; no address VGPR) a store moves 4 B per
// lane in 2 LDS cycles, half of ds_write_b32's 4: the planes are re-staged for every 1,024-row
// tile, 15 stores per lane against ~220 walk reads.  The kernel's code uses M0 nowhere else.
template <int BLOCK>
__device__ __forceinline__ void stage_words(uint32_t *s_x, int r, const uint32_t (&x)[15]) {
    static_assert(14 * kRankPlaneRows * 4 < 65536, "plane offsets fit the 16-bit instruction offset");
    const uint32_t b = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(lds_u32 *)(s_x + r * BLOCK + (threadIdx.x & ~63u)));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    asm volatile(
        "s_mov_b32 m0, %0\n\t"
        "s_nop 1\n\t"  // M0 write -> LDS add-TID: wait states (without them the first store used the old M0)
        "ds_write_addtid_b32 %1\n\t"
        "ds_write_addtid_b32 %2 offset:4096\n\t"
        "ds_write_addtid_b32 %3 offset:8192\n\t"
        "ds_write_addtid_b32 %4 offset:12288\n\t"
        "ds_write_addtid_b32 %5 offset:16384\n\t"
        "ds_write_addtid_b32 %6 offset:20480\n\t"
        "ds_write_addtid_b32 %7 offset:24576\n\t"
        "ds_write_addtid_b32 %8 offset:28672\n\t"
        "ds_write_addtid_b32 %9 offset:32768\n\t"
        "ds_write_addtid_b32 %10 offset:36864\n\t"
        "ds_write_addtid_b32 %11 offset:40960\n\t"
        "ds_write_addtid_b32 %12 offset:45056\n\t"
        "ds_write_addtid_b32 %13 offset:49152\n\t"
        "ds_write_addtid_b32 %14 offset:53248\n\t"
        "ds_write_addtid_b32 %15 offset:57344"
        :
        : "s"(b), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]),
          "v"(x[8]), "v"(x[9]), "v"(x[10]), "v"(x[11]), "v"(x[12]), "v"(x[13]), "v"(x[14])
        : "memory", "m0");
#pragma clang diagnostic pop
}
// One VALU per feature (a shift or a mask of the rank pair).  A NaN feature's rank 0xFFFF becomes
// 0xFFFF0000, the NaN-aware walk's marker (ranks are <= 0x7FFF): no second form for NaN batches
// (a form per batch kind left the compiler computing one and moving it into the other's
// registers, 15 v_mov per tile).
template <int BLOCK>
__device__ __forceinline__ void stage_planes_u32(uint32_t *s_x, int r, const uint32_t (&w)[8]) {
    uint32_t x[15];
#pragma unroll
    for (int f = 0; f < 15; ++f) x[f] = (f & 1) ? w[f >> 1] & 0xFFFF0000u : w[f >> 1] << 16;
    stage_words<BLOCK>(s_x, r, x);
}

// CL: the chunk loop (persist > 0) -- its own instantiation, so that the loop's register pressure
// stays out of the generic tile loop (small batches, leaf ids): one kernel holding both spilled
// in the generic loop (stream micro-batches 0.157 -> 0.167 ms on the device, r05bk)
template <int BLOCK, int R, int G, int P16, int PIPE, bool CL>
__global__ void __launch_bounds__(BLOCK, 1) k_forest_rank(
    const uint32_t *__restrict__ nodes, int64_t node_base, int32_t chunk_nodes, const int32_t *__restrict__ root,
    const int32_t *__restrict__ depth, int32_t t0, int32_t t1, const uint16_t *__restrict__ zr,
    const int32_t *__restrict__ nan_flag, int64_t r0, int64_t r1, const double *__restrict__ lval,
    const uint8_t *__restrict__ mleft, double *__restrict__ acc, double *__restrict__ proba,
    const int32_t *__restrict__ out_perm, int32_t *__restrict__ leaf_out, const int32_t *__restrict__ orig,
    int32_t n_trees, int first, int last, const int32_t *__restrict__ chunk_t,
    const int64_t *__restrict__ chunk_base, double *__restrict__ tv, int64_t tv_n, int32_t persist,
    int32_t n_slots) {
    // u32 planes: 1,024 rows x 16 slots; v2: u16, 1,024 rows x 32 slots; compact v2: u16, 16 slots;
    // paired v2 (P16 = 4): n_slots dword planes of 1,024 lanes x 2 rows at the top of the LDS
    constexpr int kPlaneRows = kRankPlaneRows;
    constexpr int kRowU16 = (P16 == 2 || P16 == 4) ? 32 : 16;  // u16 slots per rank row in HBM
    constexpr int kXW = P16 == 3 ? kRankXWords / 2 : kRankXWords;  // row-plane words in LDS (below the nodes)
    constexpr int kNodeW0 = P16 == 4 ? 0 : kXW;                    // first node word
    constexpr uint32_t kNB = kNodeB<P16>;
    static_assert(P16 != 4 || (R == 2 && BLOCK == kPlaneRows), "paired planes: two rows per lane, 1,024 lanes");
    // paired planes: plane s at byte pb + 4,096 s (uniform)
    const uint32_t pb = P16 == 4 ? (uint32_t)(kLdsTotal - 4096 * n_slots) & ~15u : 0u;
    if (tv) {  // all chunks at once (blockIdx.y = chunk): per-tree values out, summed by k_tree_sum
        const int c = blockIdx.y;
        t0 = chunk_t[c];
        t1 = chunk_t[c + 1];
        node_base = chunk_base[c];
        chunk_nodes = (int32_t)(chunk_base[c + 1] - node_base);
        first = 1;
        last = 0;
    }
    static_assert(BLOCK * R <= kPlaneRows * (P16 == 4 ? 2 : 1), "row planes hold 1024 rows (2048 paired)");
    static_assert(BLOCK % 64 == 0, "whole waves (the u16 plane swizzle)");
    constexpr int K = R * G;  // chains per lane of one walk group
    (void)K;
    constexpr int kRowsPerBlock = BLOCK * R;
    __shared__ __align__(16) uint32_t s_mem[kLdsTotal / 4];
    uint32_t *s_x = s_mem;
    const char *lds = reinterpret_cast<const char *>(s_mem);
    const int tid = threadIdx.x;
    // persist > 0: this one launch walks chunks [0, persist) in turn (see the chunk loop below)
    auto chunk_params = [&](int c) {
        t0 = chunk_t[c];
        t1 = chunk_t[c + 1];
        node_base = chunk_base[c];
        chunk_nodes = (int32_t)(chunk_base[c + 1] - node_base);
        first = c == 0;
        last = c + 1 == persist;
    };
    if (persist > 0) chunk_params(0);
    auto fill_nodes = [&]() {
        const uint32_t *nb = nodes + node_base;
        if constexpr (CL) {  // 4 loads in flight per thread (the chunk loop's registers are tight):
                             // the deployed model refills a one-tree chunk (~17k nodes) 100 times
#pragma unroll 1
            for (int i0 = tid; i0 < chunk_nodes; i0 += 4 * BLOCK) {
                uint32_t v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = nb[min(i0 + j * BLOCK, chunk_nodes - 1)];  // (clamped: no branch)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (i0 + j * BLOCK < chunk_nodes) s_mem[kNodeW0 + i0 + j * BLOCK] = P16 ? v[j] ^ 0xFFFF0000u : v[j];
            }
        } else {  // several loads in flight: with one tile per block (small batches) the fill is a
                  // large share of a block's work (rolled: stream micro-batches +8 us, r05bp)
            for (int i = tid; i < chunk_nodes; i += BLOCK) s_mem[kNodeW0 + i] = P16 ? nb[i] ^ 0xFFFF0000u : nb[i];
        }
    };
    fill_nodes();
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
    // (paired planes: the lane's own dword, natural order -- 64 lanes, 64 banks)
    const int pslot = (P16 == 2 || P16 == 3) ? ((tid & ~63) | ((tid & 31) << 1) | ((tid >> 5) & 1)) : tid;
    uint32_t lrow[R];
#pragma unroll
    for (int r = 0; r < R; ++r)  // compact planes: the byte address of the dword holding the lane's u16
        lrow[r] = P16 == 4 ? pb + (uint32_t)tid * 4u + 2u * r
                           : (uint32_t)(P16 == 3 ? ((r * BLOCK + pslot) & ~1) * 2 : (r * BLOCK + pslot) * (P16 ? 2 : 4));
    // paired planes: the lane's two rank rows (32 u16 slots each, as q0..q3 hold them) as n_slots
    // dwords, row 0 in the low halves
    auto stage_paired = [&](const uint4 (&a0)[R], const uint4 (&a1)[R], const uint4 (&a2)[R], const uint4 (&a3)[R]) {
        if constexpr (P16 == 4) {
            const uint32_t u[16] = {a0[0].x, a0[0].y, a0[0].z, a0[0].w, a1[0].x, a1[0].y, a1[0].z, a1[0].w,
                                    a2[0].x, a2[0].y, a2[0].z, a2[0].w, a3[0].x, a3[0].y, a3[0].z, a3[0].w};
            const uint32_t v[16] = {a0[1].x, a0[1].y, a0[1].z, a0[1].w, a1[1].x, a1[1].y, a1[1].z, a1[1].w,
                                    a2[1].x, a2[1].y, a2[1].z, a2[1].w, a3[1].x, a3[1].y, a3[1].z, a3[1].w};
            uint32_t *pl = s_mem + (pb >> 2) + tid;
#pragma unroll
            for (int f = 0; f < 32; ++f) {
                if (f >= n_slots) break;  // (uniform)
                const uint32_t w = (f & 1) ? __builtin_amdgcn_perm(v[f >> 1], u[f >> 1], 0x07060302u)   // high halves
                                           : __builtin_amdgcn_perm(v[f >> 1], u[f >> 1], 0x05040100u);  // low halves
                pl[f * kPlaneRows] = w;
            }
        }
    };
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
            if (P16 == 2 || P16 == 4) {
                q2[r] = src[2];
                q3[r] = src[3];
            }
            pacc[r] = first ? 0.0 : acc[okr ? rw : r0];  // (unconditional load: see out_slots)
        }
    };
    // fetch with 32-bit byte offsets from the uniform bases (global_load saddr + voffset: no 64-bit
    // address per lane and array); the one-group loop runs only when every offset fits (r1 * 32 B)
    auto fetch32 = [&](int64_t b) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t rw = b + r * BLOCK + tid;
            const uint32_t ro = (uint32_t)(rw < r1 ? rw : r0);
            const uint4 *src = reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(zr) + ro * (kRowU16 * 2u));
            q0[r] = src[0];
            q1[r] = src[1];
            if (P16 == 2 || P16 == 4) {
                q2[r] = src[2];
                q3[r] = src[3];
            }
            pacc[r] = first ? 0.0 : *reinterpret_cast<const double *>(reinterpret_cast<const char *>(acc) + ro * 8u);
        }
    };
    const bool small = !tv && !leaf_out && r1 * (kRowU16 * 2) <= UINT32_MAX;  // (uniform)
    if (base < r1) {
        if (small)
            fetch32(base);
        else
            fetch(base);
    }
    // A chunk of at most G trees (every chunk of the bench forest: 5-6 trees of ~3.9k nodes per
    // 94 KiB) is ONE walk group per tile, so the group pipeline below never runs and each tile
    // waited for its leaf-value loads (and, last chunk, its output slots) right after its walk.
    // Here a tile's leaf values are folded into its running sums one tile LATER -- after the next
    // tile's walk -- and its output slots are loaded with its rank rows: no global load is
    // waited on right after it is issued.  Same float64 additions in the same (tree) order.
    auto one_group = [&](auto ntag) {
        constexpr int NT = decltype(ntag)::value;
        double pv[R * NT], ap[R];
        uint32_t rowp[R];
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
            rn[g] = __builtin_amdgcn_readfirstlane(lds32(lds, rp[g]));  // uniform: SGPRs
            dmax = max(dmax, depth[t0 + g]);
        }
        // the tile's output slots, loaded with its rank rows and used one tile later.  The load is
        // unconditional (index clamped into the batch; rows past r1 are never stored: okp), in a
        // wave-uniform branch: a lane-conditional load merged into its destination at a join made
        // the compiler wait there with vmcnt(0) -- for every load in flight, i.e. for the next
        // tile's rank rows right after issuing them, once per tile (r04 ISA; ~100 us per launch)
        const bool perm_out = last && out_perm;
        auto out_slots = [&](int64_t b) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int64_t rw = b + r * BLOCK + tid;
                const uint32_t rc = (uint32_t)(rw < r1 ? rw : r1 - 1);  // (32-bit offsets: see fetch32)
                dst_n[r] = perm_out ? *reinterpret_cast<const int32_t *>(reinterpret_cast<const char *>(out_perm) + rc * 4u)
                                    : (int32_t)rw;
            }
        };
        out_slots(base);
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
                    *reinterpret_cast<double *>(reinterpret_cast<char *>(acc) + rowp[r] * 8u) = ap[r];
                }
            }
        };
        // Tile loop: the next tile's rank rows, running sums and output slots are loaded at the TOP
        // of an iteration and staged at its END (after this tile's walk, fold and leaf-value
        // loads), so no prefetched register is carried around the loop.  Carried prefetch
        // registers were copied at the latch or the head, behind a vmcnt(0) that waited for every
        // load in flight (the next tile's rows right after issuing them, or the leaf gather just
        // issued), once per tile (r04 ISA: ~100 us per launch).  The wait before the staging
        // leaves the leaf loads in flight (in-order vmcnt: they are younger).
        uint32_t row[R];
        bool ok[R];
        double a[R];
        int32_t dst[R];
        auto stage_tile = [&]() {
            stage_paired(q0, q1, q2, q3);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                row[r] = (uint32_t)(base + r * BLOCK + tid);
                ok[r] = row[r] < (uint32_t)r1;
                if constexpr (P16 == 4) {
                } else if constexpr (P16 == 2) {
                    const uint32_t w16[16] = {q0[r].x, q0[r].y, q0[r].z, q0[r].w, q1[r].x, q1[r].y, q1[r].z, q1[r].w,
                                              q2[r].x, q2[r].y, q2[r].z, q2[r].w, q3[r].x, q3[r].y, q3[r].z, q3[r].w};
#pragma unroll
                    for (int f = 0; f < 32; ++f)
                        s_x16[f * kPlaneRows + r * BLOCK + pslot] = (uint16_t)((w16[f >> 1] >> ((f & 1) * 16)) & 0xFFFFu);
                } else {
                    const uint32_t w8[8] = {q0[r].x, q0[r].y, q0[r].z, q0[r].w, q1[r].x, q1[r].y, q1[r].z, q1[r].w};
                    if constexpr (P16 == 0) {
                        stage_planes_u32<BLOCK>(s_x, r, w8);
                    } else {
#pragma unroll
                        for (int f = 0; f < 16; ++f)
                            s_x16[f * kPlaneRows + r * BLOCK + pslot] = (uint16_t)((w8[f >> 1] >> ((f & 1) * 16)) & 0xFFFFu);
                    }
                }
                a[r] = pacc[r];
                dst[r] = dst_n[r];
            }
        };
        if (base < r1) stage_tile();  // (the first tile's rows were fetched before the node fill)
        while (base < r1) {
            // unconditional (fetch clamps rows past r1 to r0): a conditional load left its
            // registers to be merged at a join, behind a vmcnt(0) right after the loads
            fetch32(base + stride);
            out_slots(base + stride);
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
            base += stride;
            if (base >= r1) break;
            stage_tile();
        }
        fold();
    };
    // (9+ trees: register spills)
    auto one_chunk = [&]() {
#define FDX_ONE_GROUP(NT) \
    if constexpr (G >= NT && (!CL || NT <= kClMaxTrees)) \
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
    };
    if constexpr (CL) {
        // Chunk loop (persist > 0, small; the host checks that every chunk is one group): a block
        // walks the same tiles (blockIdx.x + k * gridDim.x) in every chunk, so a row's running sum
        // is only ever handed between chunks by the lane that holds it -- no grid-wide sync
        // between chunks, only the block's own barrier around the node refill.
        for (int c = 0;;) {
            one_chunk();
            if (++c >= persist) return;
            chunk_params(c);
            ml = mleft + node_base;
            base = r0 + (int64_t)blockIdx.x * kRowsPerBlock;
            if (base < r1) fetch32(base);  // (this lane stored these rows' running sums itself)
            __syncthreads();  // every wave is done with the previous chunk's nodes
            fill_nodes();
            __syncthreads();
        }
    } else if (small && t1 - t0 <= (G < 8 ? G : 8)) {
        one_chunk();
        return;
    }
    // the generic tile loop (leaf ids, per-tree values, chunks of more trees than one group):
    // two rows per lane walk groups of 3 trees (6 chains) to stay within the register budget
    constexpr int GG = R == 2 ? (G < 3 ? G : 3) : G;
    for (; base < r1; base += stride) {
        int64_t row[R];
        bool ok[R];
        double a[R];
        stage_paired(q0, q1, q2, q3);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            row[r] = base + r * BLOCK + tid;
            ok[r] = row[r] < r1;
            if constexpr (P16 == 4) {
            } else if constexpr (P16 == 2) {
                const uint32_t w[16] = {q0[r].x, q0[r].y, q0[r].z, q0[r].w, q1[r].x, q1[r].y, q1[r].z, q1[r].w,
                                        q2[r].x, q2[r].y, q2[r].z, q2[r].w, q3[r].x, q3[r].y, q3[r].z, q3[r].w};
#pragma unroll
                for (int f = 0; f < 32; ++f)
                    s_x16[f * kPlaneRows + r * BLOCK + pslot] = (uint16_t)((w[f >> 1] >> ((f & 1) * 16)) & 0xFFFFu);
            } else {
                const uint32_t w[8] = {q0[r].x, q0[r].y, q0[r].z, q0[r].w, q1[r].x, q1[r].y, q1[r].z, q1[r].w};
                if constexpr (P16 == 0) {
                    stage_planes_u32<BLOCK>(s_x, r, w);
                } else {
#pragma unroll
                    for (int f = 0; f < 16; ++f)
                        s_x16[f * kPlaneRows + r * BLOCK + pslot] = (uint16_t)((w[f >> 1] >> ((f & 1) * 16)) & 0xFFFFu);
                }
            }
            a[r] = pacc[r];
        }
        if (base + stride < r1) fetch(base + stride);
        double pv[R * GG];
        bool pending = false;
        int t = t0;
        for (; t + GG <= t1; t += GG) {
            uint32_t pa[R * GG];
            rank_trees<R, GG, P16, PIPE>(lds, lrow, t, root, depth, node_base, any_nan, ml, pa);
            if (pending) rank_accumulate<R, GG>(a, pv);
            rank_leaf_values<R * GG>(pa, node_base, lval, pv, kNB);
            if (tv) rank_tree_values<R, GG>(pv, t, row, ok, tv, tv_n);
            pending = true;
            if (leaf_out) rank_leaf_ids<R, GG>(pa, node_base, t, row, ok, out_perm, leaf_out, orig, n_trees, kNB);
        }
        const int nt = t1 - t;
#define FDX_RANK_TAIL(NT)                                                                                  \
    if constexpr (GG > NT) {                                                                                \
        if (nt == NT) {                                                                                    \
            uint32_t pt[R * NT];                                                                           \
            double vt[R * NT];                                                                             \
            rank_trees<R, NT, P16, PIPE>(lds, lrow, t, root, depth, node_base, any_nan, ml, pt);           \
            if (pending) rank_accumulate<R, GG>(a, pv);                                                     \
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
        if (pending) rank_accumulate<R, GG>(a, pv);
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

}  // namespace

bool rank_mode(const fdx_forest_s *F) { return kVariants[F->variant].rank != 0; }

}  // namespace fdx

using namespace fdx;

namespace fdx {
namespace {
int install_rank_layout(fdx_forest_s *F, bool v2, hipStream_t st);
// node format a variant runs on: 1 = rank layout v1, 2 = v2
int variant_format(const Variant &v) { return v.p16 >= 2 ? 2 : 1; }
int forest_format(const fdx_forest_s *F) { return F->rank_v2 ? 2 : 1; }
int variant_group(const fdx_forest_s *F) { return F->zstride == 16 ? kVariants[F->variant].group : 4; }


// Cut the trees into chunks whose nodes fit the variant's LDS budget; whole groups of G trees
// where more than G fit (a partial group idles walk slots); oversized trees run from global
// (wide layout only: a rank-layout forest has every tree within the budget by construction).
void build_chunks(fdx_forest_s *F) {
    const Variant v = F->zstride == 16 ? kVariants[F->variant] : kVariants[0];
    const int64_t cap_nodes = v.rank ? (v.p16 == 3 ? kRankNodeCapCompact
                                                   : (v.p16 == 4 ? rank_node_cap_paired(F->rn_slots) : kRankNodeCap))
                                     : lds_node_bytes(F->zstride, v.block, v.rows) / 8;
    const int G = variant_group(F);
    const auto &off = v.rank ? F->rank_offsets : F->node_offsets;
    F->chunks.clear();
    if (v.rank) {
        // rank layouts (every tree fits the budget): packed greedily from the LAST tree, so the
        // partial chunk is walked first and the last chunk -- the one that scatters proba to the
        // scoring slots' input rows, one random 8-byte store per row -- is a full one beside those
        // stores (same contiguous tree ranges in tree order, same float64 sums; measured with one
        // launch per chunk, profiles/r05ax_chunk_pack_ab.txt)
        for (int32_t u = F->n_trees; u > 0;) {
            int32_t t = u - 1;
            while (t > 0 && off[u] - off[t - 1] <= cap_nodes) --t;
            fdx_forest_s::Chunk c;
            c.t0 = t;
            c.t1 = u;
            c.node_base = off[t];
            c.nodes = off[u] - off[t];
            c.in_lds = c.nodes <= cap_nodes;
            F->chunks.insert(F->chunks.begin(), c);
            u = t;
        }
        return;
    }
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


extern "C" int fdx_forest_layout(fdx_forest F, int32_t *layout, int32_t *n_slots) {
    FDX_REQUIRE(F && layout && n_slots, "null pointer");
    *layout = !F->rank_ok ? 0 : (F->rank_v2 ? (F->rank_identity ? 3 : 2) : 1);
    *n_slots = F->rank_v2 ? F->rn_slots : (F->rank_ok ? 16 : 0);
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
        if (m <= (v2 ? kMaxRankSamplesV2 : kMaxRankSamples)) break;
    }
    F->rseg = seg;
    for (int f = 0; f < nfs; ++f) {
        const int32_t c = F->rthr_cnt[f], ns = (int32_t)ceil_div(c, seg);
        F->ruoff[f] = (int32_t)useg.size();
        F->rsoff[f] = (int32_t)smp.size();
        F->rscnt[f] = ns;
        for (int32_t j = 0; j < ns * seg; ++j)  // (+ 0.0f: -0.0 as +0.0, see lt_bit in fdx_assemble.hip)
            useg.push_back(j < c ? RL.thr[(size_t)(RL.thr_off[f] + j)] + 0.0f : INFINITY);
        for (int32_t j = 0; j < ns; ++j) smp.push_back(RL.thr[(size_t)(RL.thr_off[f] + j * seg)]);
    }
    F->rnsmp = (int32_t)smp.size();
    // S-trees of the searched features of k_zfill_grouped_w3 (RankTab::etab; 15-feature
    // forests with the v1 row format, build_search_trees)
    std::vector<float> etab;
    F->rnetab = 0;
    if (F->n_features == 15 && seg % kW3Gap == 0 && (!v2 || F->rank_identity)) {
        build_search_trees(RL, etab, F->reoff, F->relev);
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
    if (F->variant == kDefaultRankV2Variant) {
        // paired planes when every tree fits below the forest's slot planes: the deployed model
        // (22 slots, one tree per chunk) 42.7 -> 39.2 ms for 20M rows (profiles/r06l_*)
        bool fits = true;
        for (int32_t t = 0; t < F->n_trees && fits; ++t)
            fits = F->rank_offsets[t + 1] - F->rank_offsets[t] <= rank_node_cap_paired(F->rn_slots);
        if (fits) F->variant = kPairedRankV2Variant;
    }
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


namespace fdx {
int forest_ws(fdx_forest F, int64_t n, void *ws, size_t ws_bytes, float **z, double **acc,
                     int32_t **nan_flag) {
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

}  // namespace fdx

// One k_forest_rank launch for every chunk (its chunk loop) when each chunk is one walk group:
// 10.16 vs 10.28 ms/step at configs[1], the 18 launches' drain and ramp gone
// (profiles/r05ba_one_launch_ab.txt)
static bool one_launch_ok(const fdx_forest_s *F, int64_t n, bool leaves) {
    const int64_t row_bytes = v2_rows(kVariants[F->variant].p16) ? 64 : 32;  // (the kernel's 32-bit offsets)
    bool ok = rank_mode(F) && !leaves && F->chunks.size() > 1 && n * row_bytes <= (int64_t)UINT32_MAX;
    for (const auto &ch : F->chunks) ok = ok && ch.t1 - ch.t0 <= std::min(kClMaxTrees, kVariants[F->variant].group);
    return ok;
}
// Rows per k_forest_rank row range: the one-group tile loop addresses rank rows, running sums and
// output slots by 32-bit byte offsets, so a larger batch is walked range by range (128M rows at
// 32-B rank rows), each launch over base pointers moved to its range.
static int64_t rank_range_rows(const fdx_forest_s *F) {
    const int64_t row_bytes = v2_rows(kVariants[F->variant].p16) ? 64 : 32;
    const int64_t rr = ((int64_t)UINT32_MAX / row_bytes) & ~(int64_t)1023;
    return F->range_rows > 0 ? std::min(rr, std::max<int64_t>(F->range_rows & ~(int64_t)1023, 1024)) : rr;
}

extern "C" int fdx_forest_set_range_rows(fdx_forest F, int64_t rows) {
    FDX_REQUIRE(F, "null forest");
    FDX_REQUIRE(rows >= 0, "rows < 0");
    F->range_rows = rows;
    return FDX_OK;
}

extern "C" int fdx_forest_traverse_launches(fdx_forest F, int64_t n, int32_t with_leaves, int32_t *launches) {
    FDX_REQUIRE(F && launches, "null pointer");
    FDX_REQUIRE(n >= 0, "n < 0");
    const int64_t nc = (int64_t)F->chunks.size();
    if (n == 0)
        *launches = 0;
    else if (rank_mode(F) && nc > 1 && n <= concurrent_rows(F))
        *launches = 1;  // all chunks at once (grid.y = chunk), + k_tree_sum
    else if (!rank_mode(F))
        *launches = (int32_t)nc;
    else {
        const int64_t rr = rank_range_rows(F), ranges = ceil_div(n, rr);
        *launches = (int32_t)((ranges - 1) * (one_launch_ok(F, rr, with_leaves != 0) ? 1 : nc) +
                              (one_launch_ok(F, n - (ranges - 1) * rr, with_leaves != 0) ? 1 : nc));
    }
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
        const int64_t rr = tv ? n : rank_range_rows(F);
        const int64_t row_u16 = v2_rows(kVariants[F->variant].p16) ? 32 : 16;
        for (int64_t q0 = 0; q0 < n; q0 += rr) {  // row ranges (one unless n > rank_range_rows)
        const int64_t qn = std::min(rr, n - q0);
        const uint16_t *zq = zr + q0 * row_u16;
        double *accq = acc + q0;
        // output slots: through out_perm (absolute) or at the row (moved with the range)
        double *probaq = out_perm_d ? proba_d : proba_d + q0;
        const int32_t *permq = out_perm_d ? out_perm_d + q0 : nullptr;
        int32_t *leafq = leaf_d ? (out_perm_d ? leaf_d : leaf_d + q0 * F->n_trees) : nullptr;
        const bool one_launch = !tv && one_launch_ok(F, qn, leaf_d != nullptr);
        const int32_t persist = one_launch ? (int32_t)nc : 0;
        for (size_t c = 0; c < (tv || one_launch ? 1 : nc); ++c) {
            const auto &ch = F->chunks[c];
            const int first = c == 0, last = c + 1 == nc;
#define FDX_LAUNCH_RANK(B, R, G, P, PIPE)                                                                      \
    do {                                                                                                      \
        const int64_t tiles_ = ceil_div(qn, (int64_t)(B) * (R));                                              \
        const dim3 grid(tv ? (unsigned)tiles_ : (unsigned)std::min<int64_t>(tiles_, F->n_cu), tv ? (unsigned)nc : 1u); \
        if (persist)                                                                                          \
            hipLaunchKernelGGL((k_forest_rank<B, R, G, P, PIPE, true>), grid, dim3(B), 0, st, F->rnodes_d,      \
                               ch.node_base, (int32_t)ch.nodes, F->rroot_d, F->rdepth_d, ch.t0, ch.t1, zq, flag,  \
                               (int64_t)0, qn, F->rlval_d, F->rml_d, accq, probaq, permq, leafq, F->rorig_d,     \
                               F->n_trees, first, last, F->chunk_t_d, F->chunk_base_d, tv, n, persist, F->rn_slots);\
        else                                                                                                  \
            hipLaunchKernelGGL((k_forest_rank<B, R, G, P, PIPE, false>), grid, dim3(B), 0, st, F->rnodes_d,     \
                               ch.node_base, (int32_t)ch.nodes, F->rroot_d, F->rdepth_d, ch.t0, ch.t1, zq, flag,  \
                               (int64_t)0, qn, F->rlval_d, F->rml_d, accq, probaq, permq, leafq, F->rorig_d,     \
                               F->n_trees, first, last, F->chunk_t_d, F->chunk_base_d, tv, n, 0, F->rn_slots);      \
    } while (0)
            switch (F->variant) {
                case 2: FDX_LAUNCH_RANK(1024, 1, 6, 2, 2); break;
                case 3: FDX_LAUNCH_RANK(1024, 1, 6, 3, 2); break;
                case 4: FDX_LAUNCH_RANK(1024, 1, 10, 2, 2); break;
                case 5: FDX_LAUNCH_RANK(1024, 2, 2, 4, 2); break;
                default: FDX_LAUNCH_RANK(1024, 1, 10, 0, 102); break;
            }
#undef FDX_LAUNCH_RANK
            FDX_LAUNCHED("k_forest_rank");
        }
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

