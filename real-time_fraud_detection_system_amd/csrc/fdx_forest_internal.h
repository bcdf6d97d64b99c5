// fdx_forest_internal.h -- what the three translation units of K3 share: fdx_forest.hip (the
// forest walk, the forest object and its variants), fdx_assemble.hip (the scoring-row assembly
// / prepare kernels: flags, averages, risks, StandardScaler, threshold ranks) and
// fdx_forest_layout.cpp (host-side node packing: the wide 8-byte layout and rank layouts
// v1 / v2).  Numerics and layouts are described where they are built.
#pragma once

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
    int64_t range_rows = 0;  // rows per traversal range (0: as many as 32-bit offsets allow)
};

namespace fdx {

constexpr uint32_t kInternal = 0x80000000u;

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
// position; NaN row values are 0xFFFF (u16) / 0xFFFF0000 (LDS), resolved by
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
    // S-trees of the reference layout's searched features (kW3Search: amount + the three
    // averages), for k_zfill_grouped_w3: feature kW3Search[s]'s every kW3Gap-th threshold as a
    // complete 9-ary tree of elev[s] levels, 8 keys per node (32 B; node k's children are
    // 9k+1..9k+9; keys padded with +inf), keys in in-order = sorted order, so the digits of a
    // descent (keys of the node < v) spell #samples < v in base 9; node k of feature s at
    // etab[8 * (eoff[s] + k)].  NULL when the trees exceed the LDS budget (kW3TreeFloats).
    const float *etab;
    int32_t eoff[4], elev[4], n_etab;
};
constexpr int kW3Search[4] = {0, 4, 6, 8};  // TX_AMOUNT, CUSTOMER_ID_AVG_AMOUNT_{1,7,30}DAY_WINDOW
constexpr int kMaxRankSamples = 8192;  // LDS sample table of the prepare kernels (32 KiB)
// rank layout v2 (only k_prepare_v2 reads its tables): 80 KiB of samples, so that the deployed
// model's 313k thresholds take 16-float segments (64 B per feature and row) instead of 64-float ones
constexpr int kMaxRankSamplesV2 = 20480;
constexpr int kW3Gap = 4;              // thresholds per S-tree sample (one 16-byte segment read)
constexpr int kW3TreeFloats = 28672;   // LDS budget of the S-trees (112 KiB)
constexpr int kIntTab = 256;           // integer rank table entries per feature (8 KiB in LDS)
constexpr int kRatN = 128;             // ratio rank table: nb, fr < kRatN (32 KiB per feature, global)

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
    {1024, 1, 10, 1, 0, 102},  // 1: rank layout v1, 10 chains per lane (the default: r03 sweep, 7.63 vs
                               //    8.43 ms for 6 chains at config 2; 12 chains spill, 11.7 ms), each
                               //    step's VALU interleaved over chain pairs (r05: 6.51 -> 6.43 ms)
    {1024, 1, 6, 1, 2, 2},   // 2: rank layout v2 (forests v1 cannot hold: the deployed model)
    {1024, 1, 6, 1, 3, 2},   // 3: v2 nodes over 16 u16 planes (a third more nodes per LDS chunk)
    {1024, 1, 10, 1, 2, 2},  // 4: v2, 10 chains
    {1024, 2, 2, 1, 4, 2},   // 5: v2 over paired planes (two rows per lane, the forest's slots only)
};
// the variant's rank rows in HBM are v2's 32 u16 slots (64 B)
constexpr bool v2_rows(int p16) { return p16 == 2 || p16 == 4; }
// (Round 6 measured and removed: speculative children -- the node's rank read AND both children's
// reads issued together, one dependent LDS round trip per level for 3 reads instead of 2:
// bit-exact, deployed model 42.4 -> 48.9 ms and bench model 6.57 -> 10.57 ms; the level-1 node
// from SGPR words of the root's children (one read and one round trip less per tree): 6.48-6.55
// -> 6.61-6.62 ms; the deployed model's 64-B rank rows read as 48 B: 42.4 -> 41.8 ms, i.e. not
// bound by the rows' re-stream; profiles/r06_forest_studies.txt.)
// (Round 5 also measured a one-round-trip study form (rank address from the node's address, wrong
// results: 7.05 vs 6.70 ms) and two-level packets (commit 654bb3b: bit-exact, 12 % slower per
// tree-step; profiles/r05uz_forest_walk_studies.txt) and removed them.)
// (Round 5 measured v1 over paired u16 planes, two rows per lane with 768 / 512 lanes (12 chains
// per lane, 12 / 8 waves per CU): 7.90 / 8.74 ms against 6.66 -- the walk's throughput follows
// the waves per CU, not the chains per lane -- and removed them.)
// (Round 4 measured compact v2 with 8 / 10 chains as well -- 7.27 ms against 6.91 for variant 1,
// the extra depth of its jump nodes, profiles/r04e_forest_launches.txt -- and removed them.)
// (Round 3 also measured v1 with 6 / 8 / 9 chains, compact v2 with 10 chains and register
// ranks -- the lane's rank row in 8 VGPRs, one ds_read per step: 16.3 vs 7.6 ms -- and removed
// them; DESIGN.md §4 keeps their numbers.)
constexpr int kDefaultRankVariant = 1;
constexpr int kDefaultRankV2Variant = 2;
constexpr int kDefaultRankCompactVariant = 3;
constexpr int kPairedRankV2Variant = 5;  // the v2 default when every tree fits its node budget
// trees per chunk the one-launch chunk loop walks as one group: the bench forest's chunks hold <= 6
// (3.9k-node trees in 94 KiB), and the loop instantiated for 7-8 as well spilled 17 VGPRs
constexpr int kClMaxTrees = 6;
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
constexpr int kLdsTotal = 160 * 1024 - 2048;  // leave room for the static bookkeeping

constexpr int lds_node_bytes(int fs, int block, int rows) { return kLdsTotal - fs * block * rows * 4; }

constexpr int64_t kRankNodeCap = (kLdsTotal - kRankXWords * 4) / 4 - 1;  // - the parking leaf
constexpr int64_t kRankNodeCapCompact = (kLdsTotal - kRankXWords * 2) / 4 - 1;  // 32 KiB of planes
// paired planes (variant 5): n_slots planes of 4 KiB at the top of the LDS, nodes below them
constexpr int64_t rank_node_cap_paired(int n_slots) { return ((kLdsTotal - 4096 * n_slots) & ~15) / 4 - 1; }

// ---- shared helpers (definitions: fdx_forest_layout.cpp, fdx_forest.hip, fdx_assemble.hip)
float round_down_f32(double t);  // largest float <= t
size_t align_up(size_t x);       // to 256 bytes
bool rank_mode(const fdx_forest_s *F);  // the current variant walks a rank layout
RankTab rank_tab(const fdx_forest_s *F);
// the traversal workspace's rank / float rows, running sums and NaN flag word
int forest_ws(fdx_forest F, int64_t n, void *ws, size_t ws_bytes, float **z, double **acc,
              int32_t **nan_flag = nullptr);
// Host-side validation + pre-order re-layout + 8-byte node packing (see fdx_forest.hip's header).
int pack_forest(const fdx_forest_desc *d, std::vector<uint64_t> &packed, std::vector<int32_t> &orig,
                std::vector<int32_t> &root, std::vector<int32_t> &depth);

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
constexpr int64_t kSlotSpan = 32767;  // thresholds per rank-layout-v2 slot (build_rank_layout)
// The S-trees of k_zfill_grouped_w3 (RankTab::etab) over a v1 rank layout's thresholds of the
// kW3Search features: trees (floats, 8 per node), eoff (node offset) and elev (levels) per
// searched feature.  Empty when they exceed kW3TreeFloats.
void build_search_trees(const RankLayout &L, std::vector<float> &trees, int32_t eoff[4], int32_t elev[4]);
int build_rank_layout(const fdx_forest_desc *d, const std::vector<uint64_t> &packed,
                      const std::vector<int32_t> &worig, const std::vector<int32_t> &wdepth, int64_t max_tree_nodes,
                      RankLayout &L, bool v2 = false);

}  // namespace fdx
