// fdx_forest_layout.cpp -- host side of K3's node layouts: validation of a sklearn forest
// (tree_.children_left / children_right / feature / threshold / missing_go_to_left / value,
// model_training.ipynb:506, fraud_detection.py:193), the pre-order 8-byte packing (wide layout)
// and the 4-byte rank layouts v1 / v2 (fdx_forest.hip's "Rank layout" comment).  Host code only.
#include "fdx_forest_internal.h"

#include <functional>

namespace fdx {

float round_down_f32(double t) {
    float f = (float)t;
    if ((double)f > t) f = std::nextafter(f, -INFINITY);
    return f;
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

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
int build_rank_layout(const fdx_forest_desc *d, const std::vector<uint64_t> &packed,
                      const std::vector<int32_t> &worig, const std::vector<int32_t> &wdepth, int64_t max_tree_nodes,
                      RankLayout &L, bool v2) {
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

}  // namespace fdx

using namespace fdx;

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

// Every kW3Gap-th threshold of each searched feature as a complete 9-ary tree of 8-key nodes
// (node k's children 9k+1..9k+9), keys filled by an in-order walk (= sorted order), +inf past
// the samples: a descent's digits (keys of the node < v) spell #samples < v in base 9.
void fdx::build_search_trees(const RankLayout &L, std::vector<float> &trees, int32_t eoff[4], int32_t elev[4]) {
    trees.clear();
    for (int s = 0; s < 4; ++s) {
        const int f = kW3Search[s];
        const int32_t c = L.thr_off[f + 1] - L.thr_off[f], ns = (c + kW3Gap - 1) / kW3Gap;
        const float *thr = L.thr.data() + L.thr_off[f];
        int lv = 0;
        int64_t keys = 0;  // 9^lv - 1
        while (keys < ns) {
            ++lv;
            keys = keys * 9 + 8;
        }
        const int64_t nn = keys / 8;
        eoff[s] = (int32_t)(trees.size() / 8);
        elev[s] = lv;
        std::vector<float> t((size_t)keys, INFINITY);
        int32_t i = 0;
        std::function<void(int64_t)> fill = [&](int64_t k) {
            if (k >= nn) return;
            for (int j = 0; j < 8; ++j) {
                fill(9 * k + 1 + j);
                // (-0.0 stored as +0.0: the same comparisons, and the kernel's sign-bit compare needs it)
                t[(size_t)(8 * k + j)] = i < ns ? thr[(size_t)i * kW3Gap] + 0.0f : INFINITY;
                ++i;
            }
            fill(9 * k + 9);
        };
        fill(0);
        trees.insert(trees.end(), t.begin(), t.end());
    }
    if (trees.size() > (size_t)kW3TreeFloats) trees.clear();  // over the LDS budget
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

// Host form of the row assembly's search tables (tests): the S-trees of a 15-feature forest's
// v1 rank layout.  trees_out may be NULL (sizes only); *n_floats = 0 when none are built.
extern "C" int fdx_forest_search_trees(const fdx_forest_desc *d, float *trees_out, int64_t cap, int64_t *n_floats,
                                       int32_t *eoff_out, int32_t *elev_out) {
    FDX_REQUIRE(d && n_floats && eoff_out && elev_out, "null argument");
    FDX_REQUIRE(d->n_features == 15, "the assembly's search tables serve 15-feature forests");
    RankLayout RL;
    int rc = rank_layout_host(d, RL);
    if (rc) return rc;
    std::vector<float> trees;
    build_search_trees(RL, trees, eoff_out, elev_out);
    *n_floats = (int64_t)trees.size();
    if (trees_out) {
        FDX_REQUIRE(cap >= (int64_t)trees.size(), "trees_out holds %lld floats, %lld needed", (long long)cap,
                    (long long)trees.size());
        memcpy(trees_out, trees.data(), 4 * trees.size());
    }
    return FDX_OK;
}
