"""The rank layout of the forest traversal (host only, no GPU): fdx_forest_pack_rank's
4-byte nodes walked by a numpy model of k_forest_rank's step must give sklearn's leaves
and probabilities bit for bit (golden vectors from sklearn, and the C oracle of
sklearn's Tree._apply_dense for random forests -- incl. trees large enough to need
jump nodes, and NaN rows routed by missing_go_to_left)."""
import ctypes
import os

import numpy as np
import pytest

import oracle
from forest_gen import random_forest

LEAF = 0x0000F000


def _desc(a, n_features):
    from fdx import _lib

    keep = {k: np.ascontiguousarray(a[k], dt) for k, dt in
            (("node_offsets", np.int64), ("left", np.int64), ("right", np.int64), ("feature", np.int64),
             ("threshold", np.float64), ("missing_left", np.uint8), ("value1", np.float64))}
    nt = len(keep["node_offsets"]) - 1
    d = _lib.ForestDesc(nt, n_features, keep["node_offsets"].ctypes.data, keep["left"].ctypes.data,
                        keep["right"].ctypes.data, keep["feature"].ctypes.data, keep["threshold"].ctypes.data,
                        keep["missing_left"].ctypes.data, keep["value1"].ctypes.data, None, None)
    return d, keep


def pack_rank(a, n_features=15):
    from fdx import _lib

    L = _lib.load()
    d, keep = _desc(a, n_features)
    nn, nthr = ctypes.c_int64(), ctypes.c_int32()
    rc = L.fdx_forest_rank_layout_size(ctypes.byref(d), ctypes.byref(nn), ctypes.byref(nthr))
    if rc != 0:
        return None
    n, nt = nn.value, d.n_trees
    out = dict(nodes=np.zeros(n, np.uint32), orig=np.zeros(n, np.int32), lval=np.zeros(n), ml=np.zeros(n, np.uint8),
               root=np.zeros(nt, np.int32), depth=np.zeros(nt, np.int32), thr=np.zeros(max(nthr.value, 1), np.float32),
               thr_off=np.zeros(17, np.int32))
    rc = L.fdx_forest_pack_rank(ctypes.byref(d), *[out[k].ctypes.data for k in
                                                   ("nodes", "orig", "lval", "ml", "root", "depth", "thr", "thr_off")])
    assert rc == 0, L.fdx_last_error()
    return out


def walk_rank(R, z32, p16=False):
    """numpy model of k_forest_rank: ranks r = #{u < x}, x = r << 16, step =
    med3(x - node, 1, node & 0xFFF) as int32 (NaN rows: missing_go_to_left), a fixed number
    of steps (depth), leaves are fixed points, float64 sum in tree order.
    p16: the u16-plane form -- raw ranks r, LDS node S = node ^ 0xFFFF0000 and
    d = int32((r << 16) + S) (the kernel's v_lshl_add_u32), same med3 step."""
    n = z32.shape[0]
    xv = np.zeros((n, 16), np.int64)
    nanm = np.zeros((n, 16), bool)
    for f in range(min(z32.shape[1], 15)):
        u = R["thr"][R["thr_off"][f]:R["thr_off"][f + 1]]
        r = np.searchsorted(u, z32[:, f], side="left").astype(np.int64)
        xv[:, f] = r << 16
        nanm[:, f] = np.isnan(z32[:, f])
    xv[:, 15] = 0x4000 << 16
    nodes = R["nodes"].astype(np.int64)
    assert (nodes < 2**31).all() and (xv < 2**31).all()
    acc = np.zeros(n)
    nt = len(R["root"])
    leaves = np.zeros((n, nt), np.int32)
    rows = np.arange(n)
    for t in range(nt):
        p = np.full(n, R["root"][t], np.int64)
        for _ in range(int(R["depth"][t])):
            nd = nodes[p]
            f = (nd >> 12) & 15
            if p16:
                S = nd ^ 0xFFFF0000
                d = (((xv[rows, f] >> 16) << 16) + S) & 0xFFFFFFFF
                d = np.where(d >= 2**31, d - 2**32, d)
            else:
                d = xv[rows, f] - nd
            off = nd & 0xFFF
            st = np.median(np.stack([d, np.ones_like(d), off]), axis=0).astype(np.int64)
            st = np.where(nanm[rows, f], np.where(R["ml"][p] != 0, 1, off), st)
            p = p + st
        assert ((nodes[p] & 0xFFF) == 0).all(), "walk did not end on leaves within depth"
        acc = acc + R["lval"][p]
        leaves[:, t] = R["orig"][p]
    return acc / nt, leaves


def _z32(X, mean, scale):
    return ((X - mean) / scale).astype(np.float32)


@pytest.mark.parametrize("name", ["forest_dt2.npz", "forest_rf5d8.npz", "forest_rf3.npz"])
def test_rank_layout_reproduces_sklearn(golden, name):
    z = golden(name)
    R = pack_rank(z)
    assert R is not None
    assert (R["nodes"][R["orig"] >= 0] & 0xFFF).min() >= 0
    for p16 in (False, True):
        proba, leaves = walk_rank(R, _z32(z["X"], z["mean"], z["scale"]), p16)
        np.testing.assert_array_equal(leaves, z["leaves"])
        np.testing.assert_array_equal(proba, z["proba"])


def test_rank_layout_jump_nodes():
    """Complete-ish depth-13 trees: root left subtrees of ~8k nodes exceed the 12-bit right
    offset, so the packer must forward those pointers through jump nodes."""
    rng = np.random.default_rng(13)
    a = random_forest(rng, 3, 13, p_leaf=0.02)
    R = pack_rank(a)
    assert R is not None
    jumps = int((R["orig"] == -1).sum())
    assert jumps > 0
    assert len(R["nodes"]) == int(a["node_offsets"][-1]) + jumps
    X = rng.normal(size=(3000, 15))
    X[rng.random(X.shape) < 0.05] = np.nan
    op, ol = oracle.forest_predict(X, a, want_leaves=True)
    for p16 in (False, True):
        proba, leaves = walk_rank(R, X.astype(np.float32), p16)
        np.testing.assert_array_equal(leaves, ol)
        np.testing.assert_array_equal(proba, op)


def test_rank_layout_bench_model():
    """The config-3 model (RF 100 trees, depth 20) fits the rank layout and reproduces the
    sklearn predict_proba saved with it."""
    import os

    from conftest import ROOT

    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    R = pack_rank(z)
    assert R is not None
    for p16 in (False, True):
        proba, _ = walk_rank(R, _z32(z["check_X"], z["mean"], z["scale"]), p16)
        np.testing.assert_array_equal(proba, z["check_proba"])


def test_rank_threshold_edge_cases():
    """x32 <= thr64 <=> rank(x32) <= k for thresholds between floats, at floats, +-0, +-inf."""
    thr = np.array([0.1, -0.1, 1e-40, -1e-40, 3.4e38, 1.0, 0.5 + 2**-30, -2.5 - 2**-40, 0.0, -0.0], np.float64)
    n = len(thr)
    a = dict(node_offsets=np.arange(0, 3 * n + 1, 3, dtype=np.int64),
             left=np.tile(np.array([1, -1, -1], np.int64), n), right=np.tile(np.array([2, -1, -1], np.int64), n),
             feature=np.zeros(3 * n, np.int64), threshold=np.repeat(thr, 3), missing_left=np.zeros(3 * n, np.uint8),
             value1=np.tile(np.array([0.0, 1.0, 0.0]), n))
    R = pack_rank(a)
    f32 = thr.astype(np.float32)
    cand = np.concatenate([np.nextafter(f32, np.float32(np.inf)), f32, np.nextafter(f32, np.float32(-np.inf)),
                           np.array([np.inf, -np.inf, 0.0, -0.0], np.float32)])
    z32 = np.zeros((len(cand), 15), np.float32)
    z32[:, 0] = cand
    _, leaves = walk_rank(R, z32)
    expect = np.stack([(cand.astype(np.float64) <= t) for t in thr], axis=1)
    np.testing.assert_array_equal(leaves == 1, expect)


def test_rank_layout_ineligible_forest_falls_back():
    """> 15 features: no rank layout (the wide layout serves it)."""
    rng = np.random.default_rng(2)
    a = random_forest(rng, 2, 5, n_feat=20)
    assert pack_rank(a, n_features=20) is None


def pack_rank2(a, n_features=15, version=2):
    from fdx import _lib

    L = _lib.load()
    d, keep = _desc(a, n_features)
    nn, nthr, ns = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32()
    rc = L.fdx_forest_rank_layout_size2(ctypes.byref(d), version, ctypes.byref(nn), ctypes.byref(nthr), ctypes.byref(ns))
    if rc != 0:
        return None
    n, nt = nn.value, d.n_trees
    out = dict(nodes=np.zeros(n, np.uint32), orig=np.zeros(n, np.int32), lval=np.zeros(n), ml=np.zeros(n, np.uint8),
               root=np.zeros(nt, np.int32), depth=np.zeros(nt, np.int32), thr=np.zeros(max(nthr.value, 1), np.float32),
               thr_off=np.zeros(33, np.int32), slot_feat=np.zeros(32, np.int32), slot_base=np.zeros(32, np.int32))
    rc = L.fdx_forest_pack_rank2(ctypes.byref(d), version, *[out[k].ctypes.data for k in
                                                             ("nodes", "orig", "lval", "ml", "root", "depth", "thr",
                                                              "thr_off", "slot_feat", "slot_base")])
    assert rc == 0, L.fdx_last_error()
    out["n_slots"] = ns.value
    return out


def walk_rank_v2(R, z32):
    """numpy model of k_forest_rank<.., P16 = 2>: slot s holds the clamped rank
    min(max(r_f - base_s, 0), 32767) of its feature (0xFFFF for NaN), LDS node S = node ^
    0xFFFF0000, d = int32((x << 16) + S), step = med3(d, 1, node & 0x7FF), slot = node[15:11]."""
    n = z32.shape[0]
    xs = np.zeros((n, 32), np.int64)
    for s in range(R["n_slots"]):
        f = R["slot_feat"][s]
        u = R["thr"][R["thr_off"][f]:R["thr_off"][f + 1]]
        r = np.searchsorted(u, z32[:, f], side="left").astype(np.int64)
        xs[:, s] = np.clip(r - R["slot_base"][s], 0, 32767)
        xs[np.isnan(z32[:, f]), s] = 0xFFFF
    nodes = R["nodes"].astype(np.int64)
    acc = np.zeros(n)
    rows = np.arange(n)
    nt = len(R["root"])
    leaves = np.zeros((n, nt), np.int32)
    for t in range(nt):
        p = np.full(n, R["root"][t], np.int64)
        for _ in range(int(R["depth"][t])):
            nd = nodes[p]
            x = xs[rows, (nd >> 11) & 31]
            S = nd ^ 0xFFFF0000
            d = ((x << 16) + S) & 0xFFFFFFFF
            d = np.where(d >= 2**31, d - 2**32, d)
            off = nd & 0x7FF
            st = np.median(np.stack([d, np.ones_like(d), off]), axis=0).astype(np.int64)
            st = np.where(x == 0xFFFF, np.where(R["ml"][p] != 0, 1, off), st)
            p = p + st
        assert ((nodes[p] & 0x7FF) == 0).all(), "walk did not end on leaves within depth"
        acc = acc + R["lval"][p]
        leaves[:, t] = R["orig"][p]
    return acc / nt, leaves


def test_rank_layout_v2_small_forests_match_v1(golden):
    """v2 (slot field, 11-bit offsets, no sentinel) gives sklearn's leaves on the golden forests."""
    for name in ("forest_dt2.npz", "forest_rf5d8.npz", "forest_rf3.npz"):
        z = golden(name)
        R = pack_rank2(z)
        assert R is not None and R["n_slots"] == 15
        proba, leaves = walk_rank_v2(R, _z32(z["X"], z["mean"], z["scale"]))
        np.testing.assert_array_equal(leaves, z["leaves"])
        np.testing.assert_array_equal(proba, z["proba"])


def test_rank_layout_v2_jump_nodes_and_many_thresholds():
    """Deep random trees with more than 32,767 distinct thresholds on feature 0 (two slots)
    and far right subtrees (jumps past the 11-bit offset), NaN rows included: v1 cannot hold
    them, v2 reproduces the oracle."""
    rng = np.random.default_rng(5)
    a = random_forest(rng, 10, 13, p_leaf=0.01)
    internal = a["left"] >= 0
    a["feature"][internal] = 0
    a["threshold"][internal] = rng.normal(size=int(internal.sum()))
    assert len(np.unique(a["threshold"][internal].astype(np.float32))) > 32767
    assert pack_rank(a) is None
    R = pack_rank2(a)
    n0 = len(np.unique(a["threshold"][internal].astype(np.float32)))
    assert R is not None and R["n_slots"] == -(-n0 // 32767) + 14 and R["n_slots"] >= 16
    assert int((R["orig"] == -1).sum()) > 0
    X = rng.normal(size=(3000, 15))
    X[rng.random(X.shape) < 0.05] = np.nan
    op, ol = oracle.forest_predict(X, a, want_leaves=True)
    proba, leaves = walk_rank_v2(R, X.astype(np.float32))
    np.testing.assert_array_equal(leaves, ol)
    np.testing.assert_array_equal(proba, op)


def test_rank_layout_v2_deployed_model():
    """The reference's deployed RandomForestClassifier(random_state=0) (100 unlimited-depth trees,
    bench_assets/rf_deployed.npz, model_training.ipynb:2212): v1 rejects it (features with up to
    96k thresholds), v2 reproduces sklearn's predict_proba of the served pipeline
    (scaler.transform then the forest, fraud_detection.py:190-193) bit for bit."""
    import os

    from conftest import ROOT

    z = np.load(os.path.join(ROOT, "bench_assets", "rf_deployed.npz"))
    assert pack_rank(z) is None
    R = pack_rank2(z)
    assert R is not None and R["n_slots"] <= 32
    sel = np.arange(0, len(z["test_X"]), 16)
    proba, _ = walk_rank_v2(R, _z32(z["test_X"][sel], z["mean"], z["scale"]))
    np.testing.assert_array_equal(proba, z["test_proba1"][sel])


def _search_trees(a):
    from fdx import _lib

    L = _lib.load()
    d, keep = _desc(a, 15)
    nf = ctypes.c_int64()
    eoff, elev = (ctypes.c_int32 * 4)(), (ctypes.c_int32 * 4)()
    assert L.fdx_forest_search_trees(ctypes.byref(d), None, 0, ctypes.byref(nf), eoff, elev) == 0
    trees = np.zeros(max(nf.value, 1), np.float32)
    assert L.fdx_forest_search_trees(ctypes.byref(d), trees.ctypes.data, trees.size, ctypes.byref(nf), eoff,
                                     elev) == 0
    return trees[: nf.value], list(eoff), list(elev)


@pytest.mark.parametrize("which", ["bench", "random"])
def test_search_trees_count_samples(which):
    """k_zfill_grouped_w3's search tables (fdx_forest_search_trees, the same host builder the
    forest object uploads): descending each searched feature's S-tree and counting the 4
    thresholds of the segment it leaves gives lower_bound over the feature's thresholds (the
    rank the forest walk compares), for every threshold, its float32 neighbours, random and
    extreme values."""
    if which == "bench":
        z = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench_assets",
                                 "rf100_d20.npz"))
        a = {k: z[k] for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    else:
        a = random_forest(np.random.default_rng(5), n_trees=12, depth=12)
    trees, eoff, elev = _search_trees(a)
    assert trees.size > 0
    packed = pack_rank(a)
    thr_all, thr_off = packed["thr"], packed["thr_off"]
    rng = np.random.default_rng(11)
    for s, f in enumerate((0, 4, 6, 8)):
        thr = thr_all[thr_off[f]:thr_off[f + 1]].astype(np.float32)
        v = np.concatenate([thr, np.nextafter(thr, np.float32(np.inf)), np.nextafter(thr, np.float32(-np.inf)),
                            rng.normal(0, 3, 5000).astype(np.float32),
                            np.array([-3e38, 3e38, np.inf, -np.inf], np.float32)]).astype(np.float32)
        ek = np.zeros(v.size, np.int64)
        cs = np.zeros(v.size, np.int64)
        for _ in range(elev[s]):
            nd = trees.reshape(-1, 8)[eoff[s] + ek]
            c = (nd < v[:, None]).sum(1)
            cs, ek = cs * 9 + c, ek * 9 + 1 + c
        useg = np.concatenate([thr, np.full(16, np.inf, np.float32)])
        seg = useg[(np.maximum(cs - 1, 0) * 4)[:, None] + np.arange(4)]
        rank = np.where(cs > 0, (cs - 1) * 4 + (seg < v[:, None]).sum(1), 0)
        np.testing.assert_array_equal(rank, np.searchsorted(thr, v, side="left"))
