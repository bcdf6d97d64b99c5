"""HIP kernels (through the C ABI) vs the CPU oracle and the reference's golden vectors.

Bar: bit-exact for counts, flags, permutations, leaf ids; float64 averages / risks /
probabilities are also required bit-exact here (the kernels emulate pandas' Kahan
roll_sum and sklearn's float32 traversal exactly), which is stricter than the 1e-6
relative tolerance north_star allows.
"""
import numpy as np
import pytest
import torch

import oracle
from record_decode import unpack_term_records
from forest_gen import random_forest
from fdx import ops
from fdx.pipeline import FraudPipeline

pytestmark = pytest.mark.gpu

DAY = 86_400 * 10**9
HOUR = 3600 * 10**9


def T(a, dtype, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=dev, dtype=dtype)


# ----------------------------------------------------------------------------- flags
@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 1000, 100_003])
def test_time_flags(dev, n):
    rng = np.random.default_rng(n)
    ts = rng.integers(-400 * DAY, 20_000 * DAY, size=n, dtype=np.int64)
    if n >= 8:  # hour / day boundaries
        ts[:4] = [0, 7 * HOUR - 1, 7 * HOUR, 20 * HOUR]
        ts[4:8] = [-1, -DAY, 6 * HOUR + 59 * 60 * 10**9, DAY - 1]
    for mode, wf, nf in ((0, oracle.weekend_flag, oracle.night_flag),
                         (1, oracle.spark_weekend_flag, oracle.spark_night_flag)):
        we, ni = ops.time_flags(T(ts, torch.int64, dev), mode)
        np.testing.assert_array_equal(we.cpu().numpy(), wf(ts))
        np.testing.assert_array_equal(ni.cpu().numpy(), nf(ts))


# ---------------------------------------------------------------------------- re-key
@pytest.mark.parametrize("n,n_keys", [(0, 5), (1, 1), (5000, 1), (4096, 256), (4097, 257),
                                      (100_000, 50_000), (300_001, 100_000), (2_000_000, 1 << 21),
                                      (200_000, 1 << 18), (70_000, 1 << 25)])  # 9-bit digits: 2 and 3 passes
def test_rekey_stable(dev, n, n_keys):
    rng = np.random.default_rng(n + n_keys)
    keys = rng.integers(0, n_keys, size=n).astype(np.int32)
    perm, seg, sk = ops.rekey(T(keys, torch.int32, dev), n_keys, want_sorted_keys=True)
    ref = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(perm.cpu().numpy(), ref)
    np.testing.assert_array_equal(sk.cpu().numpy(), keys[ref])
    np.testing.assert_array_equal(seg.cpu().numpy(), np.r_[0, np.cumsum(np.bincount(keys, minlength=n_keys))])
    if n:  # the histogram form (no sort) gives the same offsets; out-of-range keys are counted
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        np.testing.assert_array_equal(ops.key_segments(T(keys, torch.int32, dev), n_keys, bad=bad).cpu().numpy(),
                                      seg.cpu().numpy())
        assert int(bad.item()) == 0
        k2 = keys.copy()
        k2[::3] = -1 - k2[::3]
        ops.key_segments(T(k2, torch.int32, dev), n_keys, bad=bad)
        assert int(bad.item()) == len(k2[::3])
    # the checked re-key counts the same keys inside its first histogram pass (and still groups)
    bad = torch.full((1,), 77, dtype=torch.int32, device=dev)
    pp, sp, _, _ = ops.rekey_payload(T(keys, torch.int32, dev), n_keys, bad=bad)
    np.testing.assert_array_equal(pp.cpu().numpy(), ref)
    np.testing.assert_array_equal(sp.cpu().numpy(), seg.cpu().numpy())
    assert int(bad.item()) == 0
    if n:
        k3 = keys.copy()
        k3[::5] = -1 - k3[::5]                       # negative ids
        k3[1::7] = n_keys + k3[1::7] % 3             # ids at and just past n_keys
        k3[2::11] = np.int32(2**31 - 1)              # the largest int32
        exp = int(np.count_nonzero((k3 < 0) | (k3 >= n_keys)))
        ops.rekey_payload(T(k3, torch.int32, dev), n_keys, T(np.arange(n, dtype=np.int64), torch.int64, dev), bad=bad)
        assert int(bad.item()) == exp


def test_rekey_sorted_keys_unaligned_output(dev):
    """fdx_rekey with the caller's sorted_keys_d 4 bytes off a 16-byte boundary: the segment
    offsets come from the scalar boundary pass (the 4-keys-per-thread one needs alignment)."""
    from fdx import _lib

    rng = np.random.default_rng(11)
    n, n_keys = 100_003, 3_000
    keys = rng.integers(0, n_keys, size=n).astype(np.int32)
    L = _lib.load()
    kb = ops.key_bits_for(n_keys)
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    seg = torch.empty(n_keys + 1, dtype=torch.int64, device=dev)
    skbuf = torch.empty(n + 4, dtype=torch.int32, device=dev)
    ws = ops.workspace(L.fdx_rekey_workspace_size(n, kb), dev)
    kd = T(keys, torch.int32, dev)
    ops.check(L.fdx_rekey(ops._ptr(kd), n, kb, n_keys, ops._ptr(perm),
                          skbuf.data_ptr() + 4, ops._ptr(seg), ops._ptr(ws), ws.numel(), None), "fdx_rekey")
    ref = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(perm.cpu().numpy(), ref)
    np.testing.assert_array_equal(skbuf[1:n + 1].cpu().numpy(), keys[ref])
    np.testing.assert_array_equal(seg.cpu().numpy(), np.r_[0, np.cumsum(np.bincount(keys, minlength=n_keys))])


@pytest.mark.parametrize("n,n_keys", [(0, 5), (1, 1), (5000, 1), (100_000, 50_000), (300_001, 100_000)])
def test_rekey_payload_sorted_keys_then_offsets(dev, n, n_keys):
    """fdx_rekey_payload_keys (the fused step's customer re-key: sorted keys to the caller's
    buffer, no offsets) + fdx_segment_offsets_sorted == fdx_rekey_payload with offsets: perm,
    payload, offsets; the id-range count too."""
    rng = np.random.default_rng(n + 3 * n_keys)
    keys = rng.integers(0, n_keys, size=n).astype(np.int32)
    ts = rng.integers(0, 1 << 60, size=n, dtype=np.int64)
    amt = rng.random(n)
    args = (T(keys, torch.int32, dev), n_keys, T(ts, torch.int64, dev), T(amt, torch.float64, dev))
    p0, s0, t0, a0 = ops.rekey_payload(*args)
    sk = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    bad = torch.full((1,), 9, dtype=torch.int32, device=dev)
    p1, s1, t1, a1 = ops.rekey_payload(*args, keys_out=sk, bad=bad)
    assert s1 is None
    seg = ops.segment_offsets_sorted(sk, n_keys, n=n)
    ref = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(p1.cpu().numpy(), ref)
    np.testing.assert_array_equal(p1.cpu().numpy(), p0.cpu().numpy())
    np.testing.assert_array_equal(sk[:n].cpu().numpy(), keys[ref])
    np.testing.assert_array_equal(seg.cpu().numpy(), s0.cpu().numpy())
    np.testing.assert_array_equal(t1.cpu().numpy(), t0.cpu().numpy())
    np.testing.assert_array_equal(a1.cpu().numpy(), a0.cpu().numpy())
    assert int(bad.item()) == 0
    if n:  # a misaligned keys_out is refused
        with pytest.raises(ops.FdxError):
            ops.rekey_payload(*args, keys_out=torch.empty(n + 1, dtype=torch.int32, device=dev)[1:])


@pytest.mark.parametrize("n,n_keys", [(0, 5), (1, 1), (5000, 1), (4097, 257), (100_000, 50_000),
                                      (300_001, 100_000), (70_000, 1 << 25)])  # 8- and 9-bit first digits
def test_rekey_payload_with_first_table_ahead(dev, n, n_keys):
    """fdx_rekey_hist0 (the first pass's scanned table + the id-range count, computed ahead) +
    fdx_rekey_payload_hist0 == fdx_rekey_payload_checked: perm with the packed flag, payload,
    offsets and the count of out-of-range ids."""
    rng = np.random.default_rng(7 * n + n_keys)
    keys = rng.integers(0, n_keys, size=n).astype(np.int32)
    ts = rng.integers(0, 1 << 60, size=n, dtype=np.int64)
    fr = (rng.random(n) < 0.2).astype(np.uint8)
    for k in (keys, np.where(np.arange(n) % 9 == 4, -1 - keys, keys).astype(np.int32)):
        kd = T(k, torch.int32, dev)
        b0 = torch.full((1,), 5, dtype=torch.int32, device=dev)
        b1 = torch.full((1,), 6, dtype=torch.int32, device=dev)
        p0, s0, t0, _ = ops.rekey_payload(kd, n_keys, T(ts, torch.int64, dev), flag=T(fr, torch.uint8, dev), bad=b0)
        h = ops.rekey_hist0(kd, n_keys, bad=b1)
        p1, s1, t1, _ = ops.rekey_payload(kd, n_keys, T(ts, torch.int64, dev), flag=T(fr, torch.uint8, dev), hist0=h)
        assert int(b1.item()) == int(b0.item()) == int(np.count_nonzero((k < 0) | (k >= n_keys)))
        np.testing.assert_array_equal(p1.cpu().numpy(), p0.cpu().numpy())
        np.testing.assert_array_equal(t1.cpu().numpy(), t0.cpu().numpy())
        if int(b0.item()) == 0:  # (with ids out of range the offsets are unspecified: the caller raises)
            np.testing.assert_array_equal(p1.cpu().numpy() & 0x7FFFFFFF, np.argsort(k, kind="stable"))
            np.testing.assert_array_equal(s1.cpu().numpy(), s0.cpu().numpy())


def test_argsort_i64_and_perm_ops(dev):
    rng = np.random.default_rng(3)
    k = rng.integers(-(1 << 62), 1 << 62, size=200_001, dtype=np.int64)
    k[::7] = k[0]  # ties
    perm = ops.argsort_i64(T(k, torch.int64, dev)).cpu().numpy()
    np.testing.assert_array_equal(perm, np.argsort(k, kind="stable"))
    assert not ops.is_sorted_i64(T(k, torch.int64, dev))
    assert ops.is_sorted_i64(T(np.sort(k), torch.int64, dev))
    p = rng.permutation(len(k)).astype(np.int32)
    for dt, tdt in ((np.int64, torch.int64), (np.int32, torch.int32), (np.uint8, torch.uint8)):
        src = k.astype(dt)
        g = ops.gather(T(src, tdt, dev), T(p, torch.int32, dev)).cpu().numpy()
        np.testing.assert_array_equal(g, src[p])
        s = ops.scatter(T(src, tdt, dev), T(p, torch.int32, dev)).cpu().numpy()
        exp = np.empty_like(src)
        exp[p] = src
        np.testing.assert_array_equal(s, exp)


# --------------------------------------------------------------------------- windows
def _gpu_customer(dev, ts, amount, seg, windows=(1, 7, 30)):
    nb, avg = ops.customer_windows(T(ts, torch.int64, dev), T(amount, torch.float64, dev),
                                   T(seg, torch.int64, dev), windows)
    return nb.cpu().numpy(), avg.cpu().numpy()


def _gpu_terminal(dev, ts, fraud, seg, delay=7, windows=(1, 7, 30)):
    nb, risk = ops.terminal_windows(T(ts, torch.int64, dev), T(fraud, torch.uint8, dev),
                                    T(seg, torch.int64, dev), delay, windows)
    return nb.cpu().numpy(), risk.cpu().numpy()


@pytest.mark.parametrize("name", ["tiny_a.npz", "tiny_b.npz"])
def test_windows_match_reference_golden(dev, golden, name):
    z = golden(name)
    o = np.argsort(z["TRANSACTION_ID"], kind="stable")
    cols = {k: z[k][o] for k in z.files}
    order, seg = oracle.group_order(cols["CUSTOMER_ID"], cols["TX_DATETIME"])
    nb, avg = _gpu_customer(dev, cols["TX_DATETIME"][order], cols["TX_AMOUNT"][order], seg)
    for k, w in enumerate((1, 7, 30)):
        np.testing.assert_array_equal(nb[k], cols[f"CUSTOMER_ID_NB_TX_{w}DAY_WINDOW"][order])
        np.testing.assert_array_equal(avg[k], cols[f"CUSTOMER_ID_AVG_AMOUNT_{w}DAY_WINDOW"][order])
    order, seg = oracle.group_order(cols["TERMINAL_ID"], cols["TX_DATETIME"])
    nb, risk = _gpu_terminal(dev, cols["TX_DATETIME"][order], cols["TX_FRAUD"][order].astype(np.uint8), seg)
    for k, w in enumerate((1, 7, 30)):
        np.testing.assert_array_equal(nb[k], cols[f"TERMINAL_ID_NB_TX_{w}DAY_WINDOW"][order])
        np.testing.assert_array_equal(risk[k], cols[f"TERMINAL_ID_RISK_{w}DAY_WINDOW"][order])


def test_customer_windows_ties_reference_order(dev, golden):
    z = golden("ties.npz")
    order = np.lexsort((z["CUSTOMER_ID_NB_TX_1DAY_WINDOW"], z["TX_DATETIME"], z["CUSTOMER_ID"]))
    sk = z["CUSTOMER_ID"][order]
    seg = np.r_[np.flatnonzero(np.r_[True, sk[1:] != sk[:-1]]), len(sk)]
    nb, avg = _gpu_customer(dev, z["TX_DATETIME"][order], z["TX_AMOUNT"][order], seg)
    for k, w in enumerate((1, 7, 30)):
        np.testing.assert_array_equal(nb[k], z[f"CUSTOMER_ID_NB_TX_{w}DAY_WINDOW"][order])
        np.testing.assert_array_equal(avg[k], z[f"CUSTOMER_ID_AVG_AMOUNT_{w}DAY_WINDOW"][order])


def _edge_segments(rng, n_seg, max_len):
    """Segments with ties, gaps exactly equal to the windows, repeated amounts, empties."""
    ts_all, amt_all, fr_all, seg = [], [], [], [0]
    for s in range(n_seg):
        L = int(rng.integers(0, max_len + 1)) if s % 17 else (0 if s % 2 else 1)
        t0 = int(rng.integers(0, 400)) * DAY
        steps = rng.choice([0, 1, HOUR, DAY, 7 * DAY, 8 * DAY, 14 * DAY, 30 * DAY, 37 * DAY,
                            int(rng.integers(1, 3 * DAY))], size=L, p=[.1, .02, .1, .1, .05, .03, .03,
                                                                        .03, .04, .5])
        ts = t0 + np.cumsum(steps)
        amt = np.round(rng.gamma(2.0, 40.0, size=L), 2)
        if s % 5 == 0:
            amt[:] = 12.34  # n-consecutive-equal-values branch of roll_sum
        elif s % 5 == 1:
            amt[rng.random(L) < 0.5] = 7.0
        ts_all.append(ts); amt_all.append(amt); fr_all.append((rng.random(L) < 0.3).astype(np.uint8))
        seg.append(seg[-1] + L)
    return (np.concatenate(ts_all).astype(np.int64), np.concatenate(amt_all), np.concatenate(fr_all),
            np.asarray(seg, np.int64))


@pytest.mark.parametrize("max_len", [3, 300, 2500])
def test_windows_random_edge_cases(dev, max_len):
    rng = np.random.default_rng(max_len)
    ts, amt, fr, seg = _edge_segments(rng, 400 if max_len < 1000 else 40, max_len)
    for windows in ((1, 7, 30), (2, 5)):
        nb, avg = _gpu_customer(dev, ts, amt, seg, windows)
        onb, oavg = oracle.customer_windows(ts, amt, seg, windows)
        np.testing.assert_array_equal(nb, onb)
        np.testing.assert_array_equal(avg, oavg)
        nb, risk = _gpu_terminal(dev, ts, fr, seg, 7, windows)
        onb, orisk = oracle.terminal_windows(ts, fr, seg, 7, windows)
        np.testing.assert_array_equal(nb, onb)
        np.testing.assert_array_equal(risk, orisk)
        gts, gfr, gseg = T(ts, torch.int64, dev), T(fr, torch.uint8, dev), T(seg, torch.int64, dev)
        rec = ops.terminal_windows_grouped(gts, gseg, gfraud=gfr, delay_days=7, windows_days=windows)
        W = len(windows)
        rnb, rrisk = unpack_term_records(rec)
        np.testing.assert_array_equal(rnb, onb)
        np.testing.assert_array_equal(rrisk, orisk)
        # rows=perm: the record of grouped position q lands at row perm[q]
        perm = np.random.default_rng(W).permutation(len(ts)).astype(np.int32)
        rec2 = ops.terminal_windows_grouped(gts, gseg, rows=T(perm, torch.int32, dev), gfraud=gfr, delay_days=7,
                                            windows_days=windows)
        np.testing.assert_array_equal(rec2.cpu().numpy()[perm], rec.cpu().numpy())
        inv = ops.invert_perm(T(perm, torch.int32, dev)).cpu().numpy()
        np.testing.assert_array_equal(inv[perm], np.arange(len(ts)))


# ---------------------------------------------------------------------------- forest
def _forest(golden_z):
    return {k: golden_z[k] for k in ("left", "right", "feature", "threshold", "missing_left", "value1",
                                     "node_offsets")}


@pytest.mark.parametrize("name", ["forest_dt2.npz", "forest_rf5d8.npz", "forest_rf3.npz"])
def test_forest_matches_sklearn_golden(dev, golden, name):
    z = golden(name)
    f = ops.Forest(_forest(z), 15, z["mean"], z["scale"])
    proba, leaves = f.predict(T(z["X"], torch.float64, dev), want_leaves=True)
    np.testing.assert_array_equal(leaves.cpu().numpy(), z["leaves"])
    np.testing.assert_array_equal(proba.cpu().numpy(), z["proba"])
    # column-major input (Spark columns) gives the same answer
    Xc = T(np.asfortranarray(z["X"]).T.copy(), torch.float64, dev).t()
    np.testing.assert_array_equal(f.predict(Xc).cpu().numpy(), z["proba"])


@pytest.mark.parametrize("n_rows", [1, 777, 20_000, 131_072])
def test_forest_small_batch_concurrent_chunks(dev, n_rows):
    """batches that cannot fill the CUs run all LDS chunks in one launch and sum the per-tree
    values in tree order (k_tree_sum): same bits as the chunk-sequential launches (forced by
    a workspace without room for the per-tree values) and as the oracle"""
    rng = np.random.default_rng(n_rows)
    arr = random_forest(rng, 80, 11)
    X = rng.normal(size=(n_rows, 15))
    X[rng.random(X.shape) < 0.01] = np.nan
    mean, scale = rng.normal(size=15) * 0.1, rng.uniform(0.5, 2.0, size=15)
    f = ops.Forest(arr, 15, mean, scale)
    assert f.n_chunks >= 2
    Xd = T(X, torch.float64, dev)
    p1, l1 = f.predict(Xd, want_leaves=True)                      # full workspace: concurrent chunks
    base = 4 * 16 * n_rows + 8 * n_rows + 1024
    ws = ops.workspace(base, dev)
    assert ws.numel() < f.workspace_size(n_rows)
    p2, l2 = f.predict(Xd, want_leaves=True, ws=ws)              # sequential chunk launches
    np.testing.assert_array_equal(p1.cpu().numpy(), p2.cpu().numpy())
    np.testing.assert_array_equal(l1.cpu().numpy(), l2.cpu().numpy())
    if n_rows <= 20_000:
        op, ol = oracle.forest_predict(X, arr, mean, scale, want_leaves=True)
        np.testing.assert_array_equal(p1.cpu().numpy(), op)
        np.testing.assert_array_equal(l1.cpu().numpy(), ol)


@pytest.mark.parametrize("n_trees,depth", [(60, 10), (2, 15)])
def test_forest_chunks_and_global_path(dev, n_trees, depth):
    rng = np.random.default_rng(depth)
    arr = random_forest(rng, n_trees, depth)
    X = rng.normal(size=(20_000, 15))
    X[rng.random(X.shape) < 0.01] = np.nan
    mean, scale = rng.normal(size=15) * 0.1, rng.uniform(0.5, 2.0, size=15)
    op, ol = oracle.forest_predict(X, arr, mean, scale, want_leaves=True)
    for variant in (None, 0):  # default (rank layout) and the wide layout, whose trees spill
        f = ops.Forest(arr, 15, mean, scale)
        if variant is not None:
            f.set_variant(variant)
            assert f.n_chunks >= 2
        proba, leaves = f.predict(T(X, torch.float64, dev), want_leaves=True)
        np.testing.assert_array_equal(leaves.cpu().numpy(), ol)
        np.testing.assert_array_equal(proba.cpu().numpy(), op)


def test_standard_scale(dev, golden):
    z = golden("forest_rf5d8.npz")
    X = z["X"]
    out = ops.standard_scale(T(X, torch.float64, dev), T(z["mean"], torch.float64, dev),
                             T(z["scale"], torch.float64, dev)).cpu().numpy()
    np.testing.assert_array_equal(out, (X - z["mean"]) / z["scale"])


# -------------------------------------------------------------------------- pipeline
@pytest.mark.parametrize("shuffle", [False, True])
def test_pipeline_matches_reference_golden(dev, golden, shuffle):
    z = golden("tiny_a.npz")
    o = np.argsort(z["TRANSACTION_ID"], kind="stable")
    if shuffle:
        o = np.random.default_rng(0).permutation(o)
    cols = {k: z[k][o] for k in z.files}
    pipe = FraudPipeline()
    f = pipe.featurize(T(cols["TX_DATETIME"], torch.int64, dev), T(cols["CUSTOMER_ID"], torch.int32, dev),
                       T(cols["TERMINAL_ID"], torch.int32, dev), T(cols["TX_AMOUNT"], torch.float64, dev),
                       T(cols["TX_FRAUD"], torch.uint8, dev), int(cols["CUSTOMER_ID"].max()) + 1,
                       int(cols["TERMINAL_ID"].max()) + 1, time_sort=shuffle)
    X = f.X.cpu().numpy()
    feats = ["TX_AMOUNT", "TX_DURING_WEEKEND", "TX_DURING_NIGHT"] + oracle.CUSTOMER_COLS + oracle.TERMINAL_COLS
    for j, c in enumerate(feats):
        np.testing.assert_array_equal(X[:, j], cols[c].astype(np.float64), err_msg=c)


def test_pipeline_large_sampled_segments(dev):
    """Full-size run (synthetic config-2-shaped data); every customer and terminal segment of
    a random sample is re-computed by the oracle and must match bit for bit, and global
    invariants hold for all rows."""
    from fdx import synth

    data = synth.generate(n_customers=20_000, n_terminals=40_000, nb_days=183, seed=5)
    n = len(data["ts"])
    pipe = FraudPipeline()
    f = pipe.featurize(T(data["ts"], torch.int64, dev), T(data["customer"], torch.int32, dev),
                       T(data["terminal"], torch.int32, dev), T(data["amount"], torch.float64, dev),
                       T(data["fraud"], torch.uint8, dev), 20_000, 40_000)
    X = f.X.cpu().numpy()
    assert X.shape == (n, 15)
    # invariants: every row counts itself in its customer windows; nb grows with w
    assert (X[:, 3] >= 1).all() and (X[:, 5] >= X[:, 3]).all() and (X[:, 7] >= X[:, 5]).all()
    assert ((X[:, 10] >= 0) & (X[:, 10] <= 1)).all()
    rng = np.random.default_rng(1)
    for key, cols in (("customer", slice(3, 9)), ("terminal", slice(9, 15))):
        ids = rng.choice(int(data[key].max()) + 1, size=50, replace=False)
        m = np.flatnonzero(np.isin(data[key], ids))
        sub = {k: v[m] for k, v in data.items()}
        of = oracle.featurize_arrays(sub["ts"], sub["customer"], sub["terminal"], sub["amount"], sub["fraud"])
        names = oracle.CUSTOMER_COLS if key == "customer" else oracle.TERMINAL_COLS
        exp = np.stack([of[c] for c in names], axis=1)
        np.testing.assert_array_equal(X[m][:, cols], exp)


@pytest.mark.parametrize("max_len,windows", [(300, (1, 7, 30)), (2500, (1, 7, 30)), (300, (2, 5)), (40, (3,))])
def test_customer_interleaved_layout_matches_oracle(dev, max_len, windows):
    """The pipeline's lane-major customer layout: same bits as the oracle for every row."""
    rng = np.random.default_rng(max_len + len(windows))
    ts, amt, _, seg = _edge_segments(rng, 700 if max_len < 1000 else 60, max_len)
    _check_interleaved(dev, rng, ts, amt, seg, windows)


@pytest.mark.parametrize("max_len", [300, 2500])
def test_customer_walk_nan_amounts_matches_oracle(dev, max_len):
    """NaN amounts (pandas leaves them out of count and sum) arriving mid-segment: a walk wave
    takes the NaN-free remove loop until it first stages a NaN, the NaN-skipping one after; the
    NaN rows then leave the windows from the LDS ring and, past 128 / 256 rows, from HBM.  -NaN
    (sign bit set) in half the segments that get NaNs; two thirds of the segments get none."""
    rng = np.random.default_rng(11 + max_len)
    ts, amt, _, seg = _edge_segments(rng, 700 if max_len < 1000 else 60, max_len)
    for s in range(0, len(seg) - 1, 3):
        a, b = int(seg[s]), int(seg[s + 1])
        if b - a >= 3:
            pos = rng.integers(a + (b - a) // 3, b, size=max(1, (b - a) // 20))
            amt[pos] = np.nan if s % 2 else np.copysign(np.nan, -1.0)
    assert np.isnan(amt).any()
    _check_interleaved(dev, rng, ts, amt, seg, (1, 7, 30))


def _check_interleaved(dev, rng, ts, amt, seg, windows):
    n = len(ts)
    perm = rng.permutation(n).astype(np.int32)          # grouped position -> "time row"
    ts_time = np.empty_like(ts); ts_time[perm] = ts
    amt_time = np.empty_like(amt); amt_time[perm] = amt
    lay = ops.customer_layout(T(seg, torch.int64, dev), T(perm, torch.int32, dev), T(ts_time, torch.int64, dev),
                              T(amt_time, torch.float64, dev), len(windows))
    nb, sm = ops.customer_windows_interleaved(lay, T(seg, torch.int64, dev), windows)
    irow = lay.irow.cpu().numpy()[: lay.n_slots]
    nb, sm = nb.cpu().numpy(), sm.cpu().numpy()
    with np.errstate(all="ignore"):
        avg = sm / nb  # the consumer's float64 division
    onb, oavg = oracle.customer_windows(ts, amt, seg, windows)
    inv = np.empty(n, np.int64); inv[perm] = np.arange(n)   # time row -> grouped position
    real = irow >= 0
    assert real.sum() == n and len(np.unique(irow[real])) == n
    g = inv[irow[real]]
    np.testing.assert_array_equal(nb[:, real], onb[:, g])
    np.testing.assert_array_equal(avg[:, real], oavg[:, g])
    assert lay.n_slots <= n + (64 // len(windows)) * (np.diff(seg).max())


@pytest.mark.parametrize("variant", list(range(6)))
def test_forest_variants_bit_identical(dev, golden, variant):
    """Every traversal kernel shape gives sklearn's leaves and probabilities."""
    z = golden("forest_rf3.npz")
    f = ops.Forest(_forest(z), 15, z["mean"], z["scale"])
    f.set_variant(variant)
    X = np.vstack([z["X"]] * 3)  # > one block of rows per lane slot
    proba, leaves = f.predict(T(X, torch.float64, dev), want_leaves=True)
    np.testing.assert_array_equal(leaves.cpu().numpy(), np.vstack([z["leaves"]] * 3))
    np.testing.assert_array_equal(proba.cpu().numpy(), np.concatenate([z["proba"]] * 3))
    rng = np.random.default_rng(variant)
    arr = random_forest(rng, 24, 9)
    Xr = rng.normal(size=(7000, 15))
    g = ops.Forest(arr, 15)
    g.set_variant(variant)
    p, l = g.predict(T(Xr, torch.float64, dev), want_leaves=True)
    op, ol = oracle.forest_predict(Xr, arr, want_leaves=True)
    np.testing.assert_array_equal(l.cpu().numpy(), ol)
    np.testing.assert_array_equal(p.cpu().numpy(), op)


def test_layout_starts_walk_equals_interleaved(dev):
    """fdx_customer_layout_starts + fdx_customer_windows_walk (window starts found in the
    layout kernel) == fdx_customer_windows_interleaved, bit for bit, incl. a segment longer
    than the 1,024-row LDS stage of the start search."""
    from fdx import synth

    d = synth.generate(n_customers=400, n_terminals=500, nb_days=120, seed=31)
    # one very busy customer: > 1024 rows in its segment
    busy = np.nonzero(d["customer"] < 40)[0]
    cust = d["customer"].copy()
    cust[busy] = 0
    T = lambda a, t: torch.from_numpy(np.ascontiguousarray(a)).to(dev, t)  # noqa: E731
    ts, c, amt = T(d["ts"], torch.int64), T(cust, torch.int32), T(d["amount"], torch.float64)
    cperm, cseg, _ = ops.rekey(c, 400)
    assert int((cseg[1:] - cseg[:-1]).max()) > 1024
    lay = ops.customer_layout(cseg, cperm, ts, amt, 3)
    nb_ref, sm_ref = ops.customer_windows_interleaved(lay, cseg)
    lay2 = ops.customer_layout(cseg, cperm, ts, amt, 3, windows_days=(1, 7, 30))
    nb, sm = ops.customer_windows_walk(lay2, cseg)
    n = lay.n_slots
    valid = (lay.irow[:n] >= 0).cpu().numpy()
    np.testing.assert_array_equal(nb.cpu().numpy()[:, valid], nb_ref.cpu().numpy()[:, valid])
    np.testing.assert_array_equal(sm.cpu().numpy()[:, valid], sm_ref.cpu().numpy()[:, valid])


def test_layout_plan_fill_equals_layout(dev):
    """fdx_customer_layout_plan (from fdx_key_segments' offsets, no sort) + _fill_starts_grouped
    == fdx_customer_layout_starts_grouped: same segment order, slots, rows and window starts
    (absent customers and a segment longer than the 1,024-row LDS stage included)."""
    from fdx import synth

    d = synth.generate(n_customers=400, n_terminals=500, nb_days=120, seed=32)
    cust = d["customer"].copy()
    cust[cust < 40] = 0
    T = lambda a, t: torch.from_numpy(np.ascontiguousarray(a)).to(dev, t)  # noqa: E731
    ts, c, amt = T(d["ts"], torch.int64), T(cust, torch.int32), T(d["amount"], torch.float64)
    cperm, cseg, gts, gamt = ops.rekey_payload(c, 400, ts, amt)
    ref = ops.customer_layout(cseg, cperm, gts, gamt, 3, windows_days=(1, 7, 30), grouped=True)
    seg2 = ops.key_segments(c, 400)
    assert torch.equal(seg2, cseg)
    plan = ops.customer_layout_plan(seg2, 3)
    lay = ops.customer_layout_fill(plan, seg2, cperm, gts, gamt, (1, 7, 30))
    m = ref.n_slots
    assert lay.n_slots == m
    for a, b in ((lay.sorder, ref.sorder), (lay.goff, ref.goff), (lay.its[:m], ref.its[:m]),
                 (lay.iamt[:m], ref.iamt[:m]), (lay.irow[:m], ref.irow[:m])):
        assert torch.equal(a, b)
    valid = (ref.irow[:m] >= 0)
    # the window starts (segment-contiguous, padding unwritten) through the walk that reads them
    for x, y in zip(ops.customer_windows_walk(lay, seg2), ops.customer_windows_walk(ref, cseg)):
        assert torch.equal(x[:, valid], y[:, valid])


@pytest.mark.parametrize("case", ["short", "long", "too_many_long", "ragged", "w4"])
def test_layout_plan_order(dev, case):
    """fdx_customer_layout_plan's one-launch plan == the radix plan's order: segments by
    decreasing length (clamped at 65535), ties by index; group slot offsets and count.  Long
    segments (>= 2047 rows) are ranked exactly; more than 512 of them take the radix path."""
    rng = np.random.default_rng(7)
    if case == "short":
        lens = rng.integers(0, 800, size=50_000)
    elif case == "long":
        lens = np.r_[rng.integers(0, 2100, size=20_000), rng.integers(2040, 70_000, size=300), [70_000] * 3]
        rng.shuffle(lens)
    elif case == "w4":
        lens = rng.integers(0, 300, size=60_000)
    elif case == "too_many_long":
        lens = np.r_[rng.integers(0, 50, size=3_000), rng.integers(2047, 2200, size=600)]
        rng.shuffle(lens)
    else:
        lens = rng.integers(0, 5, size=65_536)
    W = 4 if case == "w4" else 3  # 4 windows: 16 segments per group, more groups than the one-launch plan holds
    seg = np.r_[0, np.cumsum(lens)].astype(np.int64)
    plan = ops.customer_layout_plan(T(seg, torch.int64, dev), W)
    exp = np.argsort(65535 - np.minimum(lens, 65535), kind="stable")
    n = len(lens)
    np.testing.assert_array_equal(plan.sorder.cpu().numpy()[:n], exp)
    S = 64 // W
    gslots = S * lens[exp[::S]]
    np.testing.assert_array_equal(plan.goff.cpu().numpy()[: len(gslots) + 1].astype(np.int64),
                                  np.r_[0, np.cumsum(gslots)])
    assert plan.n_slots == gslots.sum()
    pa = ops.customer_layout_plan_async(T(seg, torch.int64, dev), W).result()  # incl. its fallback
    assert pa.n_slots == plan.n_slots and torch.equal(pa.sorder[:n], plan.sorder[:n])
    assert torch.equal(pa.goff[: len(gslots) + 1], plan.goff[: len(gslots) + 1])


@pytest.mark.parametrize("compact", [False, True])
def test_fused_scoring_rank_table_overflows(dev, compact):
    """The scoring-row assembly of the fused path (k_zfill_grouped_w3: integer rank table for
    counts < 256, ratio table for terminal windows with NB < 128, searched otherwise; 24-byte
    or compact terminal records) scores bit-identically to the float64-X path (full two-level
    search of every feature) when customer counts reach >= 256 and terminal counts >= 128,
    with thresholds placed there."""
    from fdx import synth

    d = synth.generate(n_customers=400, n_terminals=500, nb_days=60, seed=41)
    rng = np.random.default_rng(3)
    cust, term = d["customer"].copy(), d["terminal"].copy()
    day = (d["ts"] - d["ts"].min()) // DAY
    cust[rng.choice(np.flatnonzero((day >= 10) & (day < 40)), 700, replace=False)] = 0
    term[rng.choice(np.flatnonzero((day >= 5) & (day < 45)), 900, replace=False)] = 0
    arrays = random_forest(np.random.default_rng(5), 12, 9)
    mean = np.array([50, .5, .5, 2, 50, 10, 50, 280, 50, 20, .1, 130, .1, 150, .1], np.float64)
    scale = np.array([30, .5, .5, 2, 30, 10, 30, 30, 30, 10, .1, 20, .1, 20, .1], np.float64)
    forest = ops.Forest(arrays, 15, mean, scale)
    args = (T(d["ts"], torch.int64, dev), T(cust, torch.int32, dev), T(term, torch.int32, dev),
            T(d["amount"], torch.float64, dev), T(d["fraud"], torch.uint8, dev))
    n = len(d["ts"])
    pipe = FraudPipeline(forest=forest, compact_records=compact)
    f, p_ref = pipe.run(*args, 400, 500)
    X = f.X.cpu().numpy()
    assert X[:, 7].max() >= 256 and X[:, 13].max() >= 128  # both table overflows occur
    ws = ops.workspace(forest.workspace_size(n * 11 // 10), dev)
    p1 = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, 400, 500, p1, ws)
    np.testing.assert_array_equal(p1.cpu().numpy(), p_ref.cpu().numpy())
    np.testing.assert_array_equal(p_ref.cpu().numpy(), oracle.forest_predict(X, arrays, mean, scale))


def test_fused_scoring_nan_amounts(dev):
    """NaN amounts through the fused path: the assembly's NaN flag routes the traversal through
    missing_go_to_left, equal to the float64-X path."""
    from fdx import synth

    d = synth.generate(n_customers=300, n_terminals=400, nb_days=40, seed=43)
    amt = d["amount"].copy()
    amt[np.random.default_rng(1).choice(len(amt), 25, replace=False)] = np.nan
    arrays = random_forest(np.random.default_rng(8), 8, 7)
    mean, scale = np.zeros(15), np.ones(15)
    forest = ops.Forest(arrays, 15, mean, scale)
    args = (T(d["ts"], torch.int64, dev), T(d["customer"], torch.int32, dev), T(d["terminal"], torch.int32, dev),
            T(amt, torch.float64, dev), T(d["fraud"], torch.uint8, dev))
    n = len(d["ts"])
    pipe = FraudPipeline(forest=forest)
    f, p_ref = pipe.run(*args, 300, 400)
    assert np.isnan(f.X.cpu().numpy()[:, 0]).sum() == 25
    p = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, 300, 400, p, ops.workspace(forest.workspace_size(n * 11 // 10), dev))
    np.testing.assert_array_equal(p.cpu().numpy(), p_ref.cpu().numpy())


def test_negative_nan_in_the_s_tree_searches(dev):
    """a NaN with its sign bit set (what x86 0/0 or inf - inf give) in the four
    features the S-trees rank (amount and the three customer averages), with the bench model
    (whose four continuous features are searched by S-trees): through fdx_forest_predict
    (k_prepare_st) against the oracle, and through the fused step (k_zfill_grouped_w3) against
    the float64 path.  [a < NaN] by the sign of a - NaN was 1 for every key there, the descent
    counted past the samples and the segment read left the feature's thresholds."""
    import os

    from fdx import synth

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    z = np.load(os.path.join(root, "bench_assets", "rf100_d20.npz"))
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    neg_nan = np.copysign(np.nan, -1.0)
    assert np.signbit(neg_nan)
    X = z["check_X"].copy()
    rng = np.random.default_rng(5)
    for f in (0, 4, 6, 8):
        X[rng.random(len(X)) < 0.1, f] = neg_nan
    assert np.signbit(X[np.isnan(X)]).all()
    got = forest.predict(T(X, torch.float64, dev)).cpu().numpy()
    np.testing.assert_array_equal(got, oracle.forest_predict(X, arrays, z["mean"], z["scale"]))
    # the fused step: -NaN amounts (and the customer averages they make NaN)
    d = synth.generate(n_customers=300, n_terminals=400, nb_days=40, seed=44)
    amt = d["amount"].copy()
    amt[rng.choice(len(amt), 40, replace=False)] = neg_nan
    args = (T(d["ts"], torch.int64, dev), T(d["customer"], torch.int32, dev), T(d["terminal"], torch.int32, dev),
            T(amt, torch.float64, dev), T(d["fraud"], torch.uint8, dev))
    n = len(d["ts"])
    pipe = FraudPipeline(forest=forest)
    f, p_ref = pipe.run(*args, 300, 400)
    assert np.isnan(f.X.cpu().numpy()[:, 0]).sum() == 40
    np.testing.assert_array_equal(p_ref.cpu().numpy(),
                                  oracle.forest_predict(f.X.cpu().numpy(), arrays, z["mean"], z["scale"]))
    p = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, 300, 400, p, ops.workspace(forest.workspace_size(n * 11 // 10), dev))
    np.testing.assert_array_equal(p.cpu().numpy(), p_ref.cpu().numpy())


@pytest.mark.parametrize("variant", [1, 3])
def test_fused_scoring_every_rank_format(dev, golden, variant):
    """The fused scoring path (rank rows prepared in-pipeline) on each rank node format the
    fused rows serve -- v1 (1) and compact v2 (3) -- equals
    featurize + float64 X + predict on the wide layout (variant 0)."""
    from fdx import synth
    from fdx.pipeline import FraudPipeline

    z = golden("forest_rf5d8.npz")
    f = ops.Forest(_forest(z), 15, z["mean"], z["scale"])
    d = synth.generate(n_customers=1500, n_terminals=3000, nb_days=50, seed=17)
    args = (T(d["ts"], torch.int64, dev), T(d["customer"], torch.int32, dev), T(d["terminal"], torch.int32, dev),
            T(d["amount"], torch.float64, dev), T(d["fraud"], torch.uint8, dev))
    n = len(d["ts"])
    pipe = FraudPipeline(forest=f)
    f.set_variant(0)
    _, p_ref = pipe.run(*args, 1500, 3000)
    f.set_variant(variant)
    p = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, 1500, 3000, p, ops.workspace(f.workspace_size(n * 2), dev))
    np.testing.assert_array_equal(p.cpu().numpy(), p_ref.cpu().numpy())


def test_terminal_windows_caller_workspace_abi(dev):
    """fdx_terminal_windows through ctypes with a caller workspace (the call allocates
    nothing): a workspace below fdx_terminal_windows_workspace_size(n) is refused with
    FDX_E_WORKSPACE, the sized one gives the oracle's windows -- incl. a segment longer than
    the kernel's 1,024-row LDS stage (its prefix counts live in the workspace)."""
    import ctypes

    from fdx import _lib

    rng = np.random.default_rng(77)
    ts, _, fr, seg = _edge_segments(rng, 30, 2500)
    assert np.diff(seg).max() > 1024
    n, W = len(ts), 3
    L = _lib.load()
    need = L.fdx_terminal_windows_workspace_size(n)
    assert need >= 4 * n
    win = (ctypes.c_int64 * W)(*[d * 86_400 * 10**9 for d in (1, 7, 30)])
    tsd, frd, segd = T(ts, torch.int64, dev), T(fr, torch.uint8, dev), T(seg, torch.int64, dev)
    nb = torch.empty((W, n), dtype=torch.int32, device=dev)
    risk = torch.empty((W, n), dtype=torch.float64, device=dev)
    small = torch.empty(need - 256, dtype=torch.uint8, device=dev)
    args = lambda ws: (ops._ptr(tsd), ops._ptr(frd), ops._ptr(segd), len(seg) - 1, n, 7 * 86_400 * 10**9, win, W,  # noqa: E731
                       ops._ptr(nb), ops._ptr(risk), ops._ptr(ws), ws.numel(), ops._s())
    assert L.fdx_terminal_windows(*args(small)) == -4  # FDX_E_WORKSPACE
    assert b"workspace" in L.fdx_last_error()
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    assert L.fdx_terminal_windows(*args(ws)) == 0
    onb, orisk = oracle.terminal_windows(ts, fr, seg, 7, (1, 7, 30))
    np.testing.assert_array_equal(nb.cpu().numpy(), onb)
    np.testing.assert_array_equal(risk.cpu().numpy(), orisk)
