"""The payload-carrying re-key and the grouped-input window kernels (round 2): the scoring
pipeline now moves ts / amount (customer side) and ts + TX_FRAUD (terminal side) through the
radix passes, so the window kernels read every segment sequentially.

fdx_rekey_payload: perm = numpy stable argsort (| fraud << 31), seg offsets, both payload
streams = the gathered columns, for 1 / 2 / 3 radix passes and tile-edge sizes.
fdx_terminal_windows_grouped: records / columns against the C oracle, incl. segments longer
than the 1,024-row LDS stage (a hot terminal, O(L log L) path with the prefix scratch),
segments of several time-sorted runs (the multi-GPU owner side) and more runs than the per-run
search handles.  fdx_customer_layout_starts_grouped: identical layout to the gathering form,
its tiled copy for 1 / 2 / 4 windows (empty customers, a hot one past the start stage) and its
window starts against numpy's searchsorted."""
import numpy as np
import pytest
import torch

import oracle
from record_decode import compact_records_unpack, unpack_term_records
from fdx import ops, synth
from fdx.pipeline import FraudPipeline

pytestmark = pytest.mark.gpu
DAY = 86_400 * 10**9


def T(a, dtype, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=dev, dtype=dtype)


@pytest.mark.parametrize("n,n_keys", [(1, 1), (4096, 256), (4097, 257), (300_001, 100_000), (200_000, 1 << 18),
                                      (70_000, 1 << 25), (1_000_000, 50_000)])
def test_rekey_payload(dev, n, n_keys):
    rng = np.random.default_rng(n ^ n_keys)
    keys = rng.integers(0, n_keys, size=n).astype(np.int32)
    p0 = rng.integers(-(1 << 62), 1 << 62, size=n, dtype=np.int64)
    p1 = rng.normal(size=n)
    fl = (rng.random(n) < 0.3).astype(np.uint8)
    ref = np.argsort(keys, kind="stable")
    seg_ref = np.r_[0, np.cumsum(np.bincount(keys, minlength=n_keys))]
    for flag in (None, fl):
        perm, seg, o0, o1 = ops.rekey_payload(T(keys, torch.int32, dev), n_keys, T(p0, torch.int64, dev),
                                              T(p1, torch.float64, dev),
                                              None if flag is None else T(flag, torch.uint8, dev))
        pm = perm.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        np.testing.assert_array_equal(pm & 0x7FFFFFFF, ref)
        np.testing.assert_array_equal(pm >> 31, 0 if flag is None else fl[ref])
        np.testing.assert_array_equal(seg.cpu().numpy(), seg_ref)
        np.testing.assert_array_equal(o0.cpu().numpy(), p0[ref])
        np.testing.assert_array_equal(o1.cpu().numpy(), p1[ref])
    perm, seg, o0, o1 = ops.rekey_payload(T(keys, torch.int32, dev), n_keys, T(p0, torch.int64, dev))
    assert o1 is None
    np.testing.assert_array_equal(o0.cpu().numpy(), p0[ref])


def _oracle_records(ts, fraud, term, n_terms, W=(1, 7, 30)):
    order, seg = oracle.group_order(term, ts)
    nb, risk = oracle.terminal_windows(ts[order], fraud[order], seg, 7, W)
    fr = np.rint(risk * nb).astype(np.int64)
    rec = np.zeros((len(ts), len(W)), np.int64)
    rec[order] = (nb.astype(np.int64) | (fr << 32)).T
    return rec


def _hot_table(rng, n_terms=40, rows_hot=6000, rows_cold=4000, days=60):
    """terminal 0 is hot (far more rows than the 1,024-row LDS stage); the others are small"""
    ts = np.concatenate([rng.integers(0, days * DAY, rows_hot), rng.integers(0, days * DAY, rows_cold)])
    ts = (ts // 10**9) * 10**9  # whole seconds: ties
    term = np.concatenate([np.zeros(rows_hot, np.int32), rng.integers(1, n_terms, rows_cold).astype(np.int32)])
    fraud = (rng.random(len(ts)) < 0.2).astype(np.uint8)
    o = np.argsort(ts, kind="stable")
    return ts[o].astype(np.int64), term[o], fraud[o]


def test_terminal_grouped_hot_terminal_records_and_columns(dev):
    rng = np.random.default_rng(21)
    ts, term, fraud = _hot_table(rng)
    ref = _oracle_records(ts, fraud, term, 40)
    perm, seg, gts, _ = ops.rekey_payload(T(term, torch.int32, dev), 40, T(ts, torch.int64, dev),
                                          flag=T(fraud, torch.uint8, dev))
    rec = ops.terminal_windows_grouped(gts, seg, rows=perm).cpu().numpy()
    np.testing.assert_array_equal(rec, ref)
    # column form at grouped positions, fraud from a grouped byte column
    p = perm.cpu().numpy() & 0x7FFFFFFF
    nb, risk = ops.terminal_windows_grouped(gts, seg, gfraud=T(fraud[p], torch.uint8, dev), records=False)
    onb, orisk = unpack_term_records(ref[p])
    np.testing.assert_array_equal(nb.cpu().numpy(), onb)
    np.testing.assert_array_equal(risk.cpu().numpy(), orisk)


@pytest.mark.parametrize("parts", [1, 3, 8, 100])
def test_terminal_grouped_runs_hot_terminal(dev, parts):
    """owner side: the receive buffer holds one time-sorted run per source part; the hot
    terminal's segment (> 1,024 rows) is cut into `parts` runs (100 > the per-run search's 64:
    direct counts)."""
    rng = np.random.default_rng(parts)
    ts, term, fraud = _hot_table(rng, rows_hot=3000 if parts == 100 else 6000)
    ref = _oracle_records(ts, fraud, term, 40)
    src = rng.integers(0, parts, len(ts))
    order = np.argsort(src, kind="stable")  # receive buffer: grouped by source, time order inside
    perm, seg, gts, _ = ops.rekey_payload(T(term[order], torch.int32, dev), 40, T(ts[order], torch.int64, dev),
                                          flag=T(fraud[order], torch.uint8, dev))
    rec = ops.terminal_windows_grouped(gts, seg, rows=perm, runs=True).cpu().numpy()
    np.testing.assert_array_equal(rec, ref[order])


def test_customer_layout_grouped_equals_gathering_form(dev):
    d = synth.generate(3000, 6000, 90, seed=8)
    ts, amt = T(d["ts"], torch.int64, dev), T(d["amount"], torch.float64, dev)
    cust = T(d["customer"], torch.int32, dev)
    cperm, cseg, _ = ops.rekey(cust, 3000)
    a = ops.customer_layout(cseg, cperm, ts, amt, 3, windows_days=(1, 7, 30))
    perm2, seg2, gts, gamt = ops.rekey_payload(cust, 3000, ts, amt)
    assert torch.equal(perm2, cperm) and torch.equal(seg2, cseg)
    b = ops.customer_layout(cseg, cperm, gts, gamt, 3, windows_days=(1, 7, 30), grouped=True)
    assert a.n_slots == b.n_slots
    for k in ("its", "iamt", "irow"):
        assert torch.equal(getattr(a, k)[: a.n_slots], getattr(b, k)[: b.n_slots]), k
    # the window starts (only defined for real rows; padding entries are never written):
    # compare what the walk computes from them
    valid = (a.irow[: a.n_slots] >= 0).cpu().numpy()
    for x, y in zip(ops.customer_windows_walk(a, cseg), ops.customer_windows_walk(b, cseg)):
        np.testing.assert_array_equal(x.cpu().numpy()[:, valid], y.cpu().numpy()[:, valid])


@pytest.mark.parametrize("days", [(1,), (1, 7), (1, 7, 30, 60)])
def test_customer_layout_grouped_tiles_and_starts(dev, days):
    """The grouped fill's tiled copy (R = 1,024 / S rows of each of a group's S = 64 / W
    segments per tile) equals the gathering form's row-at-a-time copy for 1 / 2 / 4 windows,
    with empty customers and a hot one longer than the 1,024-row start stage; every window
    start equals numpy's searchsorted over the customer's time-sorted rows (first row with
    ts > ts_t - window: the variable-window start of `feature_transformation.ipynb:613-614`)."""
    rng = np.random.default_rng(len(days))
    n, n_cust = 40_000, 700
    ts = np.sort(rng.integers(0, 90 * 86_400, n)) * 10**9  # the table in time order
    cust = rng.integers(0, 600, n)  # customers 600..699 have no rows
    cust[rng.choice(n, 1_500, replace=False)] = 5
    amt = np.round(rng.random(n) * 100, 2)
    perm, seg, gts, gamt = ops.rekey_payload(T(cust, torch.int32, dev), n_cust, T(ts, torch.int64, dev),
                                             T(amt, torch.float64, dev))
    W = len(days)
    a = ops.customer_layout(seg, perm, T(ts, torch.int64, dev), T(amt, torch.float64, dev), W, windows_days=days)
    b = ops.customer_layout(seg, perm, gts, gamt, W, windows_days=days, grouped=True)
    m = b.n_slots
    assert a.n_slots == m
    for k in ("its", "iamt", "irow"):
        assert torch.equal(getattr(a, k)[:m], getattr(b, k)[:m]), k
    seg_np, gts_np = seg.cpu().numpy(), gts.cpu().numpy()
    sorder, goff, st = b.sorder.cpu().numpy(), b.goff.cpu().numpy(), b.starts.cpu().numpy()
    S = 64 // W
    checked = 0
    for g in range(len(goff) - 1):
        segs = sorder[g * S:min((g + 1) * S, n_cust)]
        Lg = seg_np[segs[0] + 1] - seg_np[segs[0]]
        for l, s in enumerate(segs):
            tss = gts_np[seg_np[s]:seg_np[s + 1]]
            for w, d in enumerate(days):
                exp = np.searchsorted(tss, tss - d * DAY, side="right")
                o = w * m + goff[g] + l * Lg
                np.testing.assert_array_equal(st[o:o + len(tss)], exp)
            checked += len(tss)
    assert checked == n


def test_fused_pipeline_hot_terminal_matches_oracle(dev, golden):
    """run_fused end to end on a table with a hot terminal (> LDS stage): proba equals the
    float64 path and the terminal features equal the oracle."""
    z = golden("forest_rf5d8.npz")
    arrays = {k: z[k] for k in ("left", "right", "feature", "threshold", "missing_left", "value1", "node_offsets")}
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    rng = np.random.default_rng(5)
    ts, term, fraud = _hot_table(rng)
    cust = rng.integers(0, 300, len(ts)).astype(np.int32)
    amt = np.round(rng.uniform(1, 300, len(ts)), 2)
    args = (T(ts, torch.int64, dev), T(cust, torch.int32, dev), T(term, torch.int32, dev), T(amt, torch.float64, dev),
            T(fraud, torch.uint8, dev))
    pipe = FraudPipeline(forest=forest)
    f, p64 = pipe.run(*args, 300, 40)
    proba = torch.empty(len(ts), dtype=torch.float64, device=dev)
    pipe.run_fused(*args, 300, 40, proba)
    np.testing.assert_array_equal(proba.cpu().numpy(), p64.cpu().numpy())
    ref = oracle.featurize_arrays(ts, cust, term, amt, fraud)
    X = f.X.cpu().numpy()
    for j, c in enumerate(oracle.TERMINAL_COLS):
        np.testing.assert_array_equal(X[:, 9 + j], ref[c], err_msg=c)
    for j, c in enumerate(oracle.CUSTOMER_COLS):
        np.testing.assert_array_equal(X[:, 3 + j], ref[c], err_msg=c)


def test_compact_records_equal_full_records(dev):
    """fdx_terminal_windows_grouped_compact: the 16-byte records unpack to the full count
    records (oracle), for the sorted single-run form and the multi-run owner form."""
    rng = np.random.default_rng(33)
    ts, term, fraud = _hot_table(rng)
    ref = _oracle_records(ts, fraud, term, 40)
    perm, seg, gts, _ = ops.rekey_payload(T(term, torch.int32, dev), 40, T(ts, torch.int64, dev),
                                          flag=T(fraud, torch.uint8, dev))
    rec = ops.terminal_windows_compact(gts, seg, rows=perm)
    assert rec.numel() == 5 * len(ts)
    assert not bool((rec[: 2 * len(ts)].view(-1, 2)[:, 0] < 0).any())  # everything fits 21 bits
    np.testing.assert_array_equal(compact_records_unpack(rec, len(ts)), ref)
    src = rng.integers(0, 8, len(ts))
    order = np.argsort(src, kind="stable")
    perm, seg, gts, _ = ops.rekey_payload(T(term[order], torch.int32, dev), 40, T(ts[order], torch.int64, dev),
                                          flag=T(fraud[order], torch.uint8, dev))
    rec = ops.terminal_windows_compact(gts, seg, rows=perm, runs=True)
    np.testing.assert_array_equal(compact_records_unpack(rec, len(ts)), ref[order])


def test_compact_records_overflow_rows(dev, golden):
    """Window counts above 2^21 - 1 (one terminal with 2.2M rows in one day, then later rows
    whose delayed windows hold all of them): those rows escape to full records in the overflow
    area -- exact; the run_fused row assembly reads both kinds."""
    n_hot, n_late = 2_200_000, 300
    rng = np.random.default_rng(44)
    # late rows at 7.6 days: their 1-day delayed window (6.6, 7.6] days back covers every hot row
    ts = np.concatenate([np.sort(rng.integers(0, DAY // 2, n_hot)), 7 * DAY + 6 * DAY // 10 + np.arange(n_late) * 10**9])
    ts = ts.astype(np.int64)
    term = np.zeros(len(ts), np.int32)
    term[rng.random(len(ts)) < 0.001] = 1  # a second, small terminal
    fraud = (rng.random(len(ts)) < 0.01).astype(np.uint8)
    tsd, termd, frd = T(ts, torch.int64, dev), T(term, torch.int32, dev), T(fraud, torch.uint8, dev)
    perm, seg, gts, _ = ops.rekey_payload(termd, 2, tsd, flag=frd)
    full = ops.terminal_windows_grouped(gts, seg, rows=perm)
    rec = ops.terminal_windows_compact(gts, seg, rows=perm)
    n = len(ts)
    esc = (rec[: 2 * n].view(n, 2)[:, 0] < 0).cpu().numpy()
    assert esc.sum() > 0 and esc[:n_hot].sum() == 0
    np.testing.assert_array_equal(compact_records_unpack(rec, n), full.cpu().numpy())
    assert int((full[:, 0] & 0xFFFFFFFF).max()) > (1 << 21)
    z = golden("forest_rf5d8.npz")
    arrays = {k: z[k] for k in ("left", "right", "feature", "threshold", "missing_left", "value1", "node_offsets")}
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    cust = T(rng.integers(0, 100, n).astype(np.int32), torch.int32, dev)
    amt = T(np.round(rng.uniform(1, 300, n), 2), torch.float64, dev)
    pipe = FraudPipeline(forest=forest)
    _, p64 = pipe.run(tsd, cust, termd, amt, frd, 100, 2)
    proba = torch.empty(n, dtype=torch.float64, device=dev)  # the fused path on compact records
    FraudPipeline(forest=forest, compact_records=True).run_fused(tsd, cust, termd, amt, frd, 100, 2, proba)
    assert torch.equal(proba, p64)
