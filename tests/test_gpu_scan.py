"""Customer windows in SCAN mode (the §8(b) `exact|scan` mode flag):
float64 prefix sums instead of pandas' sequential Kahan add/remove recurrence.

The counts are exact; the averages are checked against the reference's own values (golden
frames from the reference notebook) and the C oracle at a relative tolerance of 1e-10 plus
1e-9 absolute (the prefix difference carries ~1e-13 relative error -- it is NOT bit-exact,
by design -- and a window of zero amounts comes out ~1e-13 instead of 0); NaN
amounts, empty customers and segments longer than the kernel's 1,024-row LDS stage are
covered.  Within scan mode everything downstream is exact: the fused scoring path equals
featurize + float64 X + predict bit for bit, and the slot-layout outputs equal the grouped
ones.
"""
import os

import numpy as np
import pytest
import torch

import oracle
from fdx import ops, synth
from fdx.pipeline import FraudPipeline

pytestmark = pytest.mark.gpu
RTOL = 1e-10
ATOL = 1e-9   # a window of zero amounts: pandas 0.0, the prefix difference ~1e-13
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def T(a, dt, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)


def _close(got, ref):
    """equal NaN positions; values within RTOL relative (+ ATOL absolute: the prefix
    difference of a window whose amounts sum to 0 is ~1e-13, not 0)"""
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    m = ~np.isnan(ref)
    np.testing.assert_allclose(got[m], ref[m], rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("name", ["tiny_a.npz", "tiny_b.npz"])
def test_scan_matches_reference_golden(dev, golden, name):
    z = golden(name)
    o = np.argsort(z["TRANSACTION_ID"], kind="stable")
    cols = {k: z[k][o] for k in z.files}
    order, seg = oracle.group_order(cols["CUSTOMER_ID"], cols["TX_DATETIME"])
    nb, avg = ops.customer_windows_scan(T(cols["TX_DATETIME"][order], torch.int64, dev),
                                        T(cols["TX_AMOUNT"][order], torch.float64, dev), T(seg, torch.int64, dev))
    nb, avg = nb.cpu().numpy(), avg.cpu().numpy()
    for k, w in enumerate((1, 7, 30)):
        np.testing.assert_array_equal(nb[k], cols[f"CUSTOMER_ID_NB_TX_{w}DAY_WINDOW"][order])
        _close(avg[k], cols[f"CUSTOMER_ID_AVG_AMOUNT_{w}DAY_WINDOW"][order])


def test_scan_nan_amounts_empty_and_long_segments(dev):
    """NaN amounts (pandas skips them: count and sum of the non-NaN rows, NaN average when a
    window holds none), customers without rows, and hot customers of 3,000+ rows (the global
    prefix path) -- against the C oracle (pandas' roll_sum restated)."""
    rng = np.random.default_rng(8)
    n_cust = 40
    lens = rng.integers(0, 60, n_cust)
    lens[[3, 17]] = [3100, 1500]   # longer than the 1,024-row LDS stage
    lens[[5, 6]] = 0               # empty customers
    seg = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    n = int(seg[-1])
    ts = np.empty(n, np.int64)
    for s in range(n_cust):
        a, b = seg[s], seg[s + 1]
        ts[a:b] = np.sort(rng.integers(0, 40 * 86400, b - a)) * 1_000_000_000
    amt = np.round(rng.uniform(1, 200, n), 2)
    amt[rng.random(n) < 0.05] = np.nan
    onb, oavg = oracle.customer_windows(ts, amt, seg)
    nb, avg = ops.customer_windows_scan(T(ts, torch.int64, dev), T(amt, torch.float64, dev), T(seg, torch.int64, dev))
    np.testing.assert_array_equal(nb.cpu().numpy(), onb)
    _close(avg.cpu().numpy(), oavg)


def test_scan_slot_layout_equals_grouped_and_fused_path_is_consistent(dev, golden):
    """customer_windows_scan(lay=...) writes the walk's slot layout (NB, SUM): the same values
    as the grouped form; and FraudPipeline(avg_mode="scan").run_fused equals featurize(scan)
    + float64 X + Forest.predict on every row, bit for bit (the average is SUM / NB in both)."""
    z = golden("forest_rf5d8.npz")
    arrays = {k: z[k] for k in ("left", "right", "feature", "threshold", "missing_left", "value1", "node_offsets")}
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    d = synth.generate(n_customers=2000, n_terminals=4000, nb_days=80, seed=31)
    n = len(d["ts"])
    args = (T(d["ts"], torch.int64, dev), T(d["customer"], torch.int32, dev), T(d["terminal"], torch.int32, dev),
            T(d["amount"], torch.float64, dev), T(d["fraud"], torch.uint8, dev))
    cperm, cseg, gts, gamt = ops.rekey_payload(args[1], 2000, args[0], args[3])
    lay = ops.customer_layout(cseg, cperm, gts, gamt, 3, grouped=True)
    snb, ssum = ops.customer_windows_scan(gts, gamt, cseg, lay=lay)
    gnb, gsum = ops.customer_windows_scan(gts, gamt, cseg, val_is_sum=True)
    irow = lay.irow[: lay.n_slots].cpu().numpy()
    real = irow >= 0
    inv = np.empty(n, np.int64)
    inv[cperm.cpu().numpy()] = np.arange(n)
    g = inv[irow[real]]
    np.testing.assert_array_equal(snb.cpu().numpy()[:, real], gnb.cpu().numpy()[:, g])
    np.testing.assert_array_equal(ssum.cpu().numpy()[:, real], gsum.cpu().numpy()[:, g])
    pipe = FraudPipeline(forest=forest, avg_mode="scan")
    feats = pipe.featurize(*args, 2000, 4000)
    p_ref = pipe.score(feats.X).cpu().numpy()
    p = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, 2000, 4000, p, ops.workspace(forest.workspace_size(n * 2), dev))
    np.testing.assert_array_equal(p.cpu().numpy(), p_ref)
    # the customer averages against the exact pipeline's, within RTOL
    Xe = FraudPipeline(forest=forest).featurize(*args, 2000, 4000).X.cpu().numpy()
    Xs = feats.X.cpu().numpy()
    np.testing.assert_array_equal(Xs[:, [3, 5, 7]], Xe[:, [3, 5, 7]])
    for c in (4, 6, 8):
        _close(Xs[:, c], Xe[:, c])
    np.testing.assert_array_equal(Xs[:, 9:15], Xe[:, 9:15])


def test_scan_config2_against_exact_pipeline(dev):
    """configs[1] at full size (17.7M tx): the scan-mode fused scores against the exact ones.
    The averages differ from pandas' only in the last bits, so a scaled feature can land on
    the other side of a float32 threshold on a handful of rows (2 of 1.75M at
    config 1); every other row's probability is identical."""
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    g = synth.generate_device(50_000, 100_000, 183, seed=1234, device=dev)
    n = g["ts"].numel()
    args = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"])
    ws = ops.workspace(forest.workspace_size(n * 11 // 10), dev)
    pe = torch.empty(n, dtype=torch.float64, device=dev)
    ps = torch.empty(n, dtype=torch.float64, device=dev)
    FraudPipeline(forest=forest).run_fused(*args, 50_000, 100_000, pe, ws)
    FraudPipeline(forest=forest, avg_mode="scan").run_fused(*args, 50_000, 100_000, ps, ws)
    diff = int((pe != ps).sum())
    assert diff <= n // 100_000, f"{diff} of {n} rows scored differently"
