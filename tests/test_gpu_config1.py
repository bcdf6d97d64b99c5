"""BASELINE.json configs[0] on the GPU: the handbook-default set (5k customers / 10k terminals /
183 days, ~1.75M tx) + DecisionTree(max_depth=2) scoring (model_training.ipynb:1276-1280), and
the reference's own config-1 rows behind the values its notebook printed.

  * notebook known answers: the reference generator's rows behind the values printed in
    feature_transformation.ipynb (:1414-1440 tx 2051326, :1798-1863 tx 3527 / 9583 / row
    10355, :3013-3031 latest terminal rows, ...), featurized by FraudPipeline.featurize and by
    the pandas drop-ins (driven like the notebook, :1092-1093 / :2435-2436), every printed
    value to its printed decimals -- the same check tests/test_oracle_golden.py applies to the
    CPU oracle;
  * a 5k / 10k / 183-day synthetic set (the handbook distributions, fdx.synth.generate_device):
    every feature of every row equal to the C oracle; the fused scoring path's
    probabilities equal to the float64 path's on every row and to the oracle forest on the
    oracle's features, for DT(depth 2) (configs[0]'s model) and the RF(100, depth 20) bench
    model.
"""
import os

import numpy as np
import pandas as pd
import pytest
import torch

import fdx
import oracle
from fdx import ops, synth
from fdx.pipeline import FraudPipeline
from kat_check import check_notebook_kat

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FEATS = oracle.INPUT_FEATURES


def T(a, dt, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)


def test_notebook_known_answers_pipeline(dev):
    """FraudPipeline.featurize (re-keys, customer / terminal windows, flags, assembly)."""
    pipe = FraudPipeline()

    def featurize(ts, c, t, a, fr, tids):
        f = pipe.featurize(T(ts, torch.int64, dev), T(c, torch.int32, dev), T(t, torch.int32, dev),
                           T(a, torch.float64, dev), T(fr, torch.uint8, dev), int(c.max()) + 1, int(t.max()) + 1)
        X = f.X.cpu().numpy()
        assert np.array_equal(X[:, 0], a)
        return {name: X[:, j] for j, name in enumerate(FEATS)}

    assert check_notebook_kat(featurize) >= 500


def test_notebook_known_answers_dropins(dev):
    """The pandas drop-ins driven exactly like the notebook: groupby-free whole-frame calls,
    sort_values('TX_DATETIME') between them (:1093, :2436), flags by is_weekend / is_night."""

    def featurize(ts, c, t, a, fr, tids):
        df = pd.DataFrame({"TRANSACTION_ID": tids, "TX_DATETIME": pd.to_datetime(ts, unit="ns"),
                           "CUSTOMER_ID": c, "TERMINAL_ID": t, "TX_AMOUNT": a, "TX_FRAUD": fr})
        df["TX_DURING_WEEKEND"] = fdx.is_weekend(df.TX_DATETIME)
        df["TX_DURING_NIGHT"] = fdx.is_night(df.TX_DATETIME)
        out = fdx.get_customer_spending_behaviour_features(df, windows_size_in_days=[1, 7, 30])
        out = out.sort_values("TX_DATETIME", kind="stable").reset_index(drop=True)
        out = fdx.get_count_risk_rolling_window(out, delay_period=7, windows_size_in_days=[1, 7, 30],
                                                feature="TERMINAL_ID")
        out = out.sort_values("TX_DATETIME", kind="stable").reset_index(drop=True)
        out = out.set_index("TRANSACTION_ID").loc[tids]
        return {name: out[name].values for name in FEATS[1:]}

    assert check_notebook_kat(featurize) >= 500


@pytest.fixture(scope="module")
def config1(dev):
    g = synth.generate_device(5_000, 10_000, 183, seed=20240601, device=dev)
    d = {k: g[k].cpu().numpy() for k in ("ts", "customer", "terminal", "amount", "fraud")}
    assert 1_500_000 < len(d["ts"]) < 2_100_000
    ref = oracle.featurize_arrays(d["ts"], d["customer"], d["terminal"], d["amount"], d["fraud"])
    Xo = np.column_stack([d["amount"]] + [ref[c] for c in FEATS[1:]])
    return g, d, Xo


def test_config1_every_feature_of_every_row(dev, config1):
    g, d, Xo = config1
    pipe = FraudPipeline()
    X = pipe.featurize(g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 5_000, 10_000).X.cpu().numpy()
    for j, c in enumerate(FEATS):
        np.testing.assert_array_equal(X[:, j], Xo[:, j], err_msg=c)


def _load(name):
    if name == "dt2":
        z = np.load(os.path.join(ROOT, "tests", "golden", "forest_dt2.npz"))
    else:
        z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    return arrays, z["mean"], z["scale"]


@pytest.mark.parametrize("model", ["dt2", "rf100_d20"])
def test_config1_scoring_fused_vs_f64_vs_oracle(dev, config1, model):
    """configs[0]'s DecisionTree(max_depth=2) and the bench RF: fused path == float64 path on
    every row; == the oracle forest on the oracle's features (every row for DT2, 200k sampled
    rows for the RF)."""
    g, d, Xo = config1
    arrays, mean, scale = _load(model)
    forest = ops.Forest(arrays, 15, mean, scale)
    pipe = FraudPipeline(forest=forest)
    n = len(d["ts"])
    args = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 5_000, 10_000)
    fused = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, fused)
    _, p64 = pipe.run(*args)
    fused, p64 = fused.cpu().numpy(), p64.cpu().numpy()
    np.testing.assert_array_equal(fused, p64)
    sel = np.arange(n) if model == "dt2" else np.random.default_rng(3).choice(n, 200_000, replace=False)
    np.testing.assert_array_equal(fused[sel], oracle.forest_predict(Xo[sel], arrays, mean, scale))
    if model == "dt2":  # a depth-2 tree has 4 leaves: every one of them must be reached
        assert len(np.unique(fused)) >= 3


@pytest.mark.parametrize("order", ["input", "slot"])
def test_config1_featurized_table_rows(dev, config1, order):
    """run_fused(rows_out=...): the featurized table the reference writes
    (feature_transformation.ipynb:2890-2905) from the scoring path's own assembly pass -- one
    fdx_feature_row per transaction, by input row or by scoring slot (each record carrying its
    row) -- equal to the C oracle on every feature of every row (counts as exact integers,
    averages / risks bit for bit, flags), and the scores unchanged by emitting it."""
    g, d, Xo = config1
    arrays, mean, scale = _load("rf100_d20")
    pipe = FraudPipeline(forest=ops.Forest(arrays, 15, mean, scale))
    n = len(d["ts"])
    args = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 5_000, 10_000)
    rows = ops.FeatureTable(n * 11 // 10, dev) if order == "slot" else ops.FeatureRecords(n, dev)
    rows.buf.fill_(0xAB)
    p_rows = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, p_rows, rows_out=rows)
    p_plain = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, p_plain)
    assert torch.equal(p_rows, p_plain)
    if order == "slot":  # slots 0..n_slots-1: every row exactly once, padding slots row -1 and zero
        m = pipe.last_slots
        assert n <= m <= rows.cap
        col = {k: v.cpu().numpy() for k, v in rows.columns(m).items()}
        real = col["row"] >= 0
        assert real.sum() == n and not col["cust_nb"][:, ~real].any() and not col["term_risk"][:, ~real].any()
        assert not col["weekend"][~real].any() and not col["night"][~real].any()
        o = np.argsort(col["row"][real], kind="stable")
        col = {k: (v[..., real][..., o]) for k, v in col.items()}
    else:
        col = {k: v.cpu().numpy() for k, v in rows.columns().items()}
    np.testing.assert_array_equal(col["row"], np.arange(n, dtype=np.int32))
    np.testing.assert_array_equal(col["weekend"], Xo[:, 1].astype(np.uint8))
    np.testing.assert_array_equal(col["night"], Xo[:, 2].astype(np.uint8))
    for w in range(3):
        np.testing.assert_array_equal(col["cust_nb"][w], Xo[:, 3 + 2 * w].astype(np.int32))
        np.testing.assert_array_equal(col["cust_avg"][w].view(np.int64), Xo[:, 4 + 2 * w].view(np.int64))
        np.testing.assert_array_equal(col["term_nb"][w], Xo[:, 9 + 2 * w].astype(np.int32))
        np.testing.assert_array_equal(col["term_risk"][w].view(np.int64), Xo[:, 10 + 2 * w].view(np.int64))
    small = ops.FeatureTable(64, dev) if order == "slot" else ops.FeatureRecords(n - 1, dev)
    with pytest.raises(ValueError):
        pipe.run_fused(*args, p_rows, rows_out=small)


def _many_threshold_forest():
    """14 complete depth-11 trees whose 28,658 internal nodes all test TX_AMOUNT at distinct
    thresholds: more than the 26,240 thresholds per searched feature whose S-tree fits
    k_zfill_grouped_w3's LDS budget, within rank layout v1's 32,766."""
    rng = np.random.default_rng(5)
    L, R, F, TH, ML, V, off = [], [], [], [], [], [], [0]
    thr = rng.permutation(np.unique(np.round(rng.uniform(-1.2, 3.0, 60_000), 6)))[: 14 * 2047]
    k = 0
    for _ in range(14):
        left, right, feat, th, ml, val = [], [], [], [], [], []

        def build(d):
            nonlocal k
            i = len(left)
            left.append(-1); right.append(-1); feat.append(-2); th.append(-2.0); ml.append(0)
            val.append(float(rng.integers(0, 1000)) / 999.0)
            if d < 11:
                feat[i] = 0
                th[i] = float(thr[k])
                k += 1
                left[i] = build(d + 1)
                right[i] = build(d + 1)
            return i

        build(0)
        L += left; R += right; F += feat; TH += th; ML += ml; V += val
        off.append(off[-1] + len(left))
    arrays = dict(left=np.array(L, np.int64), right=np.array(R, np.int64), feature=np.array(F, np.int64),
                  threshold=np.array(TH), missing_left=np.array(ML, np.uint8), value1=np.array(V),
                  node_offsets=np.array(off, np.int64))
    return arrays


@pytest.mark.parametrize("order", ["input", "slot"])
def test_featurized_table_without_search_trees(dev, config1, order):
    """the featurized table must not depend on the scoring rows' LDS budget.  A forest
    whose searched feature has too many thresholds for k_zfill_grouped_w3's S-trees is scored
    through the general assembly (k_zfill_grouped) and its table written by k_feature_rows:
    every feature of every row equal to the C oracle, scores equal to the float64 path's."""
    from table_check import assert_same_features, table_as_X

    g, d, Xo = config1
    _, mean, scale = _load("rf100_d20")
    arrays = _many_threshold_forest()
    forest = ops.Forest(arrays, 15, mean, scale)
    import ctypes

    from fdx import _lib
    lay, ns = ctypes.c_int32(), ctypes.c_int32()
    _lib.load().fdx_forest_layout(forest._h, ctypes.byref(lay), ctypes.byref(ns))
    assert lay.value == 1  # rank layout v1 (ranks fit), S-trees refused by their LDS budget
    pipe = FraudPipeline(forest=forest)
    n = len(d["ts"])
    args = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 5_000, 10_000)
    rows = ops.FeatureTable(n * 11 // 10, dev) if order == "slot" else ops.FeatureRecords(n, dev)
    rows.buf.fill_(0xAB)
    p = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, p, rows_out=rows)
    _, p64 = pipe.run(*args)
    np.testing.assert_array_equal(p.cpu().numpy(), p64.cpu().numpy())
    if order == "slot":
        Xt = table_as_X(rows, pipe.last_slots, d["amount"])
    else:
        col = {k: v.cpu().numpy() for k, v in rows.columns().items()}
        np.testing.assert_array_equal(col["row"], np.arange(n, dtype=np.int32))
        Xt = np.zeros((n, 15))
        Xt[:, 0] = d["amount"]
        Xt[:, 1], Xt[:, 2] = col["weekend"], col["night"]
        for w in range(3):
            Xt[:, 3 + 2 * w], Xt[:, 4 + 2 * w] = col["cust_nb"][w], col["cust_avg"][w]
            Xt[:, 9 + 2 * w], Xt[:, 10 + 2 * w] = col["term_nb"][w], col["term_risk"][w]
    assert_same_features(Xt, Xo, f"table ({order} order) without S-trees vs oracle")


def test_serving_snapshots_from_the_step_table(dev, config1):
    """the featurized table the scoring step writes has a consumer.  The serving
    snapshots built straight from run_fused's FeatureTable (fdx_table_select) equal the
    reference's pandas expressions on the featurized frame (the oracle's features, the
    notebook's column order, time order):
      latest per terminal  feature_transformation.ipynb:2914-2918
      customers of a date  :3606-3635 (lower-case, filter, date rows, dt, drop_duplicates)"""
    import datetime

    from fdx import serving

    g, d, Xo = config1
    arrays, mean, scale = _load("rf100_d20")
    pipe = FraudPipeline(forest=ops.Forest(arrays, 15, mean, scale))
    n = len(d["ts"])
    args = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 5_000, 10_000)
    rows = ops.FeatureTable(n * 11 // 10, dev)
    p = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, p, rows_out=rows)
    m = pipe.last_slots
    # the reference's featurized frame (time order, the notebook's columns)
    df = pd.DataFrame({"TRANSACTION_ID": np.arange(n), "TX_DATETIME": d["ts"].astype("datetime64[ns]"),
                       "CUSTOMER_ID": d["customer"], "TERMINAL_ID": d["terminal"], "TX_AMOUNT": d["amount"],
                       "TX_FRAUD": d["fraud"]})
    for j, c in enumerate(FEATS[1:], start=1):
        df[c] = Xo[:, j]
    df["TX_DURING_WEEKEND"] = df["TX_DURING_WEEKEND"].astype(np.int64)
    df["TX_DURING_NIGHT"] = df["TX_DURING_NIGHT"].astype(np.int64)
    want = df.loc[df.groupby("TERMINAL_ID").TX_DATETIME.idxmax()].filter(regex="TERMINAL_ID|TERMINAL_ID_RISK")
    got = serving.latest_terminal_features_from_table(rows, m, g["ts"], g["terminal"], 10_000)
    pd.testing.assert_frame_equal(got, want, check_dtype=False, check_exact=True, check_index_type=False)
    for day in (datetime.date(2024, 6, 2), datetime.date(2024, 8, 15), datetime.date(2024, 11, 29)):
        low = df.copy()
        low.columns = map(str.lower, low.columns)
        low = low.filter(regex="customer_id|tx_datetime")
        low = low[low.tx_datetime.dt.date == day].copy()
        low["dt"] = day
        want_c = low.drop(columns=["tx_datetime"]).drop_duplicates(subset=["customer_id"])
        got_c = serving.customer_features_on_from_table(rows, m, g["ts"], g["customer"], 5_000, day)
        assert len(got_c) > 100, day
        pd.testing.assert_frame_equal(got_c, want_c, check_dtype=False, check_exact=True, check_index_type=False)
    # the frame's own ids through a dense-key -> id map, int64 like pandas' id column;
    # a slot count past the table, or ts / key of different lengths, are refused
    ids = np.arange(10_000, dtype=np.int64) * 7 + 1_000
    got_i = serving.latest_terminal_features_from_table(rows, m, g["ts"], g["terminal"], 10_000, ids=ids)
    assert got_i["TERMINAL_ID"].dtype == np.int64
    np.testing.assert_array_equal(got_i["TERMINAL_ID"].values, ids[want["TERMINAL_ID"].values])
    with pytest.raises(ValueError, match="n_slots"):
        serving.table_select(rows, rows.cap + 64, g["ts"], g["terminal"], 10_000, 0)
    with pytest.raises(ValueError, match="rows"):
        serving.table_select(rows, m, g["ts"][:-1], g["terminal"], 10_000, 0)
