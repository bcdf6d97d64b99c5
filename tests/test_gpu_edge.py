"""Edge cases of the hot path on the GPU (through the C ABI), against the C oracle:
an empty table, a single row, one customer / one terminal holding every row (segments far
longer than every LDS stage), all-tied timestamps, id ranges with many empty segments, and
the drop-in frames at those sizes."""
import numpy as np
import pandas as pd
import pytest
import torch

import oracle
from fdx import ops
from fdx.pipeline import FraudPipeline
from table_check import assert_same_features, table_as_X

pytestmark = pytest.mark.gpu
NS = 1_000_000_000
CUST_COLS, TERM_COLS = oracle.CUSTOMER_COLS, oracle.TERMINAL_COLS


def T(a, dt, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)


def _forest(golden):
    z = golden("forest_rf5d8.npz")
    arrays = {k: z[k] for k in ("left", "right", "feature", "threshold", "missing_left", "value1", "node_offsets")}
    return ops.Forest(arrays, 15, z["mean"], z["scale"]), arrays, z


def _check(d, X, n_c, n_t):
    f = oracle.featurize_arrays(d["ts"], d["customer"], d["terminal"], d["amount"], d["fraud"])
    np.testing.assert_array_equal(X[:, 1], f["TX_DURING_WEEKEND"])
    np.testing.assert_array_equal(X[:, 2], f["TX_DURING_NIGHT"])
    for j, c in enumerate(CUST_COLS):
        np.testing.assert_array_equal(X[:, 3 + j], f[c], err_msg=c)
    for j, c in enumerate(TERM_COLS):
        np.testing.assert_array_equal(X[:, 9 + j], f[c], err_msg=c)


def _run_all(dev, golden, d, n_c, n_t):
    """featurize (exact and scan), run_fused vs featurize + predict; returns X."""
    forest, arrays, z = _forest(golden)
    args = (T(d["ts"], torch.int64, dev), T(d["customer"], torch.int32, dev), T(d["terminal"], torch.int32, dev),
            T(d["amount"], torch.float64, dev), T(d["fraud"], torch.uint8, dev))
    n = len(d["ts"])
    pipe = FraudPipeline(forest=forest)
    feats = pipe.featurize(*args, n_c, n_t)
    X = feats.X.cpu().numpy()
    assert X.shape == (n, 15)
    p_ref = pipe.score(feats.X).cpu().numpy()
    p = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
    # the fused path (interleave + walk + assembly: the kernels the bench times) writes its own
    # featurized table; every feature of every row must equal the oracle's, not only the proba
    rows = ops.FeatureTable(max(n, 1) * 21 + 4096, dev)  # (a lone long customer pads its group of 21)
    rows.buf.fill_(0xAB)
    pipe.run_fused(*args, n_c, n_t, p, ops.workspace(forest.workspace_size(max(n, 1) * 2 + 4096), dev),
                   rows_out=rows)
    np.testing.assert_array_equal(p.cpu().numpy(), p_ref)
    if n:
        np.testing.assert_array_equal(p_ref, oracle.forest_predict(X, arrays, z["mean"], z["scale"]))
        Xt = table_as_X(rows, pipe.last_slots, d["amount"])
        _check(d, Xt, n_c, n_t)
        assert_same_features(Xt, X, "fused table vs featurize")
    Xs = FraudPipeline(forest=forest, avg_mode="scan").featurize(*args, n_c, n_t).X.cpu().numpy()
    np.testing.assert_array_equal(Xs[:, [0, 1, 2, 3, 5, 7, 9, 10, 11, 12, 13, 14]],
                                  X[:, [0, 1, 2, 3, 5, 7, 9, 10, 11, 12, 13, 14]])
    return X


def test_empty_table(dev, golden):
    d = {k: np.zeros(0, dt) for k, dt in (("ts", np.int64), ("customer", np.int32), ("terminal", np.int32),
                                          ("amount", np.float64), ("fraud", np.uint8))}
    X = _run_all(dev, golden, d, 10, 10)
    assert X.shape == (0, 15)
    forest, _, _ = _forest(golden)
    assert forest.predict(torch.zeros((0, 15), dtype=torch.float64, device=dev)).numel() == 0


def test_single_row(dev, golden):
    d = {"ts": np.array([5 * 86400 * NS + 3 * 3600 * NS], np.int64), "customer": np.array([2], np.int32),
         "terminal": np.array([7], np.int32), "amount": np.array([42.5]), "fraud": np.array([1], np.uint8)}
    X = _run_all(dev, golden, d, 5, 9)
    _check(d, X, 5, 9)


def test_one_customer_one_terminal_long_segments(dev, golden):
    """Every row on one customer and one terminal: 6,000-row segments (past the 1,024-row LDS
    stages of the layout starts, the scan and the terminal kernel), bursts of equal
    timestamps, and 3 % fraud."""
    rng = np.random.default_rng(12)
    n = 6000
    ts = np.sort(rng.integers(0, 90 * 86400, n)) * NS
    ts[100:140] = ts[100]                               # a burst of equal timestamps
    d = {"ts": ts.astype(np.int64), "customer": np.zeros(n, np.int32), "terminal": np.zeros(n, np.int32),
         "amount": np.round(rng.uniform(1, 300, n), 2), "fraud": (rng.random(n) < 0.03).astype(np.uint8)}
    X = _run_all(dev, golden, d, 1, 1)
    _check(d, X, 1, 1)


def test_walk_rings_overflow_at_chunk_boundaries(dev, golden):
    """Customers whose 30-day windows hold more rows than the customer walk's LDS rings (128
    rows in the short class, 256 in the long class, which takes groups whose longest customer
    has >= 480 rows): lengths on both sides of 16-row chunk, ring and class boundaries, dense in
    time so that every window is full, beside a crowd of short customers; then the fused path's
    own featurized table row by row against the oracle (a ring overwrite that moves
    no leaf must still fail a test)."""
    rng = np.random.default_rng(21)
    lens = [15, 16, 17, 127, 128, 129, 255, 256, 257, 300, 479, 480, 481, 700, 1500]
    cust, ts = [], []
    for c, m in enumerate(lens):  # m rows within 20 days: all inside the 30-day window
        cust.append(np.full(m, c))
        ts.append(rng.integers(40 * 86400, 60 * 86400, m))
    n_small = 3000
    cust.append(len(lens) + rng.integers(0, 400, n_small))
    ts.append(rng.integers(0, 90 * 86400, n_small))
    cust, ts = np.concatenate(cust), np.concatenate(ts)
    o = np.argsort(ts, kind="stable")
    n = len(o)
    d = {"ts": (ts[o] * NS).astype(np.int64), "customer": cust[o].astype(np.int32),
         "terminal": rng.integers(0, 50, n).astype(np.int32), "amount": np.round(rng.uniform(1, 300, n), 2),
         "fraud": (rng.random(n) < 0.05).astype(np.uint8)}
    d["ts"][500:530] = d["ts"][500]  # ties inside the busy windows
    X = _run_all(dev, golden, d, len(lens) + 400, 50)
    _check(d, X, len(lens) + 400, 50)


def test_all_rows_same_timestamp(dev, golden):
    """All rows at one instant: every window holds every earlier-tied row (closed='right'
    includes the tie), the delayed terminal windows hold none."""
    rng = np.random.default_rng(3)
    n = 500
    d = {"ts": np.full(n, 40 * 86400 * NS, np.int64), "customer": rng.integers(0, 7, n).astype(np.int32),
         "terminal": rng.integers(0, 5, n).astype(np.int32), "amount": np.round(rng.uniform(1, 300, n), 2),
         "fraud": (rng.random(n) < 0.2).astype(np.uint8)}
    X = _run_all(dev, golden, d, 7, 5)
    _check(d, X, 7, 5)


def test_sparse_ids_many_empty_segments(dev, golden):
    """2,000 rows over id ranges of 200,000 customers and 300,000 terminals (most segments
    empty; the re-key's widest digit counts)."""
    rng = np.random.default_rng(4)
    n = 2000
    d = {"ts": np.sort(rng.integers(0, 60 * 86400, n)).astype(np.int64) * NS,
         "customer": rng.integers(0, 200_000, n).astype(np.int32),
         "terminal": rng.integers(0, 300_000, n).astype(np.int32),
         "amount": np.round(rng.uniform(1, 300, n), 2), "fraud": (rng.random(n) < 0.1).astype(np.uint8)}
    X = _run_all(dev, golden, d, 200_000, 300_000)
    _check(d, X, 200_000, 300_000)


def test_dropin_frames_empty_and_single(dev):
    """The reference's per-group functions on an empty frame and on a one-row frame."""
    from fdx import features

    cols = ["TRANSACTION_ID", "TX_DATETIME", "CUSTOMER_ID", "TERMINAL_ID", "TX_AMOUNT", "TX_FRAUD"]
    one = pd.DataFrame({"TRANSACTION_ID": [0], "TX_DATETIME": [pd.Timestamp("2024-06-03 10:00:00")],
                        "CUSTOMER_ID": [3], "TERMINAL_ID": [4], "TX_AMOUNT": [12.0], "TX_FRAUD": [0]})
    c = features.get_customer_spending_behaviour_features(one)
    assert c["CUSTOMER_ID_NB_TX_1DAY_WINDOW"].tolist() == [1.0]
    assert c["CUSTOMER_ID_AVG_AMOUNT_30DAY_WINDOW"].tolist() == [12.0]
    t = features.get_count_risk_rolling_window(one)
    assert t["TERMINAL_ID_NB_TX_7DAY_WINDOW"].tolist() == [0.0]
    assert t["TERMINAL_ID_RISK_7DAY_WINDOW"].tolist() == [0.0]
    empty = one.iloc[:0][cols]
    assert len(features.get_customer_spending_behaviour_features(empty)) == 0
    assert len(features.get_count_risk_rolling_window(empty)) == 0


def test_sharded_rank_without_rows(dev, golden):
    """A rank whose customer range holds no rows still takes part in the exchange (RCCL,
    world 1) and returns an empty result."""
    import os
    import socket

    import torch.distributed as dist

    from fdx.distributed import ShardedPipeline

    forest, _, _ = _forest(golden)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        sp = ShardedPipeline(FraudPipeline(forest=forest), 1, 0, 100, customer_base=50, n_customers_local=10)
        e = lambda dt: torch.zeros(0, dtype=dt, device=dev)  # noqa: E731
        p = sp.run(e(torch.int64), e(torch.int32), e(torch.int32), e(torch.float64), e(torch.uint8),
                   e(torch.float64), ops.workspace(forest.workspace_size(4096), dev))
        assert p.numel() == 0
        X = sp.featurize(e(torch.int64), e(torch.int32), e(torch.int32), e(torch.float64), e(torch.uint8))
        assert X.shape == (0, 15)
    finally:
        dist.destroy_process_group()


def test_arena_reuse_across_steps(dev, golden):
    """run_fused keeps its intermediates in an arena of the pipeline's own (ops.Arena): steps of
    different sizes enqueued back to back on one pipeline (the arena grows, then serves smaller
    steps from larger buffers, the two re-keys share one scratch buffer) give every table the
    probabilities and featurized table of a fresh pipeline; a steady run allocates nothing."""
    from fdx import synth

    forest, _, _ = _forest(golden)
    tabs = [synth.generate_device(n_c, 2 * n_c, days, seed=s, device=dev)
            for n_c, days, s in ((3000, 60, 1), (800, 20, 2), (3000, 60, 3))]
    n_max = max(g["ts"].numel() for g in tabs)
    ws = ops.workspace(forest.workspace_size(n_max * 2 + 4096), dev)
    want = []
    for g in tabs:  # fresh pipeline per table
        n = g["ts"].numel()
        p = torch.empty(n, dtype=torch.float64, device=dev)
        rows = ops.FeatureTable(n * 2 + 4096, dev)
        pf = FraudPipeline(forest=forest)
        pf.run_fused(g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 3000, 6000, p, ws, rows_out=rows)
        torch.cuda.synchronize()
        want.append((p.cpu().numpy(), table_as_X(rows, pf.last_slots, g["amount"].cpu().numpy())))
    pipe = FraudPipeline(forest=forest)
    outs = []
    for g in tabs + tabs:  # no host synchronisation between the steps
        n = g["ts"].numel()
        p = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
        rows = ops.FeatureTable(n * 2 + 4096, dev)
        pipe.run_fused(g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 3000, 6000, p,
                       ops.workspace(forest.workspace_size(n * 2 + 4096), dev), rows_out=rows)
        outs.append((p, rows, pipe.last_slots, g))
    torch.cuda.synchronize()
    for k, (p, rows, slots, g) in enumerate(outs):
        np.testing.assert_array_equal(p.cpu().numpy(), want[k % 3][0], err_msg=f"step {k}")
        assert_same_features(table_as_X(rows, slots, g["amount"].cpu().numpy()), want[k % 3][1], f"step {k}")
    nb = pipe._arena.nbytes
    g = tabs[0]
    p = torch.empty(g["ts"].numel(), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    stats0 = torch.cuda.memory_stats(dev).get("num_device_alloc", 0)
    pipe.run_fused(g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 3000, 6000, p, ws)
    torch.cuda.synchronize()
    assert pipe._arena.nbytes == nb
    assert torch.cuda.memory_stats(dev).get("num_device_alloc", 0) == stats0
